"""The benchmark configurations of BASELINE.json as concrete key vectors.

Each config is restated from the reference's own call paths:

C1  generator --puts 100000 (seed 13141), tree flags -b 100 -r 10: the buffer
    holds 100*4096/8 = 51,200 entries (src/main.cpp:89); the first flush is a
    run of the first 51,200 DISTINCT keys (Buffer::put, src/buffer.cpp:37-58),
    written sorted as entry_t {key, val} (src/lsm_tree.cpp:124-129) — an AoS
    run read at stride 8.  m = (long)(51200 * 10.0f) (src/run.cpp:15).
C2  one run of 16,777,216 keys (generator --puts 16777216), 10 bits/key.
C3  generator --puts 22347776 --gets 16777216 --gets-skewness 0.2
    --gets-misses-ratio 0.3; tree -b 128 -d 5 -f 4 -r 10: level i holds one run
    of capacity 65,536*4^i (src/lsm_tree.cpp:28-42); level 4 (oldest) is built
    from puts[0, 16.78M), level 3 the next 4.19M, ... level 0 the newest
    65,536.  Every GET probes all five filters.
C4  one run of 268,435,456 keys, 12 bits/key.
C5  runs r = 0..7 of 67,108,864 keys each (generator seed 13141 + r), 10 bits/key.
F10 the reference's own published tree (doc/final/final.tex:195-212: b = 1000,
    t = 4, f = 10) at -r 10: the buffer holds 1000*4096/8 = 512,000 entries
    (src/main.cpp:89), level i one run of capacity 512,000*10^i
    (src/lsm_tree.cpp:36-41), so m_i = 5,120,000*10^i bits (src/run.cpp:15):
    15625 << 15 for level 2 -- an odd part 625*5^i, which no d | 255 p2 or
    ladder path covers.  f10_build: 16,777,216 keys into level 2's filter
    (m = 512,000,000); f10: 16.8M GETs (skew 0.2, misses 0.3, as C3) against
    full runs of levels 0..2.

k = 3 everywhere: the reference has three fixed hashes and no k parameter
(src/bloom_filter.h:8-10), so config 2's "k=7" is not expressible bit-exactly.
"""
from __future__ import annotations

import numpy as np

from . import gen_puts, gen_workload, m_bits

SEED = 13141

C2_N = 16_777_216
C2_BPE = 10.0
C3_PUTS = 22_347_776
C3_GETS = 16_777_216
C3_LEVELS = 5
C3_BASE_CAP = 65_536
C3_FANOUT = 4
C4_N = 268_435_456
C4_BPE = 12.0
C5_N = 67_108_864
C5_RUNS = 8
F10_BUFFER = 1000 * 4096 // 8   # -b 1000: buffer_max_entries, src/main.cpp:89
F10_FANOUT = 10
F10_LEVELS = 3
F10_BPE = 10.0
F10_BUILD_N = 16_777_216


def c1_run(n_puts: int = 100_000, buffer_entries: int = 51_200, seed: int = SEED):
    """(AoS entry_t run as int32[n, 2], m) for the first buffer flush."""
    keys, vals = gen_puts(seed, n_puts, with_vals=True)
    seen = {}
    for k, v in zip(keys.tolist(), vals.tolist()):
        if k in seen:
            seen[k] = v          # Buffer::put updates an existing key
            continue
        if len(seen) == buffer_entries:
            break                # buffer full: the flush happens here
        seen[k] = v
    items = sorted(seen.items())
    run = np.array(items, dtype=np.int32).reshape(-1, 2)
    return run, m_bits(buffer_entries, 10.0)


def c2(seed: int = SEED, n: int = C2_N):
    return gen_puts(seed, n), m_bits(n, C2_BPE)


def c3_caps():
    return [C3_BASE_CAP * C3_FANOUT ** i for i in range(C3_LEVELS)]


def c3(seed: int = SEED):
    """(gets, [(level, keys, m) for level 0..4]) — level 0 is the newest run."""
    puts, gets = gen_workload(seed, C3_PUTS, C3_GETS, 0.2, 0.3)
    caps = c3_caps()
    levels = []
    start = 0
    for lvl in reversed(range(C3_LEVELS)):   # oldest (largest) run first in the stream
        cap = caps[lvl]
        levels.append((lvl, puts[start:start + cap], m_bits(cap, 10.0)))
        start += cap
    levels.sort(key=lambda t: t[0])
    return gets, levels


def c3_runs(seed: int = SEED):
    """(gets, [(level, run_keys, m)]) with each level's run as the reference
    writes it: its distinct keys in ascending order (a flush sorts the buffer,
    src/lsm_tree.cpp:124-129; a merge emits sorted, deduplicated output,
    src/merge.cpp:6-39).  Same filters as c3(): set() is idempotent."""
    gets, levels = c3(seed)
    return gets, [(lvl, np.unique(keys), m) for lvl, keys, m in levels]


def compaction_fanin(seed: int = SEED, fanout: int = 4, cap: int = C2_N // 4):
    """A level's compaction fan-in (LSMTree::merge_down, src/lsm_tree.cpp:48-95):
    `fanout` runs of `cap` entries each (generator --puts streams, seeds seed+j,
    each run its distinct keys ascending with their last-written values, as a
    flush writes it), newest first, merged into one run whose filter is sized
    for fanout * cap entries at 10 bits/key (C2's m for the defaults)."""
    runs = []
    for j in range(fanout):
        keys, vals = gen_puts(seed + j, cap, with_vals=True)
        # the newest value of a repeated key: last occurrence in the stream
        rk, rv = keys[::-1], vals[::-1]
        uk, first = np.unique(rk, return_index=True)
        runs.append(np.ascontiguousarray(np.stack([uk, rv[first]], axis=1)))
    return runs, m_bits(fanout * cap, C2_BPE)


def c4(seed: int = SEED, n: int = C4_N):
    return gen_puts(seed, n), m_bits(n, C4_BPE)


def c5_run(r: int, n: int = C5_N):
    return gen_puts(SEED + r, n), m_bits(n, 10.0)


def f10_caps():
    return [F10_BUFFER * F10_FANOUT ** i for i in range(F10_LEVELS)]


def f10_build(seed: int = SEED, n: int = F10_BUILD_N):
    """(keys, m): a run of n keys into the filter of the f = 10 tree's level 2
    (m = m_bits(51,200,000, 10.0) = 512,000,000 = 15625 << 15)."""
    return gen_puts(seed, n), m_bits(f10_caps()[2], F10_BPE)


def f10(seed: int = SEED):
    """(gets, [(level, keys, m) for level 0..2]) for the f = 10 tree: full runs
    of capacity 512,000 * 10^i (oldest, largest first in the put stream, as
    c3), 16.8M GETs at skew 0.2 / misses 0.3."""
    caps = f10_caps()
    puts, gets = gen_workload(seed, sum(caps), C3_GETS, 0.2, 0.3)
    levels = []
    start = 0
    for lvl in reversed(range(F10_LEVELS)):
        cap = caps[lvl]
        levels.append((lvl, puts[start:start + cap], m_bits(cap, F10_BPE)))
        start += cap
    levels.sort(key=lambda t: t[0])
    return gets, levels


def f10_runs(seed: int = SEED):
    """f10() with each level's run as the reference writes it (distinct keys
    ascending, as c3_runs): the same filters, plus fences for GET routing."""
    gets, levels = f10(seed)
    return gets, [(lvl, np.unique(keys), m) for lvl, keys, m in levels]
