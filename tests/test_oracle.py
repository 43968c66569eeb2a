"""The oracle against the reference's own known answers (CPU only).

Pins (tests/golden/): SURVEY.md §8a known-answer positions and §0 F4 sizing
from the compiled reference, §8c C2/C3 popcounts and GET hit counts, and the
reference's golden test test-6 (`g 1535` must hit: no false negative,
test/test-6/in + out line 2).
"""
import json
import os

import numpy as np
import pytest

from bloom_oracle import (np_build, np_m_bits, np_positions, np_test_batch, pack_bools,
                          unpack_bools)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("row", _kat()["positions"], ids=lambda r: f"m{r['m']}_k{r['key']}")
def test_known_answer_positions(coracle, row):
    assert coracle.positions([row["key"]], row["m"])[0].tolist() == row["h"]
    assert np_positions([row["key"]], row["m"])[0].tolist() == row["h"]


@pytest.mark.parametrize("row", _kat()["m_bits"], ids=lambda r: f"{r['max_size']}x{r['bpe']}")
def test_m_bits_float_semantics(coracle, row):
    assert coracle.m_bits(row["max_size"], row["bpe"]) == row["m"]
    assert np_m_bits(row["max_size"], row["bpe"]) == row["m"]


def test_m_zero_rejected(coracle):
    # reference: (long)(512*0.001f) == 0 then `% 0` -> SIGFPE; here an error
    with pytest.raises(ValueError):
        coracle.m_bits(512, 0.001)


def test_two_restatements_agree():
    import bloom_oracle as bo
    c = bo.COracle()
    rng = np.random.default_rng(7)
    keys = rng.integers(-2**31, 2**31, size=50_000, dtype=np.int64).astype(np.int32)
    keys[:4] = [0, -1, 2**31 - 1, -2**31]
    for m in [1, 2, 63, 64, 65, 1000, 1_000_003, 2**32 - 1, 2**32, 2**32 + 7, 2**45 + 3, 2**63 - 1]:
        assert (c.positions(keys, m) == np_positions(keys, m)).all(), m
    for m in [64, 1000, 65_537, 1_000_003]:
        a = c.build(m, keys)
        b = np_build(m, keys)
        assert (a == b).all()
        probe = rng.integers(-2**31, 2**31, size=20_000, dtype=np.int64).astype(np.int32)
        probe[:1000] = keys[:1000]
        assert (c.test(a, m, probe) == pack_bools(np_test_batch(b, m, probe))).all()


def test_aos_stride_matches_packed(coracle):
    rng = np.random.default_rng(3)
    run = rng.integers(-2**31, 2**31, size=(4096, 2), dtype=np.int64).astype(np.int32)
    m = 40_961
    a = coracle.build(m, run.reshape(-1), stride=8, n=4096)
    b = coracle.build(m, np.ascontiguousarray(run[:, 0]))
    assert (a == b).all()


def test_pack_roundtrip():
    rng = np.random.default_rng(1)
    for n in [0, 1, 63, 64, 65, 1000]:
        b = rng.random(n) < 0.5
        assert (unpack_bools(pack_bools(b), n) == b).all()


def test_reference_golden_test6(coracle):
    """test/test-6: puts 0..1535 with -b 1 (512-entry buffer) -> runs of 512
    sorted keys, each with a filter of m = (long)(512*0.5f) = 256 bits
    (src/run.cpp:15); `g 1535` must find the key, so is_set(1535) is true in
    its run's filter (test/test-6/out line 2)."""
    m = coracle.m_bits(512, 0.5)
    assert m == 256
    for lo in (0, 512, 1024):
        keys = np.arange(lo, lo + 512, dtype=np.int32)
        w = coracle.build(m, keys)
        hits = unpack_bools(coracle.test(w, m, keys), 512)
        assert hits.all()
    w = coracle.build(m, np.arange(1024, 1536, dtype=np.int32))
    assert unpack_bools(coracle.test(w, m, np.array([1535], np.int32)), 1)[0]


def test_c2_popcount_pin(coracle, golden):
    import bloomhip.workloads as W
    keys, m = W.c2()
    w = coracle.build(m, keys)
    assert coracle.popcount(w) == golden["reference"]["c2_popcount"]


@pytest.mark.slow
def test_c3_pins(coracle, golden):
    import bloomhip.workloads as W
    gets, levels = W.c3()
    for lvl, keys, m in levels:
        w = coracle.build(m, keys)
        assert coracle.popcount(w) == golden["reference"]["c3_popcount"][lvl]
        hits = coracle.test(w, m, gets)
        assert int(np.unpackbits(hits.view(np.uint8)).sum()) == golden["reference"]["c3_hits"][lvl]


def test_f10_level0_pin_by_the_numpy_restatement(golden):
    """The f = 10 tree's geometry (m = 5,120,000 = 625 << 13: an odd part no
    p2 form covers) through the independent numpy restatement: level 0's
    bitmap and its hit row over all 16.8M GETs equal the C oracle's pins."""
    import hashlib
    import bloomhip.workloads as W
    gets, levels = W.f10()
    lvl, keys, m = levels[0]
    pin = golden["oracle"]["f10"]["levels"][0]
    assert (lvl, m, keys.size) == (0, pin["m"], pin["n"]) == (0, 5_120_000, 512_000)
    w = np_build(m, keys)
    assert hashlib.sha256(w.tobytes()).hexdigest() == pin["sha256"]
    hits = pack_bools(np_test_batch(w, m, gets))
    assert hashlib.sha256(hits.tobytes()).hexdigest() == pin["hits_sha256"]


def test_route_restatement_matches_python_loops(coracle):
    """bo_run_meta / bo_route against a direct Python restatement of
    Run::put (src/run.cpp:158-174), Run::get's checks (:94-99) and
    LSMTree::get's newest-run pick (src/lsm_tree.cpp:141-151,195-201)."""
    import bisect
    from bloom_oracle import np_build, np_test_batch
    rng = np.random.default_rng(4)
    runs = []
    for n in (0, 3, 5000, 9000, 20000):
        keys = np.unique(rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32))
        m = max(1, n * 10)
        fences = [int(k) for i, k in enumerate(keys) if i % 4096 == 0]
        mk = int(keys.max()) if keys.size else -2**31
        f2, mk2 = coracle.run_meta(keys)
        assert list(f2) == fences and mk2 == mk
        runs.append((np_build(m, keys), m, np.array(fences, np.int32), mk, keys))
    pool = np.concatenate([r[4] for r in runs])
    gets = np.concatenate([pool[rng.integers(0, pool.size, 3000)],
                           rng.integers(-2**31, 2**31, 3000, dtype=np.int64).astype(np.int32)])
    cand, first, page = coracle.route([r[:4] for r in runs], gets)
    bits = [np_test_batch(w, m, gets) for w, m, *_ in runs]
    for i, k in enumerate(gets.tolist()):
        want_first, want_page = -1, -1
        for r, (w, m, fences, mk, _) in enumerate(runs):
            c = len(fences) > 0 and fences[0] <= k <= mk and bool(bits[r][i])
            assert bool((int(cand[r][i // 64]) >> (i % 64)) & 1) == c
            if c and want_first < 0:
                want_first = r
                want_page = bisect.bisect_right(list(fences), k) - 1
        assert (first[i], page[i]) == (want_first, want_page), i


def test_compact_restatement_matches_python(coracle):
    """bo_compact against a dict-based restatement: newest run wins per key,
    tombstones dropped only when asked (src/merge.cpp:6-39,
    src/lsm_tree.cpp:81-88)."""
    rng = np.random.default_rng(8)
    runs = []
    for n in (0, 50, 400, 1000, 3):
        keys = np.unique(rng.integers(-300, 300, size=n, dtype=np.int64).astype(np.int32))
        vals = rng.integers(-5, 5, size=keys.size, dtype=np.int64).astype(np.int32)
        vals[vals == -5] = np.iinfo(np.int32).min           # tombstones
        runs.append(np.stack([keys, vals], axis=1))
    for drop in (False, True):
        newest = {}
        for r in reversed(runs):                            # oldest first, newer overwrite
            for k, v in r.tolist():
                newest[k] = v
        want = [(k, v) for k, v in sorted(newest.items())
                if not (drop and v == np.iinfo(np.int32).min)]
        got = coracle.compact(runs, drop)
        assert [tuple(x) for x in got.tolist()] == want


def test_threaded_oracle_entries_match_sequential(coracle):
    """bench.py's CPU baseline at T threads computes exactly the sequential
    restatement's bitmap and hits (the OR of bits commutes)."""
    rng = np.random.default_rng(11)
    keys = rng.integers(-2**31, 2**31, size=300_007, dtype=np.int64).astype(np.int32)
    m = 2_000_003
    want = coracle.build(m, keys)
    for T in (1, 3, 16):
        assert (coracle.build_mt(m, keys, T) == want).all()
        assert (coracle.test_mt(want, m, keys[:70_001], T) == coracle.test(want, m, keys[:70_001])).all()
    many = coracle.build_many(m, keys[:300_000].reshape(3, -1))
    for f in range(3):
        assert (many[f] == coracle.build(m, keys[f * 100_000:(f + 1) * 100_000])).all()
