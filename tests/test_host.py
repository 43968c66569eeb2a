"""Host-side checks of the engine library (CPU only, no kernel launches).

* libbloomhip.so loads and exports every symbol include/*.h declares;
* the kernels' position arithmetic (bloom_math.h, evaluated on the host via
  bloomhip_host_positions) equals the oracle for edge and random m;
* Run::Run sizing (bloomhip_m_bits) and argument validation;
* the workload generator restatement against independent RNGs.
"""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

import bloomhip as bh
from bloom_oracle import np_m_bits, np_positions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        syms.update(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(bloomhip_\w+)\s*\(", text, re.M))
    return sorted(syms)


def test_library_exports_every_declared_symbol():
    syms = _declared_symbols()
    assert len(syms) >= 25
    L = ctypes.CDLL(bh.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(bh.EXPORTED_SYMBOLS)


def test_abi_version():
    assert bh.lib().bloomhip_abi_version() == 1


EDGE_M = [1, 2, 3, 31, 32, 33, 63, 64, 65, 255, 256, 257, 1000, 65_536, 524_288, 1_000_003,
          655_360, 167_772_160, 671_088_640, 2**31 - 1, 2**31, 2**31 + 1, 3_221_225_472,
          2**32 - 2, 2**32 - 1, 2**32, 2**32 + 1, 2**33 + 5, 2**46]


@pytest.fixture(scope="module")
def fuzz_keys():
    rng = np.random.default_rng(11)
    k = rng.integers(-2**31, 2**31, size=40_000, dtype=np.int64).astype(np.int32)
    k[:8] = [0, -1, 1, 2**31 - 1, -2**31, -2**31 + 1, 13141, -2_652_462]
    return k


@pytest.mark.parametrize("m", EDGE_M)
def test_engine_mod_arithmetic_edge_m(m, fuzz_keys):
    assert (bh.host_positions(m, fuzz_keys) == np_positions(fuzz_keys, m)).all()


def test_engine_mod_arithmetic_random_m(fuzz_keys):
    rng = np.random.default_rng(5)
    ms = np.concatenate([rng.integers(1, 2**32, size=300), rng.integers(1, 2**20, size=100),
                         (rng.integers(1, 64, size=50) << rng.integers(0, 26, size=50))])
    for m in ms.tolist():
        assert (bh.host_positions(int(m), fuzz_keys[:2000]) ==
                np_positions(fuzz_keys[:2000], int(m))).all(), m


def test_m_bits_matches_reference_sizing():
    rng = np.random.default_rng(2)
    for size, bpe in [(16_777_217, 10.0), (33_554_431, 0.5), (51_200, 7.7), (512, 0.5)] + [
            (int(s), float(np.float32(b))) for s, b in zip(rng.integers(1, 2**31, 200),
                                                          rng.uniform(0.1, 20, 200))]:
        assert bh.m_bits(size, bpe) == np_m_bits(size, bpe)


@pytest.mark.parametrize("size,bpe", [(512, 0.001), (0, 10.0), (100, -1.0), (100, float("nan"))])
def test_m_bits_rejects_empty_filter(size, bpe):
    with pytest.raises(bh.BloomHipError) as e:
        bh.m_bits(size, bpe)
    assert e.value.status == bh.EINVAL


def test_create_rejects_zero_bits():
    h = ctypes.c_void_p()
    assert bh.lib().bloomhip_create(0, 0, ctypes.byref(h)) == bh.EINVAL


def test_null_arguments_rejected():
    L = bh.lib()
    assert L.bloomhip_size(None, None) == bh.EINVAL
    assert L.bloomhip_set_batch(None, None, 0, 4, 0, None) == bh.EINVAL
    assert L.bloomhip_test_batch(None, 1, None, 0, 4, 0, None, 0, None) == bh.EINVAL
    assert L.bloomhip_destroy(None) == bh.EINVAL
    assert L.bloomhip_host_positions(0, None, 0, None) == bh.EINVAL


def test_no_gpu_fails_loudly_not_silently():
    """Without a device the engine must refuse, never fall back to the CPU."""
    if bh.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(bh.BloomHipError) as e:
        bh.BloomFilter(1024)
    assert e.value.status in (bh.ENODEV, bh.EIO)


def test_mt19937_matches_numpy():
    for seed in (13141, 13142, 0, 5489):
        ref = np.random.RandomState(seed if seed else 4357).randint(
            0, 2**32, size=3000, dtype=np.uint64).astype(np.uint32)
        assert (bh.gen_mt19937(seed, 3000) == ref).all()


def test_glibc_rand_matches_libc():
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 2, 13141):
        libc.srand(seed)
        ref = np.array([libc.rand() for _ in range(4000)], dtype=np.int32)
        assert (bh.gen_glibc_rand(seed, 4000) == ref).all()
    libc.srand(1)


def test_puts_stream_is_even_mt_outputs():
    keys, vals = bh.gen_puts(13141, 1000, with_vals=True)
    mt = bh.gen_mt19937(13141, 2000).view(np.int32)
    assert (keys == mt[0::2]).all() and (vals == mt[1::2]).all()


def test_workload_small_stream_shape():
    puts, gets = bh.gen_workload(13141, 5000, 3000, 0.2, 0.3)
    assert puts.size == 5000 and gets.size == 3000
    # A puts-only prefix of the MT stream: puts draw key,value; miss-GETs draw
    # one value, so every put key is an MT output.
    mt = set(bh.gen_mt19937(13141, 20000).view(np.int32).tolist())
    assert set(puts.tolist()) <= mt
    # ~70% of non-repeated GETs come from earlier puts (miss ratio 0.3).
    frac = np.isin(gets, puts).mean()
    assert 0.55 < frac < 0.85


def test_c1_run_is_sorted_distinct_prefix():
    from bloomhip import workloads as W
    run, m = W.c1_run()
    assert m == 512_000 and run.shape == (51_200, 2)
    assert (np.diff(run[:, 0].astype(np.int64)) > 0).all()


def test_load_of_a_non_filter_file_fails_before_touching_the_gpu(tmp_path):
    """bloomhip_load validates the file on the host first (no GPU needed)."""
    import ctypes
    p = tmp_path / "junk.bloom"
    p.write_bytes(b"not a filter at all" * 10)
    h = ctypes.c_void_p()
    L = bh._lib()
    assert L.bloomhip_load(str(p).encode(), 0, ctypes.byref(h)) == bh.EINVAL
    assert L.bloomhip_load(str(tmp_path / "none").encode(), 0, ctypes.byref(h)) == -5  # EIO
    assert not h.value


def test_load_rejects_oversized_header_without_allocating(tmp_path):
    """A header whose sizes disagree with the file (here: 2^46 bits and 2^32-1
    fences in a 48-byte file) is refused before anything is sized from it."""
    import ctypes
    import struct
    L = bh._lib()
    h = ctypes.c_void_p()
    for m, nf in [((1 << 46), 0xFFFFFFFF), ((1 << 62), 0), (1000, 5)]:
        hdr = b"BLOOMHP1" + struct.pack("<IIQQIi", 1, 1, m, (m + 63) // 64, nf, 0)
        p = tmp_path / f"big_{m}_{nf}.bloom"
        p.write_bytes(hdr + b"\0" * 8)
        assert L.bloomhip_load(str(p).encode(), 0, ctypes.byref(h)) == bh.EINVAL
        assert not h.value


def test_binding_refuses_keys_that_are_not_int32():
    """Keys are KEY_t = int32 (src/types.h:4): an int64 array read as int32
    words would build the wrong keys, so the binding converts integer arrays
    at stride 4 (when they fit) and refuses anything else."""
    ptr, on_dev, keep = bh._keys_ptr(np.arange(10), 4)  # numpy's default int64
    assert keep.dtype == np.int32 and list(keep) == list(range(10)) and on_dev == 0
    with pytest.raises(ValueError):
        bh._keys_ptr(np.array([2**31]), 4)          # out of range
    with pytest.raises(ValueError):
        bh._keys_ptr(np.zeros((4, 2), dtype=np.int64), 8)  # int64 entries at stride 8
    with pytest.raises(ValueError):
        bh._keys_ptr(np.zeros(4, dtype=np.float32), 4)
    _, _, keep = bh._keys_ptr(np.zeros(8, dtype=np.int32), 8)
    assert bh._key_count(keep, 8, None) == 4
    with pytest.raises(ValueError):
        bh._key_count(keep, 8, 5)                  # 5 keys at stride 8 need 36 bytes
    with pytest.raises(ValueError):
        bh._out_ptr(np.zeros(3, dtype=np.uint64), 32, 8, "out")   # too small
    with pytest.raises(ValueError):
        bh._out_ptr(np.zeros(8, dtype=np.int32), 16, 8, "out")    # wrong element size
    with pytest.raises(ValueError):
        bh.compact([np.zeros((4, 2), dtype=np.int64)])


P2_D = (3, 5, 15, 17, 51, 85, 255)


def test_engine_p2_mod_every_form(fuzz_keys):
    """The p2 remainder (bloom_math.h mod_p2: m = d << t with d | 255, the
    byte-sum congruence and one multiply-high) against the exact remainder
    for every d and t it takes, and the m either side of each (general path)."""
    checked = 0
    for d in P2_D:
        for t in range(12, 32):
            m = d << t
            if m >= 2**32:
                continue
            for mm in (m, m - 1, m + 1):
                assert (bh.host_positions(mm, fuzz_keys[:4000]) ==
                        np_positions(fuzz_keys[:4000], mm)).all(), (d, t, mm)
            checked += 1
    assert checked > 100


def test_engine_wide_mod_random_m(fuzz_keys):
    """mod_wide (2^32 <= m <= 2^46: double-estimated quotient + one exact
    correction) against the exact remainder, m spread over the whole range
    and packed near powers of two and near quotient boundaries."""
    rng = np.random.default_rng(17)
    ms = np.concatenate([rng.integers(2**32, 2**46 + 1, size=200, dtype=np.uint64),
                         (np.uint64(1) << rng.integers(32, 47, size=60).astype(np.uint64)) +
                         rng.integers(-3, 4, size=60).astype(np.int64).astype(np.uint64),
                         np.array([2**32, 2**32 + 1, 2**32 + 1_000_003, 2**46, 2**46 - 1],
                                  dtype=np.uint64)])
    for m in ms.tolist():
        if not 2**32 <= m <= 2**46:
            continue
        assert (bh.host_positions(int(m), fuzz_keys[:3000]) ==
                np_positions(fuzz_keys[:3000], int(m))).all(), m


def test_library_is_built_from_these_kernel_sources():
    # the in-tree library carries the digest of the kernel sources it was
    # compiled from: a stale lib/ (sources edited, not rebuilt) fails here
    # before any GPU run measures the wrong kernels
    import hashlib
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    h = hashlib.sha256()
    for name in bench.kernel_sources():
        with open(os.path.join(root, "cs265-lsm-tree_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    assert bh.lib().bloomhip_kernel_sha().decode() == h.hexdigest()[:16]


def test_digest_covers_every_kernel_source():
    """csrc/Makefile's KERNEL_SRCS (the digest compiled into the library, read
    by bench.kernel_sources) lists every device source and header of the
    product: a kernel unit left out would change without changing the digest."""
    import glob
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    csrc = os.path.join(root, "cs265-lsm-tree_amd", "csrc")
    listed = bench.kernel_sources()
    assert len(set(listed)) == len(listed)
    for name in listed:
        assert os.path.exists(os.path.join(csrc, name)), name
    product = {os.path.basename(p) for p in glob.glob(os.path.join(csrc, "bloom_*"))
               if p.endswith((".hip", ".h"))}
    assert product <= set(listed), product - set(listed)
    assert "bloom_capi.cpp" in listed


@pytest.mark.parametrize("shift", [31, 32])
def test_planner_magic_bound_implies_exact(shift):
    """The planners (bloom_kernels.hip seg_magic, plan_ladder's computed
    tuple) skip their exhaustive check of a multiply-high divisor when
    x * e < 2^shift for every x they divide (M = ceil(2^shift / g),
    e = M g - 2^shift): the bound is checked here against brute force over
    every x it admits, for random and edge divisors."""
    rng = np.random.default_rng(7)
    gs = [1, 2, 3, 5, 7, 640, 4095, 4096, 40961, (1 << 20) - 1] + list(rng.integers(1, 1 << 22, 40))
    for g in gs:
        g = int(g)
        M = ((1 << shift) + g - 1) // g
        e = M * g - (1 << shift)
        xmax = (1 << shift) // e if e else 1 << 22  # x e < 2^shift for x < xmax
        xmax = min(xmax, 1 << 22)
        x = np.arange(xmax, dtype=np.uint64)
        got = (x * np.uint64(M)) >> np.uint64(32)
        want = x // np.uint64(2 * g) if shift == 31 else x // np.uint64(g)
        assert np.array_equal(got, want), g
