"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle.

Bit-exact: the same bitmap blocks after set_batch, the same packed is_set
booleans after test_batch.  Small cases compare with the C oracle directly;
full-size configs compare with the SHA-256 fixtures the pinned oracle wrote
(tests/golden/pins.json) plus size-independent properties (no false
negatives, idempotence, order independence, merge = union).
"""
import hashlib

import numpy as np
import pytest

import bloomhip as bh
from bloom_oracle import unpack_bools

pytestmark = pytest.mark.gpu

STRATEGIES = [bh.BUILD_ATOMIC, bh.BUILD_LDS, bh.BUILD_PARTITION]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rand_keys(n, seed=0):
    rng = np.random.default_rng(seed)
    k = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    if n >= 6:
        k[:6] = [0, -1, 1, 2**31 - 1, -2**31, 13141]
    return k


def supported(f, strategy):
    try:
        f.set_strategy(strategy)
        return True
    except bh.BloomHipError:
        return False


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


# ---------------------------------------------------------------- build ----
@pytest.mark.parametrize("m", [1, 2, 31, 32, 33, 64, 65, 256, 1000, 65_537, 512_000, 524_288,
                               1_000_003, 4_194_304, 10_485_761, 167_772_160, 671_088_640,
                               5_120_000, 51_200_000, 512_000_000,  # the f = 10 tree: 625 << 13 ...
                               2**32 - 1, 2**32, 2**32 + 1_000_003, 2**33 - 7])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=["atomic", "lds", "partition"])
def test_build_matches_oracle(coracle, m, strategy):
    n = 200_000 if m > 100_000 else 5_000
    keys = rand_keys(n, seed=m % 1000)
    f = bh.BloomFilter(m)
    if not supported(f, strategy):
        pytest.skip("strategy not applicable to this m")
    f.set_batch(keys)
    assert (f.words() == coracle.build(m, keys)).all()


# ----------------------------------------------- super-tile pass 1 builds ----
# Builds on >= 1024 segments (m > ~1.07 Gbit, below 2^32) sort super-tiles of
# 16,384 keys (k_part_bin2: half A stashed in LDS, half B in registers, one
# joint histogram, two output phases): m = 1.4e9 (general remainder, 1,187
# segments), C4's 3 << 30 (p2 remainder, 2,458) and 2^32 - 1 (3,277).
SUPER_MS = [1_400_000_000, 3 * 2**30, 2**32 - 1]


@pytest.mark.parametrize("m", SUPER_MS)
@pytest.mark.parametrize("n", [1, 8191, 8192, 8193, 16_383, 16_385, 40_000, 100_003])
def test_super_tile_build_matches_oracle(coracle, m, n):
    """Tiles whose B half is empty, partial or full, a short last super-tile,
    several tiles: every case bit-exact against the oracle."""
    keys = rand_keys(n, seed=n % 977 + m % 13)
    f = bh.BloomFilter(m)
    f.set_strategy(bh.BUILD_PARTITION)  # AUTO takes atomics below 2^16 keys
    f.set_batch(keys)
    assert (f.words() == coracle.build(m, keys)).all()


@pytest.mark.parametrize("m", SUPER_MS[:2])
def test_super_tile_build_layouts_and_skew(coracle, m):
    """entry_t keys at stride 8 (16-B aligned: the vector key loads), keys at
    stride 12, and a skewed batch (one key repeated across a whole tile: a
    run of 49,152 entries, the rank field's maximum) mixed with random keys."""
    rng = np.random.default_rng(5)
    keys = rand_keys(70_001, seed=11)
    aos = np.zeros((keys.size, 3), dtype=np.int32)
    aos[:, 0] = keys
    want = coracle.build(m, keys)
    f = bh.BloomFilter(m)
    f.set_strategy(bh.BUILD_PARTITION)
    f.set_batch(np.ascontiguousarray(aos[:, :2]).reshape(-1), n=keys.size, stride=8)
    assert (f.words() == want).all()
    g = bh.BloomFilter(m)
    g.set_strategy(bh.BUILD_PARTITION)
    g.set_batch(aos.reshape(-1), n=keys.size, stride=12)
    assert (g.words() == want).all()
    skew = np.concatenate([np.full(16_384, 12345, dtype=np.int32), keys[:30_000],
                           np.full(20_000, -7, dtype=np.int32)])
    rng.shuffle(skew[16_384:])
    h = bh.BloomFilter(m)
    h.set_strategy(bh.BUILD_PARTITION)
    h.set_batch(skew)
    assert (h.words() == coracle.build(m, skew)).all()
    # a second batch into the same filter: pass 2 ORs into the existing bitmap
    more = rand_keys(33_333, seed=12)
    h.set_batch(more)
    assert (h.words() == coracle.build(m, np.concatenate([skew, more]))).all()


@pytest.mark.parametrize("strategy", STRATEGIES, ids=["atomic", "lds", "partition"])
def test_build_device_keys_and_accumulation(coracle, torch_cuda, strategy):
    torch = torch_cuda
    m = 4_000_037 if strategy != bh.BUILD_LDS else 400_009
    a, b = rand_keys(300_000, 1), rand_keys(300_000, 2)
    f = bh.BloomFilter(m)
    if not supported(f, strategy):
        pytest.skip("n/a")
    f.set_batch(torch.from_numpy(a).cuda())
    f.sync()
    f.set_batch(torch.from_numpy(b).cuda())   # second batch ORs into the first
    f.sync()
    assert (f.words() == coracle.build(m, np.concatenate([a, b]))).all()


def test_build_generic_mod_path_m_above_2_32(coracle):
    m = 2**32 + 1_000_003    # 512 MiB bitmap; 64-bit remainder path
    keys = rand_keys(100_000, 9)
    f = bh.BloomFilter(m)
    f.set_batch(keys)
    ref = coracle.build(m, keys)
    w = f.words()
    assert (w == ref).all()


def test_entry_t_run_stride8_c1(coracle, golden):
    """C1: the first flushed run as AoS entry_t (src/types.h:14-22) at stride 8."""
    from bloomhip import workloads as W
    run, m = W.c1_run()
    ref = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__),
                                             "golden", "c1_bitmap.npy"))
    for strategy in STRATEGIES:
        f = bh.BloomFilter(m)
        if not supported(f, strategy):
            continue
        f.set_batch(run.reshape(-1), n=run.shape[0], stride=8)
        w = f.words()
        assert (w == ref).all(), strategy
        assert sha(w) == golden["oracle"]["c1"]["sha256"]


def test_unaligned_and_strided_keys(coracle):
    keys = rand_keys(100_003, 4)
    m = 1_048_583
    buf = np.zeros(keys.size + 1, dtype=np.int32)
    buf[1:] = keys                            # 4-byte offset: not 16-byte aligned
    f = bh.BloomFilter(m)
    f.set_batch(buf[1:])
    assert (f.words() == coracle.build(m, keys)).all()
    wide = np.zeros((keys.size, 3), dtype=np.int32)  # stride 12
    wide[:, 0] = keys
    g = bh.BloomFilter(m)
    g.set_batch(wide.reshape(-1), n=keys.size, stride=12)
    assert (g.words() == f.words()).all()


def test_empty_and_single_key(coracle):
    f = bh.BloomFilter(1000)
    f.set_batch(np.zeros(0, dtype=np.int32))
    assert not f.words().any()
    f.set(-2**31)
    assert (f.words() == coracle.build(1000, np.array([-2**31], np.int32))).all()
    assert f.is_set(-2**31)


def test_adversarial_single_key_overflows_bins(coracle):
    """All positions in three segments: bins overflow and spill to atomics."""
    keys = np.full(3_000_000, 777, dtype=np.int32)
    keys[::1000] = np.arange(3000, dtype=np.int32)
    m = 167_772_160
    f = bh.BloomFilter(m)
    f.set_strategy(bh.BUILD_PARTITION)
    f.set_batch(keys)
    assert (f.words() == coracle.build(m, keys)).all()


def test_order_independence_and_idempotence():
    keys = rand_keys(500_000, 12)
    m = 5_000_011
    f = bh.BloomFilter(m)
    f.set_batch(keys)
    w1 = f.words()
    g = bh.BloomFilter(m)
    g.set_batch(keys[::-1].copy())
    g.set_batch(keys)                         # idempotent
    assert (g.words() == w1).all()


def test_upload_download_roundtrip_and_validation():
    m = 100_003
    keys = rand_keys(10_000, 13)
    f = bh.BloomFilter(m)
    f.set_batch(keys)
    w = f.words()
    g = bh.BloomFilter(m)
    g.load_words(w)
    assert (g.words() == w).all()
    assert unpack_bools(bh.test_batch([g], keys)[0], keys.size).all()
    bad = w.copy()
    bad[-1] |= np.uint64(1) << np.uint64(63)   # bit >= m
    with pytest.raises(bh.BloomHipError):
        g.load_words(bad)


def test_clear_resets():
    f = bh.BloomFilter(1_000_000)
    f.set_batch(rand_keys(1000, 1))
    f.clear()
    assert not f.words().any()


@pytest.mark.parametrize("strategy", STRATEGIES, ids=["atomic", "lds", "partition"])
def test_deferred_clear_then_build_and_probe(coracle, strategy):
    """clear() defers its memset; every later use must still see zeros first."""
    m = 120_000 if strategy == bh.BUILD_LDS else 10_000_019
    a, b = rand_keys(300_000, 40), rand_keys(300_000, 41)
    f = bh.BloomFilter(m)
    if not supported(f, strategy):
        pytest.skip("n/a")
    f.set_batch(a)
    f.clear()
    f.set_batch(b)                      # build straight after the deferred clear
    assert (f.words() == coracle.build(m, b)).all()
    f.clear()
    probe = np.concatenate([b[:1000], a[:1000]])
    got = bh.test_batch([f], probe)[0]  # probe of a cleared filter: all miss
    assert not got.any()
    f.clear()
    f.set_batch(a)
    f.set_batch(b)                      # second batch merges
    assert (f.words() == coracle.build(m, np.concatenate([a, b]))).all()


# ---------------------------------------------------------------- probe ----
PROBES = [bh.PROBE_GATHER, bh.PROBE_PARTITION, bh.PROBE_LDS, bh.PROBE_STACKED]
PROBE_IDS = ["gather", "partition", "lds", "stacked"]


@pytest.mark.parametrize("m", [1, 64, 65, 1000, 655_360, 1_000_003, 167_772_160, 671_088_640,
                               0xFFFFFF00, 2**32 - 1, 2**32 + 15])
@pytest.mark.parametrize("probe", PROBES, ids=PROBE_IDS)
def test_probe_matches_oracle(coracle, m, probe):
    keys = rand_keys(100_000 if m < 2**32 else 20_000, 21)
    f = bh.BloomFilter(m)
    f.set_probe_strategy(probe)   # partition / lds fall back to gathers where they cannot apply
    f.set_batch(keys)
    probe = np.concatenate([keys[:30_000], rand_keys(70_001, 22)])
    got = bh.test_batch([f], probe)[0]
    assert (got == coracle.test(coracle.build(m, keys), m, probe)).all()
    assert unpack_bools(got, probe.size)[:min(30_000, keys.size)].all()   # no false negatives


def test_probe_many_filters_chunks_past_16(coracle):
    """20 filters, mixed strategies: gathered ones go out in launches of <= 16
    consecutive rows around the partitioned and LDS-probed ones."""
    rng = np.random.default_rng(3)
    filters, refs = [], []
    for j in range(20):
        m = int(rng.integers(1000, 1_300_000 if j in (5, 6, 15) else 30_000_000))
        keys = rand_keys(20_000, 100 + j)
        f = bh.BloomFilter(m)
        f.set_probe_strategy(bh.PROBE_PARTITION if j in (3, 11, 12) else
                             bh.PROBE_LDS if j in (5, 6, 15) else bh.PROBE_GATHER)
        f.set_batch(keys)
        filters.append(f)
        refs.append((m, coracle.build(m, keys)))
    probe = rand_keys(50_017, 99)
    probe[:20_000] = rand_keys(20_000, 105)
    got = bh.test_batch(filters, probe)
    for j, (m, w) in enumerate(refs):
        assert (got[j] == coracle.test(w, m, probe)).all(), j


@pytest.mark.parametrize("probe", PROBES, ids=PROBE_IDS)
def test_probe_device_buffers_and_strides(coracle, torch_cuda, probe):
    torch = torch_cuda
    m = 1_000_003 if probe == bh.PROBE_LDS else 2_000_003
    keys = rand_keys(64 * 1000 + 37, 31)
    f = bh.BloomFilter(m)
    f.set_probe_strategy(probe)
    f.set_batch(keys)
    ref = coracle.test(coracle.build(m, keys), m, keys)
    dk = torch.from_numpy(keys).cuda()
    dout = torch.zeros((1, (keys.size + 63) // 64), dtype=torch.int64, device="cuda")
    bh.test_batch([f], dk, out=dout)
    torch.cuda.synchronize()
    f.sync()
    assert (dout.cpu().numpy().view(np.uint64)[0] == ref).all()
    aos = np.zeros((keys.size, 2), dtype=np.int32)
    aos[:, 0] = keys
    got = bh.test_batch([f], aos.reshape(-1), n=keys.size, stride=8)[0]
    assert (got == ref).all()


def _stack_case(coracle, ms, probe_keys, strategies=None, stride=4, seed=0):
    filters, refs = [], []
    for j, m in enumerate(ms):
        keys = rand_keys(int(min(40_000, max(64, m // 10))), 500 + seed + j)
        f = bh.BloomFilter(m)
        f.set_probe_strategy(strategies[j] if strategies else bh.PROBE_STACKED)
        f.set_batch(keys)
        filters.append(f)
        refs.append((m, coracle.build(m, keys)))
        lo, hi = j * 1000, min((j + 1) * 1000, probe_keys.size)
        if lo < hi:
            probe_keys[lo:hi] = keys[:hi - lo]   # some hits per filter
    if stride in (8, 12):
        aos = np.zeros((probe_keys.size, stride // 4), dtype=np.int32)
        aos[:, 0] = probe_keys
        got = bh.test_batch(filters, aos.reshape(-1), n=probe_keys.size, stride=stride)
    else:
        got = bh.test_batch(filters, probe_keys)
    for j, (m, w) in enumerate(refs):
        assert (got[j] == coracle.test(w, m, probe_keys)).all(), (j, m)


@pytest.mark.parametrize("ms", [
    [10_240 * 4**i for i in range(5)],            # C3's level geometry, scaled down 64x
    [655_360 * 4**i for i in range(4)],           # C3 levels 0-3
    [2**22, 2**20, 2**22, 2**16],                 # powers of two, a repeated size
    [1_000_000, 1_000_000],                       # no 128-bit-multiple w divides 10^6
    [3 * 2**20, 2**20, 3 * 2**18, 2**18, 2**19, 3 * 2**17, 2**17, 2**16, 2**15],  # 9 members
    [5 * 2**21, 2**21, 1_000_003, 5 * 2**19, 2**32 + 15],  # non-divisors, > 2^32 mixed in
    [5_120_000 * 10**i for i in range(3)],        # the f = 10 tree: gcd 625 << 13 (w = 320,000)
    [256_000 * 10**i for i in range(4)],          # f = 10 at the default r = 0.5: 125 << 11
    [3**7 * 2**9 * 7**i for i in range(3)],       # odd parts 2187 * 7^i, fanout 7
    [256_000 * 10**i for i in range(1, 4)],       # 625 segments on 250 strided workgroups (2-3 each)
], ids=["c3x64", "c3_l0-3", "pow2", "no_w", "nine", "mixed", "f10", "f10_r05", "fan7", "r05_l1-3"])
def test_stacked_probe_matches_oracle(coracle, ms):
    probe = rand_keys(300_001, 77)
    _stack_case(coracle, ms, probe)


@pytest.mark.parametrize("ms", [
    [655_360 * 4**i for i in range(5)],           # C3's levels: d = 5, t = 17..25
    [3 * 2**(16 + 2 * i) for i in range(4)],      # 12 bits/key levels: d = 3
    [5 * 2**25, 5 * 2**21, 5 * 2**20],            # uneven spacing (fanout 16, then 2)
    [5 * 2**22, 5 * 2**22, 5 * 2**20],            # a repeated size
    [5 * 2**(14 + 2 * i) for i in range(6)],      # six members, 2 KiB blocks
    [17 * 2**24, 17 * 2**20],                     # d = 17
    [5 * 2**20, 3 * 2**20, 5 * 2**18],            # two odd parts: not a ladder (segment stack)
    [3 * 2**(14 + 2 * i) for i in range(8)][::-1],  # eight members: 7 packed, byte image
    [5 * 2**(13 + 2 * i) for i in range(7)][::-1],  # seven members
], ids=["c3", "d3", "uneven", "repeat", "six", "d17", "not_ladder", "eight", "seven"])
def test_ladder_stack_matches_oracle(coracle, ms):
    """Levels d << t_j probed in one ladder pass (bins = hash bits, the
    members' blocks staged per bin); every member's rows against the oracle."""
    probe = rand_keys(300_001, 83)
    _stack_case(coracle, ms, probe, seed=11)


@pytest.mark.parametrize("n", [1, 63, 64, 8191, 8193])
def test_ladder_stack_tiny_ragged_and_strided(coracle, n):
    """A ladder over batches smaller than one 8192-key tile or one tile plus
    one key, and entry_t keys at stride 8."""
    ms = [655_360 * 4**i for i in range(4)]
    _stack_case(coracle, ms, rand_keys(n, 90 + n), seed=3)
    _stack_case(coracle, ms, rand_keys(n, 91 + n), stride=8, seed=4)


@pytest.mark.parametrize("n", [1, 63, 16_383, 16_385, 40_001])
def test_stacked_probe_super_tiles_ragged_and_strided(coracle, n):
    """The f = 10 tree's stack (1,250 segments: pass 1 on 16,384-key
    super-tiles with the slot plane, pass 2 at 16,384 keys per tile, the
    two-pass combine) on batches below one super-tile and one key past it,
    packed keys, entry_t keys and 12-byte records (the strided loads)."""
    ms = [5_120_000 * 10**i for i in range(3)]
    _stack_case(coracle, ms, rand_keys(n, 95 + n), seed=5)
    _stack_case(coracle, ms, rand_keys(n, 96 + n), stride=8, seed=6)
    _stack_case(coracle, ms, rand_keys(n, 97 + n), stride=12, seed=7)


def test_stacked_probe_auto_and_strided(coracle):
    """AUTO stacks a divisible group at >= 2^18 keys; AoS entry_t keys."""
    ms = [655_360 * 4**i for i in range(5)]
    probe = rand_keys(270_000, 78)
    _stack_case(coracle, ms, probe, strategies=[bh.PROBE_AUTO] * 5)
    _stack_case(coracle, ms[:3], rand_keys(263_001, 79), stride=8, seed=7)


@pytest.mark.parametrize("n", [1, 63, 64, 4095, 4097])
def test_stacked_probe_tiny_and_ragged_batches(coracle, n):
    """Explicit STACKED on batches smaller than a tile or one tile plus one key."""
    ms = [40_960 * 4**i for i in range(3)]
    probe = rand_keys(n, 80 + n)
    _stack_case(coracle, ms, probe)


def test_stacked_probe_with_cleared_and_empty_members(coracle):
    """A member that was never built and one that was cleared (deferred memset)
    probe as all-miss rows inside the stack."""
    ms = [655_360 * 4**i for i in range(4)]
    filters, refs = [], []
    for j, m in enumerate(ms):
        f = bh.BloomFilter(m)
        f.set_probe_strategy(bh.PROBE_STACKED)
        keys = rand_keys(30_000, 300 + j)
        if j != 1:
            f.set_batch(keys)
        if j == 2:
            f.clear()
        filters.append(f)
        refs.append((m, coracle.build(m, keys) if j in (0, 3) else np.zeros((m + 63) // 64, np.uint64)))
    probe = rand_keys(280_001, 81)
    got = bh.test_batch(filters, probe)
    for j, (m, w) in enumerate(refs):
        assert (got[j] == coracle.test(w, m, probe)).all(), j
    assert not got[1].any() and not got[2].any()


def test_stacked_probe_ladder_and_segment_geometries(coracle):
    """AUTO/STACKED groups of both stack kinds in one process: C3's levels
    (5 << 17, 5 << 19, ...: one odd part, a ladder stack with padded runs)
    and a mix of odd parts (3 << 20 with powers of two: no ladder, the
    segment stack, w | every member so each member's segment is staged
    without wrapping).  Each member's own keys are planted in the probe."""
    rng = np.random.default_rng(9)
    for ms in ([655_360 * 4**i for i in range(5)], [3 * 2**20, 2**20, 3 * 2**18, 2**18]):
        fs, refs = [], []
        for j, m in enumerate(ms):
            keys = rng.integers(-2**31, 2**31, size=40_000, dtype=np.int64).astype(np.int32)
            f = bh.BloomFilter(m)
            f.set_probe_strategy(bh.PROBE_STACKED)
            f.set_batch(keys)
            fs.append(f)
            refs.append((m, coracle.build(m, keys), keys))
        probe = rng.integers(-2**31, 2**31, size=300_001, dtype=np.int64).astype(np.int32)
        for j, (m, w, keys) in enumerate(refs):
            probe[j * 1000:(j + 1) * 1000] = keys[:1000]
        got = bh.test_batch(fs, probe)
        for j, (m, w, keys) in enumerate(refs):
            assert (got[j] == coracle.test(w, m, probe)).all(), (ms, j)


# m = d << t with d | 255 takes the p2 remainder on the device (bloom_math.h
# mod_p2_hi: alignbit, v_sad_u8, mulhi, mad_i32_i24); host fuzzing covers only
# its host form.  Every odd d | 255 across t, through the atomic build, the
# partition build (pass-1 kinds kModP2 / kModLadder0 where t allows), the
# gather probe and the LDS probe (m/8 <= 160 KiB).
P2_CASES = [(d, t) for d in (3, 5, 15, 17, 51, 85, 255) for t in (12, 14, 17, 20, 21, 22)
            if (d << t) <= (1 << 28)]


@pytest.mark.parametrize("d,t", P2_CASES)
def test_p2_remainder_every_odd_part(coracle, d, t):
    m = d << t
    keys = rand_keys(120_000, seed=d * 64 + t)
    ref = coracle.build(m, keys)
    built = None
    for strategy in (bh.BUILD_ATOMIC, bh.BUILD_PARTITION, bh.BUILD_LDS):
        f = bh.BloomFilter(m)
        if not supported(f, strategy):
            continue
        f.set_batch(keys)
        assert (f.words() == ref).all(), (d, t, strategy)
        built = f
    probe = np.concatenate([keys[:20_000], rand_keys(60_000, seed=7 + d + t)])
    want = coracle.test(ref, m, probe)
    for ps in (bh.PROBE_GATHER, bh.PROBE_LDS):  # LDS falls back to gathers above 160 KiB
        built.set_probe_strategy(ps)
        assert (bh.test_batch([built], probe)[0] == want).all(), (d, t, ps)


@pytest.mark.parametrize("ms", [[655_360 * 4**i for i in range(5)],
                                [5_120_000 * 10**i for i in range(3)]], ids=["c3", "f10"])
def test_stacked_probe_profile_slot(ms):
    """The stacked pass runs (and is timed) when AUTO should pick it: C3's
    levels (a ladder) and the f = 10 tree's (a segment stack whose width
    has a large odd part)."""
    filters = []
    for j, m in enumerate(ms):
        f = bh.BloomFilter(m)
        f.set_batch(rand_keys(10_000, j))
        filters.append(f)
    f0 = filters[0]
    f0.profile(True)
    f0.profile_reset()
    bh.test_batch(filters, rand_keys(1 << 19, 5))
    prof = f0.profile_read()
    f0.profile(False)
    assert prof.get("probe_stacked", {}).get("launches") == 1, prof


def test_probe_empty():
    f = bh.BloomFilter(100)
    out = bh.test_batch([f], np.zeros(0, dtype=np.int32))
    assert out.shape == (1, 0)


# -------------------------------------------------------- full configs ----
@pytest.mark.parametrize("m", [167_772_160, 3 * 2**26, 100_000_007], ids=["ladder", "segments", "odd_m"])
@pytest.mark.parametrize("stride", [4, 8])
def test_host_keys_build(torch_cuda, m, stride):
    """A partition build from host keys (staged by the library, packed or
    entry_t at stride 8) gives the same bitmap as one from device-resident
    keys, also when merging into a built filter."""
    torch = torch_cuda
    n = (1 << 22) + 12_345
    keys = rand_keys(n, 41)
    if stride == 8:
        host = np.zeros((n, 2), dtype=np.int32)
        host[:, 0] = keys
        host = host.reshape(-1)
    else:
        host = keys
    f = bh.BloomFilter(m)
    f.set_strategy(bh.BUILD_PARTITION)
    f.set_batch(host, n=n, stride=stride)
    g = bh.BloomFilter(m)
    g.set_strategy(bh.BUILD_PARTITION)
    g.set_batch(torch.from_numpy(keys).cuda())
    assert (f.words() == g.words()).all()
    more = rand_keys(n, 42)
    f.set_batch(more)
    g.set_batch(torch.from_numpy(more).cuda())
    assert (f.words() == g.words()).all()


def test_c2_full_bitmap(golden):
    from bloomhip import workloads as W
    keys, m = W.c2()
    for strategy in STRATEGIES:
        f = bh.BloomFilter(m)
        if not supported(f, strategy):
            continue
        f.set_batch(keys)
        w = f.words()
        assert sha(w) == golden["oracle"]["c2"]["sha256"], strategy
        assert int(np.unpackbits(w.view(np.uint8)).sum()) == golden["reference"]["c2_popcount"]


@pytest.mark.parametrize("probe", [bh.PROBE_AUTO] + PROBES, ids=["auto"] + PROBE_IDS)
def test_c3_probe_five_levels(golden, probe):
    from bloomhip import workloads as W
    gets, levels = W.c3()
    filters = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_probe_strategy(probe)
        f.set_batch(keys)
        lv = golden["oracle"]["c3"]["levels"][lvl]
        assert sha(f.words()) == lv["sha256"], lvl
        filters.append(f)
    got = bh.test_batch(filters, gets)
    for lvl in range(5):
        lv = golden["oracle"]["c3"]["levels"][lvl]
        assert sha(got[lvl]) == lv["hits_sha256"], lvl
        assert int(np.unpackbits(got[lvl].view(np.uint8)).sum()) == golden["reference"]["c3_hits"][lvl]


def test_c4_full_bitmap(golden):
    from bloomhip import workloads as W
    keys, m = W.c4()
    f = bh.BloomFilter(m)
    f.set_batch(keys)
    w = f.words()
    assert sha(w) == golden["oracle"]["c4"]["sha256"]
    # probe property at full size: every inserted key tests positive
    got = bh.test_batch([f], keys[::97].copy())[0]
    assert unpack_bools(got, keys[::97].size).all()


@pytest.mark.parametrize("m", [5 << 23, 3 << 24, 41_943_053])
def test_partition_merge_then_clear_rebuild(coracle, m):
    """The partition build's two writebacks: a second batch ORs into the
    first (merge: plain stores of the words it read) and, after clear(), a
    fresh build writes every word of the bitmap (non-temporal stores, no
    memset before it), on plan_build's ladder (d | 255) and on segments."""
    a, b, c = rand_keys(400_000, 31), rand_keys(300_000, 32), rand_keys(500_000, 33)
    f = bh.BloomFilter(m)
    f.set_strategy(bh.BUILD_PARTITION)
    f.set_batch(a)
    f.set_batch(b)
    assert (f.words() == coracle.build(m, np.concatenate([a, b]))).all()
    f.clear()
    f.set_batch(c)
    assert (f.words() == coracle.build(m, c)).all()


@pytest.mark.parametrize("m", [671_088_640, 360_000_007])
def test_hbm_resident_pass2_ragged(coracle, m):
    """Builds whose sorted entries exceed the Infinity Cache (> 256 MiB, more
    than 33.5M keys) walk pass 2 with two vectors per lane (WALK 3): a ragged
    batch (a short last tile) on C5's ladder geometry (5 << 27) and on a
    general m (segments), against the oracle."""
    n = 33_554_432 + 3 * 8192 + 777
    keys = rand_keys(n, seed=m % 101)
    f = bh.BloomFilter(m)
    f.set_strategy(bh.BUILD_PARTITION)
    f.set_batch(keys)
    assert (f.words() == coracle.build(m, keys)).all()


def test_c5_run0_full_bitmap(golden):
    from bloomhip import workloads as W
    keys, m = W.c5_run(0)
    f = bh.BloomFilter(m)
    f.set_batch(keys)
    assert sha(f.words()) == golden["oracle"]["c5"][0]["sha256"]


def test_f10_build_full_bitmap(golden):
    """The reference's published tree (b = 1000, f = 10, -r 10): 16.8M keys
    into level 2's filter, m = 512,000,000 = 15625 << 15 (workloads.f10_build),
    against the oracle's pin, by every build strategy that applies."""
    from bloomhip import workloads as W
    keys, m = W.f10_build()
    pin = golden["oracle"]["f10"]["build"]
    assert (m, keys.size) == (pin["m"], pin["n"])
    for strategy in STRATEGIES:
        f = bh.BloomFilter(m)
        if not supported(f, strategy):
            continue
        f.set_batch(keys)
        assert sha(f.words()) == pin["sha256"], strategy


@pytest.mark.parametrize("probe", [bh.PROBE_AUTO] + PROBES, ids=["auto"] + PROBE_IDS)
def test_f10_probe_three_levels(golden, probe):
    """The f = 10 tree's levels 0..2 (m = 5.12M, 51.2M, 512M bits) built from
    their full runs and probed with the 16.8M GETs in one call: every
    level's bitmap and hit row against the oracle's pins, per probe kind."""
    from bloomhip import workloads as W
    gets, levels = W.f10()
    pins = golden["oracle"]["f10"]["levels"]
    filters = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_probe_strategy(probe)
        f.set_batch(keys)
        assert sha(f.words()) == pins[lvl]["sha256"], lvl
        filters.append(f)
    got = bh.test_batch(filters, gets)
    for lvl in range(len(levels)):
        assert sha(got[lvl]) == pins[lvl]["hits_sha256"], lvl
