"""GPU parity of §8f row 3: compaction (k-way merge, newest wins, optional
tombstone drop) fused with the new run's filter + metadata build, against
the oracle's MergeContext restatement (oracle/bloom_oracle.c bo_compact)."""
import numpy as np
import pytest

import bloomhip as bh

pytestmark = pytest.mark.gpu
TOMB = np.iinfo(np.int32).min


def make_runs(sizes, key_range, seed, tomb_frac=0.05):
    rng = np.random.default_rng(seed)
    runs = []
    for n in sizes:
        keys = np.unique(rng.integers(-key_range, key_range, size=n, dtype=np.int64)
                         .astype(np.int32))
        vals = rng.integers(-2**31 + 1, 2**31, size=keys.size, dtype=np.int64).astype(np.int32)
        vals[rng.random(keys.size) < tomb_frac] = TOMB
        runs.append(np.ascontiguousarray(np.stack([keys, vals], axis=1)))
    return runs


@pytest.mark.parametrize("sizes", [[0], [1], [5000], [3000, 0, 7000], [1, 1, 1, 1, 1],
                                   [10_000] * 7, [2049, 2047, 4096, 1]])
@pytest.mark.parametrize("drop", [False, True])
def test_compact_matches_oracle(coracle, sizes, drop):
    runs = make_runs(sizes, 20_000, len(sizes) * 7 + sum(sizes) % 97)
    got = bh.compact(runs, drop_tombstones=drop)
    want = coracle.compact(runs, drop)
    assert np.array_equal(got, want)


def test_compact_extreme_keys_and_all_duplicates(coracle):
    ext = np.array([[TOMB, 1], [-1, 2], [0, 3], [2**31 - 1, 4]], dtype=np.int32)
    runs = [ext.copy(), ext.copy(), ext.copy()]
    runs[1][:, 1] = 9
    runs[0][2, 1] = TOMB
    for drop in (False, True):
        assert np.array_equal(bh.compact(runs, drop), coracle.compact(runs, drop))


def test_compact_builds_the_new_runs_filter(coracle):
    runs = make_runs([400_000, 250_000, 120_000, 60_000], 2**30, 3)
    total = sum(r.shape[0] for r in runs)
    m = bh.m_bits(total, 10.0)
    f = bh.BloomFilter(m)
    got = bh.compact(runs, drop_tombstones=True, filter=f)
    want = coracle.compact(runs, True)
    assert np.array_equal(got, want)
    assert (f.words() == coracle.build(m, want[:, 0].copy())).all()
    fences, mk = f.run_meta()
    wf, wmk = coracle.run_meta(want[:, 0].copy())
    assert np.array_equal(fences, wf) and mk == wmk


def test_compact_device_buffers(coracle):
    torch = pytest.importorskip("torch")
    runs = make_runs([300_001, 100_000, 7], 2**31 - 1, 5)
    druns = [torch.from_numpy(r).cuda() for r in runs]
    total = sum(r.shape[0] for r in runs)
    dout = torch.empty((total, 2), dtype=torch.int32, device="cuda")
    f = bh.BloomFilter(bh.m_bits(total, 8.0))
    got = bh.compact(druns, drop_tombstones=False, filter=f, out=dout)
    torch.cuda.synchronize()
    want = coracle.compact(runs, False)
    assert np.array_equal(got.cpu().numpy(), want)
    assert (f.words() == coracle.build(f.m, want[:, 0].copy())).all()


@pytest.mark.parametrize("sizes", [[1], [4096], [4097], [8192, 1], [12_289, 4095, 3]])
def test_compact_filter_and_fences_at_fence_boundaries(coracle, sizes):
    # the compaction builds its filter from the kept keys (packed) and reads
    # the sorted run's fences + last key directly: fence counts around 4096
    runs = make_runs(sizes, 2**31 - 1, sum(sizes) % 1009, tomb_frac=0.0)
    total = sum(r.shape[0] for r in runs)
    f = bh.BloomFilter(bh.m_bits(max(total, 1), 10.0))
    got = bh.compact(runs, drop_tombstones=True, filter=f)
    want = coracle.compact(runs, True)
    assert np.array_equal(got, want)
    assert (f.words() == coracle.build(f.m, want[:, 0].copy())).all()
    fences, mk = f.run_meta()
    wf, wmk = coracle.run_meta(want[:, 0].copy())
    assert np.array_equal(fences, wf) and mk == wmk


def test_compact_everything_dropped_leaves_an_empty_run(coracle):
    runs = [np.array([[5, TOMB], [9, TOMB]], dtype=np.int32),
            np.array([[5, 1], [9, 2]], dtype=np.int32)]
    f = bh.BloomFilter(bh.m_bits(4, 10.0))
    got = bh.compact(runs, drop_tombstones=True, filter=f)
    assert got.shape[0] == 0 and np.array_equal(got.reshape(-1, 2), coracle.compact(runs, True))
    assert not f.words().any()
    fences, mk = f.run_meta()
    assert fences.size == 0 and mk == np.iinfo(np.int32).min


def test_compact_device_runs_at_odd_entry_offsets(coracle):
    # device runs that start 8 B past a 16-B boundary: the merge stages each
    # share in address-aligned 16-B vectors at the matching LDS parity
    torch = pytest.importorskip("torch")
    runs = make_runs([70_001, 33_333, 4097, 2], 2**31 - 1, 11)
    views = []
    for r in runs:
        buf = torch.zeros((r.shape[0] + 2, 2), dtype=torch.int32, device="cuda")
        buf[1:1 + r.shape[0]] = torch.from_numpy(r).cuda()
        views.append(buf[1:1 + r.shape[0]])
    assert all((v.data_ptr() % 16) == 8 for v in views)
    f = bh.BloomFilter(bh.m_bits(sum(r.shape[0] for r in runs), 10.0))
    got = bh.compact(views, drop_tombstones=False, filter=f)
    want = coracle.compact(runs, False)
    assert np.array_equal(np.asarray(got), want)
    assert (f.words() == coracle.build(f.m, want[:, 0].copy())).all()


def _dup_runs(sizes, key_range, seed):
    # sorted runs WITH repeated keys inside each run (the reference's runs
    # never repeat a key, but MergeContext's order defines them: the first
    # entry of the newest run holding a key wins)
    rng = np.random.default_rng(seed)
    runs = []
    for n in sizes:
        keys = np.sort(rng.integers(-key_range, key_range, size=n, dtype=np.int64).astype(np.int32))
        vals = rng.integers(-2**31 + 1, 2**31, size=n, dtype=np.int64).astype(np.int32)
        vals[rng.random(n) < 0.1] = TOMB
        runs.append(np.ascontiguousarray(np.stack([keys, vals], axis=1)))
    return runs


@pytest.mark.parametrize("sizes,key_range", [([100_000] * 4, 5_000), ([70_000, 3, 40_000], 50),
                                             ([300_000, 300_000], 1), ([20_000] * 8, 2_000_000)])
@pytest.mark.parametrize("drop", [False, True])
def test_compact_repeated_keys_across_partitions(coracle, sizes, key_range, drop):
    # one-pass k-way path (<= 8 runs): partition starts fall inside long runs
    # of equal keys, within and across runs; a single key repeated 600,000
    # times still splits into bounded partitions ((key, run, index) order)
    runs = _dup_runs(sizes, key_range, sum(sizes) % 101 + key_range)
    got = bh.compact(runs, drop_tombstones=drop)
    assert np.array_equal(got, coracle.compact(runs, drop))


@pytest.mark.parametrize("drop", [False, True])
def test_compact_more_runs_than_one_pass_takes(coracle, drop):
    # 12 runs: beyond the one-pass kernel's 8, the pairwise merge tree + dedup
    runs = make_runs([30_000] * 12, 200_000, 12)
    f = bh.BloomFilter(bh.m_bits(360_000, 10.0))
    got = bh.compact(runs, drop_tombstones=drop, filter=f)
    want = coracle.compact(runs, drop)
    assert np.array_equal(got, want)
    assert (f.words() == coracle.build(f.m, want[:, 0].copy())).all()


@pytest.mark.parametrize("k", range(1, 9))
def test_compact_every_fan_in_of_the_one_pass_kernel(coracle, k):
    # the one-pass kernel sizes its partitions by the fan-in (q = 16 - k
    # samples of 256 entries each): every k it takes, with repeated keys
    # inside and across runs, both tombstone modes, and the fused filter
    runs = _dup_runs([60_000 + 777 * r for r in range(k)], 40_000, 31 * k)
    total = sum(r.shape[0] for r in runs)
    for drop in (False, True):
        f = bh.BloomFilter(bh.m_bits(total, 10.0))
        got = bh.compact(runs, drop_tombstones=drop, filter=f)
        want = coracle.compact(runs, drop)
        assert np.array_equal(got, want)
        if want.shape[0]:
            assert (f.words() == coracle.build(f.m, want[:, 0].copy())).all()


@pytest.mark.parametrize("repeated", [False, True], ids=["unique", "repeated"])
def test_compact_large_beyond_one_lookback_window(coracle, repeated):
    # 4 x 2.6M entries: ~1,450 partitions at fan-in 4, so the merge's
    # decoupled look-back crosses its 1024-partition window (q0 -= the
    # window) and partitions wait on predecessors that were not resident
    # with them (more than the 512 workgroups the chip holds at once); both
    # tombstone modes, the fused filter and fences, against the oracle
    sizes = [2_600_000, 2_600_001, 2_599_999, 2_600_003]
    runs = (_dup_runs(sizes, 3_000_000, 77) if repeated
            else make_runs(sizes, 2**31 - 1, 78))
    total = sum(r.shape[0] for r in runs)
    assert total > 10_000_000
    for drop in (False, True):
        f = bh.BloomFilter(bh.m_bits(total, 10.0))
        got = bh.compact(runs, drop_tombstones=drop, filter=f)
        want = coracle.compact(runs, drop)
        assert np.array_equal(got, want)
        assert (f.words() == coracle.build(f.m, want[:, 0].copy())).all()
        fences, mk = f.run_meta()
        wf, wmk = coracle.run_meta(want[:, 0].copy())
        assert np.array_equal(fences, wf) and mk == wmk
