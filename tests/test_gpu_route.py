"""GPU parity of §8f rows 1 and 4: run metadata (fence pointers, max key)
built beside the filter, and batched GET routing (range check + filter probe
+ newest candidate run + page index), against the C oracle's restatement of
Run::put / Run::get / LSMTree::get (oracle/bloom_oracle.c bo_run_meta,
bo_route).  Bit-exact: same fences and max key, same candidate rows, same
first-run and page per key."""
import hashlib

import numpy as np
import pytest

import bloomhip as bh

pytestmark = pytest.mark.gpu


def sorted_run(n, seed):
    rng = np.random.default_rng(seed)
    k = np.unique(rng.integers(-2**31, 2**31, size=n + n // 8 + 8, dtype=np.int64).astype(np.int32))
    return k[:n] if k.size >= n else k


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 12_289, 300_000])
def test_run_meta_matches_oracle(coracle, n):
    keys = sorted_run(n, n + 1)
    f = bh.BloomFilter(bh.m_bits(max(n, 1), 10.0))
    f.set_batch_run(keys)
    fences, mk = f.run_meta()
    want_f, want_mk = coracle.run_meta(keys)
    assert np.array_equal(fences, want_f)
    assert mk == want_mk
    if n:
        assert (f.words() == coracle.build(f.m, keys)).all()


def test_run_meta_strided_unsorted_and_device(coracle):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    keys = rng.integers(-2**31, 2**31, size=50_001, dtype=np.int64).astype(np.int32)  # unsorted
    aos = np.zeros((keys.size, 2), dtype=np.int32)
    aos[:, 0] = keys
    f = bh.BloomFilter(600_000)
    f.set_batch_run(aos.reshape(-1), n=keys.size, stride=8)
    want = coracle.run_meta(keys)
    got = f.run_meta()
    assert np.array_equal(got[0], want[0]) and got[1] == want[1]
    g = bh.BloomFilter(600_000)
    g.set_batch_run(torch.from_numpy(keys).cuda())
    got = g.run_meta()
    assert np.array_equal(got[0], want[0]) and got[1] == want[1]


def test_run_meta_upload_round_trip():
    f = bh.BloomFilter(1000)
    fences = np.array([-5, 3, 3, 90], dtype=np.int32)
    f.set_run_meta(fences, 1234)
    got = f.run_meta()
    assert np.array_equal(got[0], fences) and got[1] == 1234
    with pytest.raises(bh.BloomHipError):
        f.set_run_meta(np.array([4, 1], dtype=np.int32), 9)   # fences must ascend


def build_runs(sizes, bpe=10.0, seed=0, probe=bh.PROBE_AUTO):
    runs, refs = [], []
    for j, n in enumerate(sizes):
        keys = sorted_run(n, 1000 * seed + j)
        m = bh.m_bits(max(n, 1), bpe)
        f = bh.BloomFilter(m)
        f.set_probe_strategy(probe)
        f.set_batch_run(keys)
        runs.append(f)
        refs.append((keys, m))
    return runs, refs


def oracle_runs(coracle, refs):
    out = []
    for keys, m in refs:
        fences, mk = coracle.run_meta(keys)
        out.append((coracle.build(m, keys), m, fences, mk))
    return out


def get_keys(refs, n, seed):
    rng = np.random.default_rng(seed)
    pool = np.concatenate([k for k, _ in refs])
    hits = pool[rng.integers(0, pool.size, size=n // 2)]
    miss = rng.integers(-2**31, 2**31, size=n - n // 2, dtype=np.int64).astype(np.int32)
    g = np.concatenate([hits, miss])
    rng.shuffle(g)
    g[:4] = [np.iinfo(np.int32).min, np.iinfo(np.int32).max, refs[0][0][0], refs[0][0][-1]]
    return g


def routed_by(runs, call):
    """Runs call() with profiling on runs[0] (the handle a multi-run call
    records its launches on) and returns (path, call's result): path is
    "fused" when the routing ran inside the stacked probe's combine
    (k_probe_combine_route), "k_route" when k_route ran after the probes."""
    f0 = runs[0]
    f0.profile(True)
    f0.profile_reset()
    try:
        out = call()
        prof = f0.profile_read()
    finally:
        f0.profile(False)
    fused = prof.get("probe_stacked+route", {}).get("launches", 0)
    plain = prof.get("k_route", {}).get("launches", 0)
    assert (fused > 0) != (plain > 0), prof
    return ("fused" if fused else "k_route"), out


def packed_matches(runs, gets, wc, wf, wp, path=None, **kw):
    """bloomhip_route_gets_packed against the oracle's rows, first and page
    (route[i] = first << 28 | page, or ROUTE_NONE), and the path it took."""
    p, (cand, route) = routed_by(runs, lambda: bh.route_gets_packed(runs, gets, **kw))
    if path is not None:
        assert p == path
    want = np.where(wf < 0, np.uint32(bh.ROUTE_NONE),
                    (wf.astype(np.uint32) << np.uint32(bh.ROUTE_PAGE_BITS)) | wp.astype(np.uint32))
    assert np.array_equal(cand, wc) and np.array_equal(route, want)
    f, pg = bh.unpack_route(route)
    assert np.array_equal(f, wf) and np.array_equal(pg, wp)
    return route


@pytest.mark.parametrize("probe", [bh.PROBE_AUTO, bh.PROBE_GATHER, bh.PROBE_PARTITION,
                                   bh.PROBE_LDS], ids=["auto", "gather", "partition", "lds"])
def test_route_matches_oracle(coracle, probe):
    runs, refs = build_runs([20_000, 70_000, 300_000, 1_200_000, 9], seed=1, probe=probe)
    gets = get_keys(refs, 400_001, 7)
    cand, first, page = bh.route_gets(runs, gets)
    wc, wf, wp = coracle.route(oracle_runs(coracle, refs), gets)
    assert np.array_equal(cand, wc)
    assert np.array_equal(first, wf)
    assert np.array_equal(page, wp)
    assert (first >= 0).sum() > 0 and (page[first >= 0] >= 0).all()
    packed_matches(runs, gets, wc, wf, wp)


def test_route_skewed_and_duplicate_fences(coracle):
    """Runs whose keys are far from uniform (a dense cluster plus a sparse
    tail), so the interpolation guess of k_route's page search misses and the
    full binary search runs; runs with long stretches of equal keys (equal
    fences: upper_bound must pass them all); GETs at, just below and just
    above every fence."""
    rng = np.random.default_rng(21)
    dense = rng.integers(0, 200_000, size=270_000, dtype=np.int64)
    tail = rng.integers(-2**31, 2**31, size=30_000, dtype=np.int64)
    skewed = np.sort(np.concatenate([dense, tail])).astype(np.int32)
    dup = np.sort(np.repeat(rng.integers(-2**31, 2**31, size=40, dtype=np.int64), 5000)).astype(np.int32)
    small = np.sort(rng.integers(-1000, 1000, size=9000, dtype=np.int64)).astype(np.int32)
    runs, refs = [], []
    for keys in (small, skewed, dup):
        m = bh.m_bits(keys.size, 10.0)
        f = bh.BloomFilter(m)
        f.set_batch_run(keys)
        runs.append(f)
        refs.append((keys, m))
    fences = np.concatenate([k[::4096] for k, _ in refs]).astype(np.int64)
    edge = np.concatenate([fences - 1, fences, fences + 1])
    edge = np.clip(edge, -2**31, 2**31 - 1).astype(np.int32)
    pool = np.concatenate([k for k, _ in refs])
    gets = np.concatenate([edge, pool[rng.integers(0, pool.size, size=150_000)],
                           rng.integers(-2**31, 2**31, size=50_000, dtype=np.int64).astype(np.int32)])
    rng.shuffle(gets)
    cand, first, page = bh.route_gets(runs, gets)
    wc, wf, wp = coracle.route(oracle_runs(coracle, refs), gets)
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    assert (page[first == 1] > 0).any()  # pages past the first in the skewed run
    packed_matches(runs, gets, wc, wf, wp, path="k_route")


def test_route_many_runs_and_missing_meta(coracle):
    """40 runs (probe launches chunked past 16 filters); one run has no
    metadata (never a candidate), one is empty."""
    sizes = [int(s) for s in np.random.default_rng(2).integers(1000, 120_000, size=40)]
    sizes[7] = 0
    runs, refs = build_runs(sizes, seed=2)
    nometa = bh.BloomFilter(bh.m_bits(5000, 10.0))
    nometa.set_batch(refs[3][0][:5000])           # filter only, no set_batch_run
    runs[12] = nometa
    gets = get_keys(refs, 100_003, 9)
    path, (cand, first, page) = routed_by(runs, lambda: bh.route_gets(runs, gets))
    assert path == "k_route"  # 40 runs: no single stack takes them all
    orefs = oracle_runs(coracle, refs)
    orefs[12] = (coracle.build(nometa.m, refs[3][0][:5000]), nometa.m, np.zeros(0, np.int32), 0)
    wc, wf, wp = coracle.route(orefs, gets)
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    assert not cand[12].any() and not cand[7].any()
    # the packed form holds a run index in 4 bits: more than 16 runs refused
    with pytest.raises(bh.BloomHipError):
        bh.route_gets_packed(runs, gets)
    packed_matches(runs[:16], gets, *coracle.route(orefs[:16], gets), path="k_route")


def test_route_device_buffers_and_strides(coracle):
    torch = pytest.importorskip("torch")
    runs, refs = build_runs([50_000, 200_000], seed=3)
    gets = get_keys(refs, 70_001, 11)
    wc, wf, wp = coracle.route(oracle_runs(coracle, refs), gets)
    n = gets.size
    dc = torch.zeros((2, (n + 63) // 64), dtype=torch.int64, device="cuda")
    df = torch.empty(n, dtype=torch.int32, device="cuda")
    dp = torch.empty(n, dtype=torch.int32, device="cuda")
    bh.route_gets(runs, torch.from_numpy(gets).cuda(), cand=dc, first=df, page=dp)
    torch.cuda.synchronize()
    assert np.array_equal(dc.cpu().numpy().view(np.uint64), wc)
    assert np.array_equal(df.cpu().numpy(), wf) and np.array_equal(dp.cpu().numpy(), wp)
    aos = np.zeros((n, 2), dtype=np.int32)
    aos[:, 0] = gets
    c2, f2, p2 = bh.route_gets(runs, aos.reshape(-1), n=n, stride=8)
    assert np.array_equal(c2, wc) and np.array_equal(f2, wf) and np.array_equal(p2, wp)
    dr = torch.empty(n, dtype=torch.int32, device="cuda")
    dc.zero_()
    bh.route_gets_packed(runs, torch.from_numpy(gets).cuda(), cand=dc, route=dr)
    torch.cuda.synchronize()
    f3, p3 = bh.unpack_route(dr.cpu().numpy().view(np.uint32))
    assert np.array_equal(dc.cpu().numpy().view(np.uint64), wc)
    assert np.array_equal(f3, wf) and np.array_equal(p3, wp)


def test_route_c3_full(coracle, golden):
    """C3 at full size: 16.8M GETs over the five level runs."""
    from bloomhip import workloads as W
    gets, levels = W.c3_runs()
    runs, orefs = [], []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch_run(keys)
        runs.append(f)
        fences, mk = coracle.run_meta(keys)
        orefs.append((coracle.build(m, keys), m, fences, mk))
    path, (cand, first, page) = routed_by(runs, lambda: bh.route_gets(runs, gets))
    assert path == "fused"  # the five levels are one ladder stack (the bench's route_c3)
    wc, wf, wp = coracle.route(orefs, gets)
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    route = packed_matches(runs, gets, wc, wf, wp, path="fused")  # the bench's route_c3 form
    rc3 = golden["oracle"]["route_c3"]
    assert hashlib.sha256(wc.tobytes()).hexdigest() == rc3["cand_sha256"]
    assert hashlib.sha256(route.tobytes()).hexdigest() == rc3["route_sha256"]
    # filter bits are the pinned C3 probe results restricted by the range check
    probe = bh.test_batch(runs, gets)
    assert ((cand & ~probe) == 0).all()


def test_route_f10_full(coracle, golden):
    """The reference's published tree (b = 1000, f = 10: runs of 512,000 *
    10^i keys): 16.8M GETs over its three level runs, whose 13,875 fences
    (55 KB) are staged in LDS by the combine with routing fused in at one
    workgroup per CU; against the oracle, and the path asserted."""
    from bloomhip import workloads as W
    gets, levels = W.f10_runs()
    runs, orefs = [], []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch_run(keys)
        runs.append(f)
        fences, mk = coracle.run_meta(keys)
        orefs.append((coracle.build(m, keys), m, fences, mk))
    assert sum(o[2].size for o in orefs) * 4 > 48 << 10  # beyond the round-4 fence budget
    path, (cand, first, page) = routed_by(runs, lambda: bh.route_gets(runs, gets))
    assert path == "fused"
    wc, wf, wp = coracle.route(orefs, gets)
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    route = packed_matches(runs, gets, wc, wf, wp, path="fused")  # the bench's f10 route form
    rf = golden["oracle"]["f10"]["route"]
    assert hashlib.sha256(wc.tobytes()).hexdigest() == rf["cand_sha256"]
    assert hashlib.sha256(route.tobytes()).hexdigest() == rf["route_sha256"]
    probe = bh.test_batch(runs, gets)
    for lvl in range(len(levels)):
        assert hashlib.sha256(probe[lvl].tobytes()).hexdigest() == \
            golden["oracle"]["f10"]["levels"][lvl]["hits_sha256"]


@pytest.mark.parametrize("layout", ["packed", "entry", "device"])
def test_route_fused_into_stacked_combine(coracle, layout):
    """Every run in one ladder stack (sizes 4096 * 4^i at 10 bits/key: m = 5 <<
    (13 + 2i)), STACKED: the routing runs inside the stack's combine
    (k_probe_combine_route) instead of k_route.  A skewed run (the page
    guess misses), a run without metadata (never a candidate), a ragged
    batch, packed / entry_t / device keys and outputs."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(31)
    sizes = [4096, 16_384, 65_536, 262_144]
    refs, runs = [], []
    for j, n in enumerate(sizes):
        if j == 2:  # skewed: a dense cluster plus a sparse tail
            keys = np.sort(np.concatenate([rng.integers(0, 100_000, size=n - 900, dtype=np.int64),
                                           rng.integers(-2**31, 2**31, size=900, dtype=np.int64)]))
            keys = keys.astype(np.int32)
        else:
            keys = sorted_run(n, 77 + j)
        m = bh.m_bits(n, 10.0)
        f = bh.BloomFilter(m)
        f.set_probe_strategy(bh.PROBE_STACKED)
        if j == 1:
            f.set_batch(keys)  # filter only: no run metadata
        else:
            f.set_batch_run(keys)
        runs.append(f)
        refs.append((keys, m))
    orefs = oracle_runs(coracle, refs)
    orefs[1] = (orefs[1][0], orefs[1][1], np.zeros(0, np.int32), 0)
    gets = get_keys(refs, 300_001, 13)
    wc, wf, wp = coracle.route(orefs, gets)
    if layout == "packed":
        path, (cand, first, page) = routed_by(runs, lambda: bh.route_gets(runs, gets))
    elif layout == "entry":
        aos = np.zeros((gets.size, 2), dtype=np.int32)
        aos[:, 0] = gets
        path, (cand, first, page) = routed_by(
            runs, lambda: bh.route_gets(runs, aos.reshape(-1), n=gets.size, stride=8))
    else:
        n = gets.size
        dc = torch.zeros((len(runs), (n + 63) // 64), dtype=torch.int64, device="cuda")
        df = torch.empty(n, dtype=torch.int32, device="cuda")
        dp = torch.empty(n, dtype=torch.int32, device="cuda")
        path, _ = routed_by(runs, lambda: bh.route_gets(runs, torch.from_numpy(gets).cuda(),
                                                         cand=dc, first=df, page=dp))
        torch.cuda.synchronize()
        cand, first, page = dc.cpu().numpy().view(np.uint64), df.cpu().numpy(), dp.cpu().numpy()
    assert path == "fused"  # the kernel under test really ran
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    assert not cand[1].any() and (first >= 0).sum() > 1000
    if layout == "packed":
        packed_matches(runs, gets, wc, wf, wp, path="fused")
    elif layout == "entry":
        packed_matches(runs, aos.reshape(-1), wc, wf, wp, path="fused", n=gets.size, stride=8)
    else:
        dr = torch.empty(n, dtype=torch.int32, device="cuda")
        dc.zero_()
        path, _ = routed_by(runs, lambda: bh.route_gets_packed(runs, torch.from_numpy(gets).cuda(),
                                                                cand=dc, route=dr))
        torch.cuda.synchronize()
        assert path == "fused"
        f3, p3 = bh.unpack_route(dr.cpu().numpy().view(np.uint32))
        assert np.array_equal(dc.cpu().numpy().view(np.uint64), wc)
        assert np.array_equal(f3, wf) and np.array_equal(p3, wp)


def test_route_fused_duplicate_fences_and_edges(coracle):
    """The fused routing (one ladder stack, STACKED) on runs whose fences
    repeat (long stretches of equal keys: upper_bound must pass them all),
    a run clustered in a narrow range next to one spread over all of int32
    (page guesses off by many fences), and GETs at, just below and just above
    every fence plus both int32 extremes."""
    rng = np.random.default_rng(41)
    sizes = [4096, 16_384, 65_536, 262_144]
    small = np.sort(rng.integers(-1000, 1000, size=sizes[0], dtype=np.int64)).astype(np.int32)
    dup = np.sort(np.repeat(rng.integers(-2**31, 2**31, size=sizes[1] // 4096, dtype=np.int64),
                            4096)).astype(np.int32)
    clustered = np.sort(np.concatenate([
        rng.integers(0, 50_000, size=sizes[2] - 300, dtype=np.int64),
        rng.integers(-2**31, 2**31, size=300, dtype=np.int64)])).astype(np.int32)
    spread = sorted_run(sizes[3], 5)
    runs, refs = [], []
    for keys in (small, dup, clustered, spread):
        assert keys.size in sizes
        m = bh.m_bits(keys.size, 10.0)
        f = bh.BloomFilter(m)
        f.set_probe_strategy(bh.PROBE_STACKED)
        f.set_batch_run(keys)
        runs.append(f)
        refs.append((keys, m))
    fences = np.concatenate([k[::4096] for k, _ in refs]).astype(np.int64)
    edge = np.clip(np.concatenate([fences - 1, fences, fences + 1]), -2**31, 2**31 - 1).astype(np.int32)
    pool = np.concatenate([k for k, _ in refs])
    gets = np.concatenate([edge, pool[rng.integers(0, pool.size, size=200_000)],
                           rng.integers(-2**31, 2**31, size=60_000, dtype=np.int64).astype(np.int32),
                           np.array([np.iinfo(np.int32).min, np.iinfo(np.int32).max], dtype=np.int32)])
    rng.shuffle(gets)
    path, (cand, first, page) = routed_by(runs, lambda: bh.route_gets(runs, gets))
    assert path == "fused"
    wc, wf, wp = coracle.route(oracle_runs(coracle, refs), gets)
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    assert (first == 1).any() and (page[first == 2] > 0).any()
    packed_matches(runs, gets, wc, wf, wp, path="fused")


@pytest.mark.parametrize("n", [100_001, 16_385])
def test_route_fused_on_super_tiles(coracle, n):
    """The f = 10 tree's filter sizes (m = 5.12M * 10^i) over runs of 5,120 *
    10^i keys (1,000 bits per key): one segment stack of 1,250 segments, so
    the probe sorts 16,384-key super-tiles and the combine with routing fused
    in takes each super-tile in two passes; a ragged batch and one key past a
    super-tile, against the oracle, the path asserted."""
    runs, refs = build_runs([5_120, 51_200, 512_000], bpe=1000.0, seed=6, probe=bh.PROBE_STACKED)
    assert [m for _, m in refs] == [5_120_000 * 10**i for i in range(3)]
    gets = get_keys(refs, n, 17)
    path, (cand, first, page) = routed_by(runs, lambda: bh.route_gets(runs, gets))
    assert path == "fused"
    wc, wf, wp = coracle.route(oracle_runs(coracle, refs), gets)
    assert np.array_equal(cand, wc) and np.array_equal(first, wf) and np.array_equal(page, wp)
    assert (first >= 0).sum() > n // 4
    packed_matches(runs, gets, wc, wf, wp, path="fused")
