"""The C ABI's lock order under concurrent callers: handles are
locked in address order, workspaces after handles, and the workspace map
(bloomhip_trim) never inside a workspace lock.  Each scenario runs its
threads against a deadline: a deadlock fails the test instead of hanging it,
and every result is still checked against the oracle."""
import threading

import numpy as np
import pytest

import bloomhip as bh

pytestmark = pytest.mark.gpu
DEADLINE_S = 90


def _run_all(fns):
    errors = []

    def wrap(fn):
        def go():
            try:
                fn()
            except Exception as e:  # noqa: BLE001 - reported below
                errors.append(repr(e))
        return go
    threads = [threading.Thread(target=wrap(fn), daemon=True) for fn in fns]
    for t in threads:
        t.start()
    for t in threads:
        t.join(DEADLINE_S)
    stuck = [t for t in threads if t.is_alive()]
    assert not stuck, f"{len(stuck)} thread(s) still blocked after {DEADLINE_S} s: lock-order deadlock"
    assert not errors, errors


def _runs(seed, sizes):
    rng = np.random.default_rng(seed)
    out = []
    for n in sizes:
        k = np.unique(rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32))
        out.append(np.ascontiguousarray(np.stack([k, k], axis=1)))
    return out


def test_trim_during_compaction_with_filter(coracle):
    # bloomhip_compact(filter=f) holds its workspace across the build of f
    # (partition strategy: m beyond LDS, >= 64K keys), which looks the
    # workspace up again; bloomhip_trim takes the workspace map and then
    # each workspace.  r02 took them in opposite orders.
    runs = _runs(1, [300_000, 200_000, 100_000])
    total = sum(r.shape[0] for r in runs)
    m = bh.m_bits(total, 10.0)
    f = bh.BloomFilter(m)
    assert f.resolve_strategy(total) == bh.BUILD_PARTITION
    want = coracle.compact(runs, False)
    got = {}

    def compactions():
        for _ in range(15):
            f.clear()
            got["run"] = bh.compact(runs, filter=f)

    def trims():
        for _ in range(60):
            bh.lib().bloomhip_trim()

    _run_all([compactions, trims])
    assert np.array_equal(got["run"], want)
    assert (f.words() == coracle.build(m, want[:, 0].copy())).all()


def test_multi_filter_probes_in_opposite_orders_with_a_compaction(coracle):
    ka = np.random.default_rng(2).integers(-2**31, 2**31, size=400_000, dtype=np.int64).astype(np.int32)
    kb = np.random.default_rng(3).integers(-2**31, 2**31, size=400_000, dtype=np.int64).astype(np.int32)
    ma, mb = bh.m_bits(ka.size, 10.0), bh.m_bits(kb.size, 8.0)
    a, b = bh.BloomFilter(ma), bh.BloomFilter(mb)
    a.set_batch(ka)
    b.set_batch(kb)
    probe = np.concatenate([ka[:100_000], kb[:100_000],
                            np.random.default_rng(4).integers(-2**31, 2**31, size=100_000,
                                                              dtype=np.int64).astype(np.int32)])
    want_a = coracle.test(coracle.build(ma, ka), ma, probe)
    want_b = coracle.test(coracle.build(mb, kb), mb, probe)
    runs = _runs(5, [200_000, 150_000])
    total = sum(r.shape[0] for r in runs)
    c = bh.BloomFilter(bh.m_bits(total, 10.0))
    bad = []

    def ab():
        for _ in range(20):
            r = bh.test_batch([a, b], probe)
            if not ((r[0] == want_a).all() and (r[1] == want_b).all()):
                bad.append("ab")

    def ba():
        for _ in range(20):
            r = bh.test_batch([b, a], probe)
            if not ((r[0] == want_b).all() and (r[1] == want_a).all()):
                bad.append("ba")

    def compactions():
        for _ in range(10):
            c.clear()
            bh.compact(runs, filter=c)

    def trims():
        for _ in range(30):
            bh.lib().bloomhip_trim()

    _run_all([ab, ba, compactions, trims])
    assert not bad, bad


def test_trim_returns_device_memory_to_baseline(coracle):
    # a caller that looked a workspace up just before bloomhip_trim
    # took the map could regrow its buffers after trim freed them, in a
    # workspace no longer in the map (never freed again).  Trim now retires
    # the workspaces it takes and late callers look the map up again, so
    # after a final trim the device's free memory is back where it was.
    import torch
    runs = _runs(6, [300_000, 200_000, 100_000])
    total = sum(r.shape[0] for r in runs)
    m = bh.m_bits(total, 10.0)
    f = bh.BloomFilter(m)
    want = coracle.compact(runs, False)
    bh.compact(runs, filter=f)  # the handle's own staging exists from here on
    bh.lib().bloomhip_trim()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]

    def compactions():
        for _ in range(20):
            f.clear()
            assert np.array_equal(bh.compact(runs, filter=f), want)

    def trims():
        for _ in range(80):
            bh.lib().bloomhip_trim()

    _run_all([compactions, compactions, trims])
    bh.lib().bloomhip_trim()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    # one workspace of this size is ~20 MB: a leaked one shows
    assert free1 >= free0 - (4 << 20), (free0 - free1) / 2**20
