"""The N>1 path on CPU: world_size-2 gloo processes shard C5-style runs one
per rank (run r on rank r mod N), build them (with the oracle standing in for
the GPU), and check the gathered per-run digests and the max-time reduction
bench.py uses.  No collective touches filter data."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from bloomhip import shard

N_RUNS = 8
RUN_KEYS = 20_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_keys(r):
    import bloomhip as bh
    return bh.gen_puts(13141 + r, RUN_KEYS), bh.m_bits(RUN_KEYS, 10.0)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path[:0] = [p for p in os.environ.get("BLOOMHIP_TEST_PATH", "").split(":") if p]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bloom_oracle import COracle
        C = COracle()

        def build(r):
            keys, m = _run_keys(r)
            return C.build(m, keys)

        local = shard.build_my_runs(N_RUNS, rank, world, build)
        allr = shard.gather_digests(local, dist)
        t = shard.max_over_ranks(float(rank + 1), dist)
        ok = shard.all_ranks_ok(True, dist)
        q.put((rank, sorted(local), allr, t, ok))
    finally:
        dist.destroy_process_group()


def test_probe_slices_partition_the_gets():
    for n in (0, 1, 63, 64, 65, 16_777_216, 1_000_003):
        for world in (1, 2, 3, 4, 8):
            sl = [shard.probe_slice(n, r, world) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == n
            for (a, b), (c, d) in zip(sl, sl[1:]):
                assert b == c and a <= b
            for a, b in sl[:-1]:
                assert a % 64 == 0 and b % 64 == 0     # packed words never straddle ranks
    with pytest.raises(ValueError):
        shard.probe_slice(10, 2, 2)


def _probe_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path[:0] = [p for p in os.environ.get("BLOOMHIP_TEST_PATH", "").split(":") if p]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bloomhip as bh
        from bloom_oracle import COracle
        C = COracle()
        # every rank holds replicas of the same run filters ...
        filters = []
        for r in range(3):
            keys, m = _run_keys(r)
            filters.append((C.build(m, keys), m))
        gets = bh.gen_puts(777, 50_017)
        gets[:20_000] = _run_keys(1)[0][:20_000]
        # ... and probes its own contiguous slice of the GETs
        lo, hi = shard.probe_slice(gets.size, rank, world)
        rows = [C.test(w, m, gets[lo:hi]) for w, m in filters]
        parts = [None] * world
        dist.all_gather_object(parts, (lo, hi, rows))
        hits = shard.sum_over_ranks(sum(int(np.unpackbits(r.view(np.uint8)).sum()) for r in rows),
                                    dist)
        q.put((rank, parts, hits))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_probe(coracle):
    """Probe side of §8e: replicated filters, GETs sharded by probe_slice; the
    ranks' packed rows concatenate into the single-process result."""
    import bloomhip as bh
    world = 2
    port = _free_port()
    os.environ["BLOOMHIP_TEST_PATH"] = ":".join(sys.path[:3])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_probe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gets = bh.gen_puts(777, 50_017)
    gets[:20_000] = _run_keys(1)[0][:20_000]
    for rank, parts, hits in res:
        total = 0
        for r in range(3):
            keys, m = _run_keys(r)
            want = coracle.test(coracle.build(m, keys), m, gets)
            got = np.concatenate([p[2][r] for p in parts])
            assert np.array_equal(got, want), r
            total += int(np.unpackbits(want.view(np.uint8)).sum())
        assert hits == total


def test_assignment_is_a_partition():
    for world in (1, 2, 4, 8):
        runs = [r for k in range(world) for r in shard.runs_for_rank(N_RUNS, k, world)]
        assert shard.covers(runs, N_RUNS)
    assert shard.runs_for_rank(8, 1, 2) == [1, 3, 5, 7]
    with pytest.raises(ValueError):
        shard.runs_for_rank(8, 2, 2)


def test_gloo_world2_sharded_builds(coracle):
    world = 2
    port = _free_port()
    os.environ["BLOOMHIP_TEST_PATH"] = ":".join(sys.path[:3])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {}
    for r in range(N_RUNS):
        keys, m = _run_keys(r)
        want[r] = shard.digest(coracle.build(m, keys))
    for rank, mine, allr, t, ok in res:
        assert mine == shard.runs_for_rank(N_RUNS, rank, world)
        assert allr == want                      # every run built once, correctly
        assert t == float(world)                 # max over ranks
        assert ok
