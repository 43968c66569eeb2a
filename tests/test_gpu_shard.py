"""Filter replication (bloomhip_clone) for the probe side of per-run
sharding: on a one-GPU box the clone is a device-to-device copy;
between GPUs it is a peer copy over xGMI (same code path, hipMemcpyPeer)."""
import numpy as np
import pytest

import bloomhip as bh

pytestmark = pytest.mark.gpu


def rand_keys(n, seed):
    return np.random.default_rng(seed).integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)


@pytest.mark.parametrize("m", [1000, 655_360, 167_772_160])
def test_clone_is_identical_and_independent(coracle, m):
    keys = np.sort(rand_keys(200_000, m % 97))
    f = bh.BloomFilter(m)
    f.set_batch_run(keys)
    c = f.clone()
    assert (c.words() == f.words()).all()
    assert (c.words() == coracle.build(m, keys)).all()
    fa, ma = f.run_meta()
    fb, mb = c.run_meta()
    assert np.array_equal(fa, fb) and ma == mb
    probe = rand_keys(100_003, 5)
    probe[:50_000] = keys[:50_000]
    assert (bh.test_batch([c], probe)[0] == bh.test_batch([f], probe)[0]).all()
    # independent storage: changing the clone leaves the source alone
    before = f.words().copy()
    c.set_batch(rand_keys(50_000, 6))
    assert (f.words() == before).all()


def test_clone_of_cleared_and_fresh_filters():
    f = bh.BloomFilter(10_000)
    f.set_batch(rand_keys(1000, 1))
    f.clear()
    assert not f.clone().words().any()
    assert not bh.BloomFilter(777).clone().words().any()


def test_clone_to_a_missing_device_fails():
    f = bh.BloomFilter(1000)
    with pytest.raises(bh.BloomHipError):
        f.clone(device=bh.device_count() + 3)


def test_sharded_probe_slices_concatenate(coracle):
    """One process standing in for N ranks: each slice probed against a replica."""
    from bloomhip import shard
    m = 10_485_760
    keys = rand_keys(1_000_000, 9)
    f = bh.BloomFilter(m)
    f.set_batch(keys)
    gets = rand_keys(300_017, 10)
    gets[:100_000] = keys[:100_000]
    want = coracle.test(coracle.build(m, keys), m, gets)
    for world in (2, 3, 8):
        rows = []
        for r in range(world):
            lo, hi = shard.probe_slice(gets.size, r, world)
            rows.append(bh.test_batch([f.clone()], gets[lo:hi].copy())[0])
        assert np.array_equal(np.concatenate(rows), want), world


# ---- two or more GPUs in one process (skipped on a one-GPU box; the
# driver's 8-GPU node runs them): the cross-device paths of SURVEY §8e.
multi_gpu = pytest.mark.skipif(bh.device_count() < 2, reason="needs >= 2 GPUs")


@multi_gpu
@pytest.mark.parametrize("m", [655_360, 167_772_160])
def test_clone_across_devices_peer_copy(coracle, m):
    """bloomhip_clone to another GPU: hipMemcpyPeer over xGMI; the replica
    probes on its own device with the source's answers."""
    keys = np.sort(rand_keys(300_000, m % 89))
    f = bh.BloomFilter(m, device=0)
    f.set_batch_run(keys)
    want = coracle.build(m, keys)
    probe = rand_keys(200_003, 7)
    probe[:100_000] = keys[:100_000]
    ref = bh.test_batch([f], probe)[0]
    for dev in range(1, bh.device_count()):
        c = f.clone(device=dev)
        assert c.device == dev
        assert (c.words() == want).all(), dev
        fa, ma = f.run_meta()
        fb, mb = c.run_meta()
        assert np.array_equal(fa, fb) and ma == mb
        assert (bh.test_batch([c], probe)[0] == ref).all(), dev


@multi_gpu
def test_per_run_builds_on_two_devices_match_pins(golden):
    """configs[4]'s sharding rule in one process: run r of the C5 fan-in on
    device r % G (bloomhip/shard.py), every bitmap equal to its pinned digest
    (two runs per device keeps it short)."""
    import hashlib
    from bloomhip import shard
    from bloomhip import workloads as W
    G = min(2, bh.device_count())
    for r in range(2 * G):
        dev = shard.rank_for_run(r, G)  # one device standing for each rank
        assert dev == r % G
        keys, m = W.c5_run(r)
        f = bh.BloomFilter(m, device=dev)
        f.set_batch(keys)
        assert hashlib.sha256(f.words().tobytes()).hexdigest() == golden["oracle"]["c5"][r]["sha256"], r
