"""GPU tests of §8f row 2: a filter saved beside its run and loaded back,
and a filter rebuilt from the run file (entry_t AoS records, 8-B stride)
— bit-exact against the C oracle."""
import numpy as np
import pytest

import bloomhip as bh

pytestmark = pytest.mark.gpu


def run_entries(n, seed):
    rng = np.random.default_rng(seed)
    keys = np.unique(rng.integers(-2**31, 2**31, size=n + n // 4 + 8, dtype=np.int64)
                     .astype(np.int32))[:n]
    run = np.zeros((keys.size, 2), dtype=np.int32)
    run[:, 0] = keys
    run[:, 1] = rng.integers(0, 2**31, size=keys.size, dtype=np.int64).astype(np.int32)
    return run


@pytest.mark.parametrize("m", [1, 65, 655_360, 167_772_160])
def test_save_load_round_trip(coracle, tmp_path, m):
    run = run_entries(min(200_000, max(10, m // 10)), m % 97)
    f = bh.BloomFilter(m)
    f.set_batch_run(run.reshape(-1), n=run.shape[0], stride=8)
    p = str(tmp_path / "run.bloom")
    f.save(p)
    g = bh.BloomFilter.load(p)
    assert g.m == m
    assert (g.words() == coracle.build(m, run[:, 0])).all()
    fences, mk = g.run_meta()
    want = coracle.run_meta(run[:, 0])
    assert np.array_equal(fences, want[0]) and mk == want[1]
    probe = np.concatenate([run[:1000, 0], np.arange(-500, 500, dtype=np.int32)])
    assert (bh.test_batch([g], probe)[0] == coracle.test(coracle.build(m, run[:, 0]), m, probe)).all()


def test_load_rejects_damaged_and_foreign_files(tmp_path):
    f = bh.BloomFilter(10_000)
    f.set_batch_run(np.arange(0, 3000, dtype=np.int32))
    p = tmp_path / "a.bloom"
    f.save(str(p))
    data = bytearray(p.read_bytes())
    for cut in (0, 20, len(data) - 1):
        q = tmp_path / f"cut{cut}.bloom"
        q.write_bytes(bytes(data[:cut]))
        with pytest.raises(bh.BloomHipError):
            bh.BloomFilter.load(str(q))
    data[100] ^= 0x10                       # one flipped bit: checksum mismatch
    q = tmp_path / "flip.bloom"
    q.write_bytes(bytes(data))
    with pytest.raises(bh.BloomHipError):
        bh.BloomFilter.load(str(q))
    with pytest.raises(bh.BloomHipError):
        bh.BloomFilter.load(str(tmp_path / "missing.bloom"))


@pytest.mark.parametrize("n", [0, 1, 51_200, 300_001])
def test_build_from_run_file(coracle, tmp_path, n):
    """A run file as Run::map_write leaves it: max_size entry_t slots, the
    first n written (src/run.cpp:34-72, src/run.h:19)."""
    max_size = max(n, 1) + 1000
    run = run_entries(n, n + 3)
    n = run.shape[0]
    buf = np.zeros((max_size, 2), dtype=np.int32)
    buf[:n] = run
    p = tmp_path / "run.dat"
    p.write_bytes(buf.tobytes())
    f = bh.BloomFilter.from_run_file(str(p), n, max_size, 10.0)
    m = coracle.m_bits(max_size, 10.0)
    assert f.m == m
    assert (f.words() == coracle.build(m, run[:, 0])).all()
    fences, mk = f.run_meta()
    want = coracle.run_meta(run[:, 0])
    assert np.array_equal(fences, want[0]) and mk == want[1]
    with pytest.raises(bh.BloomHipError):     # file shorter than n entries
        bh.BloomFilter.from_run_file(str(p), max_size + 1, max_size, 10.0)
