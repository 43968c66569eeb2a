"""The C++ drop-in class (include/bloomhip_bloom_filter.hpp) compiles against
the C ABI and, on a GPU, gives the oracle's bitmap and hits when driven the
way src/run.cpp drives BloomFilter."""
import os
import subprocess

import numpy as np
import pytest

import bloomhip as bh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "facade_run.cpp")


@pytest.fixture(scope="module")
def facade_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("facade") / "facade_run")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), SRC,
                           "-L", bh.LIB_DIR, "-lbloomhip", f"-Wl,-rpath,{bh.LIB_DIR}", "-o", out])
    return out


def _expect(max_size, bpe, coracle):
    m = coracle.m_bits(max_size, bpe)
    keys = (np.arange(max_size, dtype=np.uint64) * np.uint64(2654435761)).astype(np.uint32).view(np.int32)
    probe = (np.arange(2 * max_size, dtype=np.uint64) * np.uint64(2654435761)).astype(np.uint32).view(np.int32)
    w = coracle.build(m, keys)
    hits = int(np.unpackbits(coracle.test(w, m, probe).view(np.uint8)).sum())
    s = 0
    for x in w.tolist():
        s = (s * 1099511628211 + x) % 2**64
    return m, coracle.popcount(w), hits, s


def test_facade_compiles_and_fails_loudly_without_gpu(facade_bin):
    if bh.device_count() > 0:
        pytest.skip("GPU present")
    r = subprocess.run([facade_bin], capture_output=True, text=True)
    assert r.returncode == 3 and "error" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("max_size,bpe", [(512, 0.5), (51_200, 10.0), (300_000, 7.7)])
def test_facade_matches_oracle(facade_bin, coracle, max_size, bpe):
    r = subprocess.run([facade_bin, str(max_size), str(bpe)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = dict(kv.split("=") for kv in r.stdout.split())
    m, pop, hits, s = _expect(max_size, bpe, coracle)
    assert int(got["m"]) == m
    assert int(got["pop"]) == pop
    assert int(got["hits"]) == hits == int(got["batch_hits"])
    assert int(got["sum"]) == s
