"""The drop-in boundary, end to end.

1. src/run.cpp compiles UNCHANGED against the 3-line src/bloom_filter.h of
   INTEGRATION.md (include/dropin/bloom_filter.h), with the reference
   Makefile's own `g++ -std=c++11` (Makefile:4).
2. The reference's whole LSM binary, built from its own sources with that
   header and linked against libbloomhip (oracle/Makefile `ref`), passes the
   reference's own golden tests (test/test-{1..6}, scripts/test.py:15-46):
   tests 1-4 never flush (no filter is built: they run on the CPU), tests 5
   and 6 flush runs, so their filters are built and probed on the GPU.
3. test-6, the only reference test whose output depends on the filter
   (`g 1535` -> out line 2 `1535`), replayed through the C++ facade: three
   256-bit run filters, bitmaps equal to the oracle's, is_set(1535) true on
   the newest run.

The reference sources are read only at build time in the build container
(skipped where /root/reference is absent); the golden tests' inputs and
outputs travel as data (tests/golden/ref_tests.json, made by
tests/golden/make_ref_tests.py).
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import bloomhip as bh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
INCLUDE = os.path.join(ROOT, "include")
LSM_BIN = os.path.join(ROOT, "oracle", "_ref", "lsm_bloomhip")
with open(os.path.join(ROOT, "tests", "golden", "ref_tests.json")) as _f:
    REF_TESTS = json.load(_f)["tests"]
# tests whose workload flushes the buffer (builds run filters): GPU only
FLUSHING = {"test-5", "test-6"}

needs_reference = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")),
                                     reason="reference sources only in the build container")


def dsl(ops):
    """The reference's workload lines (src/main.cpp:15-47) from fixture ops."""
    out = []
    for op in ops:
        if op[0] == "l":
            out.append(f'l "{op[1]}"')
        else:
            out.append(" ".join(str(x) for x in op))
    return "\n".join(out) + "\n"


@needs_reference
def test_reference_run_cpp_compiles_unchanged(tmp_path):
    # run.cpp, run.h, types.h as they are, bloom_filter.h
    # replaced by the drop-in header, the reference's own compiler line.
    for name in ("run.cpp", "run.h", "types.h"):
        shutil.copy(os.path.join(REF, "src", name), tmp_path / name)
    shutil.copy(os.path.join(INCLUDE, "dropin", "bloom_filter.h"), tmp_path / "bloom_filter.h")
    r = subprocess.run(["g++", "-std=c++11", "-g", "-I", str(tmp_path), "-I", INCLUDE, "-c",
                        str(tmp_path / "run.cpp"), "-o", str(tmp_path / "run.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # Run's filter calls resolve to the engine's C ABI
    syms = subprocess.run(["nm", "-u", str(tmp_path / "run.o")], capture_output=True,
                          text=True).stdout
    for s in ("bloomhip_create", "bloomhip_set_batch", "bloomhip_is_set"):
        assert s in syms


@needs_reference
def test_reference_lsm_links_against_engine():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "ref"])
    assert os.access(LSM_BIN, os.X_OK)
    ldd = subprocess.run(["ldd", LSM_BIN], capture_output=True, text=True).stdout
    assert "libbloomhip.so" in ldd and "boost" not in ldd


def run_reference_test(name, tmp_path):
    t = REF_TESTS[name]
    for fname, hexdata in t["files"].items():
        (tmp_path / fname).write_bytes(bytes.fromhex(hexdata))
    r = subprocess.run([LSM_BIN] + t["params"], input=dsl(t["ops"]), capture_output=True,
                       text=True, cwd=tmp_path, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout == t["expected_stdout"]


needs_lsm = pytest.mark.skipif(not os.access(LSM_BIN, os.X_OK),
                               reason="oracle/_ref/lsm_bloomhip not built (no reference tree)")


@needs_lsm
@pytest.mark.parametrize("name", sorted(set(REF_TESTS) - FLUSHING))
def test_reference_golden_test_buffer_only(name, tmp_path):
    run_reference_test(name, tmp_path)


@needs_lsm
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FLUSHING))
def test_reference_golden_test_through_gpu_filter(name, tmp_path):
    run_reference_test(name, tmp_path)


def _test6_runs():
    """The three runs test-6's `-b 1` flushes: the 1537 puts in order, 512 per
    flush (src/lsm_tree.cpp:104-139), the last put stays in the buffer."""
    puts = [op for op in REF_TESTS["test-6"]["ops"] if op[0] == "p"]
    assert len(puts) == 1537
    buffer_max = 512  # 1 page * 4096 B / sizeof(entry_t) (src/main.cpp:89)
    runs = [puts[i:i + buffer_max] for i in range(0, 3 * buffer_max, buffer_max)]
    return [[k for _, k, _ in r] for r in runs]


def test_test6_fixture_shape(coracle):
    runs = _test6_runs()
    assert runs[2][-1] == 1535 and ["g", 1535] in REF_TESTS["test-6"]["ops"]
    assert REF_TESTS["test-6"]["expected_stdout"].splitlines()[1] == "1535"
    assert coracle.m_bits(512, 0.5) == 256
    # the oracle agrees that 1535 is set in the newest run's filter
    w = coracle.build(256, np.array(runs[2], dtype=np.int32))
    assert coracle.test(w, 256, np.array([1535], dtype=np.int32))[0] & 1


@pytest.fixture(scope="module")
def test6_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("test6") / "test6_runs")
    subprocess.check_call(["g++", "-O2", "-std=c++11", "-I", INCLUDE,
                           os.path.join(ROOT, "tests", "cpp", "test6_runs.cpp"),
                           "-L", bh.LIB_DIR, "-lbloomhip", f"-Wl,-rpath,{bh.LIB_DIR}", "-o", out])
    return out


@pytest.mark.gpu
def test_reference_test6_through_facade(test6_bin, coracle):
    runs = _test6_runs()
    stdin = "".join(f"{r} {k}\n" for r, keys in enumerate(runs) for k in keys)
    r = subprocess.run([test6_bin, "1535", "1", "0"], input=stdin, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    # newest first, as the level's deque
    for i, keys in enumerate(reversed(runs)):
        want = coracle.build(256, np.array(keys, dtype=np.int32))
        f = lines[i].split()
        assert f[0] == f"run{i}" and f[1] == "m=256"
        assert [int(x, 16) for x in f[2:]] == [int(x) for x in want]
    ans = {int(l.split()[1]): int(l.split()[2]) for l in lines if l.startswith("is_set")}
    assert ans[1535] == 1  # out line 2 of test-6
    newest = coracle.build(256, np.array(runs[2], dtype=np.int32))
    for k in (1, 0):
        assert ans[k] == int(coracle.test(newest, 256, np.array([k], dtype=np.int32))[0] & 1)
