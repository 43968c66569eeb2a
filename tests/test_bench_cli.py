"""bench.py's launch contract (CPU only, no GPU touched).

`python bench.py --gpus N` must either measure N GPUs or fail: it starts N
ranks itself when no launcher set WORLD_SIZE (one process per
GPU), refuses a WORLD_SIZE that differs from --gpus, and propagates a rank's
failure as its own non-zero exit status.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr


def test_bad_gpu_count_exits_nonzero():
    r = _run(["--gpus", "0"], {})
    assert r.returncode == 2


def test_self_launch_starts_ranks_and_propagates_failure():
    # No GPU here: the two ranks it starts fail at device selection, and the
    # parent must report that as a non-zero exit, never as a 1-GPU line.
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-extras",
              "--no-cpu-baseline", "--prewarm-s", "0"], {"BLOOMHIP_DIST_BACKEND": "gloo"})
    assert r.returncode != 0
    assert "exited with" in r.stderr
    assert '"n_gpus": 1' not in r.stdout


def test_launch_ranks_sets_rank_environment(tmp_path, monkeypatch):
    # launch_ranks re-runs bench.py; point it at a stand-in script that
    # reports the rank environment it was given.
    sys.path.insert(0, ROOT)
    import bench
    probe = tmp_path / "probe.py"
    out = tmp_path / "ranks"
    out.mkdir()
    probe.write_text(
        "import os, sys\n"
        f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write(\n"
        "    ' '.join(os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', "
        "'MASTER_ADDR')) + ' ' + ' '.join(sys.argv[1:]))\n")
    monkeypatch.setattr(bench, "__file__", str(probe))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "3", "--steps", "7"])
    assert bench.launch_ranks(3) == 0
    got = sorted(p.read_text() for p in out.iterdir())
    assert got == [f"{r} {r} 3 127.0.0.1 --gpus 3 --steps 7" for r in range(3)]
