set -o pipefail
D=gpurun_out/xp18; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $D/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline > $D/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline > $D/bench_c5.log 2>&1 || exit 1
