set -o pipefail
D=gpurun_out/xp22; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c5 > $D/bench.log 2>&1 || exit 1
