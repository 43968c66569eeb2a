set -o pipefail
D=gpurun_out/xp12; mkdir -p $D
UB_T4K=1 timeout -k 10 200 python tools/ubench.py part_c5 > $D/part_c5_t4k.log 2>&1 || exit 1
UB_P1=1 timeout -k 10 200 python tools/ubench.py part > $D/part_p1.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-extras --no-cpu-baseline > $D/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline > $D/bench_c5.log 2>&1 || exit 1
