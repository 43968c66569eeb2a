set -o pipefail
D=gpurun_out/xp14; mkdir -p $D
timeout -k 10 200 python tools/ubench.py stack > $D/stack.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stack" --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit 1
