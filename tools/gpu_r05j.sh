set -o pipefail
mkdir -p gpurun_out/r05j
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread -k "route" > gpurun_out/r05j/pytest.log 2>&1 || { tail -30 gpurun_out/r05j/pytest.log; exit 1; }
tail -2 gpurun_out/r05j/pytest.log
true
