# The plain combine stages its result bytes with every load first: tests, C3 / f10 A/B
# stack / ladder / f10 / C3 tests, then the C3 and f10 probe A/B
set -o pipefail
mkdir -p gpurun_out/r05ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread -k "stack or ladder or f10 or c3 or route or super" > gpurun_out/r05ab/pytest.log 2>&1 || { tail -40 gpurun_out/r05ab/pytest.log; exit 1; }
tail -2 gpurun_out/r05ab/pytest.log
timeout -k 10 300 python -u tools/probe_ab.py 4 c3 > gpurun_out/r05ab/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05ab/ab_c3.log; exit 1; }
tail -2 gpurun_out/r05ab/ab_c3.log
timeout -k 10 300 python -u tools/probe_ab.py 3 f10 > gpurun_out/r05ab/ab_f10.log 2>&1 || { tail -20 gpurun_out/r05ab/ab_f10.log; exit 1; }
tail -2 gpurun_out/r05ab/ab_f10.log
