# f10 routing back on 8192-key tiles when the fused super-tile combine would
# run one workgroup per CU: route tests, then the f10 / C3 A/B
set -o pipefail
mkdir -p gpurun_out/r05o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_route.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "route or super or f10 or stack" > gpurun_out/r05o/pytest.log 2>&1 || { tail -40 gpurun_out/r05o/pytest.log; exit 1; }
tail -2 gpurun_out/r05o/pytest.log
timeout -k 10 300 python -u tools/probe_ab.py 4 f10 > gpurun_out/r05o/ab_f10.log 2>&1 || { tail -20 gpurun_out/r05o/ab_f10.log; exit 1; }
tail -2 gpurun_out/r05o/ab_f10.log
timeout -k 10 300 python -u tools/probe_ab.py 3 c3 > gpurun_out/r05o/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05o/ab_c3.log; exit 1; }
tail -2 gpurun_out/r05o/ab_c3.log
