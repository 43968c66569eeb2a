# Strided segment-stack pass 2: stack / f10 tests, then the f10 and C3 probe
# A/B against lib_alt (tools/build_alt.sh HEAD)
set -o pipefail
mkdir -p gpurun_out/r05l
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread -k "stack or f10 or c3_probe" > gpurun_out/r05l/pytest.log 2>&1 || { tail -30 gpurun_out/r05l/pytest.log; exit 1; }
tail -2 gpurun_out/r05l/pytest.log
timeout -k 10 300 python -u tools/probe_ab.py 4 f10 > gpurun_out/r05l/ab_f10.log 2>&1 || { tail -20 gpurun_out/r05l/ab_f10.log; exit 1; }
tail -10 gpurun_out/r05l/ab_f10.log
timeout -k 10 300 python -u tools/probe_ab.py 3 c3 > gpurun_out/r05l/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05l/ab_c3.log; exit 1; }
tail -3 gpurun_out/r05l/ab_c3.log
