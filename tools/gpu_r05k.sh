# Route page search A/B: route tests on the new build, then the C3 probe /
# routing A/B against lib_alt (tools/build_alt.sh HEAD)
set -o pipefail
mkdir -p gpurun_out/r05k
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05k/pytest.log 2>&1 || { tail -30 gpurun_out/r05k/pytest.log; exit 1; }
tail -2 gpurun_out/r05k/pytest.log
timeout -k 10 400 python -u tools/probe_ab.py 4 c3 > gpurun_out/r05k/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05k/ab_c3.log; exit 1; }
tail -12 gpurun_out/r05k/ab_c3.log
timeout -k 10 300 python -u tools/probe_ab.py 3 f10 > gpurun_out/r05k/ab_f10.log 2>&1 || { tail -20 gpurun_out/r05k/ab_f10.log; exit 1; }
tail -10 gpurun_out/r05k/ab_f10.log
