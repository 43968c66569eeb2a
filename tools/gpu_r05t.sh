# Experiment: C3's ladder stack on 16,384-key super-tiles at 512 bins
# (BH_LADDER_SUPER=1): ladder / C3 tests, C3 A/B against lib_alt, rocprofv3
set -o pipefail
mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
export BH_LADDER_SUPER=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread -k "ladder or c3 or route_fused" > gpurun_out/r05t/pytest.log 2>&1 || { tail -40 gpurun_out/r05t/pytest.log; exit 1; }
tail -2 gpurun_out/r05t/pytest.log
timeout -k 10 300 python -u tools/probe_ab.py 4 c3 > gpurun_out/r05t/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05t/ab_c3.log; exit 1; }
tail -2 gpurun_out/r05t/ab_c3.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t/new -o run --output-format csv -- python tools/probe_prof.py auto 30 > gpurun_out/r05t/new.log 2>&1 || { tail -20 gpurun_out/r05t/new.log; exit 1; }
echo ok
