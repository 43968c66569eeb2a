# Experiment: builds of 257-511 segments on 4096-key tiles (three pass-1
# workgroups per CU, runs of ~24): build tests, then the f10 build A/B
set -o pipefail
mkdir -p gpurun_out/r05u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "build" > gpurun_out/r05u/pytest.log 2>&1 || { tail -40 gpurun_out/r05u/pytest.log; exit 1; }
tail -2 gpurun_out/r05u/pytest.log
timeout -k 10 300 python -u tools/build_ab.py 4 f10 > gpurun_out/r05u/ab_f10.log 2>&1 || { tail -20 gpurun_out/r05u/ab_f10.log; exit 1; }
tail -10 gpurun_out/r05u/ab_f10.log
timeout -k 10 300 python -u tools/build_ab.py 2 c2 > gpurun_out/r05u/ab_c2.log 2>&1 || { tail -20 gpurun_out/r05u/ab_c2.log; exit 1; }
tail -2 gpurun_out/r05u/ab_c2.log
