# Stacked probe on super-tiles: the whole GPU suite, then the f10 and C3
# probe / routing A/B against lib_alt (tools/build_alt.sh HEAD)
set -o pipefail
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05m/pytest.log 2>&1 || { tail -40 gpurun_out/r05m/pytest.log; exit 1; }
tail -2 gpurun_out/r05m/pytest.log
timeout -k 10 300 python -u tools/probe_ab.py 4 f10 > gpurun_out/r05m/ab_f10.log 2>&1 || { tail -20 gpurun_out/r05m/ab_f10.log; exit 1; }
tail -10 gpurun_out/r05m/ab_f10.log
timeout -k 10 300 python -u tools/probe_ab.py 3 c3 > gpurun_out/r05m/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05m/ab_c3.log; exit 1; }
tail -3 gpurun_out/r05m/ab_c3.log
