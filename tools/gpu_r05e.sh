set -o pipefail
mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -x -q --timeout 300 --timeout-method thread -k "build or c4 or c5 or c2 or compact or f10 or host_keys or super" > gpurun_out/r05e/pytest.log 2>&1 || { tail -30 gpurun_out/r05e/pytest.log; exit 1; }
tail -2 gpurun_out/r05e/pytest.log
bash tools/gpu_ab_r05.sh r05e c4,c2
timeout -k 10 300 python tools/ubench.py ladder > gpurun_out/r05e/ub_ladder.log 2>&1 || { tail -5 gpurun_out/r05e/ub_ladder.log; exit 1; }; grep -v amdgpu.ids gpurun_out/r05e/ub_ladder.log | grep "round\": 1" | cut -c1-250
bash tools/gpu_steps.sh r05e_prof stats_f10 && python tools/kstats.py gpurun_out/r05e_prof/stats_f10 2>/dev/null | head -20
