# The loads-first run-table transpose: build / C4 / compaction / super tests, C4 A/B
set -o pipefail
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -x -q --timeout 300 --timeout-method thread -k "build or c4 or compact or super" > gpurun_out/r05w/pytest.log 2>&1 || { tail -30 gpurun_out/r05w/pytest.log; exit 1; }
tail -2 gpurun_out/r05w/pytest.log
bash tools/gpu_ab_r05.sh r05w c4
