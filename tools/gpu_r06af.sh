#!/bin/bash
# Round-6: the merge / clear-and-rebuild writeback test.
set -o pipefail
OUT=gpurun_out/r06af; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "merge_then_clear" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -5 $OUT/pytest.log
