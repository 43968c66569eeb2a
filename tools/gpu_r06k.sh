#!/bin/bash
# Round-6: the f = 10 tree's stacked probe pass 2 on two interleaved chains
# (WALK 7) vs two vectors per lane (WALK 3, lib_alt = HEAD); stacked-probe tests.
set -o pipefail
OUT=gpurun_out/r06k; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stack" --timeout 300 --timeout-method thread > $OUT/pytest_stack.log 2>&1 || { tail -30 $OUT/pytest_stack.log; exit 1; }
tail -1 $OUT/pytest_stack.log
timeout -k 10 500 python tools/probe_ab.py 4 f10 > $OUT/probe_ab_f10.log 2>&1 || exit 1
tail -4 $OUT/probe_ab_f10.log
