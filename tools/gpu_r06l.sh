#!/bin/bash
# Round-6: the f = 10 tree's stacked probe pass 2 on two interleaved chains
# at 8192-key tiles (the fused f10 route) on two chains of one vector (WALK 11) vs WALK 2; stacked-probe tests.
set -o pipefail
OUT=gpurun_out/r06l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py -m gpu -x -q -k "stack or route" --timeout 300 --timeout-method thread > $OUT/pytest_stack.log 2>&1 || { tail -30 $OUT/pytest_stack.log; exit 1; }
tail -1 $OUT/pytest_stack.log
timeout -k 10 500 python tools/probe_ab.py 4 f10 > $OUT/probe_ab_f10.log 2>&1 || exit 1
tail -4 $OUT/probe_ab_f10.log
