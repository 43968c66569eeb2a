#!/bin/bash
# Round-6: the fused route page search between per-run sentinels (unguarded halving, one two-word window check)
set -o pipefail
OUT=gpurun_out/r06o; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_route.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_route.log 2>&1 || { tail -30 $OUT/pytest_route.log; exit 1; }
tail -1 $OUT/pytest_route.log
timeout -k 10 500 python tools/probe_ab.py 3 c3 > $OUT/probe_ab_c3.log 2>&1 || exit 1
tail -2 $OUT/probe_ab_c3.log
timeout -k 10 500 python tools/probe_ab.py 3 f10 > $OUT/probe_ab_f10.log 2>&1 || exit 1
tail -2 $OUT/probe_ab_f10.log
