#!/bin/bash
# Round-6 (throwaway): the fused route's answers stored non-temporal
# (lib_alt = HEAD): routing tests, C3 / f10 routing A/B, one bench A/B.
set -o pipefail
OUT=gpurun_out/r06ae; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_route.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_route.log 2>&1 || { tail -30 $OUT/pytest_route.log; exit 1; }
tail -1 $OUT/pytest_route.log
timeout -k 10 500 python tools/probe_ab.py 3 c3 > $OUT/probe_ab_c3.log 2>&1 || exit 1
tail -2 $OUT/probe_ab_c3.log
tools/ab.sh r06ae/ab 2 --steps 100 --no-c4 --no-c5 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
