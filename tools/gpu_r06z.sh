#!/bin/bash
# Round-6: pass 1's sorted tiles stored non-temporal when they exceed the
# Infinity Cache (C5's k_part_bin at 1024 lanes by template, C4's k_part_bin2
# by a uniform branch) against plain stores (lib_alt = HEAD): parity tests,
# C5 build A/B, default bench A/B.
set -o pipefail
OUT=gpurun_out/r06z2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c5 or c4 or super_tile or hbm_resident or build_matches" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python tools/build_ab.py 5 c5 > $OUT/build_ab_c5.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c5.log
tools/ab.sh r06z2/ab 2 --steps 100 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
