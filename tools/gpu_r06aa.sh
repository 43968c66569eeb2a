#!/bin/bash
# Round-6: pass 2 of builds beyond the Infinity Cache (C4 WALK 7, C5 WALK 3)
# reads the sorted tiles with non-temporal loads, against plain loads
# (lib_alt = HEAD): parity tests,
# C5 build A/B, default bench A/B.
set -o pipefail
OUT=gpurun_out/r06aa; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c5 or c4 or super_tile or hbm_resident or build_matches" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python tools/build_ab.py 5 c5 > $OUT/build_ab_c5.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c5.log
tools/ab.sh r06aa/ab 2 --steps 100 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
