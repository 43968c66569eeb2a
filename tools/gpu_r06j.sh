#!/bin/bash
# Round-6: GPU suite at the two-chain C4 pass 2 (WALK 7); C5 pass 2 on two
# chains x one vector (WALK 10) vs WALK 1; bench-level A/B against lib_alt
# (368c29c: before the probe mask and WALK 7).
set -o pipefail
OUT=gpurun_out/r06j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
UB_VARIANTS=2401,2410 timeout -k 10 400 python tools/ubench.py p2ab_c5 > $OUT/p2ab_c5_walk10.log 2>&1 || exit 1
grep -h '"op"' $OUT/p2ab_c5_walk10.log | cut -c1-200
tools/ab.sh r06j/ab 3 --steps 100 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
