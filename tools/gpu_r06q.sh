#!/bin/bash
# Round-6: C2's ladder-build pass 2 with two vectors per lane (WALK 3) and on
# two chains (WALK 7) against the product's WALK 1; C5 repeated.
set -o pipefail
OUT=gpurun_out/r06q; mkdir -p $OUT
UB_VARIANTS=2401,2413,2417 timeout -k 10 400 python tools/ubench.py p2ab > $OUT/p2ab_c2.log 2>&1 || exit 1
grep -h '"op"\|check' $OUT/p2ab_c2.log | cut -c1-220
UB_VARIANTS=2413 timeout -k 10 400 python tools/ubench.py p2ab_c5 > $OUT/p2ab_c5.log 2>&1 || exit 1
grep -h '"op"\|check' $OUT/p2ab_c5.log | cut -c1-220
