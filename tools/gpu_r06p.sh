#!/bin/bash
# Round-6: C5's ladder-build pass 2 with two vectors per lane (WALK 3) and on
# two chains of two vectors (WALK 7) against the product's WALK 1.
set -o pipefail
OUT=gpurun_out/r06p; mkdir -p $OUT
UB_VARIANTS=2401,2413,2417 timeout -k 10 400 python tools/ubench.py p2ab_c5 > $OUT/p2ab_c5.log 2>&1 || exit 1
grep -h '"op"\|check' $OUT/p2ab_c5.log | cut -c1-220
