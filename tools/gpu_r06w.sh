#!/bin/bash
# Round-6: C4's super-tile pass 2 on two chains of one redirected vector per
# lane (WALK 11) against the product's WALK 7 (two chains of two vectors).
set -o pipefail
OUT=gpurun_out/r06w; mkdir -p $OUT
UB_VARIANTS=2507,2511 timeout -k 10 400 python tools/ubench.py p2ab_c4 > $OUT/p2ab_c4.log 2>&1 || exit 1
grep -h '"op"\|check' $OUT/p2ab_c4.log | cut -c1-100,180-260
