#!/bin/bash
# Round-6 experiment: pass 2 on the WALK 4 build walk (ubench 2400) against
# WALK 1 (2401) and the product (1), C2 and C5 geometries, interleaved.
set -o pipefail
OUT=gpurun_out/r06c; mkdir -p $OUT
export UB_VARIANTS=2400,2401
timeout -k 10 200 python tools/ubench.py p2ab > $OUT/p2ab_c2.log 2>&1 || exit 1
timeout -k 10 300 python tools/ubench.py p2ab_c5 > $OUT/p2ab_c5.log 2>&1 || exit 1
grep -h '"op"\|check' $OUT/*.log
