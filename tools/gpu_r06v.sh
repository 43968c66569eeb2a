#!/bin/bash
# Round-6: C3's ladder stack on 4096-key tiles (pass 1 at three workgroups
# per CU) with pass 2 walking tile pairs (WALK 12), against 8192-key tiles:
# tools/ubench.py ladder (every phase checked against the segment stack).
set -o pipefail
OUT=gpurun_out/r06v; mkdir -p $OUT
UB_LADDER=0,1,2,5 timeout -k 10 400 python tools/ubench.py ladder > $OUT/ub_ladder.log 2>&1 || { tail -20 $OUT/ub_ladder.log; exit 1; }
grep -h 'check\|"op"' $OUT/ub_ladder.log | cut -c1-60,150-260
