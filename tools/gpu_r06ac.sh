#!/bin/bash
# Round-6: the non-temporal bitmap writeback, a second bench A/B (three
# rounds, lib_alt = HEAD) and the C2 build A/B again.
set -o pipefail
OUT=gpurun_out/r06ac; mkdir -p $OUT
tools/ab.sh r06ac/ab 3 --steps 200 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
timeout -k 10 400 python tools/build_ab.py 5 c2 > $OUT/build_ab_c2.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c2.log
