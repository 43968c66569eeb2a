#!/bin/bash
# Round-6: the C5 job on one, two and four streams with the two-vector pass 2.
set -o pipefail
OUT=gpurun_out/r06y; mkdir -p $OUT
timeout -k 10 400 python tools/c5_streams.py 3 > $OUT/c5_streams.log 2>&1 || { tail $OUT/c5_streams.log; exit 1; }
tail -6 $OUT/c5_streams.log
