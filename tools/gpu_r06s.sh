#!/bin/bash
# Round-6 (throwaway build): the fused f10 route on super-tiles (one combine
# workgroup per CU) against 8192-key tiles (lib_alt = HEAD).
set -o pipefail
OUT=gpurun_out/r06s; mkdir -p $OUT
timeout -k 10 500 python tools/probe_ab.py 3 f10 > $OUT/probe_ab_f10.log 2>&1 || exit 1
tail -2 $OUT/probe_ab_f10.log
