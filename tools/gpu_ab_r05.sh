#!/bin/bash
# Interleaved A/B (lib_alt = A, lib = B) of the builds C2 and C4 and of the
# C3 probe / route, on one box.  Usage: tools/gpu_ab_r05.sh TAG [c2,c4,c3,c5]
set -o pipefail
TAG=${1:?tag}; WHAT=${2:-c2,c4,c3}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for w in ${WHAT//,/ }; do
  case $w in
    c2) timeout -k 10 900 bash tools/ab.sh "$TAG/ab_c2" 3 --no-extras --steps 200 --warmup 20 > "$OUT/ab_c2.log" 2>&1 || { tail -5 "$OUT/ab_c2.log"; exit 1; }; cat "$OUT/ab_c2.log" ;;
    c4) timeout -k 10 900 bash tools/ab.sh "$TAG/ab_c4" 2 --workload c4 --no-extras --steps 10 --warmup 2 > "$OUT/ab_c4.log" 2>&1 || { tail -5 "$OUT/ab_c4.log"; exit 1; }; cat "$OUT/ab_c4.log" ;;
    c5) timeout -k 10 900 bash tools/ab.sh "$TAG/ab_c5" 2 --workload c5 --no-extras --steps 20 --warmup 3 > "$OUT/ab_c5.log" 2>&1 || { tail -5 "$OUT/ab_c5.log"; exit 1; }; cat "$OUT/ab_c5.log" ;;
    c3) timeout -k 10 600 python tools/probe_ab.py 3 > "$OUT/probe_ab.log" 2>&1 || { tail -5 "$OUT/probe_ab.log"; exit 1; }; tail -2 "$OUT/probe_ab.log" ;;
    f10) timeout -k 10 600 python tools/probe_ab.py 3 f10 > "$OUT/probe_ab_f10.log" 2>&1 || { tail -5 "$OUT/probe_ab_f10.log"; exit 1; }; tail -2 "$OUT/probe_ab_f10.log" ;;
  esac
done
