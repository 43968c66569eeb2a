#!/bin/bash
# A/B of two builds of libbloomhip on one GPU box, interleaved (B A B A ...)
# so clock drift hits both alike.  A = cs265-lsm-tree_amd/lib_alt/libbloomhip.so
# (build it from another commit with tools/build_alt.sh REV), B = the tree's
# lib/libbloomhip.so.  Extra args go to bench.py.
# Usage: tools/ab.sh TAG ROUNDS [bench args...]
set -o pipefail
TAG=${1:?tag}; R=${2:-3}; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
ALT=cs265-lsm-tree_amd/lib_alt/libbloomhip.so
[ -f "$ALT" ] || { echo "missing $ALT"; exit 2; }
for r in $(seq 1 "$R"); do
  for v in B A; do
    if [ $v = A ]; then export BLOOMHIP_LIB=$PWD/$ALT; else unset BLOOMHIP_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/${v}_$r.log" 2>&1 || { echo "$v round $r failed"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
    python - "$OUT/${v}_$r.log" "$v" "$r" <<'PY'
import json, sys
d = json.loads(next(l for l in open(sys.argv[1]) if l.startswith("{")))
k = d["roofline"].get("profiled_kernel_ms", {})
x = {kk: round(v * 1e3, 1) for kk, v in k.items()}
p = d.get("probe_c3", {})
c4 = d.get("c4_build", {})
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], x, "probe_c3", p.get("kernel_ms"),
      "c4", c4.get("gkeys_s"), c4.get("kernels"), "route", d.get("route_c3", {}).get("wall_ms"),
      "c5", d.get("c5_eight_runs", {}).get("gkeys_s"), "compact", d.get("compact_fanin4", {}).get("ms"))
PY
  done
done
