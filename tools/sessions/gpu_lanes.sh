#!/bin/bash
# pass-2 lanes per tile (G) at C5 / C2 / C4 geometry with the current tile sizes
mkdir -p gpurun_out/lanes
export TMPDIR=/tmp
for w in c5 c2; do
  for g in 0 4 8 16 32; do
    BLOOMHIP_APPLY_LANES=$g timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/lanes/${w}_g$g.log 2>&1 || exit 1
    echo "$w G=$g $(grep -o '"kernels": {[^}]*}[^}]*}' gpurun_out/lanes/${w}_g$g.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/lanes/${w}_g$g.log)"
  done
done
for g in 0 8; do
  BLOOMHIP_APPLY_LANES=$g timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline > gpurun_out/lanes/c4_g$g.log 2>&1 || exit 1
  echo "c4 G=$g $(grep -o '"kernels": {[^}]*}[^}]*}' gpurun_out/lanes/c4_g$g.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/lanes/c4_g$g.log)"
done
