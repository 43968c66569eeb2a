#!/bin/bash
# C5 with 160 KiB segment images (512 segments instead of 768), 4096- vs 8192-key tiles
mkdir -p gpurun_out/segmax
export TMPDIR=/tmp
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/segmax/$tag.log 2>&1 || exit 1
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/segmax/$tag.log) $(grep -o '"kernels": {[^}]*}[^}]*}' gpurun_out/segmax/$tag.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/segmax/$tag.log)"
}
run base X=1
run seg160 BLOOMHIP_SEG_MAX_KIB=160
run seg160_big256 BLOOMHIP_SEG_MAX_KIB=160 BLOOMHIP_BIG_TILE_BINS=256
run base_again X=1
