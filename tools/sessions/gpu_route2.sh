#!/bin/bash
# route + combine rework: parity (route, probe), route per-CU sweep, bench, kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-4} | cut -c1-400
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step route_sweep 300 python tools/route_sweep.py 0 4 8 || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
step stats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_rc -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline || exit 1
BLOOMHIP_BIG_TILE_BINS=512 step bench_c5_big 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
step bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
BLOOMHIP_BIG_TILE_BINS=200 step bench_c2_big 400 python bench.py --steps 100 --warmup 10 --no-extras --no-cpu-baseline || exit 1
