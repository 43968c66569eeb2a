#!/bin/bash
# parity first, then pass-2 walk sweeps at C2 / C5 / C4 sizes, then bench lines
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-3} | cut -c1-1500
  return $rc
}
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 300 -x || exit 1
TAILN=14 step ub_part 300 python tools/ubench.py part || exit 1
TAILN=14 step ub_part_c5 300 python tools/ubench.py part_c5 || exit 1
TAILN=14 step ub_part_c4 400 python tools/ubench.py part_c4 || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
step bench_c4_part 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1
step bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
