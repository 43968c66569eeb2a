#!/bin/bash
# 24-bit partition entries: parity, pass ablations (C2, C5, C4), stacked probe, bench
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-3} | cut -c1-300
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
TAILN=20 step ub_part 300 python tools/ubench.py part || exit 1
TAILN=20 step ub_part_c4 300 python tools/ubench.py part_c4 || exit 1
TAILN=16 step ub_stack 300 python tools/ubench.py stack || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
step bench_c4 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1
step bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
