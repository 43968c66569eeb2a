#!/bin/bash
# stacked probe with wrap-around member windows: parity, C3 probe wrap vs divisor-only
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
BLOOMHIP_STACK_WRAP=0 step stats_div 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_div -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1
step stats_wrap 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_wrap -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
