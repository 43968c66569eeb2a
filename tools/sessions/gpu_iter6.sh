#!/bin/bash
# parity, the C3 probe strategy sweep, the C2 bench line
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
TAILN=12 step probe_sweep 300 python tools/probe_sweep.py || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
