#!/bin/bash
# stacked probe: parity (probe tests), ablation, the C3 strategy sweep, the bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-3} | cut -c1-400
  return $rc
}
step pytest_probe 600 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "probe or stack" --timeout 120 --timeout-method thread || exit 1
TAILN=30 step ub_stack 300 python tools/ubench.py stack || exit 1
TAILN=20 step probe_sweep 300 python tools/probe_sweep.py || exit 1
