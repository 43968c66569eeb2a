#!/bin/bash
# routing: parity + the bench line (route leg)
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
step pytest_route 600 python -u -m pytest tests/test_gpu_route.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
