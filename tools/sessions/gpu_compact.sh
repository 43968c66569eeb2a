#!/bin/bash
# compaction rework: full GPU parity, bench, kernel stats
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
step stats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_cp -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline || exit 1
