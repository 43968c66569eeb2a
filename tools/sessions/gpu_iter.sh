#!/bin/bash
# Iteration session: parity tests, bench, rocprofv3 kernel stats of the bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-iter}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -4 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 300 -x
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 400 python bench.py --steps 50 --warmup 5 || exit 1
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit 1
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -3
