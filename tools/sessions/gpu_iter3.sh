#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 300 -x
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 400 python bench.py --no-cpu-baseline || exit 1
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_it3 -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit 1
