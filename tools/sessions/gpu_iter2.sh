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
TAILN=5 step ubench_part 300 python tools/ubench.py part || exit 1
step bench 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline || exit 1
