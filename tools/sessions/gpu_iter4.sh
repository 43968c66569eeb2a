#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} "gpurun_out/$name.log" | cut -c1-1500
  return $rc
}
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 300 -x
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 400 python bench.py --no-cpu-baseline || exit 1
step bench_c4_part 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1
step bench_c4_atomic 400 python bench.py --workload c4 --steps 2 --warmup 1 --strategy atomic --no-extras --no-cpu-baseline || exit 1
step bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
