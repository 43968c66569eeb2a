#!/bin/bash
# Round-end evidence: GPU parity, the default bench line (with CPU baseline),
# the C4/C5 lines, and rocprofv3 kernel stats of the C2 bench.  TAG names the
# profiles/ directory the summaries are copied to afterwards.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-3} | cut -c1-600
  return $rc
}
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 300 -x || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py || exit 1
step bench_c4 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1
step bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
step stats_c2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_c2 -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline || exit 1
