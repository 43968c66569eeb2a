#!/bin/bash
# Round evidence at HEAD: GPU parity, smoke, the default bench line (with CPU
# baseline), C4/C5 lines, rocprofv3 kernel stats of the C2 bench and of the
# C3 probe, and the C2 PMC traffic passes (FETCH_SIZE, WRITE_SIZE separately).
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/ev/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/ev/$name.log" | tail -${TAILN:-2} | cut -c1-300
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py || exit 1
step bench_c4 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1
step bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1
step stats_c2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/stats_c2 -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline || exit 1
step stats_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/stats_c3 -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1
step pmc_fetch 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_c2_ev_FETCH_SIZE -o pmc --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras || exit 1
step pmc_write 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_c2_ev_WRITE_SIZE -o pmc --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras || exit 1
echo done
