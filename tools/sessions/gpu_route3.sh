#!/bin/bash
# route instruction diet: parity (route tests + full gpu suite), sweep, PMC, bench
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
step pytest_route 300 python -u -m pytest tests/test_gpu_route.py -q -m gpu -x --timeout 200 --timeout-method thread || exit 1
step route_sweep 300 python tools/route_sweep.py 0 4 || exit 1
step pmc_route1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_route1 -o pmc --output-format csv -- python tools/route_sweep.py 0 || exit 1
step stats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_rc -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline || exit 1
