#!/bin/bash
# byte-interleaved stack image: parity, C3 probe bytes vs planes, route PMC
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
BLOOMHIP_STACK_LAYOUT=planes step stats_planes 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_planes -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1
step stats_bytes 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_bytes -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1
step pmc_route1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_route1 -o pmc --output-format csv -- python tools/route_sweep.py 0 || exit 1
step pmc_route2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --kernel-trace -d gpurun_out/pmc_route2 -o pmc --output-format csv -- python tools/route_sweep.py 0 || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
