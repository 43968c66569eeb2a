#!/bin/bash
# word-interleaved stack image: parity, C3 probe stats, SQ PMC of pass 2, bench
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
step stats_il 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_il -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1
step pmc_il 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_il -o pmc --output-format csv -- python tools/probe_prof.py auto 10 || exit 1
step bench 400 python bench.py --no-cpu-baseline || exit 1
