#!/bin/bash
# PMC passes (one counter group per run) on the C3 stacked probe.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c3}
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "== pmc $i: $C $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- python tools/probe_prof.py auto 10 > gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit $?
done
echo done
