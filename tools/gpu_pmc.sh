#!/bin/bash
# PMC counter passes (no tracing domains besides kernel-trace) on the C2 build
# and the C3 probe.  Usage: tools/gpu_pmc.sh TAG
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
timeout -k 10 600 rocprofv3 -i tools/pmc/counters.txt --kernel-trace -d gpurun_out/$TAG -o pmc --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/$TAG.log; find gpurun_out/$TAG -name "*.csv" | head -20
