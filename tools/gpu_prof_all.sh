#!/bin/bash
# Round evidence: kernel stats + PMC bytes for C2 (the bench value), stats for
# C4 / C5, and kernel stats of the C3 stacked probe.  TAG names the outputs.
TAG=${1:-r01b}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof.sh c2 $TAG || exit 1
STEPS=5 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_$TAG -o run --output-format csv -- python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_c4_$TAG.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/prof_c5_$TAG.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_$TAG -o run --output-format csv -- python tools/probe_prof.py auto 30 > gpurun_out/prof_c3_$TAG.log 2>&1 || exit 1
echo done
