#!/bin/bash
# rocprofv3 kernel-trace stats of the bench, then two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE: they do not fit one pass) for roofline.traffic.
# Usage: tools/gpu_prof.sh WORKLOAD TAG   (e.g. c2 r01)
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${1:-c2}; TAG=${2:-r01}
ARGS="--workload $W --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline --no-extras"
echo "== stats $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${W}_$TAG -o run --output-format csv -- python bench.py $ARGS > gpurun_out/prof_${W}_$TAG.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_${W}_$TAG.log | cut -c1-300
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C $(date +%T)"
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${W}_${TAG}_$C -o pmc --output-format csv -- python bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/pmc_${W}_${TAG}_$C.log 2>&1 || exit $?
done
find gpurun_out/prof_${W}_$TAG gpurun_out/pmc_${W}_${TAG}_* -name "*.csv" | head -20
