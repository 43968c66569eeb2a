#!/bin/bash
# the default bench line (now with the C5 eight-run leg) at N=1, and the
# N=2 rehearsal (2 gloo ranks sharing one GPU)
mkdir -p gpurun_out/c5r
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/c5r/bench.log 2>&1 || { tail -5 gpurun_out/c5r/bench.log; exit 1; }
grep -o '"c5_eight_runs": {[^}]*}' gpurun_out/c5r/bench.log
BLOOMHIP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/c5r/bench_dist2.log 2>&1 || { tail -5 gpurun_out/c5r/bench_dist2.log; exit 1; }
grep -o '"c5_eight_runs": {[^}]*}' gpurun_out/c5r/bench_dist2.log
