#!/bin/bash
# Rehearse the N > 1 bench path on one GPU: 2 ranks over gloo sharing cuda:0.
mkdir -p gpurun_out; export TMPDIR=/tmp
BLOOMHIP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  --workload ${1:-c5} > gpurun_out/bench_dist2.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_dist2.log | cut -c1-700; echo "rc=$rc"; exit $rc
