#!/bin/bash
# stacked probe ablation (tools/ubench.py stack) at C3
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== ub_stack $(date +%T)"
timeout -k 10 300 python tools/ubench.py stack > gpurun_out/ub_stack.log 2>&1; rc=$?
echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/ub_stack.log | tail -25 | cut -c1-300
exit $rc
