#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/ubench.py part > gpurun_out/ub_depth_c2.log 2>&1 || exit 1
grep k_part_apply gpurun_out/ub_depth_c2.log
timeout -k 10 300 python tools/ubench.py part_c5 > gpurun_out/ub_depth_c5.log 2>&1 || exit 1
grep k_part_apply gpurun_out/ub_depth_c5.log
timeout -k 10 300 python tools/ubench.py part_c4 > gpurun_out/ub_depth_c4.log 2>&1 || exit 1
grep k_part_apply gpurun_out/ub_depth_c4.log
