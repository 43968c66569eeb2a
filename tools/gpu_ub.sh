#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/ubench.py ${1:-part} > gpurun_out/ubench_${1:-part}.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ubench_${1:-part}.log; exit $rc
