#!/bin/bash
# GPU parity first, then the given ubench modes (default: part)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 300 -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for mode in ${@:-part}; do
  echo "== $mode"
  timeout -k 10 300 python tools/ubench.py $mode > gpurun_out/ubench_$mode.log 2>&1 || { tail -5 gpurun_out/ubench_$mode.log; exit 1; }
  grep '^{' gpurun_out/ubench_$mode.log | grep -v '"k_part_apply", "n": [0-9]*, "variant": 1[0-9][0-9]'
done
