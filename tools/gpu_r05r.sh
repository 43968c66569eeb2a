# Experiment: C2 pass 2 with every segment done twice by two workgroups (grid
# 2 x nbins, two per CU): does doubled work at two workgroups per CU take
# much less than twice the time?  lib_exp = HEAD + the duplicate-grid hook.
set -o pipefail
mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
export BLOOMHIP_LIB=$PWD/cs265-lsm-tree_amd/lib_exp/libbloomhip.so
for r in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export BH_DUP2=1; else unset BH_DUP2; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-extras --no-cpu-baseline > gpurun_out/r05r/b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r05r/b_${v}_$r.log; exit 1; }
    python -c "
import json,sys
for l in open('gpurun_out/r05r/b_${v}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print('dup=$v round=$r value', d['value'], d['roofline']['profiled_kernel_ms'])
"
  done
done
