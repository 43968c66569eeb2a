set -o pipefail
D=gpurun_out/xp2; mkdir -p $D
export UB_GD=1
for v in xp0 xp1; do
  for w in part part_c5 part_c4; do
    UBENCH_LIB=cs265-lsm-tree_amd/lib/libbloomhip_ubench_$v.so timeout -k 10 200 python tools/ubench.py $w > $D/${v}_$w.log 2>&1 || exit 1
  done
done
UBENCH_LIB=cs265-lsm-tree_amd/lib/libbloomhip_ubench_xp0.so timeout -k 10 200 python tools/ubench.py stack > $D/xp0_stack.log 2>&1 || exit 1
