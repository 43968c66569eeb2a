set -o pipefail
D=gpurun_out/xp27; mkdir -p $D
UB_2X=1 timeout -k 10 200 python tools/ubench.py part > $D/part2x.log 2>&1 || exit 1
UB_2X=1 timeout -k 10 200 python tools/ubench.py part_c5 > $D/part2x_c5.log 2>&1 || exit 1
