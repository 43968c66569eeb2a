set -o pipefail
D=gpurun_out/xp5; mkdir -p $D
UB_P1=1 timeout -k 10 200 python tools/ubench.py part > $D/p1_part.log 2>&1 || exit 1
UB_P1=1 timeout -k 10 200 python tools/ubench.py part > $D/p1_part2.log 2>&1 || exit 1
