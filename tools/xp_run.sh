set -o pipefail
D=gpurun_out/xp10; mkdir -p $D
timeout -k 10 200 python tools/ubench.py stack > $D/stack.log 2>&1 || exit 1
