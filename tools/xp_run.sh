set -o pipefail
D=gpurun_out/xp23; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/stats_c3 -o run --output-format csv -- python tools/probe_prof.py auto 30 > $D/stats_c3.log 2>&1 || exit 1
