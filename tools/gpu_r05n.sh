# f10 probe on super-tiles: rocprofv3 kernel stats, new build (lib/) and lib_alt
set -o pipefail
mkdir -p gpurun_out/r05n
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05n/new -o run --output-format csv -- python tools/probe_prof.py auto 30 - f10 > gpurun_out/r05n/new.log 2>&1 || { tail -20 gpurun_out/r05n/new.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05n/alt -o run --output-format csv -- python tools/probe_prof.py auto 30 alt f10 > gpurun_out/r05n/alt.log 2>&1 || { tail -20 gpurun_out/r05n/alt.log; exit 1; }
echo ok
