#!/bin/bash
# C3 probe: parity of the stacked path + kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "c3 or stack" --timeout 120 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -20 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3x -o run --output-format csv -- python tools/probe_prof.py auto 30 > gpurun_out/prof_c3x.log 2>&1 || exit 1
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_c3x/run_kernel_stats.csv")):
    n = r["Name"].replace("void ", "").split("(")[0][-50:]
    print(f'{n:50s} {r["Calls"]:>4s} {float(r["AverageNs"])/1000:8.1f} us')
PY
