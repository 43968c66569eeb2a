# The driver's default bench invocation three times on one box (run-to-run spread)
set -o pipefail
mkdir -p gpurun_out/r05rep
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/r05rep/bench_$r.log 2>&1 || { tail -5 gpurun_out/r05rep/bench_$r.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/r05rep/bench_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print('run $r', d['value'], d['ms_per_step'], 'c3', d['probe_c3']['kernel_ms'], 'c4', d['c4_build']['gkeys_s'], 'route', d['route_c3']['wall_ms'], 'f10 probe', d['f10']['probe']['kernel_ms'], 'traffic', d['roofline']['traffic'])
"
done
