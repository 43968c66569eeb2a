set -o pipefail
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stack or f10 or route" > gpurun_out/r05b/pytest.log 2>&1 || { tail -30 gpurun_out/r05b/pytest.log; exit 1; }
tail -3 gpurun_out/r05b/pytest.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c4 --no-c5 > gpurun_out/r05b/bench.log 2>&1 || { tail -20 gpurun_out/r05b/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r05b/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print('value', d['value'], d['parity'])
f=d['f10']
print('f10 probe', {k:f['probe'][k] for k in ['gkeys_s','kernel_ms','wall_ms','kernels','hits_sha_match']})
print('c3', d['probe_c3']['kernel_ms'], 'route', d['route_c3']['wall_ms'])
PY
