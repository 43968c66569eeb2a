#!/bin/bash
# Round-6: routing tests with the f10 route on super-tiles, and one default
# bench line (packed routing legs, parity).
set -o pipefail
OUT=gpurun_out/r06t; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_route.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_route.log 2>&1 || { tail -30 $OUT/pytest_route.log; exit 1; }
tail -1 $OUT/pytest_route.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json, sys
d = json.loads(next(l for l in open(sys.argv[1]) if l.startswith("{")))
print(d["value"], "c3", d["probe_c3"]["kernel_ms"], "route", d["route_c3"]["wall_ms"], "f10", {k: v.get("kernel_ms") or v.get("wall_ms") for k, v in d["f10"].items() if isinstance(v, dict)}, "c5", d["c5_eight_runs"]["gkeys_s"], "c4", d["c4_build"]["gkeys_s"], d["parity"])
PY
