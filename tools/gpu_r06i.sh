#!/bin/bash
# Round-6: GPU suite with the probe pass 2's per-vector mask; C3 probe A/B
# against lib_alt (HEAD); C4 pass 2 on 2/3/4 interleaved chains.
set -o pipefail
OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python tools/probe_ab.py 4 > $OUT/probe_ab.log 2>&1 || exit 1
tail -4 $OUT/probe_ab.log
UB_VARIANTS=2507,2508,2509 timeout -k 10 400 python tools/ubench.py p2ab_c4 > $OUT/p2ab_c4_chains.log 2>&1 || exit 1
grep -h '"op"' $OUT/p2ab_c4_chains.log | cut -c1-200
