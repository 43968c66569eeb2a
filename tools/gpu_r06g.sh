#!/bin/bash
# Round-6: pass 1 with the single-wave scan at <= 256 bins (C2): GPU suite,
# then interleaved build A/B against lib_alt (6512234).
set -o pipefail
OUT=gpurun_out/r06g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python tools/build_ab.py 6 c2 > $OUT/build_ab_c2.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c2.log
