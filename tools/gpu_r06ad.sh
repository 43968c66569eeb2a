#!/bin/bash
# Round-6: non-temporal bitmap writeback for fresh builds only (merges store
# plainly): GPU suite, C2 build A/B (the merge path) and the bench A/B
# (fresh builds), lib_alt = HEAD.
set -o pipefail
OUT=gpurun_out/r06ad; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python tools/build_ab.py 5 c2 > $OUT/build_ab_c2.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c2.log
tools/ab.sh r06ad/ab 3 --steps 200 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
