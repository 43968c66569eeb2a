#!/bin/bash
# Round-6: builds whose entries exceed the Infinity Cache (C5) on WALK 3 (two
# vectors per lane): GPU suite, C5 build A/B and the default bench A/B
# against lib_alt (HEAD).
set -o pipefail
OUT=gpurun_out/r06r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python tools/build_ab.py 3 c5 > $OUT/build_ab_c5.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c5.log
tools/ab.sh r06r/ab 2 --steps 100 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
