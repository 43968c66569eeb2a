#!/bin/bash
# Round-6 (throwaway): pass 2 writes the finished bitmap with non-temporal
# stores (lib_alt = HEAD: plain stores): build tests, C2 / C5 build A/B and
# the default bench A/B.
set -o pipefail
OUT=gpurun_out/r06ab; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "build or c2 or c5 or c4 or super_tile" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python tools/build_ab.py 5 c2 > $OUT/build_ab_c2.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c2.log
timeout -k 10 400 python tools/build_ab.py 3 c5 > $OUT/build_ab_c5.log 2>&1 || exit 1
tail -2 $OUT/build_ab_c5.log
tools/ab.sh r06ab/ab 2 --steps 100 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
