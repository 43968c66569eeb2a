#!/bin/bash
# Round-6: GPU suite with the WALK 4 build walk; C4 pass 2 on WALK 5 (2500)
# against WALK 3 (2503) and the product (1), interleaved.
set -o pipefail
OUT=gpurun_out/r06d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
UB_VARIANTS=2500,2503 timeout -k 10 400 python tools/ubench.py p2ab_c4 > $OUT/p2ab_c4.log 2>&1 || exit 1
grep -h '"op"\|check' $OUT/p2ab_c4.log | cut -c1-200
