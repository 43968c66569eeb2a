#!/bin/bash
# Round-6: the HBM-resident pass-2 ragged builds (WALK 3) against the oracle.
set -o pipefail
OUT=gpurun_out/r06u; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "hbm_resident" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -4 $OUT/pytest.log
