#!/bin/bash
# Round-6 (throwaway): C4's 161 MB super-tile run table written straight as
# columns by pass 1 (threshold 256 MiB: within the Infinity Cache) against
# rows + transpose (lib_alt = HEAD); bench A/B (the c4_build leg).
set -o pipefail
OUT=gpurun_out/r06x; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c4_full or super_tile" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
tools/ab.sh r06x/ab 2 --steps 50 --no-c5 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
