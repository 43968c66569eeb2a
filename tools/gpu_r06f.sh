#!/bin/bash
# Round-6: the WALK 4 build walk in the bench context, interleaved A/B
# (A = lib_alt at fe46758, WALK 1; B = the tree's lib, WALK 4): C2 and C5.
set -o pipefail
bash tools/ab.sh r06f/ab_c2 4 --no-extras --steps 200 --warmup 20 || exit 1
timeout -k 10 500 python tools/build_ab.py 3 c5 || exit 1
