#!/bin/bash
# Builds experiment variants of the ubench library (the product kernels with
# -D overrides): tools/ub_variants.sh NAME "-DFOO=1 ..." [NAME "-D..." ...]
# -> cs265-lsm-tree_amd/lib/libbloomhip_ubench_NAME.so (UBENCH_LIB selects one
# for tools/ubench.py).
set -e
cd "$(dirname "$0")/../cs265-lsm-tree_amd/csrc"
mkdir -p ../lib/obj
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall --offload-arch=gfx950 $defs -c -o ../lib/obj/ubench_$name.o ubench.hip &
done
wait
for o in ../lib/obj/ubench_*.o; do
  n=$(basename $o .o); [ "$n" = ubench_isa ] && continue
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/lib${n/ubench/bloomhip_ubench}.so $o
done
ls ../lib
