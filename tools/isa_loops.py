#!/usr/bin/env python3
"""Instruction classes per loop body (back-edge) of one kernel in the saved
gfx950 assembly (`make isa`).  Usage: isa_loops.py MANGLED_SUBSTRING [MIN_VALU]"""
import collections
import re
import sys

import os
S = os.environ.get("ISA_S", "cs265-lsm-tree_amd/lib/obj/bloom_kernels-hip-amdgcn-amd-amdhsa-gfx950.s")
L = open(S).read().splitlines()
want, min_valu = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 50
i = next(k for k, l in enumerate(L) if re.match(r"^_Z\S*: ;", l) and want in l.split(":")[0])
j = i
while not L[j].strip().startswith(".Lfunc_end"):
    j += 1
body = L[i:j]
labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
for k, l in enumerate(body):
    m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
    if not m or m.group(1) not in labels or labels[m.group(1)] >= k:
        continue
    c = collections.Counter()
    for s in body[labels[m.group(1)]:k + 1]:
        op = s.strip().split()[0] if s.strip() else ""
        c["VALU" if op.startswith("v_") else "LDS" if op.startswith("ds_") else
          "VMEM" if op.startswith(("global_", "buffer_")) else
          "WAIT" if op.startswith(("s_waitcnt", "s_barrier")) else
          "SALU" if op.startswith("s_") else "-"] += 1
    if c["VALU"] >= min_valu:
        print(m.group(1), dict(c))
