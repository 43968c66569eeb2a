#!/usr/bin/env python3
"""Instruction mix of one kernel in the saved gfx950 assembly (`make isa`):
counts per class (VALU, SALU, LDS, VMEM, branches/waits) over the whole
kernel body, and inside the main loop when a label is given.
Usage: isa_count.py KERNEL_SUBSTRING [LOOP_LABEL]"""
import collections
import re
import subprocess
import sys

S = sys.argv[3] if len(sys.argv) > 3 else "cs265-lsm-tree_amd/lib/obj/bloom_kernels-hip-amdgcn-amd-amdhsa-gfx950.s"
want = sys.argv[1]
lines = open(S).read().splitlines()
# kernel bodies start at "<mangled>:" labels of functions marked @function
starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\S+: ;", l)]
names = subprocess.run(["c++filt"], input="\n".join(n for _, n in starts), capture_output=True,
                       text=True).stdout.splitlines()
for (i, mang), dem in zip(starts, names):
    if want not in dem:
        continue
    body = []
    for l in lines[i + 1:]:
        if l.strip().startswith(".Lfunc_end"):
            break
        body.append(l)
    cnt = collections.Counter()
    for l in body:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        cls = ("LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "flat_"))
               else "SMEM" if op.startswith("s_load") or op.startswith("s_buffer") else
               "WAIT" if op.startswith(("s_waitcnt", "s_barrier")) else
               "SALU" if op.startswith("s_") else "VALU" if op.startswith("v_") else "other")
        cnt[cls] += 1
        cnt["op:" + op] += 1
    print(dem.split("(")[0])
    print("  ", {k: v for k, v in cnt.items() if not k.startswith("op:")})
    top = sorted(((v, k[3:]) for k, v in cnt.items() if k.startswith("op:v_")), reverse=True)[:25]
    print("   top VALU:", ", ".join(f"{k}={v}" for v, k in top))
    break
