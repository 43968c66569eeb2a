#!/usr/bin/env python3
"""Compact view of hipcc -Rpass-analysis=kernel-resource-usage output
(cs265-lsm-tree_amd/lib/obj/resource_usage.txt from `make isa`): one line per
kernel with VGPRs, spills, LDS bytes and occupancy.  Usage: kres.py [FILTER]"""
import re
import subprocess
import sys

path = sys.argv[2] if len(sys.argv) > 2 else "cs265-lsm-tree_amd/lib/obj/resource_usage.txt"
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("sgpr", r"SGPRs: (\d+)")):
        m = re.search(pat, line)
        if m and key not in cur:
            cur[key] = int(m.group(1))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
for r, n in zip(rows, names):
    n = n.replace("bloomhip::(anonymous namespace)::", "").split("(")[0]
    if flt in n:
        print(f"{n:70s} vgpr={r.get('vgpr')} spill={r.get('spill')} lds={r.get('lds')} occ={r.get('occ')}")
