#!/usr/bin/env python3
"""Interleaved A/B of one partition build (clear + set_batch on device-resident
keys, the bench's step; before round 6's last change the children built
without the clear, i.e. timed merge builds)
between two builds of libbloomhip, in child processes on one GPU: A =
cs265-lsm-tree_amd/lib_alt (tools/build_alt.sh REV), B = lib/.  Workloads:
c2 (16.8M keys, m = 5 << 25), f10 (16.8M keys, m = 512,000,000), c5 (67M keys,
m = 5 << 27).  Each child prewarms 0.5 s, then times 50 builds with HIP events
on the launch stream; rounds alternate B A B A.
Usage: python tools/build_ab.py [rounds] [c2|f10|c5]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, time
sys.path.insert(0, sys.argv[1])
import torch
import bloomhip as bh
from bloomhip import workloads as W
w = sys.argv[2]
keys, m = W.c2() if w == "c2" else W.f10_build() if w == "f10" else W.c2(n=67108864)
if w == "c5":
    m = bh.m_bits(keys.size, 10.0)
dk = torch.from_numpy(keys).cuda()
f = bh.BloomFilter(m)
f.set_strategy(bh.BUILD_PARTITION)
s = torch.cuda.current_stream()
def one():  # the bench's step: a fresh filter (clear) and one build
    f.clear(stream=s)
    f.set_batch(dk, stream=s)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    one()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
for _ in range(50):
    one()
b.record(s)
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 50
print(json.dumps({"build_ms": round(ms, 5), "gkeys_s": round(keys.size / ms / 1e6, 2),
                  "kernel_sha": bh.lib().bloomhip_kernel_sha().decode()}))
'''


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    workload = sys.argv[2] if len(sys.argv) > 2 else "c2"
    alt = os.path.join(ROOT, "cs265-lsm-tree_amd", "lib_alt", "libbloomhip.so")
    res = {"A": [], "B": []}
    for r in range(rounds):
        for v in ("B", "A"):
            env = dict(os.environ)
            env.pop("BLOOMHIP_LIB", None)
            if v == "A":
                env["BLOOMHIP_LIB"] = alt
            out = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "cs265-lsm-tree_amd"),
                                  workload], env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            d.update({"side": v, "round": r, "workload": workload})
            res[v].append(d)
            print(json.dumps(d), flush=True)
    for v in ("A", "B"):
        xs = sorted(x["build_ms"] for x in res[v])
        print(json.dumps({"side": v, "workload": workload, "build_ms_median": xs[len(xs) // 2]}), flush=True)


if __name__ == "__main__":
    main()
