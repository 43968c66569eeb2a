#!/usr/bin/env python3
"""Interleaved A/B of the C3 probe (16.8M GETs x 5 level filters) and the C3
GET routing between two builds of libbloomhip, in child processes on one
GPU: A = cs265-lsm-tree_amd/lib_alt (tools/build_alt.sh REV), B = lib/.
Workload c3 (default) or f10 (the f = 10 tree's three levels; its GETs are
routed over the three level runs the same way).
Each child prewarms, then times 50 probe calls (HIP events on the launch
stream) and 30 routing calls; rounds alternate B A B A so clock drift hits
both alike.
Usage: python tools/probe_ab.py [rounds] [c3|f10]"""
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
gets, levels = W.c3_runs() if sys.argv[2] == "c3" else W.f10_runs()  # runs sorted, as written (fences)
dg = torch.from_numpy(gets).cuda()
fs = []
for _, keys, m in levels:
    f = bh.BloomFilter(m)
    f.set_batch_run(keys)
    fs.append(f)
s = torch.cuda.current_stream()
out = torch.empty((len(fs), (gets.size + 63) // 64), dtype=torch.int64, device="cuda")
fr = torch.empty(gets.size, dtype=torch.int32, device="cuda")
pg = torch.empty(gets.size, dtype=torch.int32, device="cuda")
def timed(fn, n):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(n):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n
p = timed(lambda: bh.test_batch(fs, dg, out=out, stream=s), 50)
r = timed(lambda: bh.route_gets(fs, dg, cand=out, first=fr, page=pg, stream=s), 30)
print(json.dumps({"probe_ms": round(p, 4), "route_ms": round(r, 4),
                  "kernel_sha": bh.lib().bloomhip_kernel_sha().decode()}))
'''


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    workload = sys.argv[2] if len(sys.argv) > 2 else "c3"
    alt = os.path.join(ROOT, "cs265-lsm-tree_amd", "lib_alt", "libbloomhip.so")
    res = {"A": [], "B": []}
    for r in range(rounds):
        for v in ("B", "A"):
            env = dict(os.environ)
            env.pop("BLOOMHIP_LIB", None)
            if v == "A":
                env["BLOOMHIP_LIB"] = alt
            out = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "cs265-lsm-tree_amd"),
                                  workload],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            d.update({"side": v, "round": r})
            res[v].append(d)
            print(json.dumps(d), flush=True)
    for v in ("A", "B"):
        ps = sorted(x["probe_ms"] for x in res[v])
        rs = sorted(x["route_ms"] for x in res[v])
        print(json.dumps({"side": v, "probe_ms_median": ps[len(ps) // 2],
                          "route_ms_median": rs[len(rs) // 2]}), flush=True)


if __name__ == "__main__":
    main()
