#!/usr/bin/env python3
"""Host time to enqueue one C2 build (clear + set_batch on device keys, no
synchronisation), A/B between lib_alt (tools/build_alt.sh REV) and lib/, in
child processes.  A build costs ~91 us of GPU time, so an enqueue that takes
about as long leaves the GPU waiting between builds.
Usage: python tools/host_enqueue.py [rounds]"""
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
keys, m = W.c2()
dk = torch.from_numpy(keys).cuda()
f = bh.BloomFilter(m)
s = torch.cuda.current_stream()
for _ in range(50):
    f.clear(stream=s); f.set_batch(dk, stream=s)
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for _ in range(n):
    f.clear(stream=s); f.set_batch(dk, stream=s)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(json.dumps({"enqueue_us": round((t1 - t0) / n * 1e6, 2), "per_build_us": round((t2 - t0) / n * 1e6, 2)}))
'''


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    alt = os.path.join(ROOT, "cs265-lsm-tree_amd", "lib_alt", "libbloomhip.so")
    for r in range(rounds):
        for v in ("B", "A"):
            env = dict(os.environ)
            env.pop("BLOOMHIP_LIB", None)
            if v == "A":
                env["BLOOMHIP_LIB"] = alt
            out = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "cs265-lsm-tree_amd")],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            d.update({"side": v, "round": r})
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
