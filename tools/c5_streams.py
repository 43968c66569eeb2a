#!/usr/bin/env python3
"""C5 job (8 runs x 67M keys, one GPU): the 8 builds on one stream against
the same builds alternating over 2 or 4 streams (independent runs, one
workspace per stream), interleaved rounds, wall time per job between device
syncs.  Usage: python tools/c5_streams.py [rounds]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
import bloomhip as bh  # noqa: E402
from bloomhip import workloads as W  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    built = []
    for r in range(8):
        keys, m = W.c5_run(r)
        built.append((torch.from_numpy(keys).cuda(), bh.BloomFilter(m)))
        del keys
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]

    def job(ns):
        for j, (dk, f) in enumerate(built):
            s = streams[j % ns]
            f.clear(stream=s)
            f.set_batch(dk, stream=s)

    def timed(ns, calls=20):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            job(ns)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            job(ns)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / calls

    for rnd in range(rounds):
        for ns in (1, 2, 4):
            ms = timed(ns) * 1e3
            print(json.dumps({"round": rnd, "streams": ns, "ms": round(ms, 4),
                              "gkeys_s": round(8 * W.C5_N / ms / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
