#!/usr/bin/env python3
"""C3 batched GET routing (16.8M GETs over the five level runs) timed with
BLOOMHIP_ROUTE_PER_CU = each value given (workgroups per CU of k_route):
`python tools/route_sweep.py 2 4 8`.  Prints one JSON line per value
(wall ms per route_gets call, stream-ordered, device-resident outputs)."""
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
    torch.cuda.set_device(0)
    gets, levels = W.c3_runs()
    runs = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch_run(keys)
        runs.append(f)
    n = gets.size
    dgets = torch.from_numpy(gets).cuda()
    dc = torch.empty((len(runs), (n + 63) // 64), dtype=torch.int64, device="cuda")
    df = torch.empty(n, dtype=torch.int32, device="cuda")
    dp = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    ref = None
    for v in sys.argv[1:] or ["0"]:
        if v == "0":
            os.environ.pop("BLOOMHIP_ROUTE_PER_CU", None)
        else:
            os.environ["BLOOMHIP_ROUTE_PER_CU"] = v
        for _ in range(3):
            bh.route_gets(runs, dgets, cand=dc, first=df, page=dp, stream=s)
        torch.cuda.synchronize()
        reps = 30
        t0 = time.perf_counter()
        for _ in range(reps):
            bh.route_gets(runs, dgets, cand=dc, first=df, page=dp, stream=s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        got = (df.cpu().numpy().tobytes(), dp.cpu().numpy().tobytes())
        same = None if ref is None else got == ref
        ref = ref or got
        print(json.dumps({"per_cu": v, "ms": round(ms, 4), "same_as_first": same}), flush=True)


if __name__ == "__main__":
    main()
