#!/usr/bin/env python3
"""C3 probe (16.8M GETs x 5 level filters) repeated under one strategy, for
rocprofv3 --kernel-trace --stats: `python tools/probe_prof.py [auto|stacked|
partition|gather|route] [reps] [alt|-] [c3|f10]` (route: the GET routing,
bloomhip_route_gets_packed, over runs built with their fences; f10: the f = 10
tree's three levels instead of C3's five).  A marker kernel separates the
setup from the timed calls (tools/trace_stats.py)."""
import os
import sys

import torch

if len(sys.argv) > 3 and sys.argv[3] == "alt":  # the lib_alt build (tools/build_alt.sh)
    os.environ["BLOOMHIP_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "cs265-lsm-tree_amd", "lib_alt", "libbloomhip.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
import bloomhip as bh  # noqa: E402
from bloomhip import workloads as W  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "auto"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    route = kind == "route"
    st = {"auto": bh.PROBE_AUTO, "route": bh.PROBE_AUTO, "stacked": bh.PROBE_STACKED, "partition": bh.PROBE_PARTITION,
          "gather": bh.PROBE_GATHER}[kind]
    torch.cuda.set_device(0)
    workload = sys.argv[4] if len(sys.argv) > 4 else "c3"
    # routing needs each run as the reference writes it (sorted: its fences
    # ascend); the filters are the same either way
    if route:
        gets, levels = W.c3_runs() if workload == "c3" else W.f10_runs()
    else:
        gets, levels = W.c3() if workload == "c3" else W.f10()
    dgets = torch.from_numpy(gets).cuda()
    filters = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        if route:
            f.set_batch_run(keys)
        else:
            f.set_batch(keys)
        f.set_probe_strategy(st)
        filters.append(f)
    out = torch.empty((len(filters), (gets.size + 63) // 64), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    rt = torch.empty(gets.size, dtype=torch.int32, device="cuda")
    # one untimed call, then the marker kernel tools/trace_stats.py cuts the
    # trace at (the builds above and this call stay out of the stats)
    call = (lambda: bh.route_gets_packed(filters, dgets, cand=out, route=rt, stream=s)) if route else \
        (lambda: bh.test_batch(filters, dgets, out=out, stream=s))
    call()
    torch.cuda.synchronize()
    torch.cuda._sleep(1)
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    print("done", kind, reps)


if __name__ == "__main__":
    main()
