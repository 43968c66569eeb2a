#!/usr/bin/env python3
"""The bench's fan-in-4 compaction (4 runs x 4.2M entries, filter fused)
repeated for rocprofv3 --kernel-trace --stats: `python tools/compact_prof.py
[reps] [alt]` (alt: the lib_alt build of tools/build_alt.sh).  A marker
kernel separates the setup from the timed calls (tools/trace_stats.py)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[2] == "alt":
    os.environ["BLOOMHIP_LIB"] = os.path.join(ROOT, "cs265-lsm-tree_amd", "lib_alt", "libbloomhip.so")
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
import torch  # noqa: E402

import bloomhip as bh  # noqa: E402
from bloomhip import workloads as W  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    runs, m = W.compaction_fanin()
    druns = [torch.from_numpy(r).cuda() for r in runs]
    total = sum(r.shape[0] for r in runs)
    dout = torch.empty((total, 2), dtype=torch.int32, device="cuda")
    f = bh.BloomFilter(m)
    bh.compact(druns, drop_tombstones=True, filter=f, out=dout)  # untimed, then the trace marker
    torch.cuda.synchronize()
    torch.cuda._sleep(1)
    ts = []
    for _ in range(reps):
        f.clear()
        t0 = time.perf_counter()
        bh.compact(druns, drop_tombstones=True, filter=f, out=dout)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print("compact ms median", round(ts[len(ts) // 2] * 1e3, 4))


if __name__ == "__main__":
    main()
