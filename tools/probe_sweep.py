#!/usr/bin/env python3
"""Times the C3 probe per level filter under each probe strategy (gather /
partition), and the five-filter call as the product routes it.  Prints one
JSON object per measurement.  Used to place the gather/partition threshold
(kProbeGatherMaxBytes)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
import bloomhip as bh  # noqa: E402
from bloomhip import workloads as W  # noqa: E402


def timed(fn, reps=20):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn(s)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn(s)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    torch.cuda.set_device(0)
    gets, levels = W.c3()
    dgets = torch.from_numpy(gets).cuda()
    nw = (gets.size + 63) // 64
    filters = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch(keys)
        filters.append(f)
    out = torch.empty((len(filters), nw), dtype=torch.int64, device="cuda")
    ref = None
    for (lvl, _, m), f in zip(levels, filters):
        row = {}
        for name, st in (("gather", bh.PROBE_GATHER), ("partition", bh.PROBE_PARTITION),
                         ("lds", bh.PROBE_LDS)):
            if st == bh.PROBE_LDS and (m + 7) // 8 > 160 * 1024:
                continue
            f.set_probe_strategy(st)
            ms = timed(lambda s: bh.test_batch([f], dgets, out=out[lvl:lvl + 1], stream=s))
            row[name] = round(ms * 1e3, 1)
            got = out[lvl].cpu().clone()
            if ref is None or ref[0] != lvl:
                ref = (lvl, got)
            else:
                assert torch.equal(ref[1], got), f"level {lvl}: strategies disagree"
        f.set_probe_strategy(bh.PROBE_AUTO)
        print(json.dumps({"level": lvl, "m_bits": m, "filter_bytes": (m + 7) // 8,
                          "us": row}), flush=True)
    for nf in (3, 4, 5):
        ms = timed(lambda s: bh.test_batch(filters[:nf], dgets, out=out[:nf], stream=s))
        print(json.dumps({"levels": nf, "auto_us": round(ms * 1e3, 1)}), flush=True)
    # Stacked pass vs the members probed one by one (their own best kind).
    alone = [bh.PROBE_LDS, bh.PROBE_GATHER, bh.PROBE_GATHER, bh.PROBE_GATHER, bh.PROBE_PARTITION]
    for sub in ([0, 1, 2, 3, 4], [0, 1, 2, 3], [1, 2, 3], [3, 4], [0, 4], [2, 3]):
        fs = [filters[i] for i in sub]
        o = out[:len(sub)]
        for i in sub:
            filters[i].set_probe_strategy(bh.PROBE_STACKED)
        st_us = timed(lambda s: bh.test_batch(fs, dgets, out=o, stream=s)) * 1e3
        got = o.cpu().clone()
        for i in sub:
            filters[i].set_probe_strategy(alone[i])
        al_us = timed(lambda s: bh.test_batch(fs, dgets, out=o, stream=s)) * 1e3
        assert torch.equal(got, o.cpu()), f"stacked {sub} disagrees"
        for i in sub:
            filters[i].set_probe_strategy(bh.PROBE_AUTO)
        au_us = timed(lambda s: bh.test_batch(fs, dgets, out=o, stream=s)) * 1e3
        print(json.dumps({"levels": sub, "stacked_us": round(st_us, 1),
                          "one_by_one_us": round(al_us, 1), "auto_us": round(au_us, 1)}),
              flush=True)
    for st_name, st in (("all gather", bh.PROBE_GATHER),):
        for f in filters:
            f.set_probe_strategy(st)
        ms = timed(lambda s: bh.test_batch(filters, dgets, out=out, stream=s))
        print(json.dumps({"levels": 5, st_name + "_us": round(ms * 1e3, 1)}), flush=True)
        for f in filters:
            f.set_probe_strategy(bh.PROBE_AUTO)


if __name__ == "__main__":
    sys.exit(main())
