#!/usr/bin/env python3
"""Counter calibration summary (tools/ubench.py cal under the rocprofv3 --pmc
passes of tools/gpu_steps.sh `cal`): for each access shape, the counters per
dispatch against the bytes the kernel requested.  Dispatches of ub_cal are
taken in order, three per shape (CAL_SHAPES).

  fetch_per_known  = FETCH_SIZE bytes / requested bytes (reads)
  write_per_known  = WRITE_SIZE bytes / requested bytes (writes)
  req128_frac      = TCC_BUBBLE / TCC_EA0_RDREQ (128-B read requests)
  dram_rd_per_req  = TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ (requests that reach DRAM)

Usage: pmc_cal.py TAG [out.json]  (TAG: the gpu_steps.sh tag, gpurun_out/TAG/)"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dispatches(d):
    """{dispatch id: {counter: value}} for the ub_cal dispatches of one pass."""
    out = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "ub_cal" not in r["Kernel_Name"]:
                continue
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            out[did][r["Counter_Name"]] = out[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main(tag, dest=None):
    base = os.path.join(ROOT, "gpurun_out", tag)
    shapes = [json.loads(l) for l in open(os.path.join(base, "cal.log")) if l.startswith('{"cal"')]
    passes = {}
    for p in glob.glob(os.path.join(base, "cal_*")):
        if os.path.isdir(p):
            passes[os.path.basename(p)] = dispatches(p)
    rows = []
    for i, sh in enumerate(shapes):
        ctr = {}
        for name, ds in passes.items():
            got = ds[3 * i:3 * i + 3]
            for c in set().union(*[set(x) for x in got]) if got else ():
                ctr[c] = statistics.median(x[c] for x in got if c in x)
        known = sh["known_bytes"]
        row = dict(sh)
        row["counters"] = ctr
        if "FETCH_SIZE" in ctr:
            row["fetch_per_known"] = round(ctr["FETCH_SIZE"] * 1024 / known, 4)
        if "WRITE_SIZE" in ctr:
            row["write_per_known"] = round(ctr["WRITE_SIZE"] * 1024 / known, 4)
        rd = ctr.get("TCC_EA0_RDREQ_sum")
        if rd:
            row["rdreq_bytes_per_known_at_64B"] = round(rd * 64 / known, 4)
            if "TCC_BUBBLE_sum" in ctr:
                row["req128_frac"] = round(ctr["TCC_BUBBLE_sum"] / rd, 4)
            if "TCC_EA0_RDREQ_DRAM_sum" in ctr:
                row["dram_rd_per_req"] = round(ctr["TCC_EA0_RDREQ_DRAM_sum"] / rd, 4)
        wr = ctr.get("TCC_EA0_WRREQ_sum")
        if wr and "TCC_EA0_WRREQ_64B_sum" in ctr:
            row["wrreq64_frac"] = round(ctr["TCC_EA0_WRREQ_64B_sum"] / wr, 4)
        rows.append(row)
        print(json.dumps({k: v for k, v in row.items() if k != "counters"}))
    if dest:
        json.dump({"tag": tag, "source": "tools/ubench.py cal + tools/gpu_steps.sh cal (rocprofv3 --pmc, one counter set per pass)",
                   "shapes": rows}, open(dest, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
