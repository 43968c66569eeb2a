#!/usr/bin/env python3
"""Per-kernel stats of ONE workload's timed calls from a rocprofv3
--kernel-trace CSV: the dispatches after the last marker kernel (the
profiling scripts launch torch.cuda._sleep(1), whose kernel is torch's
spin_kernel, between their setup -- filter
builds, key uploads -- and the timed calls), grouped by kernel name, written
in the layout of rocprofv3's --stats kernel CSV (Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs).  Without a marker every dispatch counts.
Usage: python tools/trace_stats.py RUN_kernel_trace.csv OUT_kernel_stats.csv"""
import collections
import csv
import sys


def main(src, dst):
    rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
    last = -1
    for i, r in enumerate(rows):
        if "spin_kernel" in r["Kernel_Name"] or "sleep" in r["Kernel_Name"].lower():
            last = i
    durs = collections.defaultdict(list)
    for r in rows[last + 1:]:
        durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in durs.values()) or 1
    with open(dst, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])
    print(f"{dst}: {sum(len(v) for v in durs.values())} dispatches after marker #{last + 1} "
          f"of {len(rows)}, {len(durs)} kernels")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
