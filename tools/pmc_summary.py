#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: per kernel, median counter value per
dispatch over dispatches of the same grid size.  Usage: pmc_summary.py DIR"""
import collections
import csv
import glob
import json
import statistics
import sys


def main(d):
    data = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = name.replace("bloomhip::(anonymous namespace)::", "").replace("void ", "")
            short = short.split("(")[0]
            key = (short, int(r["Grid_Size"]))
            data[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for (k, g), ctrs in sorted(data.items()):
        out[f"{k} grid={g}"] = {c: statistics.median(v) for c, v in ctrs.items()}
    return out


if __name__ == "__main__":
    res = main(sys.argv[1])
    for k, v in res.items():
        print(k)
        for c, x in sorted(v.items()):
            print(f"   {c:24s} {x:16.1f}")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
