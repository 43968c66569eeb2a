#!/usr/bin/env python3
"""Compact view of a rocprofv3 --stats kernel CSV: name (template args kept),
calls, average microseconds.  `python tools/kstats.py <run_kernel_stats.csv>`."""
import csv
import re
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("bloomhip::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*\)$", "", n)
    n = re.sub(r"\(bloomhip::.*", "", n)
    print(f"{n[:70]:70s} {r['Calls']:>5} {float(r['AverageNs']) / 1000:10.2f} us")
