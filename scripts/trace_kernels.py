#!/usr/bin/env python3
"""Median duration per kernel from a rocprofv3 --kernel-trace csv directory:
trace_kernels.py DIR [SUBSTRING] (kernels whose name contains SUBSTRING, > 0.05 ms)."""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("kmc::", "").split("(")[0]
    if sub in n:
        acc[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n, v in sorted(acc.items()):
    v = sorted(v)
    if v[-1] > 0.05:
        print("    %-48s %.3f ms med  (%d launches)" % (n[:48], v[len(v) // 2], len(v)))
