#!/usr/bin/env python3
"""Per-call canon_* kernel durations (ms) from a rocprofv3 kernel trace directory."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "canon_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], []
for r in rows:
    n = r["Kernel_Name"].split("canon_")[1].split("_kernel")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if n == "count" and cur:
        calls.append(cur)
        cur = []
    cur.append((n, d))
calls.append(cur)
for c in calls:
    if sum(d for _, d in c) > 1.0:
        print(" ".join("%s=%.2f" % (n, d) for n, d in c if d > 0.05), " sum=%.1f" % sum(d for _, d in c))
