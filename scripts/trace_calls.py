#!/usr/bin/env python3
"""Per-call kernel durations from a rocprofv3 --kernel-trace csv directory: a call
ends with a kernel whose name contains END.  trace_calls.py DIR END [LAST_N]."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
end = sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], []
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("kmc::", "").split("(")[0]
    if n.startswith("void at::") or n.startswith("at::"):
        continue
    cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if end in n:
        calls.append(cur)
        cur = []
for c in calls[-last:]:
    print("call: %.3f ms from first start to last end" % ((c[-1][2] - c[0][1]) / 1e6))
    for n, a, b in c:
        print("   %-50s %8.3f ms" % (n[:50], (b - a) / 1e6))
