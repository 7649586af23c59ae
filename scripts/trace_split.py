"""Per-call kernel times of a cbench run under the kernel trace, split by
configuration: the canonical kernels of the first half of the calls (C4) and the
second half (C4R) -- scripts/cbench.py runs C4 before C4R, the same number of
calls each.  Usage: python scripts/trace_split.py <rocprofv3 -d dir> [substring]"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "canon_"
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if sub not in n:
        continue
    key = n.replace("(anonymous namespace)", "").replace("void ", "").split("(")[0].split("::")[-1]
    per.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(per.items()):
    h = len(v) // 2
    a, b = v[:h], v[h:]
    if a and b:
        print("    %-40s C4 %7.3f  C4R %7.3f ms med" % (k[:40], statistics.median(a), statistics.median(b)))
