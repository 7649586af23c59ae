#!/usr/bin/env python3
"""Per-call kernel split of the canonical calls in a cbench run under the kernel
trace: the trace is cut into calls at each canon_direct_setup_kernel launch (the
first kernel of a direct-output call), every kernel's launches are summed per call,
and the calls are split in two halves (scripts/cbench.py runs C4's calls, then
C4R's, as many each).  Prints per configuration the median per-call time of every
kernel and of the whole span (first kernel start to last kernel end).
Usage: python scripts/canon_call_split.py <rocprofv3 -d dir>"""
import csv
import glob
import statistics
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        n = n.split("(")[0].split("::")[-1]
        if "canon_direct_setup_kernel" in n:
            cur = {"_t0": int(r["Start_Timestamp"]), "_t1": 0, "k": {}}
            calls.append(cur)
        if cur is None or not (n.startswith("canon_") or "scan" in n):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cur["k"][n] = cur["k"].get(n, 0.0) + d
        cur["_t1"] = max(cur["_t1"], int(r["End_Timestamp"]))
    h = len(calls) // 2
    for name, cs in (("C4", calls[:h]), ("C4R", calls[h:])):
        if not cs:
            continue
        keys = sorted({k for c in cs for k in c["k"]}, key=lambda k: -statistics.median([c["k"].get(k, 0) for c in cs]))
        span = statistics.median([(c["_t1"] - c["_t0"]) / 1e6 for c in cs])
        tot = statistics.median([sum(c["k"].values()) for c in cs])
        print("%s: %d calls, span %.2f ms, kernels %.2f ms (medians per call)" % (name, len(cs), span, tot))
        for k in keys:
            print("    %-36s %7.3f ms" % (k[:36], statistics.median([c["k"].get(k, 0.0) for c in cs])))


if __name__ == "__main__":
    main()
