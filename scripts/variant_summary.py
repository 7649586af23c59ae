#!/usr/bin/env python3
"""Summary of a scripts/gpu_variants.sh run with PROF=1: per variant and pass the
top kmc kernels (calls x average ms) from rocprofv3 --stats, then the JSON lines'
timings.  Usage: variant_summary.py gpurun_out/TAG [HEADER ...]"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    for line in sys.argv[2:]:
        print("# " + line)
    for p in sorted(glob.glob(os.path.join(d, "prof_*"))):
        f = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)
        if not f:
            continue
        rows = [r for r in csv.DictReader(open(f[0])) if "kmc::" in r["Name"]]
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        name = lambda r: r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace(
            "kmc::", "").split("(")[0]
        print("%s: %s" % (os.path.basename(p), "; ".join(
            "%s x%s %.3f ms" % (name(r), r["Calls"], float(r["AverageNs"]) / 1e6) for r in rows[:8])))
    for l in open(os.path.join(d, "variants.log")):
        if l.startswith("{"):
            x = json.loads(l)
            print(x.get("config", x.get("k")), "s_med %.3f ms" % (1e3 * x["s_med"]) if "s_med" in x else l.strip()[:200])


if __name__ == "__main__":
    main()
