#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per
dispatch for each kernel (name shortened).  Usage: pmc_summary.py DIR [DIR ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(\w+)<([^>]*)>", name)
    if m:
        return "%s<%s>" % (m.group(1), m.group(2).replace("(anonymous namespace)::", ""))
    return name.split("(")[0].split("::")[-1]


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values]
    dur = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row["Kernel_Name"])
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return vals, dur


def main():
    vals, dur = load(sys.argv[1:])
    for k in sorted(vals):
        n = max(len(v) for v in vals[k].values())
        print("== %s  (%d samples, mean dur %.3f ms)" % (k, n, sum(dur[k]) / len(dur[k]) / 1e6))
        for c in sorted(vals[k]):
            v = vals[k][c]
            print("   %-28s %16.4g" % (c, sum(v) / len(v)))


if __name__ == "__main__":
    main()
