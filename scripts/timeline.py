#!/usr/bin/env python3
"""Timeline of the last call in a rocprofv3 kernel (+ memory-copy) trace: every
kernel and copy from the last launch of kernel `first` on, with its start offset,
duration and the idle gap before it.  Usage: timeline.py TRACE_DIR FIRST_KERNEL_SUBSTRING"""
import csv
import glob
import sys


def rows(d):
    out = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n[:70]))
    for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                        "COPY %s %s B" % (r.get("Direction", "?"), r.get("Bytes", "?"))))
    return sorted(out)


def main():
    ev = rows(sys.argv[1])
    first = sys.argv[2]
    starts = [i for i, e in enumerate(ev) if first in e[2]]
    if starts:  # full-size launches only (a small check call may come last)
        big = max(ev[i][1] - ev[i][0] for i in starts)
        starts = [i for i in starts if ev[i][1] - ev[i][0] > big / 2]
    if not starts:
        print("no", first)
        return
    ev = ev[starts[-1]:]
    nxt = [i for i, e in enumerate(ev) if i > 0 and first in e[2]]
    if nxt:
        ev = ev[:nxt[0]]
    t0 = ev[0][0]
    prev_end = t0
    busy = 0
    for s, e, n in ev:
        print("%10.1f us  +%8.1f us gap  %10.1f us  %s" % ((s - t0) / 1e3, (s - prev_end) / 1e3, (e - s) / 1e3, n))
        busy += e - s
        prev_end = max(prev_end, e)
    print("span %.3f ms, busy %.3f ms" % ((prev_end - t0) / 1e6, busy / 1e6))


if __name__ == "__main__":
    main()
