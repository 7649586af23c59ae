#!/usr/bin/env python3
"""Turn gpurun_out/prof_bench/ (scripts/profile_bench.sh) into committed profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the bench command
  profiles/<tag>_bench_trace.json   the bench JSON line printed under the profiler
  profiles/<tag>_kernel_launches.json  per-launch durations of the histogram kernel
  profiles/pmc_dense_k8_10gbase.json  HBM bytes per histogram launch (bench.py reads it)
  profiles/pmc_lds_k8_10gbase.json   LDS-array cycles per window and the held clock of the
                                     histogram kernel (bench.py's roofline.lds_floor_*)
FETCH_SIZE is counted in KiB and, on gfx950, reads half the bytes of a wide
streaming read (MI355X_MICROARCH.md §HBM): bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024."""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "prof_bench")
DST = os.path.join(REPO, "profiles")


def per_launch(counter_dir, counter, name_sub, durations=False):
    vals, durs = [], []
    for f in glob.glob(os.path.join(counter_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and name_sub in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
                    durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    return (vals, durs) if durations else vals


def lds_summary(line, k, kern, cus=256, xcds=8, last=10):
    """profiles/pmc_lds_k8_10gbase.json from the LDS pass: per full-size launch (the
    last `last`, after the clock ramp) the LDS-array cycles (all CUs), conflict
    cycles, LDS atomics, and the kernel's shader cycles (GRBM_GUI_ACTIVE / 8 XCDs)."""
    d = os.path.join(SRC, "lds")
    act = per_launch(d, "SQ_LDS_IDX_ACTIVE", kern)
    con = per_launch(d, "SQ_LDS_BANK_CONFLICT", kern)
    atm = per_launch(d, "SQ_INSTS_LDS_ATOMIC", kern)
    grbm, dur = per_launch(d, "GRBM_GUI_ACTIVE", kern, durations=True)
    if not (act and con and atm and grbm and line):
        return None
    full = lambda xs: [i for i, v in enumerate(xs) if v > 0.5 * max(xs)][-last:]  # not the slice check
    mean = lambda xs, ix: sum(xs[i] for i in ix) / len(ix)
    ka, kg = full(act), full(grbm)
    windows = line["config"]["total_records"] * (line["config"]["record_len"] - k + 1)
    a, c, t = mean(act, ka), mean(con, ka), mean(atm, ka)
    cyc = mean(grbm, kg) / xcds  # shader cycles of one launch
    ms = mean(dur, kg)
    out = {
        "k": k, "kernel": kern, "windows_per_launch": windows, "cus": cus, "launches": len(ka),
        "sq_lds_idx_active": a, "sq_lds_bank_conflict": c, "sq_insts_lds_atomic": t,
        "array_cycles_per_atomic": a / t, "conflict_frac": c / a,
        "array_cycles_per_window": a / windows,  # summed over the CUs
        "kernel_cycles": cyc, "launch_ms_under_pmc": ms, "clock_ghz": cyc / (ms * 1e-3) / 1e9,
        # the binding roof: the share of the kernel's cycles in which an average CU's
        # LDS array is busy (1.0 = the kernel runs at the LDS floor)
        "lds_busy_frac": a / cus / cyc,
        # the build measured: the bench line's code-object id of count_dense_kernel
        "build_id": line.get("roofline", {}).get("build_id"),
        "source": "rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE of "
                  "python3 bench.py --steps 20 --warmup 14 (scripts/profile_bench.sh), the last %d full-size "
                  "launches; kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md DVFS note); "
                  "lds_busy_frac = SQ_LDS_IDX_ACTIVE / CUs / kernel cycles" % len(ka),
    }
    with open(os.path.join(DST, "pmc_lds_k8_10gbase.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(DST, exist_ok=True)
    stats = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(DST, "%s_kernel_stats.csv" % tag))
    line = None
    with open(os.path.join(SRC, "trace.log")) as fh:
        for l in fh:
            if l.startswith("{"):
                line = json.loads(l)
    if line:
        with open(os.path.join(DST, "%s_bench_trace.json" % tag), "w") as fh:
            json.dump(line, fh, indent=1)
    k = line["config"]["k"] if line else 8
    kern = "count_dense_kernel<%d, 1, 3," % k if k == 8 else "count_dense_kernel<%d," % k
    # per-launch durations of the histogram kernel, in launch order (warm-up first)
    traces = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_trace.csv"), recursive=True)
    if traces:
        with open(traces[0]) as fh:
            rows = [r for r in csv.DictReader(fh) if kern in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        ms = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 4) for r in rows]
        with open(os.path.join(DST, "%s_kernel_launches.json" % tag), "w") as fh:
            json.dump({"kernel": kern + " (histogram launches of the bench command, in order)",
                       "ms": ms}, fh)
    fetch = per_launch(os.path.join(SRC, "fetch"), "FETCH_SIZE", kern)
    write = per_launch(os.path.join(SRC, "write"), "WRITE_SIZE", kern)
    r128 = per_launch(os.path.join(SRC, "fetch"), "TCC_EA0_RDREQ_128B", kern)
    r64 = per_launch(os.path.join(SRC, "fetch"), "TCC_EA0_RDREQ_64B", kern)
    # full-size launches only: the warm-up's 1 Mbase slice check is the same kernel
    fetch = [v for v in fetch if v > 0.5 * max(fetch)] if fetch else fetch
    write = [v for v in write if v > 0.5 * max(write)] if write else write
    r128 = [v for v in r128 if v > 0.5 * max(r128)] if r128 else r128
    if fetch and write and line:
        f = sum(fetch) / len(fetch)
        w = sum(write) / len(write)
        out = {
            "k": k,
            "data_bytes": line["config"]["total_records"] * (line["config"]["record_len"] + 1),
            "kernel": kern,
            "fetch_size_kib_per_launch": f,
            "write_size_kib_per_launch": w,
            "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
            "correction": "gfx950: FETCH_SIZE counts a 128-B read request as 64 B (x2; MI355X_MICROARCH.md HBM "
                          "section), confirmed here by TCC_EA0_RDREQ_128B x 128 B",
            "launches_sampled": [len(fetch), len(write)],
            "build_id": line.get("roofline", {}).get("build_id"),
            "source": "rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_64B / --pmc WRITE_SIZE "
                      "(separate passes) of python3 bench.py --steps 3",
        }
        if r128:
            out["rdreq_bytes_per_launch"] = (sum(r128) / len(r128)) * 128 + (sum(r64) / len(r64) if r64 else 0) * 64
        with open(os.path.join(DST, "pmc_dense_k8_10gbase.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        print(json.dumps(out))
    lds = lds_summary(line, k, kern)
    if lds:
        print(json.dumps(lds))


if __name__ == "__main__":
    main()
