#!/usr/bin/env python3
"""HBM traffic per launch of the k = 8 histogram kernel for every rank's shard of
the strong-scaled 10 Gbase bench job at N = 1, 2, 4, 8 (bench.rank_plan), the
`roofline.traffic` that bench.py reports at each N (rocprofv3 PMC on one GPU: the
same kernel over the same shard bytes as that rank of the N-GPU job).

  run:    python scripts/pmc_shards.py run   (under rocprofv3 --pmc ..., one counter
          group per run: FETCH_SIZE TCC_EA0_RDREQ_128B, then WRITE_SIZE); every
          shard gets exactly LAUNCHES calls, in the order printed
  parse:  python scripts/pmc_shards.py parse FETCH_DIR WRITE_DIR RUN_LOG OUT.json
          (gfx950: FETCH_SIZE counts a 128-B read request as 64 B, x2; see
          MI355X_MICROARCH.md's HBM section; cross-checked by TCC_EA0_RDREQ_128B)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dna-kmeres-parallel_amd")]
LAUNCHES = 4
KERNEL = "count_dense_kernel<8, 1, 3,"


def run():
    import torch

    import bench
    import kmc
    dev = torch.device("cuda:0")
    # the build measured (bench.py reports a PMC entry only for the same build)
    print(json.dumps({"build_id": bench.dense_code_object_id(kmc.LIB_PATH)}), flush=True)
    k, L = 8, 1_000_000_000
    nb = 1 << (2 * k)
    for world in (1, 2, 4, 8):
        for rank in range(world):
            plan = bench.rank_plan("strong", world, rank, 10, L, k)
            base, hold_hi = plan["hold"]
            (wl, wh), (rl, rh) = plan["win"], plan["read"]
            data = torch.empty(max(hold_hi - base, 16), dtype=torch.uint8, device=dev)
            kmc.synth_fill_range(data, base, hold_hi, L, bench.SEED_BASE + k)
            idx = torch.from_numpy(plan["indices"]).to(dev)
            out = torch.empty((nb, plan["n_tot"]), dtype=torch.int32, device=dev)
            a = kmc.dense_args(data, idx, k, out.view(-1), read=(rl, rh), win=(wl, wh), data_offset=base)
            ws = torch.empty(max(kmc.dense_ex_workspace_size(a), 1), dtype=torch.uint8, device=dev)
            a = kmc.dense_args(data, idx, k, out.view(-1), read=(rl, rh), win=(wl, wh), workspace=ws,
                               data_offset=base)
            for _ in range(LAUNCHES):
                kmc.count_dense_ex(a)
            torch.cuda.synchronize()
            print(json.dumps({"world": world, "rank": rank, "data_bytes": wh - wl}), flush=True)
            del data, out, ws
            torch.cuda.empty_cache()


def per_dispatch(d):
    """{counter: [value per dispatch of KERNEL, in dispatch order]}"""
    rows = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KERNEL in r["Kernel_Name"].replace("(anonymous namespace)::", ""):
                    did = int(r["Dispatch_Id"])
                    rows[did][r["Counter_Name"]] = rows[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = defaultdict(list)
    for did in sorted(rows):
        for c, v in rows[did].items():
            out[c].append(v)
    return out


def parse(fetch_dir, write_dir, log, dst):
    lines = [json.loads(l) for l in open(log) if l.startswith("{")]
    build_id = next(x["build_id"] for x in lines if "build_id" in x)
    shards = [x for x in lines if "world" in x]
    f, w = per_dispatch(fetch_dir), per_dispatch(write_dir)
    assert len(f["FETCH_SIZE"]) == LAUNCHES * len(shards) == len(w["WRITE_SIZE"]), \
        (len(f["FETCH_SIZE"]), len(w["WRITE_SIZE"]), len(shards))
    res = []
    for i, s in enumerate(shards):
        sl = slice(LAUNCHES * i + 1, LAUNCHES * (i + 1))  # the first launch of a shard warms the caches
        mean = lambda xs: sum(xs[sl]) / len(xs[sl])
        fetch_kib, write_kib = mean(f["FETCH_SIZE"]), mean(w["WRITE_SIZE"])
        e = {"k": 8, "data_bytes": s["data_bytes"], "shard": "world %d rank %d" % (s["world"], s["rank"]),
             "kernel": KERNEL, "build_id": build_id, "fetch_size_kib_per_launch": fetch_kib, "write_size_kib_per_launch": write_kib,
             "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
             "correction": "gfx950: FETCH_SIZE counts a 128-B read request as 64 B (x2; MI355X_MICROARCH.md "
                           "HBM section), cross-checked by TCC_EA0_RDREQ_128B x 128 B",
             "source": "rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_128B / --pmc WRITE_SIZE (separate passes) of "
                       "scripts/pmc_shards.py run, launches 2-%d of each shard" % LAUNCHES}
        if "TCC_EA0_RDREQ_128B" in f:
            e["rdreq_bytes_per_launch"] = mean(f["TCC_EA0_RDREQ_128B"]) * 128
        res.append(e)
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    for e in res:
        print(e["shard"], e["data_bytes"], "%.4g" % e["hbm_bytes_per_launch"],
              "%.4f x data" % (e["hbm_bytes_per_launch"] / e["data_bytes"]))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(*sys.argv[2:6])
