#!/usr/bin/env python3
"""One rank of an N-way strong-scaling bench.py job, on one GPU, without the
all-reduce: what each rank's step costs when the 10 Gbase job is cut N ways
(bench.rank_plan, kmc_plan_shards).  For every N and rank it prints the step
time (the whole kmc_count_dense_ex call: histogram kernel + slab reduce + spill
fix-up, back to back), the histogram kernel's time (HIP events around it) and
the step overhead; the worst rank bounds the N-GPU step.
Usage: python scripts/shardbench.py [--worlds 1,2,4,8] [--steps 20] [--ranks all|first]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dna-kmeres-parallel_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--records", type=int, default=10)
    ap.add_argument("--record-len", type=int, default=1_000_000_000)
    ap.add_argument("--ranks", default="first", help="first: rank 0 and the last rank; all: every rank")
    a = ap.parse_args()
    import torch

    import bench
    import kmc
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    k, L = a.k, a.record_len
    seed = bench.SEED_BASE + k
    nb = 1 << (2 * k)
    for world in [int(x) for x in a.worlds.split(",")]:
        ranks = range(world) if a.ranks == "all" else sorted({0, world - 1})
        for rank in ranks:
            plan = bench.rank_plan("strong", world, rank, a.records, L, k)
            base, hold_hi = plan["hold"]
            (win_lo, win_hi), (read_lo, read_hi) = plan["win"], plan["read"]
            data = torch.empty(max(hold_hi - base, 16), dtype=torch.uint8, device=dev)
            kmc.synth_fill_range(data, base, hold_hi, L, seed)
            idx = torch.from_numpy(plan["indices"]).to(dev)
            out = torch.empty((nb, plan["n_tot"]), dtype=torch.int32, device=dev)
            args = kmc.dense_args(data, idx, k, out.view(-1), read=(read_lo, read_hi), win=(win_lo, win_hi),
                                  data_offset=base)
            ws = torch.empty(max(kmc.dense_ex_workspace_size(args), 1), dtype=torch.uint8, device=dev)
            args = kmc.dense_args(data, idx, k, out.view(-1), read=(read_lo, read_hi), win=(win_lo, win_hi),
                                  workspace=ws, data_offset=base)
            for _ in range(14):  # clock ramp
                kmc.count_dense_ex(args, stream)
            torch.cuda.synchronize()
            tot = int(out.to(torch.int64).sum())  # = the valid windows starting in [win_lo, win_hi)
            ev =[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.steps)]
            for b, e in ev:
                b.record(stream)
                e.record(stream)
            # (1) whole steps back to back, no events inside
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                kmc.count_dense_ex(args, stream)
            torch.cuda.synchronize()
            step_ms = (time.perf_counter() - t0) / a.steps * 1e3
            # (2) the histogram kernel alone
            for b, e in ev:
                kmc.trace_events(b, e)
                kmc.count_dense_ex(args, stream)
            torch.cuda.synchronize()
            kmc.trace_events(None, None)
            kern = sorted(b.elapsed_time(e) for b, e in ev)
            kern_ms = kern[len(kern) // 2]
            print(json.dumps({"world": world, "rank": rank, "win_bytes": win_hi - win_lo, "windows_counted": tot,
                              "step_ms": round(step_ms, 4), "kernel_ms": round(kern_ms, 4),
                              "overhead_us": round((step_ms - kern_ms) * 1e3, 1),
                              "GBps_kernel": round((win_hi - win_lo) / kern_ms / 1e6, 1)}), flush=True)
            del data, out, ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
