#!/usr/bin/env python3
"""DIAGNOSTIC: how the k = 8 step reacts to a concurrent kernel on a second stream,
the stand-in for the RCCL all-reduce that bench.py overlaps with the next step's
counting.  For one rank's shard of an N-way strong-scaled job
(bench.rank_plan), every step launches kmc_count_dense_ex on the compute stream
and, once it is done, a spin kernel (scripts/spin_kernel.hip: `nwg` workgroups
holding 64 KB of LDS each, so a 128 KB count workgroup cannot share their CU) for
`us` microseconds on a second stream, exactly as an all-reduce of that step's
matrix would start while the next step counts.  Prints the per-step time and the
histogram kernel's time (HIP events) with and without the spin, and with the dense
grid leaving `reserve` CUs free (kmc_set_reserved_cus).
Usage: python scripts/interfere.py [--worlds 1,8] [--nwgs 0,4,8,16,32] [--us 50] [--reserve 0,8]"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dna-kmeres-parallel_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,8")
    ap.add_argument("--nwgs", default="0,4,8,16,32")
    ap.add_argument("--us", type=float, default=50.0)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--reserve", default="0")
    a = ap.parse_args()
    import torch

    import bench
    import kmc
    spin = ctypes.CDLL(os.path.join(REPO, "scripts", "lib", "libspin.so"))
    spin.spin_launch.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    k, L = a.k, 1_000_000_000
    seed = bench.SEED_BASE + k
    nb = 1 << (2 * k)
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    for world in [int(x) for x in a.worlds.split(",")]:
        plan = bench.rank_plan("strong", world, 0, 10, L, k)
        base, hold_hi = plan["hold"]
        (wl, wh), (rl, rh) = plan["win"], plan["read"]
        data = torch.empty(max(hold_hi - base, 16), dtype=torch.uint8, device=dev)
        kmc.synth_fill_range(data, base, hold_hi, L, seed)
        idx = torch.from_numpy(plan["indices"]).to(dev)
        out = torch.empty((nb, plan["n_tot"]), dtype=torch.int32, device=dev)
        ref = None
        for rep, reserve in [(r, v) for r in range(2) for v in [int(x) for x in a.reserve.split(",")]]:
            # (two passes over the modes: the box's clock drift shows)
            kmc.set_reserved_cus(reserve)
            args = kmc.dense_args(data, idx, k, out.view(-1), read=(rl, rh), win=(wl, wh), data_offset=base)
            ws = torch.empty(max(kmc.dense_ex_workspace_size(args), 1), dtype=torch.uint8, device=dev)
            args = kmc.dense_args(data, idx, k, out.view(-1), read=(rl, rh), win=(wl, wh), workspace=ws, data_offset=base)
            for _ in range(16):
                kmc.count_dense_ex(args, s1)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            for nwg in [int(x) for x in a.nwgs.split(",")]:
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.steps)]
                for b, e in ev:
                    b.record(s1)
                    e.record(s1)
                done = [torch.cuda.Event() for _ in range(a.steps)]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.steps):
                    kmc.trace_events(ev[i][0], ev[i][1])
                    kmc.count_dense_ex(args, s1)
                    if nwg:
                        done[i].record(s1)
                        s2.wait_event(done[i])
                        rc = spin.spin_launch(nwg, int(a.us * 100), 65536, ctypes.c_void_p(sink.data_ptr()),
                                              ctypes.c_void_p(s2.cuda_stream))
                        assert rc == 0, rc
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / a.steps * 1e3
                kmc.trace_events(None, None)
                kern = sorted(b.elapsed_time(e) for b, e in ev)
                ok = bool(torch.equal(out, ref))
                print(json.dumps({"world": world, "pass": rep, "reserve": reserve, "spin_wgs": nwg,
                                  "spin_us": a.us if nwg else 0,
                                  "step_ms": round(dt, 4), "kernel_ms_med": round(kern[len(kern) // 2], 4),
                                  "kernel_ms_max": round(kern[-1], 4), "counts_unchanged": ok}), flush=True)
            del ws
        kmc.set_reserved_cus(0)
        del data, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
