#!/usr/bin/env python3
"""Kernel micro-benchmark: time the dense histogram kernel alone (HIP events
around the launch, kmc_trace_set_events) for several k on one synthetic buffer.
Usage: python scripts/kbench.py [--gbases 10] [--ks 3,7,8] [--iters 10]
Set KMC_LIB to time a diagnostic build (make -C dna-kmeres-parallel_amd ablate)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-kmeres-parallel_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gbases", type=float, default=10.0)
    ap.add_argument("--records", type=int, default=10)
    ap.add_argument("--ks", default="3,7,8")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tag", default=os.environ.get("KMC_LIB", "libkmc.so"))
    a = ap.parse_args()
    import torch
    import kmc
    dev = torch.device("cuda:0")
    L = int(a.gbases * 1e9 / a.records)
    nbytes = a.records * (L + 1)
    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    kmc.synth_fill(data, a.records, L, 0x5EED0008)
    idx = torch.from_numpy(kmc.synth_indices(a.records, L)).to(dev)
    for k in [int(x) for x in a.ks.split(",")]:
        out = torch.empty((1 << (2 * k), a.records), dtype=torch.int32, device=dev)
        args = kmc.dense_args(data, idx, k, out)
        ws = torch.empty(kmc.dense_ex_workspace_size(args), dtype=torch.uint8, device=dev)
        args = kmc.dense_args(data, idx, k, out, workspace=ws)
        for _ in range(10):  # the clock ramps over ~10 launches after idling
            kmc.count_dense_ex(args)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
        for b, e in ev:
            b.record(); e.record()
        torch.cuda.synchronize()
        for b, e in ev:
            kmc.trace_events(b, e)
            kmc.count_dense_ex(args)
        torch.cuda.synchronize()
        kmc.trace_events(None, None)
        ms = sorted(b.elapsed_time(e) for b, e in ev)
        med = ms[len(ms) // 2]
        print(json.dumps({"lib": os.path.basename(a.tag), "k": k, "bytes": nbytes, "ms_med": med, "ms_min": ms[0],
                          "GBps": nbytes / med / 1e6, "frac8TB": nbytes / med / 1e6 / 8000}))


if __name__ == "__main__":
    main()
