#!/usr/bin/env python3
"""Time kmc_count_canonical_hash on C4 / C4R (3.1 Gbase, k = 31, soft-masked) with
whatever library KMC_LIB names (timing-only ablation builds included: no result
check).  Prints the median of --iters calls per input and the per-kernel split
needs rocprofv3 around it.  Usage: KMC_LIB=... python scripts/canon_time.py"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dna-kmeres-parallel_amd"), os.path.join(REPO, "scripts")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--configs", default="c4,c4r")
    a = ap.parse_args()
    import torch
    import kmc
    import genome_synth
    dev = torch.device("cuda:0")
    for name in a.configs.split(","):
        if name == "c4":
            data, idx, _ = genome_synth.grch38_like(torch, dev, 3.1)
        else:
            data, idx, _, _ = genome_synth.repeat_genome(torch, dev, 3.1)
        ts = []
        for it in range(a.iters + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = kmc.count_canonical(data, idx, 31, flags=kmc.CANON_SOFTMASK)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del r
        ts = sorted(ts[1:])
        print("%s %s: median %.2f ms, min %.2f ms" % (os.path.basename(kmc.LIB_PATH), name, 1e3 * ts[len(ts) // 2],
                                                      1e3 * ts[0]), flush=True)
        del data, idx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
