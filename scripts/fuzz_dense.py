#!/usr/bin/env python3
"""DIAGNOSTIC fuzz: kmc_count_dense (k = 1..13: LDS kernels, packed 16-bit bins
with their scans and recounts, the radix path) vs the oracle on random record sets
with N / lowercase / low-complexity runs; bit-exact counts and invalid counts.
--sampled: k >= 9 cases take the sampled radix partition, with capacities x 1,
x 0.9 (overflow lists) or x 0.3 (the exact rerun) at random.
Usage: python scripts/fuzz_dense.py [--cases 40] [--seed 1] [--sampled]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dna-kmeres-parallel_amd"), os.path.join(REPO, "oracle")]


def make_case(rng, k):
    n = int(rng.choice([1, 2, 5, 30])) if k < 12 else int(rng.choice([1, 2, 3]))
    recs = []
    for _ in range(n):
        L = int(rng.choice([0, 1, k - 1, k, 4095, 65_000, 400_000, 3_000_000]))
        if n > 5:
            L = min(L, 65_000)
        x = rng.choice(np.frombuffer(b"ACGTacN", np.uint8), size=L,
                       p=[.2425, .2425, .2425, .2425, .01, .01, .01]).astype(np.uint8)
        if L > 1000 and rng.random() < 0.5:
            a = int(rng.integers(0, L - 500))
            b = min(L, a + int(rng.integers(500, 2_000_000)))
            unit = rng.choice([b"A", b"AC", b"ACGTTGCA", b"AAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAT"])
            x[a:b] = np.resize(np.frombuffer(unit, np.uint8), b - a)
        recs.append(np.append(x, np.uint8(0)))
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    return data, idx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=40)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--sampled", action="store_true")
    a = ap.parse_args()
    import torch
    import kmc
    import oracle
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(a.seed)
    bad = 0
    if a.sampled:  # the mode hook lives in the diagnostic library (lib/libkmc_diag.so)
        kmc.diag().__enter__()
    for c in range(a.cases):
        k = int(rng.integers(1, 14))
        data, idx = make_case(rng, k)
        mode = ""
        if a.sampled and k >= 9:
            scale = float(rng.choice([1.0, 0.9, 0.3]))
            kmc.lib().kmc_diag_radix_mode(2, scale)
            mode = " sampled x%.1f" % scale
        d = torch.from_numpy(data if data.size else np.zeros(16, np.uint8)).to(dev)
        out, inv = kmc.count_dense(d, torch.from_numpy(idx).to(dev), k, data_bytes=data.size, invalid=True)
        torch.cuda.synchronize()
        exp, exp_inv = oracle.count_dense(data, idx, k)
        ok = np.array_equal(out.cpu().numpy(), exp) and np.array_equal(inv.cpu().numpy(), exp_inv)
        print("case %2d: k=%2d %3d records %9d bytes%s %s" % (c, k, idx.size - 1, data.size, mode,
                                                            "ok" if ok else "MISMATCH"), flush=True)
        if mode:
            kmc.lib().kmc_diag_radix_mode(0, 1.0)
        bad += not ok
        del out, inv, d
    print("fuzz: %d/%d cases bit-exact" % (a.cases - bad, a.cases))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
