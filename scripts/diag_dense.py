#!/usr/bin/env python3
"""DIAGNOSTIC: per-record column sums of the dense k = 8 counter against each
record's windows, for the hot / burst / iid record mix of
tests/test_dense_gpu.py::test_k8_hot_half_scans_with_fallback and an iid mix of
the same size, with thieves on (default), off, and late owners."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dna-kmeres-parallel_amd"), os.path.join(REPO, "oracle")]


def main():
    import torch
    import kmc
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(808)
    acgt = np.frombuffer(b"ACGT", np.uint8)

    def hot(n):
        return np.where(rng.random(n) < 0.65, ord("A"), acgt[rng.integers(1, 4, n)]).astype(np.uint8)

    def burst(n, run):
        x = hot(n)
        o = (n - run) // 2
        x[o:o + run] = ord("A")
        return x
    sc = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    M = lambda x: int(x * sc)
    mixes = {
        "hot": [hot(M(100 << 20)), burst(M(5 << 20), M(3 << 20)), hot(M(60 << 20)), acgt[rng.integers(0, 4, M(20 << 20))],
                burst(M(3 << 20), M(1 << 20)), hot(M(150 << 20)), burst(M(7 << 20), M(5 << 20)), hot(M(40 << 20))],
        "iid": [acgt[rng.integers(0, 4, M(n << 20))] for n in (100, 5, 60, 20, 3, 150, 7, 40)],
    }
    hook = kmc.lib().kmc_diag_dense_steal
    for name, seqs in mixes.items():
        recs = [np.append(x, np.uint8(0)) for x in seqs]
        data = np.concatenate(recs)
        idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
        d = torch.from_numpy(data).to(dev)
        di = torch.from_numpy(idx).to(dev)
        win = np.array([r.size - 8 for r in recs])
        a_cnt = np.array([(r[:-1] == ord("A")).sum() for r in recs])
        for mode, args in (("default", (-1, 0)), ("no_thieves", (0, 0)), ("late_owners", (1, 30000))):
            hook(*args)
            out, inv = kmc.count_dense(d, di, 8, invalid=True)
            torch.cuda.synchronize()
            o = out.cpu().numpy().astype(np.int64)
            col = o.sum(axis=0)
            print(name, mode, "colsum/windows:", np.round(col / win, 4).tolist(), "bin0:", o[0].tolist(), flush=True)
        hook(-1, 0)


if __name__ == "__main__":
    main()
