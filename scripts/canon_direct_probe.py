#!/usr/bin/env python3
"""Direct-output probe (diagnostic library): for C4 / C4R at 3.1 Gbase, the share
of pairs that went through pk and the fallback copy, per call.
Usage: python scripts/canon_direct_probe.py [--gbases 3.1]"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dna-kmeres-parallel_amd"), os.path.join(REPO, "scripts")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gbases", type=float, default=3.1)
    a = ap.parse_args()
    import torch
    import kmc
    import genome_synth
    dev = torch.device("cuda:0")
    with kmc.diag() as D:
        for name in ("c4", "c4r"):
            if name == "c4":
                data, idx, lens = genome_synth.grch38_like(torch, dev, a.gbases)
            else:
                data, idx, lens, _ = genome_synth.repeat_genome(torch, dev, a.gbases)
            for it in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                keys, counts, off = kmc.count_canonical(data, idx, 31, flags=kmc.CANON_SOFTMASK)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                e, pr = ctypes.c_ulonglong(0), ctypes.c_ulonglong(0)
                D.kmc_diag_canon_fallback(ctypes.byref(e), ctypes.byref(pr))
                print("%s call %d: %.2f ms, distinct %d, fallback entries %d, pairs %d (%.2f %%)"
                      % (name, it, dt * 1e3, keys.numel(), e.value, pr.value, 100.0 * pr.value / max(keys.numel(), 1)),
                      flush=True)
                if it == 2:
                    n = len(lens)
                    per = (ctypes.c_ulonglong * n)()
                    q3 = (ctypes.c_ulonglong * 3)()
                    D.kmc_diag_canon_fallback_detail(per, n, q3)
                    offs = off.cpu().numpy()
                    print("   queued lists: big %d, table(1) %d, table(2) %d" % tuple(q3))
                    print("   fallback share per record: " + " ".join(
                        "%d:%.0f%%" % (r, 100.0 * per[r] / max(int(offs[r + 1] - offs[r]), 1)) for r in range(n)))
                del keys, counts, off
            del data, idx
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
