#!/usr/bin/env python3
"""DIAGNOSTIC: C4 with a -DKMC_CANON_PROF build (KMC_LIB=...): K4 phase split from
per-wave s_memtime cycles summed over the waves of one call."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-kmeres-parallel_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    import kmc
    import cbench
    dev = torch.device("cuda:0")
    data, idx, lens = cbench.grch38_like(torch, dev, float(os.environ.get("GB", "3.1")))
    lib = kmc.lib()
    buf = (ctypes.c_ulonglong * 16)()
    names = ["insert", "barrier1", "writeout", "barrier2", "list_end(prefetch wait)", "list_top"]
    for it in range(2):
        lib.kmc_diag_canon_prof(buf)
        kmc.count_canonical(data, idx, 31, flags=kmc.CANON_SOFTMASK)
        torch.cuda.synchronize()
        lib.kmc_diag_canon_prof(buf)
        v = list(buf)
        tot = sum(v[:6])
        waves = 256 * 16
        print("iter %d: passes/wave %d lists/wave %d | per wave %.1f Mcycles: %s" % (
            it, v[6] // waves, v[7] // waves, tot / waves / 1e6,
            ", ".join("%s %.1f%%" % (n, 100.0 * v[i] / max(tot, 1)) for i, n in enumerate(names))))
        print("   insert split: staging %.1f%%, probe loop %.1f%% (queue-read waits %.1f%%, CAS waits %.1f%%) of wave time" % (
            100.0 * v[12] / max(tot, 1), 100.0 * v[13] / max(tot, 1), 100.0 * v[14] / max(tot, 1), 100.0 * v[11] / max(tot, 1)))
        print("   probe loops %d, rounds/loop %.2f, staged keys/loop %.1f, CAS wait %.0f cycles/round (%.1f%% of wave time)" % (v[10], v[8] / max(v[10], 1), v[9] / max(v[10], 1), v[11] / max(v[8], 1), 100.0 * v[11] / max(tot, 1)))


if __name__ == "__main__":
    main()
