#!/usr/bin/env python3
"""Workload for calibrating rocprofv3 HBM byte counters on gfx950: a torch copy of
exactly 1 GiB (1 GiB read + 1 GiB written), the synthetic generator (writes the
10 GB input) and two k=8 histogram launches over it (reads 10 GB)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-kmeres-parallel_amd"))
import torch  # noqa: E402

import kmc  # noqa: E402

dev = torch.device("cuda:0")
src = torch.ones(1 << 30, dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
dst.copy_(src)
torch.cuda.synchronize()
del src, dst
n, L = 10, 1_000_000_000
data = torch.empty(n * (L + 1), dtype=torch.uint8, device=dev)
kmc.synth_fill(data, n, L, 0x5EED0008)
idx = torch.from_numpy(kmc.synth_indices(n, L)).to(dev)
for _ in range(2):
    kmc.count_dense(data, idx, 8)
torch.cuda.synchronize()
print("ok")
