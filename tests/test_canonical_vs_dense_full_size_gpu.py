"""The canonical machinery at config scale, tied to the reference-pinned dense path.

kmc_count_canonical_hash has no reference counterpart, but in
KMC_CANON_FORWARD mode at k <= 13 its per-record (key, count) lists ARE the dense
histogram: key = the window's MSB-first 2-bit code, the dense bin = the same code
with its base digits reversed (LE, the bin order of permutation(), utils.h:35-47).
The dense path (kmc_count_dense, k = 13: the radix pipeline) is pinned to the
reference's permutationsCountAll (main.cu:636-646) by tests/test_oracle.py and the
golden fixtures, and run at this size by tests/test_baseline_configs_gpu.py.

Here the canonical pipeline runs at the size it ships at -- the full 3.1 Gbase C4
stand-in (25 chromosome-sized records, 5 % N runs, 50 % soft-masked) and the
repeat-rich C4R stand-in (scripts/genome_synth.py) -- with k = 13 forward, and
every record's lists, converted to dense LE codes on the GPU, must equal the dense
count of the same buffer bin for bin: K1, K3a, K3b, both K4s instances, the table
kernel, direct output and the fallback copy all sit between the two.  With
KMC_CANON_SOFTMASK the canonical call counts lowercase a/c/g/t as bases; the
dense path counts uppercase only, so it runs on the buffer with a/c/g/t
uppercased (the soft-mask rule of kmc.h applied to the bytes).
"""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = 13
GBASES = 3.1


def msb_to_le(keys, k):
    """MSB-first 2-bit keys (int64 tensor) -> LE dense codes: the k base digits reversed."""
    import torch
    le = torch.zeros_like(keys)
    for q in range(k):
        le |= ((keys >> (2 * (k - 1 - q))) & 3) << (2 * q)
    return le


def uppercase_bases(data):
    """a/c/g/t -> A/C/G/T (other bytes unchanged), in chunks on the device."""
    import torch
    out = data.clone()
    lut = torch.arange(256, dtype=torch.uint8, device=data.device)
    for ch in b"acgt":
        lut[ch] = ch - 32
    chunk = 1 << 28
    for o in range(0, out.numel(), chunk):
        out[o:o + chunk] = lut[out[o:o + chunk].long()]
    return out


def check_forward_equals_dense(kmc, data, idx, soft):
    import torch
    n = idx.numel() - 1
    flags = kmc.CANON_FORWARD | (kmc.CANON_SOFTMASK if soft else 0)
    keys, counts, off = kmc.count_canonical(data, idx, K, flags=flags)
    torch.cuda.synchronize()
    dense_in = uppercase_bases(data) if soft else data
    dense, inv = kmc.count_dense(dense_in, idx, K, invalid=True)
    torch.cuda.synchronize()
    del dense_in
    off_h = off.cpu().tolist()
    nb = 1 << (2 * K)
    col = torch.zeros(nb, dtype=torch.int32, device=data.device)
    total = 0
    for s in range(n):
        a, b = off_h[s], off_h[s + 1]
        kk = keys[a:b]
        assert int((kk < 0).sum()) == 0 and int((kk >= nb).sum()) == 0, "record %d: key >= 4^k" % s
        le = msb_to_le(kk, K)
        col.zero_()
        col[le] = counts[a:b]
        # a key listed twice would leave one of its two counts in col: the sums differ
        assert int(counts[a:b].to(torch.int64).sum()) == int(col.to(torch.int64).sum()), \
            "record %d: a key listed twice" % s
        assert torch.equal(col, dense[:, s]), "record %d: forward canonical lists != dense histogram" % s
        total += b - a
        del kk, le
    assert total == off_h[-1]
    del keys, counts, off, dense, inv
    torch.cuda.empty_cache()
    return total


@pytest.fixture(scope="module")
def synth():
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import genome_synth
    return genome_synth


@pytest.mark.parametrize("soft", [False, True])
def test_c4_forward_k13_equals_dense(kmc, cuda, synth, soft):
    import torch
    data, idx, lens = synth.grch38_like(torch, cuda, GBASES)
    distinct = check_forward_equals_dense(kmc, data, idx, soft)
    assert distinct > 25 * 10_000_000  # each record's ~124 Mbase fill most of its 67 M bins
    del data, idx
    torch.cuda.empty_cache()


def test_c4r_forward_k13_equals_dense(kmc, cuda, synth):
    import torch
    data, idx, lens, _ = synth.repeat_genome(torch, cuda, GBASES)
    check_forward_equals_dense(kmc, data, idx, True)
    del data, idx
    torch.cuda.empty_cache()
