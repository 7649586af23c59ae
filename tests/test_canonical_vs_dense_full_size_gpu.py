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

The canonical folding itself is tied the same way (round 6): k = 13 is odd, so no
13-mer is its own reverse complement, and the canonical count of key c (c <
rc(c)) is dense[c] + dense[rc(c)] -- every record's canonical (non-forward) lists
must equal that fold of the dense histogram, key for key, and list nothing else.
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


def revcomp_msb(x, k):
    """Key of the reverse complement of 2k-bit MSB-first keys (int64 tensor)."""
    r = (x & 3) ^ 3
    for q in range(1, k):
        r = (r << 2) | (((x >> (2 * q)) & 3) ^ 3)
    return r


def check_against_dense(kmc, data, idx, soft, forward=True):
    """Forward mode: each record's lists == its dense histogram (keys as LE codes).
    Canonical mode (odd k): each record's lists == the reverse-complement fold of it."""
    import torch
    n = idx.numel() - 1
    flags = (kmc.CANON_FORWARD if forward else 0) | (kmc.CANON_SOFTMASK if soft else 0)
    keys, counts, off = kmc.count_canonical(data, idx, K, flags=flags)
    torch.cuda.synchronize()
    dense_in = uppercase_bases(data) if soft else data
    dense, inv = kmc.count_dense(dense_in, idx, K, invalid=True)
    torch.cuda.synchronize()
    del dense_in
    off_h = off.cpu().tolist()
    nb = 1 << (2 * K)
    col = torch.zeros(nb, dtype=torch.int32, device=data.device)
    if not forward:  # per MSB key: its LE bin, its reverse complement, whether it is the canonical one
        allk = torch.arange(nb, dtype=torch.int64, device=data.device)
        le_all = msb_to_le(allk, K)
        rc_all = revcomp_msb(allk, K)
        canon = allk < rc_all
        assert not bool((allk == rc_all).any())  # odd k: no palindromes
        del allk
    total = 0
    for s in range(n):
        a, b = off_h[s], off_h[s + 1]
        kk = keys[a:b]
        assert int((kk < 0).sum()) == 0 and int((kk >= nb).sum()) == 0, "record %d: key >= 4^k" % s
        col.zero_()
        if forward:
            col[msb_to_le(kk, K)] = counts[a:b]  # indexed by LE bin
            exp = dense[:, s]
        else:
            col[kk] = counts[a:b]  # indexed by MSB key
            d = dense[:, s].contiguous()[le_all]  # dense count of every MSB key
            exp = torch.where(canon, d + d[rc_all], torch.zeros_like(d))
            del d
        # a key listed twice would leave one of its two counts in col: the sums differ
        assert int(counts[a:b].to(torch.int64).sum()) == int(col.to(torch.int64).sum()), \
            "record %d: a key listed twice" % s
        assert torch.equal(col, exp), "record %d: canonical lists (forward=%s) != dense histogram" % (s, forward)
        total += b - a
        del kk, exp
    assert total == off_h[-1]
    del keys, counts, off, dense, inv
    if not forward:
        del le_all, rc_all, canon
    torch.cuda.empty_cache()
    return total


@pytest.fixture(scope="module")
def synth():
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import genome_synth
    return genome_synth


@pytest.fixture(scope="module")
def c4(cuda, synth):
    import torch
    data, idx, lens = synth.grch38_like(torch, cuda, GBASES)
    yield data, idx
    del data, idx
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c4r(cuda, synth):
    import torch
    data, idx, lens, _ = synth.repeat_genome(torch, cuda, GBASES)
    yield data, idx
    del data, idx
    torch.cuda.empty_cache()


@pytest.mark.parametrize("soft,forward", [(False, True), (True, True), (True, False)])
def test_c4_k13_equals_dense(kmc, c4, soft, forward):
    distinct = check_against_dense(kmc, *c4, soft, forward)
    assert distinct > 25 * 10_000_000  # each record's ~124 Mbase fill most of its 67 M bins


@pytest.mark.parametrize("forward", [True, False])
def test_c4r_k13_equals_dense(kmc, c4r, forward):
    check_against_dense(kmc, *c4r, True, forward)
