"""Config C4 (BASELINE configs[3]) at the size it is quoted on, key by key.

kmc_count_canonical_hash(k = 31, KMC_CANON_SOFTMASK) over the two 3.1 Gbase
GRCh38 stand-ins of scripts/genome_synth.py -- C4 (iid bases, 5 % N runs, 50 %
soft-masked, 25 chromosome-sized records) and C4R (repeat-rich: interspersed and
tandem repeats, reverse-complemented copies, 2.3 G distinct keys, the hottest seen
~160 K times) -- and the WHOLE output of that one call is checked:

  (a) per record, sum of counts == the valid windows, counted independently on the
      device (torch: a 0/1 lookup of the bytes and a windowed cumulative sum);
  (b) every key is canonical: key <= its reverse complement's key and < 4^k (torch
      ops over every key, not sampled);
  (c) no key repeats within a record: each record's keys sorted on the GPU
      (torch.sort), adjacent keys differ -- a key split into two entries is caught;
  (d) per record, sum of dg_hash(key) * count mod 2^64 equals the oracle's sum of
      dg_hash(canonical key) over every valid window of the record
      (oracle_canonical_digest, a rolling restatement of the definition on the host,
      pinned to the sort-based self-oracle by tests/test_oracle.py) -- a missing,
      substituted or miscounted key changes it;
  (e) the (key, count) pairs whose dg_hash has top 12 bits == SEL (1 key in 4 096:
      ~720 K keys spread over every list of every record, the chromosome-sized
      lists of the big K4s instance included) equal the oracle's, pair for pair.
dg_hash is splitmix64's finaliser, unrelated to the GPU's partition and list hashes.
Canonical counting has no reference counterpart (parity unpinned
by design); the oracle is the definition (kmc.h), semantics per
/root/reference/main.cu:636-646 generalised to k = 31.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = 31
GBASES = 3.1
SEL = 0x9A5


def _s64(c):
    return c - (1 << 64) if c >= 1 << 63 else c


def dg_hash_t(x):
    """oracle_dg_hash on an int64 tensor (wrapping multiplies, logical shifts)."""
    x = x ^ ((x >> 30) & ((1 << 34) - 1))
    x = x * _s64(0xBF58476D1CE4E5B9)
    x = x ^ ((x >> 27) & ((1 << 37) - 1))
    x = x * _s64(0x94D049BB133111EB)
    return x ^ ((x >> 31) & ((1 << 33) - 1))


def revcomp_t(x, k):
    """Key of the reverse complement of 2k-bit MSB-first keys (int64 tensor)."""
    v = x ^ ((1 << (2 * k)) - 1)
    for sh, m in ((2, 0x3333333333333333), (4, 0x0F0F0F0F0F0F0F0F), (8, 0x00FF00FF00FF00FF),
                  (16, 0x0000FFFF0000FFFF)):
        v = ((v >> sh) & m) | ((v & m) << sh)
    v = ((v >> 32) & 0xFFFFFFFF) | (v << 32)
    s = 64 - 2 * k
    return (v >> s) & ((1 << (64 - s)) - 1)


def valid_windows_t(torch, data, a, e, k, soft, step=1 << 28):
    """Windows of data[a:e] (e = the record's terminator) whose k bytes are all
    bases, counted with plain torch ops."""
    lut = torch.zeros(256, dtype=torch.int32, device=data.device)
    for ch in (b"ACGTacgt" if soft else b"ACGT"):
        lut[ch] = 1
    tot = 0
    nw = e - a - k + 1
    for o in range(0, max(nw, 0), step):
        m = min(step, nw - o)
        v = lut[data[a + o:a + o + m + k - 1].long()]
        cs = torch.cumsum(torch.nn.functional.pad(v, (1, 0)), 0)
        tot += int(((cs[k:] - cs[:-k]) == k).sum())
        del v, cs
    return tot


def check_full_size(torch, kmc, oracle, data, idx, lens, k=K, soft=True):
    keys, counts, off = kmc.count_canonical(data, idx, k, flags=kmc.CANON_SOFTMASK if soft else 0)
    torch.cuda.synchronize()
    exp = oracle.canonical_digest(data.cpu().numpy(), idx.cpu().numpy(), k, soft=soft, sel_val=SEL)
    return check_output(torch, exp, data, idx, len(lens), k, soft, keys, counts, off)


def check_output(torch, exp, data, idx, n, k, soft, keys, counts, off):
    """Checks (a)-(e) of one call's output against the oracle's digest `exp`."""
    off_h = off.cpu().numpy().astype(np.int64)
    idx_h = idx.cpu().numpy()
    M = (1 << 64) - 1
    chunk = 1 << 27
    n_sel = 0
    for s in range(n):
        a, b = int(off_h[s]), int(off_h[s + 1])
        rk, rc = keys[a:b], counts[a:b].to(torch.int64)
        # (a) counts sum to the valid windows (device count), and to the oracle's
        w = valid_windows_t(torch, data, int(idx_h[s]), int(idx_h[s + 1]) - 1, k, soft)
        tot = int(rc.sum())
        assert tot == w == exp[s]["valid"], "record %d: counts %d, device windows %d, oracle %d" % (
            s, tot, w, exp[s]["valid"])
        assert int((rc <= 0).sum()) == 0, "record %d: a count <= 0" % s
        dg = 0
        sk, sc = [], []
        for c0 in range(0, b - a, chunk):
            kk, cc = rk[c0:c0 + chunk], rc[c0:c0 + chunk]
            # (b) canonical and in range
            assert int((kk < 0).sum()) == 0 and int((kk >> (2 * k)).sum()) == 0, "record %d: key >= 4^k" % s
            assert bool((kk <= revcomp_t(kk, k)).all()), "record %d: key above its reverse complement" % s
            # (d) digest; (e) the selected subset
            h = dg_hash_t(kk)
            dg = (dg + int((h * cc).sum())) & M
            sel = ((h >> 52) & 0xFFF) == SEL
            sk.append(kk[sel].cpu().numpy().view(np.uint64))
            sc.append(cc[sel].cpu().numpy().astype(np.uint32))
            del kk, cc, h, sel
        assert dg == exp[s]["digest"], "record %d: sum of dg_hash(key) * count differs from the oracle" % s
        sk, sc = np.concatenate(sk), np.concatenate(sc)
        o = np.argsort(sk, kind="stable")
        np.testing.assert_array_equal(sk[o], exp[s]["keys"], err_msg="record %d: selected keys" % s)
        np.testing.assert_array_equal(sc[o], exp[s]["counts"], err_msg="record %d: selected counts" % s)
        n_sel += sk.size
        # (c) distinct within the record
        if b - a > 1:
            srt = torch.sort(rk)[0]
            assert not bool((srt[1:] == srt[:-1]).any()), "record %d: a key occurs twice" % s
            del srt
        del rk, rc
    return int(off_h[-1]), n_sel


@pytest.fixture(scope="module")
def synth():
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import genome_synth
    return genome_synth


def test_c4_grch38_like_full_size_key_level(kmc, oracle, cuda, synth):
    import torch
    data, idx, lens = synth.grch38_like(torch, cuda, GBASES)
    distinct, n_sel = check_full_size(torch, kmc, oracle, data, idx, lens)
    assert distinct > 2_900_000_000 and n_sel > 500_000  # iid input: nearly every valid window is distinct
    del data, idx
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c4r(cuda, synth):
    import torch
    data, idx, lens, _ = synth.repeat_genome(torch, cuda, GBASES)
    yield data, idx, lens
    del data, idx
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,soft", [(31, True), (21, True), (25, False)])
def test_c4r_repeat_rich_full_size_key_level(kmc, oracle, cuda, c4r, k, soft):
    """C4R at k = 31 (the config), 21, and 25 unmasked (the lowercase repeats are
    then not bases: shorter runs, other lists)."""
    import torch
    distinct, n_sel = check_full_size(torch, kmc, oracle, *c4r, k=k, soft=soft)
    if (k, soft) == (31, True):
        assert 2_000_000_000 < distinct < 2_600_000_000 and n_sel > 400_000


def test_full_size_checks_catch_tampered_output(kmc, oracle, cuda, synth):
    """The checks above are not vacuous: on a 30 Mbase repeat-rich genome the
    untouched output passes them, and each tampering fails them -- a key replaced
    by another canonical key (digest), one count moved to another key (digest), a
    key split into two entries with the same total and digest (duplicate check),
    one count lowered (window sum)."""
    import torch
    data, idx, lens, _ = synth.repeat_genome(torch, cuda, 0.03, seed=5, min_len=20_000)
    n, k = len(lens), 31
    keys, counts, off = kmc.count_canonical(data, idx, k, flags=kmc.CANON_SOFTMASK)
    torch.cuda.synchronize()
    exp = oracle.canonical_digest(data.cpu().numpy(), idx.cpu().numpy(), k, soft=True, sel_val=SEL)
    check_output(torch, exp, data, idx, n, k, True, keys, counts, off)
    a, e = int(off[0]), int(off[1])
    rep = a + int(torch.nonzero(counts[a:e] > 1)[0])  # a key of record 0 seen more than once
    oth = a if rep != a else a + 1

    def substitute():
        kk = keys.clone()
        y = int(kk[oth]) ^ 1
        kk[oth] = min(y, int(revcomp_t(torch.tensor([y], device=kk.device), k)[0]))
        return kk, counts, off

    def move_count():
        cc = counts.clone()
        cc[rep] -= 1
        cc[oth] += 1
        return keys, cc, off

    def split():  # (key, c) -> (key, c - 1), (key, 1): same windows, same digest
        kk = torch.cat([keys[:rep + 1], keys[rep:rep + 1], keys[rep + 1:]])
        cc = torch.cat([counts[:rep + 1], torch.ones_like(counts[:1]), counts[rep + 1:]])
        cc[rep] -= 1
        oo = off.clone()
        oo[1:] += 1
        return kk, cc, oo

    def lower():
        cc = counts.clone()
        cc[rep] -= 1
        return keys, cc, off

    for fn in (substitute, move_count, split, lower):
        with pytest.raises(AssertionError):
            check_output(torch, exp, data, idx, n, k, True, *fn())
    del data, idx, keys, counts, off
    torch.cuda.empty_cache()
