"""GPU parity of kmc_count_canonical_hash (k <= 31) against the canonical
self-oracle (oracle_count_canonical: scalar, sort + run-length).

No reference counterpart exists for canonical counting ("parity unpinned",
SURVEY.md §8(c)); the self-oracle is itself pinned to the reference's dense
counts for k <= 13 (tests/test_oracle.py), and the KMC_CANON_FORWARD mode is
checked here against the GPU dense path on the golden fixtures.  Bit-exact
(key, count) sets per record.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def dev(x, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def gpu_canon(kmc, cuda, data, idx, k, flags=0):
    import torch
    d = dev(data if data.size else np.zeros(16, np.uint8), cuda)
    keys, counts, off = kmc.count_canonical(d, dev(idx, cuda), k, flags=flags, capacity=max(data.size, 1))
    torch.cuda.synchronize()
    return keys.cpu().numpy().view(np.uint64), counts.cpu().numpy().view(np.uint32), off.cpu().numpy()


def per_record_sorted(keys, counts, off):
    out = []
    for s in range(off.size - 1):
        a, b = int(off[s]), int(off[s + 1])
        o = np.argsort(keys[a:b], kind="stable")
        out.append((keys[a:b][o], counts[a:b][o]))
    return out


def assert_same(got, exp, msg=""):
    g = per_record_sorted(*got)
    e = per_record_sorted(*exp)
    assert len(g) == len(e), msg
    for s, ((gk, gc), (ek, ec)) in enumerate(zip(g, e)):
        np.testing.assert_array_equal(gk, ek, err_msg="%s record %d keys" % (msg, s))
        np.testing.assert_array_equal(gc, ec, err_msg="%s record %d counts" % (msg, s))


def random_records(rng, lens, alphabet=b"ACGTN", p=(.2475, .2475, .2475, .2475, .01)):
    recs = [np.append(rng.choice(np.frombuffer(alphabet, dtype=np.uint8), size=int(L), p=p), np.uint8(0))
            for L in lens]
    data = np.concatenate(recs) if recs else np.zeros(0, np.uint8)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    return data, idx


@pytest.mark.parametrize("name,dialect", G.cases())
def test_canonical_golden(kmc, oracle, cuda, name, dialect):
    g = G.load(name, dialect)
    idx = G.full_indices(g)
    # (15 / 16: the two key-width instances of the walks, either side of the
    # dword boundary of the 2k-bit key)
    for k in (1, 3, 5, 12, 15, 16, 21, 31):
        for flags in (0, kmc.CANON_SOFTMASK, kmc.CANON_FORWARD):
            got = gpu_canon(kmc, cuda, g["data"], idx, k, flags)
            exp = oracle.count_canonical(g["data"], idx, k, soft=bool(flags & 1), forward=bool(flags & 2))
            assert_same(got, exp, "%s/%s k=%d flags=%d" % (name, dialect, k, flags))


@pytest.mark.parametrize("k", [2, 7, 8, 13])
def test_forward_mode_equals_dense_path(kmc, cuda, k):
    """KMC_CANON_FORWARD keys are the dense bins (MSB-first instead of LE)."""
    import torch
    rng = np.random.default_rng(k)
    data, idx = random_records(rng, [0, 5, 3000, 20011, 1])
    keys, counts, off = gpu_canon(kmc, cuda, data, idx, k, kmc.CANON_FORWARD)
    d = dev(data, cuda)
    dense, _ = kmc.count_dense(d, dev(idx, cuda), k)
    torch.cuda.synchronize()
    dense = dense.cpu().numpy()
    rebuilt = np.zeros_like(dense)
    for s in range(idx.size - 1):
        a, b = int(off[s]), int(off[s + 1])
        kk = keys[a:b].astype(np.uint64)
        le = np.zeros(kk.size, dtype=np.uint64)
        for q in range(k):  # MSB-first -> LE code
            le |= ((kk >> np.uint64(2 * (k - 1 - q))) & np.uint64(3)) << np.uint64(2 * q)
        rebuilt[le.astype(np.int64), s] = counts[a:b]
    np.testing.assert_array_equal(rebuilt, dense)


@pytest.mark.parametrize("k", [11, 15, 16, 25, 31])
def test_canonical_random_vs_oracle(kmc, oracle, cuda, k):
    """Ragged records (empty, shorter than k, tiny, long), N runs, lowercase."""
    rng = np.random.default_rng(100 + k)
    lens = [0, 1, k - 1, k, k + 1, 2, 3, 40, 100_000, 7, 333_333, 0, 16, 17, 31, 32, 33]
    data, idx = random_records(rng, lens, b"ACGTNacgt", (.2, .2, .2, .2, .04, .04, .04, .04, .04))
    for flags in (0, kmc.CANON_SOFTMASK):
        got = gpu_canon(kmc, cuda, data, idx, k, flags)
        exp = oracle.count_canonical(data, idx, k, soft=bool(flags & 1))
        assert_same(got, exp, "k=%d flags=%d" % (k, flags))


def test_canonical_repetitive_and_many_records(kmc, oracle, cuda):
    """Low-complexity sequence (hot keys, long probe chains) and 20 000 short records."""
    rng = np.random.default_rng(9)
    rep = np.frombuffer((b"A" * 5000 + b"AC" * 3000 + b"ACGTTGCA" * 2000 + b"T" * 777), dtype=np.uint8)
    short = [np.append(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=int(L)), np.uint8(0))
             for L in rng.integers(0, 60, size=20_000)]
    recs = [np.append(rep, np.uint8(0))] + short
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    for k in (4, 21, 31):
        assert_same(gpu_canon(kmc, cuda, data, idx, k), oracle.count_canonical(data, idx, k), "k=%d" % k)


@pytest.mark.parametrize("cap", [8, 40])
def test_canonical_pass_overflow_split(kmc, oracle, cuda, cap):
    """K4's pass split: with the per-wave claim capacity lowered (test hook) most
    passes overflow and are redone as two passes, recursively; results unchanged.
    Records from 600 K to 3 M windows (lists of 2-8 K keys), one repetitive."""
    import ctypes
    rng = np.random.default_rng(77 + cap)
    data, idx = random_records(rng, [3_000_000, 600_000, 1_500_001])
    rep = np.frombuffer(b"ACGTTGCA" * 100_000 + b"A" * 200_000, dtype=np.uint8)
    data = np.concatenate([data, rep, np.zeros(1, np.uint8)])
    idx = np.append(idx, data.size)
    with kmc.diag() as D:  # the hooks live in the diagnostic library only
        hook = D.kmc_diag_canon_claim_cap
        sort_cap = D.kmc_diag_canon_sort_cap  # 0: every list to the table kernel
        assert hook(cap) == 0 and sort_cap(0) == 0
        for k in (21, 31):
            assert_same(gpu_canon(kmc, cuda, data, idx, k), oracle.count_canonical(data, idx, k), "cap=%d k=%d" % (cap, k))


@pytest.mark.parametrize("scap,big", [(0, None), (1, 0), (2500, 0), (1, None), (2500, None), (1 << 30, None)])
def test_canonical_sort_and_table_paths(kmc, oracle, cuda, scap, big):
    """Lists split between the three counting kernels by the diagnostic hooks: the
    common K4s instance takes lists of at most `scap` keys (0: none), the big K4s
    instance those up to `big` keys (None: its default 12 288; 0: none) and the
    probed table kernel the rest (and any list with too many crowded slots) -- the
    same counts whatever the split: (0, -) every list in the table kernel; (1 or
    2500, 0) common + table; (1 or 2500, default) common + big (lists of 2 .. 12 288
    keys in the big instance); (default, default) the shipped split.  Records with
    lists of ~2-4 K keys, hot keys (a list deferred from K4s for a crowded slot),
    short records (lists of a few keys)."""
    rng = np.random.default_rng(5 + scap % 97)
    data, idx = random_records(rng, [1_200_000, 9000, 40, 700_001], b"ACGTNacgt",
                               (.2, .2, .2, .2, .04, .04, .04, .04, .04))
    rep = np.frombuffer(b"ACGTTGCAAT" * 3000 + b"G" * 900 + b"ACGATCGATCGGA" * 400, dtype=np.uint8)
    data = np.concatenate([data, rep, np.zeros(1, np.uint8)])
    idx = np.append(idx, data.size)
    with kmc.diag() as D:  # the hooks live in the diagnostic library only
        assert D.kmc_diag_canon_sort_cap(scap) == 0
        if big is not None:
            assert D.kmc_diag_canon_sort_cap_big(big) == 0
        for k in (17, 31):
            for flags in (0, kmc.CANON_SOFTMASK):
                got = gpu_canon(kmc, cuda, data, idx, k, flags)
                exp = oracle.count_canonical(data, idx, k, soft=bool(flags & 1))
                assert_same(got, exp, "scap=%d big=%s k=%d flags=%d" % (scap, big, k, flags))


def test_canonical_crowded_list_deferred(kmc, oracle, cuda):
    """K4s hands a list with more than 128 crowded slots (keys repeated > 16 times)
    to the table kernel: records of one list each (< 4 K windows), made of a 200-bp
    unit repeated 20 times (200 distinct keys x 20 copies), beside records whose
    crowded slots stay within K4s (a 12-bp unit: a dozen keys, hundreds of copies)."""
    rng = np.random.default_rng(31)
    recs = []
    for r in range(6):
        unit = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=200 if r % 2 == 0 else 12)
        reps = 20 if r % 2 == 0 else 300
        recs.append(np.append(np.tile(unit, reps), np.uint8(0)))
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([x.size for x in recs])]).astype(np.int64)
    for k in (21, 31):
        exp = oracle.count_canonical(data, idx, k)
        assert exp[1].max() >= 20
        assert_same(gpu_canon(kmc, cuda, data, idx, k), exp, "k=%d" % k)


def _list_value(key):
    """The list value of kmc_hash.hip (feistel: uint64 arrays, wrapping multiplies):
    K4s's slot and sub are its low 12 and next 4 bits."""
    with np.errstate(over="ignore"):
        return key ^ (((key >> np.uint64(17)) * np.uint64(0x9FB21C651E98DF25)) >> np.uint64(47))


@pytest.mark.parametrize("nd", [9, 64, 65, 100])
def test_canonical_crowded_slot_many_keys(kmc, oracle, cuda, nd):
    """A crowded K4s slot holding many distinct keys: nd distinct 31-mers whose
    list values (feistel of the canonical key) share the low 12 bits (one slot of the common instance's
    4 096), each written 1-5 times between N's, in a record short enough to be one
    list -- the crowded-slot rounds then find nd pivots in a slot of ~3 nd keys
    (over 128 keys: several chunk pairs per pass), and emit their results 64 at a
    time (64 / 65 / 100: one full batch, one more, a partial second), counts >= 4
    through the count side array.  Records of random keys beside it."""
    k = 31
    rng = np.random.default_rng(900 + nd)
    codes = rng.integers(0, 1 << 62, size=1 << 21, dtype=np.uint64)
    rc = np.zeros_like(codes)
    for q in range(k):  # reverse complement of the MSB-first 2-bit code
        rc |= (np.uint64(3) - ((codes >> np.uint64(2 * q)) & np.uint64(3))) << np.uint64(2 * (k - 1 - q))
    canon = np.minimum(codes, rc)
    sel = np.flatnonzero((_list_value(canon) & np.uint64(4095)) == 0)
    _, first = np.unique(canon[sel], return_index=True)
    pick = codes[sel[np.sort(first)][:nd]]
    assert pick.size == nd
    bases = np.frombuffer(b"ACGT", dtype=np.uint8)
    parts = []
    for i, c in enumerate(pick):
        kmer = bases[[(int(c) >> (2 * (k - 1 - q))) & 3 for q in range(k)]]
        for _ in range(i % 5 + 1):
            parts += [kmer, np.frombuffer(b"N", dtype=np.uint8)]
    rec = np.concatenate(parts + [np.zeros(1, np.uint8)])
    data2, idx2 = random_records(rng, [5000, 300_000])
    data = np.concatenate([rec, data2])
    idx = np.concatenate([[0], rec.size + idx2]).astype(np.int64)
    exp = oracle.count_canonical(data, idx, k)
    assert int(exp[2][1] - exp[2][0]) == nd and exp[1][:nd].max() == 5
    assert_same(gpu_canon(kmc, cuda, data, idx, k), exp, "nd=%d" % nd)


def test_canonical_slot_distinctness_test_edges(kmc, oracle, cuda):
    """K4s proves a slot's keys distinct when the high half of its word -- one
    2^sub per key, sub = bits 12-15 of the key's list value -- has as many bits set as the
    slot has keys.  Constructed edges, each group in a slot of its own of one
    list: 16 distinct keys on all 16 subs (the largest slot that passes); 2
    distinct keys on sub 15 (the sum carries out of the word: fails, pairwise
    check); 9 keys on 9 subs, one of them written twice (fails, pairwise: 10 keys,
    the second tier of its reads); 8 keys, two on one sub (fails, pairwise); 3
    keys written 5, 4 and 5 times (14 keys in one slot: pairwise, copies in both
    tiers).  Counts against the oracle."""
    k = 31
    rng = np.random.default_rng(4242)
    codes = rng.integers(0, 1 << 62, size=1 << 22, dtype=np.uint64)
    rc = np.zeros_like(codes)
    for q in range(k):
        rc |= (np.uint64(3) - ((codes >> np.uint64(2 * q)) & np.uint64(3))) << np.uint64(2 * (k - 1 - q))
    canon = np.minimum(codes, rc)
    h = _list_value(canon)
    slot = (h & np.uint64(4095)).astype(np.int64)
    sub = ((h >> np.uint64(12)) & np.uint64(15)).astype(np.int64)

    def keys_of(sl, subs):  # one forward code per requested sub (distinct canonical keys)
        out, seen = [], set()
        for su in subs:
            i = np.flatnonzero((slot == sl) & (sub == su) & ~np.isin(canon, list(seen) or [np.uint64(0)]))
            assert i.size, (sl, su)
            seen.add(canon[i[0]])
            out.append(codes[i[0]])
        return out
    groups = [(keys_of(7, range(16)), [1] * 16),
              (keys_of(8, [15, 15]), [1, 1]),
              (keys_of(9, range(9)), [2] + [1] * 8),
              (keys_of(10, [3, 3, 0, 1, 2, 4, 5, 6]), [1] * 8),
              (keys_of(11, [0, 1, 2]), [5, 4, 5])]
    bases = np.frombuffer(b"ACGT", dtype=np.uint8)
    parts = []
    for ks, reps in groups:
        for c, r in zip(ks, reps):
            kmer = bases[[(int(c) >> (2 * (k - 1 - q))) & 3 for q in range(k)]]
            parts += [kmer, np.frombuffer(b"N", dtype=np.uint8)] * r
    rec = np.concatenate(parts + [np.zeros(1, np.uint8)])
    data2, idx2 = random_records(rng, [2000])
    data = np.concatenate([rec, data2])
    idx = np.concatenate([[0], rec.size + idx2]).astype(np.int64)
    exp = oracle.count_canonical(data, idx, k)
    assert int(exp[2][1]) == 16 + 2 + 9 + 8 + 3
    assert_same(gpu_canon(kmc, cuda, data, idx, k), exp, "slot edges")


def test_canonical_size_independent_properties(kmc, cuda):
    """64 Mbase: counts sum to the valid windows; canonical == forward folded by revcomp."""
    import torch
    L = 64 << 20
    n = 4
    data = torch.empty(n * (L + 1), dtype=torch.uint8, device=cuda)
    kmc.synth_fill(data, n, L, 0x5EED001F)
    idx = dev(kmc.synth_indices(n, L), cuda)
    keys, counts, off = kmc.count_canonical(data, idx, 31)
    torch.cuda.synchronize()
    off = off.cpu().numpy()
    per = [int(counts[int(off[s]):int(off[s + 1])].to(torch.int64).sum()) for s in range(n)]
    assert per == [L - 31 + 1] * n
    # canonical keys are <= their reverse complement's key
    k = 31
    kk = keys.cpu().numpy().view(np.uint64)
    rc = np.zeros_like(kk)
    for q in range(k):
        rc |= (np.uint64(3) - ((kk >> np.uint64(2 * q)) & np.uint64(3))) << np.uint64(2 * (k - 1 - q))
    assert np.all(kk <= rc)


def test_canonical_big_lists_sort_vs_table(kmc, cuda):
    """A chromosome-sized record (240 Mbase: 2^15 lists of ~7.3 K keys, above the
    common K4s instance's 6 080) is counted by the big K4s instance; its (key, count)
    set equals the probed table kernel's (every list forced there through the
    diagnostic library), and its counts sum to the windows.  A 60 Mbase record with
    a 3 Mbase tandem repeat beside it crowds slots of its lists (deferred)."""
    import torch
    L = 240_000_000
    A = (L + 1 + 15) & ~15  # record 2's synthetic bases start 16-aligned (synth_fill), after N padding
    data = torch.empty(A + 60_000_001 + 16, dtype=torch.uint8, device=cuda)
    kmc.synth_fill(data, 1, L, 0x5EED0B16)
    data[L + 1:A] = ord("N")
    kmc.synth_fill(data[A:], 1, 60_000_000, 0x5EED0B17)
    unit = torch.from_numpy(np.frombuffer(b"ACGTTGCATTAGCCAGT" * 3, dtype=np.uint8).copy()).to(cuda)
    rep = unit.repeat(3_000_000 // unit.numel() + 1)[:3_000_000]
    data[A + 1000:A + 1000 + rep.numel()] = rep
    idx = np.array([0, L + 1, A + 60_000_001], dtype=np.int64)
    di = dev(idx, cuda)

    def run(k):
        keys, counts, off = kmc.count_canonical(data, di, k, capacity=L + 60_000_000)
        torch.cuda.synchronize()
        out = []
        for s in range(2):
            a, b = int(off[s]), int(off[s + 1])
            o = torch.argsort(keys[a:b])
            out.append((keys[a:b][o], counts[a:b][o]))
        return out

    for k in (31, 25):
        got = run(k)
        with kmc.diag() as D:
            assert D.kmc_diag_canon_sort_cap(0) == 0
            ref = run(k)
        for s, ((gk, gc), (rk, rc)) in enumerate(zip(got, ref)):
            assert torch.equal(gk, rk) and torch.equal(gc, rc), "k=%d record %d" % (k, s)
        assert int(got[0][1].to(torch.int64).sum()) == L - k + 1
        assert int(got[1][1].to(torch.int64).sum()) == 60_000_000 - k + 1


@pytest.mark.parametrize("k,soft", [(31, True), (21, False), (13, True)])
def test_canonical_direct_output_vs_pk_layout(kmc, oracle, cuda, k, soft):
    """Direct output (round 5: the pairs written by the counting kernels straight
    to their record's region when its start is known, else through pk and the
    fallback copy) against the pk + place layout (kmc_diag_canon_direct(0)) and the
    self-oracle: the same per-record sets and the same record offsets, on a
    repeat-rich genome (lists whose failing slots overflow the LDS staging, crowded
    slots) beside random records, many short ones and empty ones."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import genome_synth
    rng = np.random.default_rng(700 + k)
    g, gi, _, _ = genome_synth.repeat_genome(torch, cuda, 0.02, seed=k, min_len=20_000)
    gh, gih = g.cpu().numpy(), gi.cpu().numpy()
    d2, i2 = random_records(rng, [0, 5, 250_000, 1, 31, 32, 9000] + list(rng.integers(0, 300, size=500)),
                            b"ACGTNacgt", (.2, .2, .2, .2, .04, .04, .04, .04, .04))
    data = np.concatenate([gh, d2])
    idx = np.concatenate([gih, gih[-1] + i2[1:]]).astype(np.int64)
    flags = kmc.CANON_SOFTMASK if soft else 0
    exp = oracle.count_canonical(data, idx, k, soft=soft)
    got = {}
    with kmc.diag() as D:
        for mode in (1, 0):
            assert D.kmc_diag_canon_direct(mode) == 0
            got[mode] = gpu_canon(kmc, cuda, data, idx, k, flags)
            assert_same(got[mode], exp, "direct=%d k=%d soft=%s" % (mode, k, soft))
    np.testing.assert_array_equal(got[0][2], got[1][2])


def test_canonical_capacity_error(kmc, cuda):
    import torch
    rng = np.random.default_rng(1)
    data, idx = random_records(rng, [5000])
    d = dev(data, cuda)
    with pytest.raises(kmc.KmcError) as ei:
        kmc.count_canonical(d, dev(idx, cuda), 21, capacity=10)
    assert ei.value.code == 1009
    with pytest.raises(kmc.KmcError):
        kmc.count_canonical(d, dev(idx, cuda), 32)


@pytest.mark.parametrize("k,soft", [(31, True), (21, True), (31, False), (15, True)])
def test_canonical_repeat_rich_genome(kmc, oracle, cuda, k, soft):
    """The repeat-rich synthetic genome of config C4 (scripts/genome_synth.py: ~45 %
    interspersed repeats with 0-15 % divergence, half reverse-complemented,
    tandem repeats, N runs, soft-masked repeats) at 40 Mbase in 25 records: many
    keys occur thousands of times (the LDS table's repeat path, hot keys within
    a pass) and reverse-complement copies fold onto shared keys."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import genome_synth
    data, idx, _, _ = genome_synth.repeat_genome(torch, cuda, 0.04, seed=77, min_len=20_000)
    host, hidx = data.cpu().numpy(), idx.cpu().numpy()
    flags = kmc.CANON_SOFTMASK if soft else 0
    got = gpu_canon(kmc, cuda, host, hidx, k, flags)
    exp = oracle.count_canonical(host, hidx, k, soft=soft)
    if soft:  # the repeat path is exercised (unmasked: the lowercase repeats are not bases)
        assert exp[1].max() > 1000 and (exp[1] > 1).sum() > 100_000
    assert_same(got, exp, "repeat-rich k=%d soft=%s" % (k, soft))


@pytest.mark.parametrize("k", [11, 31])
def test_canonical_unaligned_data_and_caller_workspace(kmc, oracle, cuda, k):
    """The canonical entry point takes any data pointer (rounded down to 16 bytes,
    offsets biased, as the dense path does): data + 1, 7, 8, 15 of a buffer give the
    self-oracle's counts; kmc_count_canonical_hash_ex with a caller workspace of the
    queried size gives the same, and half that workspace is refused."""
    import torch
    rng = np.random.default_rng(900 + k)
    data, idx = random_records(rng, [0, 5, 40_000, 1, 333_333, 64], b"ACGTNacgt",
                               (.2, .2, .2, .2, .04, .04, .04, .04, .04))
    exp = oracle.count_canonical(data, idx, k, soft=True)
    di = dev(idx, cuda)
    for off in (1, 7, 8, 15):
        big = torch.zeros(data.size + 48, dtype=torch.uint8, device=cuda)
        big[off:off + data.size] = dev(data, cuda)
        d = big[off:off + data.size]
        keys, counts, ro = kmc.count_canonical(d, di, k, flags=kmc.CANON_SOFTMASK, capacity=data.size)
        torch.cuda.synchronize()
        got = (keys.cpu().numpy().view(np.uint64), counts.cpu().numpy().view(np.uint32), ro.cpu().numpy())
        assert_same(got, exp, "offset %d" % off)
        wsb = kmc.canonical_workspace_size(idx, k, torch.cuda.current_device())
        assert wsb > 0
        ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
        keys, counts, ro = kmc.count_canonical(d, di, k, flags=kmc.CANON_SOFTMASK, capacity=data.size,
                                               workspace=ws)
        torch.cuda.synchronize()
        got = (keys.cpu().numpy().view(np.uint64), counts.cpu().numpy().view(np.uint32), ro.cpu().numpy())
        assert_same(got, exp, "caller workspace, offset %d" % off)
    # ~20 B per window plus per-list tables (the size holds for every alignment)
    assert 16 * 373_367 < wsb < 32 * 373_367 + (1 << 20), wsb
    refused = []
    for frac in (2, 4, 8, 64):
        try:
            kmc.count_canonical(d, di, k, flags=kmc.CANON_SOFTMASK, capacity=data.size, workspace=ws[:wsb // frac])
            torch.cuda.synchronize()
        except kmc.KmcError as e:
            assert e.code == 1004
            refused.append(frac)
    assert refused and refused[-1] == 64, (wsb, refused)


@pytest.mark.parametrize("k", [31, 17])
def test_canonical_offsets_beyond_2gib(kmc, oracle, cuda, k):
    """Records that lie past byte 2^31 of the buffer (the C4 genome is 3.1 GB): the
    input walks address their chunks through 64-bit wave bases (a sign-extended
    32-bit half once dropped every window there), counts equal the self-oracle's."""
    import torch
    rng = np.random.default_rng(2031 + k)
    data, idx = random_records(rng, [3_000_000, 1, 1_000_001], b"ACGTNacgt",
                               (.2, .2, .2, .2, .04, .04, .04, .04, .04))
    base = (1 << 31) + 4096 + 7
    buf = torch.empty(base + data.size + 64, dtype=torch.uint8, device=cuda)
    buf[base:base + data.size] = dev(data, cuda)
    gidx = dev(idx + base, cuda)
    keys, counts, off = kmc.count_canonical(buf, gidx, k, flags=kmc.CANON_SOFTMASK, capacity=data.size)
    torch.cuda.synchronize()
    got = (keys.cpu().numpy().view(np.uint64), counts.cpu().numpy().view(np.uint32), off.cpu().numpy())
    assert_same(got, oracle.count_canonical(data, idx, k, soft=True), "k=%d" % k)
    del buf
    torch.cuda.empty_cache()
