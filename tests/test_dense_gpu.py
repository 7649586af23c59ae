"""GPU parity of the HIP dense counter against the oracle and the reference kernel.

Bit-exact integer comparisons throughout.  Run on the MI355X box (`-m gpu`).
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def dev(x, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def random_records(rng, lens, n_frac=0.0, lower_frac=0.0, other_frac=0.0):
    recs = []
    for L in lens:
        s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=int(L))
        if n_frac:
            s[rng.random(s.size) < n_frac] = ord("N")
        if lower_frac:
            m = rng.random(s.size) < lower_frac
            s[m] |= 0x20
        if other_frac:
            m = rng.random(s.size) < other_frac
            s[m] = rng.integers(0, 256, size=int(m.sum()), dtype=np.uint8)
        recs.append(np.append(s, np.uint8(0)))
    data = np.concatenate(recs) if recs else np.zeros(0, np.uint8)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    return data, idx


def run_dense(kmc, cuda, data, idx, k, **kw):
    import torch
    d = dev(data if data.size else np.zeros(16, np.uint8), cuda)
    out, inv = kmc.count_dense(d, dev(idx, cuda), k, data_bytes=data.size, invalid=True, **kw)
    torch.cuda.synchronize()
    return out.cpu().numpy(), inv.cpu().numpy()


def test_synth_kernel_matches_host(kmc, cuda):
    import torch
    for nrec, L, first in ((3, 1000, 0), (5, 4093, 17), (1, 65, 1 << 33)):
        total = nrec * (L + 1)
        buf = torch.zeros(total + 64, dtype=torch.uint8, device=cuda)
        kmc.synth_fill(buf, nrec, L, 0x5EED0008, first)
        torch.cuda.synchronize()
        got = buf[:total].cpu().numpy()
        np.testing.assert_array_equal(got, kmc.synth_host(nrec, L, 0x5EED0008, first))
        assert int(buf[total:].sum()) == 0  # nothing written past the end


@pytest.mark.parametrize("name,dialect", G.cases())
def test_dense_matches_golden(kmc, cuda, name, dialect):
    g = G.load(name, dialect)
    idx = G.full_indices(g)
    for k in g["ks"]:
        k = int(k)
        got, inv = run_dense(kmc, cuda, g["data"], idx, k)
        exp, exp_inv = G.dense_expected(g, k)
        np.testing.assert_array_equal(got, exp, err_msg="%s/%s k=%d" % (name, dialect, k))
        np.testing.assert_array_equal(inv, exp_inv, err_msg="%s/%s k=%d invalid" % (name, dialect, k))


@pytest.mark.parametrize("name", ["basic", "random", "maxseqs", "crlf", "odd"])
def test_dropin_matches_golden(kmc, cuda, name):
    import torch
    g = G.load(name, "blank")
    idx = G.full_indices(g).astype(np.int32)
    n = idx.size - 1
    d = dev(g["data"], cuda)
    out = kmc.dropin_count(d, dev(idx, cuda), n)
    torch.cuda.synchronize()
    exp, _ = G.dense_expected(g, 3)
    np.testing.assert_array_equal(out.cpu().numpy().reshape(64, n), exp)


def test_dropin_matches_reference_kernel(kmc, oracle, cuda):
    """The reference's own sumKmereCoincidencesGlobalMemory (kernels.h, compiled for
    gfx950 from /root/reference into oracle/_ref) vs the drop-in, same buffers."""
    import torch
    if not oracle.have_ref_kernel():
        pytest.skip("oracle/_ref/libref_kernel.so not built")
    L = oracle.ref_kernel()
    assert L.ref_kernel_k() == 3
    assert L.ref_kernel_upload_patterns() == 0
    rng = np.random.default_rng(3)
    for lens in ([5000, 1, 2, 3, 4, 777, 10000], list(rng.integers(0, 3000, size=101))):
        data, idx = random_records(rng, lens, 0.01, 0.01, 0.002)
        idx32 = idx.astype(np.int32)
        n = idx.size - 1
        d = dev(data, cuda)
        di = dev(idx32, cuda)
        ref = torch.zeros(64 * n, dtype=torch.int32, device=cuda)
        assert L.ref_kernel_launch(d.data_ptr(), di.data_ptr(), n, ref.data_ptr()) == 0
        ours = kmc.dropin_count(d, di, n)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(ours.cpu().numpy(), ref.cpu().numpy())


def test_dropin_unaligned_data_matches_reference_kernel(kmc, oracle, cuda):
    """kernels.h:113 takes any char *data: the drop-in on data + 1 .. 15 (a pointer
    inside a buffer) against the reference kernel on the same pointer."""
    import torch
    if not oracle.have_ref_kernel():
        pytest.skip("oracle/_ref/libref_kernel.so not built")
    L = oracle.ref_kernel()
    assert L.ref_kernel_upload_patterns() == 0
    rng = np.random.default_rng(33)
    data, idx = random_records(rng, [3000, 1, 5, 17, 1500, 4099], 0.01, 0.01, 0.002)
    idx32 = idx.astype(np.int32)
    n = idx.size - 1
    di = dev(idx32, cuda)
    for off in range(16):
        big = torch.full((data.size + 48,), ord("A"), dtype=torch.uint8, device=cuda)
        big[off:off + data.size] = dev(data, cuda)
        d = big[off:]
        assert d.data_ptr() % 16 == off % 16 or big.data_ptr() % 16 != 0
        ref = torch.zeros(64 * n, dtype=torch.int32, device=cuda)
        assert L.ref_kernel_launch(d.data_ptr(), di.data_ptr(), n, ref.data_ptr()) == 0
        ours = kmc.dropin_count(d, di, n)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(ours.cpu().numpy(), ref.cpu().numpy(), err_msg="offset %d" % off)


@pytest.mark.parametrize("k", [3, 8, 11])
def test_dense_unaligned_data_vs_oracle(kmc, oracle, cuda, k):
    """kmc_count_dense / kmc_count_dense_ex with a data pointer at every offset mod 16
    (the library aligns it down and biases the offsets), including a byte-range
    shard of the offset buffer."""
    import torch
    rng = np.random.default_rng(5000 + k)
    data, idx = random_records(rng, [0, 5, 4096 * 2 + 3, 1, 70_001, 333], 0.003, 0.003, 0.001)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    di = dev(idx, cuda)
    for off in (1, 7, 8, 15):
        big = torch.zeros(data.size + 48, dtype=torch.uint8, device=cuda)
        big[off:off + data.size] = dev(data, cuda)
        d = big[off:off + data.size]
        out, inv = kmc.count_dense(d, di, k, data_bytes=data.size, invalid=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), exp, err_msg="offset %d" % off)
        np.testing.assert_array_equal(inv.cpu().numpy(), exp_inv, err_msg="offset %d" % off)
        # two shards of the offset buffer sum to the whole
        acc = np.zeros_like(exp)
        for (a, b, rl, rh) in kmc.plan_shards(idx, k, 2, 4096):
            o = torch.empty((1 << (2 * k), idx.size - 1), dtype=torch.int32, device=cuda)
            kmc.count_dense_ex(kmc.dense_args(d, di, k, o.view(-1), read=(rl, rh), win=(a, b)))
            torch.cuda.synchronize()
            acc += o.cpu().numpy()
        np.testing.assert_array_equal(acc, exp, err_msg="shards, offset %d" % off)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8])
def test_dense_random_vs_oracle(kmc, oracle, cuda, k):
    rng = np.random.default_rng(1000 + k)
    # short, tile-straddling and multi-workgroup records; invalid bytes of every kind
    lens = [0, 1, k - 1, k, k + 1, 15, 16, 17, 1023, 1024, 1025, 70000, 3, 250000, 4096 * 3 + 5]
    data, idx = random_records(rng, lens, 0.003, 0.003, 0.001)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


@pytest.mark.parametrize("k", [7, 8])
def test_dense_chunk_boundaries_vs_oracle(kmc, oracle, cuda, k):
    """k >= 7 hands a piece's tiles to the waves in 16-tile chunks (16 KiB) from a
    workgroup counter; the halo of a chunk's last tile is loaded apart.  ~48 MB, so
    every workgroup's range holds many chunks: records ending on and around chunk
    edges (16 KiB multiples -8 .. +7), pieces shorter than one chunk, invalid bytes
    on both sides of chunk edges, and window ranges (shards) cutting chunks."""
    import torch
    rng = np.random.default_rng(7070 + k)
    lens = [16384 * m + d for m in (1, 2, 5, 33) for d in (-8, -1, 0, 1, 7)]
    lens += [5, 16383, 3 * 16384 + 1023, 6_000_000, 10_000_001, 4096 * 37 + 11]
    lens += list(rng.integers(1, 200_000, size=40)) + [12_000_000, 16_000_000]
    rng.shuffle(lens)
    data, idx = random_records(rng, lens, 0.0005, 0.0005, 0.0)
    # invalid bytes right at chunk edges of the buffer (and one past, one before)
    edges = np.arange(16384, data.size - 16, 16384 * 7)
    for off in (-1, 0, 1):
        data[edges + off] = np.uint8(ord("N"))
    data[idx[1:] - 1] = 0  # (record terminators stay)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)
    d, di = dev(data, cuda), dev(idx, cuda)
    out = torch.empty((1 << (2 * k), idx.size - 1), dtype=torch.int32, device=cuda)
    for lo, hi in ((16384 * 3 - 5, 16384 * 900 + 3), (1, data.size // 2 + 16384 - 1), (data.size // 3, data.size)):
        kmc.count_dense_ex(kmc.dense_args(d, di, k, out.view(-1), read=(lo, min(hi + k - 1, data.size)), win=(lo, hi)))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), oracle.count_dense(data, idx, k, win=(lo, hi))[0],
                                      err_msg="window range [%d, %d)" % (lo, hi))


@pytest.mark.parametrize("k", [9, 10, 11, 12, 13])
def test_radix_k9_13_vs_oracle(kmc, oracle, cuda, k):
    """9 <= k <= 13: the radix-partitioned path (67 M bins per record at k = 13)."""
    rng = np.random.default_rng(2000 + k)
    lens = [0, 1, k - 1, k, k + 1, 1025, 300_000, 17, 2_000_003]
    data, idx = random_records(rng, lens, 0.003, 0.003, 0.001)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


@pytest.mark.parametrize("k", [9, 10, 11, 12, 13])
def test_radix_wrapping_bins_recounted(kmc, oracle, cuda, k):
    """k >= 12 keeps two 16-bit bins per LDS word in R4: a k-mer seen >= 65 536
    times in one list (poly-A / poly-AC runs) wraps its bin and the list is
    recounted exactly; lists without a wrap keep the packed result (k <= 11: the
    32-bit bins, same input).  The same runs overflow R3's rings every round (one
    bucket takes a whole round's windows): its cold path, the partly-written first
    segment after an overflow and several segments per phase-B thread, at every
    ring geometry (k = 9..13)."""
    rng = np.random.default_rng(4100 + k)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    poly = np.full(300_000, ord("A"), np.uint8)
    di = np.frombuffer(b"AC" * 70_000, np.uint8)
    mixed = np.concatenate([acgt[rng.integers(0, 4, 500_000)], poly, acgt[rng.integers(0, 4, 200_000)], di])
    recs = [np.append(mixed, np.uint8(0)), np.append(acgt[rng.integers(0, 4, 1_000_000)], np.uint8(0)),
            np.append(poly[:70_000], np.uint8(0))]
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    assert exp[0, 0] > 65_536  # AAAA...A in record 0
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


@pytest.fixture
def radix_mode(kmc):
    """kmc_diag_radix_mode(mode, cap_scale): 0 auto, 1 exact offsets, 2 sampled
    regions; cap_scale < 1 shrinks the sampled capacities so regions overflow and
    the gated exact rerun takes over.  The hook exists only in the diagnostic
    library (lib/libkmc_diag.so), which every binding uses inside kmc.diag();
    restored to auto afterwards."""
    with kmc.diag() as D:
        yield D.kmc_diag_radix_mode
        assert D.kmc_diag_radix_mode(0, 1.0) == 0


@pytest.mark.parametrize("k", [9, 10, 11, 12, 13])
@pytest.mark.parametrize("scale", [1.0, 0.97, 0.25])
def test_radix_sampled_regions_vs_oracle(kmc, oracle, cuda, radix_mode, k, scale):
    """The sampled partition (C3's path): R1 replaced by a 1-in-16 tile sample that
    sizes a region per (record, bucket, workgroup), R3 writing into the regions and
    R4 walking them.  scale 1: regions fit; 0.97: a few overflow, 0.25: most do --
    either way the device-side exact rerun must give the oracle's counts.  Random
    records (short ones, tile edges, multi-MB) and the skewed poly-A / poly-AC mix
    (ring overflows, R4 bin wraps)."""
    assert radix_mode(2, scale) == 0
    rng = np.random.default_rng(7000 + k)
    data, idx = random_records(rng, [0, 1, k, 1025, 300_000, 17, 2_000_003, 4_500_000], 0.003, 0.003, 0.001)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    mixed = np.concatenate([acgt[rng.integers(0, 4, 500_000)], np.full(300_000, ord("A"), np.uint8),
                            acgt[rng.integers(0, 4, 200_000)], np.frombuffer(b"AC" * 70_000, np.uint8)])
    recs = [np.append(mixed, np.uint8(0)), np.append(acgt[rng.integers(0, 4, 3_000_000)], np.uint8(0))]
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


@pytest.mark.parametrize("k", [10, 13])
def test_radix_sampled_long_list(kmc, oracle, cuda, radix_mode, k):
    """Sampled partition with one very long list: a bucket taking a 5 Mbase poly-A
    run (one region per workgroup holding it, its bins wrapping: R4's exact
    recount of the regions), beside random records."""
    assert radix_mode(2, 1.0) == 0
    rng = np.random.default_rng(8100 + k)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    recs = [np.concatenate([acgt[rng.integers(0, 4, 700_000)], np.full(5_000_000, ord("A"), np.uint8),
                            acgt[rng.integers(0, 4, 300_001)], [0]]).astype(np.uint8),
            np.append(acgt[rng.integers(0, 4, 2_000_000)], np.uint8(0))]
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


@pytest.mark.parametrize("scale", [1.0, 0.5])
def test_radix_sampled_shards_and_workspace(kmc, oracle, cuda, radix_mode, scale):
    """Sampled partition over byte-range shards (window range + halo) with a caller
    workspace sized by kmc_count_dense_ex_workspace_size: the shards sum to the
    whole histogram; and the whole buffer through an unaligned data pointer."""
    import torch
    assert radix_mode(2, scale) == 0
    k = 13
    rng = np.random.default_rng(91)
    data, idx = random_records(rng, [2_600_000, 5, 1_400_001], 0.002, 0.002)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    d, di = dev(data, cuda), dev(idx, cuda)
    acc = np.zeros_like(exp)
    inv_acc = np.zeros_like(exp_inv)
    for a, b, rl, rh in kmc.plan_shards(idx, k, 3):
        out = torch.full((1 << (2 * k), idx.size - 1), -1, dtype=torch.int32, device=cuda)
        inv = torch.full((idx.size - 1,), -1, dtype=torch.int32, device=cuda)
        args = kmc.dense_args(d, di, k, out, read=(rl, rh), win=(a, b), invalid=inv)
        ws = torch.empty(kmc.dense_ex_workspace_size(args), dtype=torch.uint8, device=cuda)
        kmc.count_dense_ex(kmc.dense_args(d, di, k, out, read=(rl, rh), win=(a, b), invalid=inv, workspace=ws))
        torch.cuda.synchronize()
        acc += out.cpu().numpy()
        inv_acc += inv.cpu().numpy()
        del out, ws
    np.testing.assert_array_equal(acc, exp)
    np.testing.assert_array_equal(inv_acc, exp_inv)
    # the whole buffer from a data pointer 7 bytes past an aligned one
    big = torch.zeros(data.size + 48, dtype=torch.uint8, device=cuda)
    big[7:7 + data.size] = d
    out, inv = kmc.count_dense(big[7:7 + data.size], di, k, data_bytes=data.size, invalid=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    np.testing.assert_array_equal(inv.cpu().numpy(), exp_inv)


@pytest.mark.parametrize("k", [11, 13])
def test_radix_shards_sum_to_full(kmc, oracle, cuda, k):
    import torch
    rng = np.random.default_rng(31 + k)
    data, idx = random_records(rng, [600_000, 5, 400_001], 0.002, 0.002)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    d, di = dev(data, cuda), dev(idx, cuda)
    acc = np.zeros_like(exp)
    inv_acc = np.zeros_like(exp_inv)
    for a, b, rl, rh in kmc.plan_shards(idx, k, 3):
        out = torch.full((1 << (2 * k), idx.size - 1), -1, dtype=torch.int32, device=cuda)
        inv = torch.full((idx.size - 1,), -1, dtype=torch.int32, device=cuda)
        kmc.count_dense_ex(kmc.dense_args(d, di, k, out, read=(rl, rh), win=(a, b), invalid=inv))
        torch.cuda.synchronize()
        acc += out.cpu().numpy()
        inv_acc += inv.cpu().numpy()
        del out
    np.testing.assert_array_equal(acc, exp)
    np.testing.assert_array_equal(inv_acc, exp_inv)


@pytest.mark.parametrize("k", [3, 8])
def test_dense_long_records_span_workgroups(kmc, oracle, cuda, k):
    """Records of several MB: every record is cut over many workgroups (slab reduce)."""
    rng = np.random.default_rng(77)
    data, idx = random_records(rng, [3_000_001, 2_500_000, 17, 4_000_003], 0.0005, 0.0005)
    got, inv = run_dense(kmc, cuda, data, idx, k)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


def test_k8_packed_counter_wraps(kmc, oracle, cuda):
    """k = 8 keeps two 16-bit counters per LDS word: low-entropy input drives
    both halves of the same words through many wraps concurrently."""
    rng = np.random.default_rng(8)
    n = 48 * 1024 * 1024
    # 97 % A, 3 % G: bins 0 (AAAAAAAA, low half of word 0) and 0x8000 (AAAAAAAG, high
    # half of word 0) and the other single-G bins each get millions of counts
    s = np.where(rng.random(n) < 0.97, ord("A"), ord("G")).astype(np.uint8)
    s[: 4 * 1024 * 1024] = ord("A")               # one long run: > 65 536 adds per workgroup
    s[-3 * 1024 * 1024:] = np.frombuffer(b"AAAAAAAG", np.uint8)[np.arange(3 * 1024 * 1024) % 8]
    data = np.append(s, np.uint8(0))
    idx = np.array([0, data.size], dtype=np.int64)
    got, inv = run_dense(kmc, cuda, data, idx, 8)
    exp, exp_inv = oracle.count_dense(data, idx, 8)
    assert exp[0, 0] > 1 << 21 and exp[0x8000, 0] > 1 << 17
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


def test_k8_overflow_fallback_mixed(kmc, oracle, cuda):
    """Some workgroup pieces overflow their 16-bit counters (poly-A records, whole
    or cut across workgroups), others do not: only those are recounted exactly."""
    rng = np.random.default_rng(88)
    lens, seqs = [], []
    for i in range(60):
        if i % 3 == 0:
            seqs.append(np.full(70_000 + 37 * i, ord("A"), np.uint8))        # whole-record overflow
        elif i % 3 == 1:
            seqs.append(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=200_000 + i))
        else:
            s = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=300_000)
            s[50_000:250_000] = np.frombuffer(b"CCCCCCCT", np.uint8)[np.arange(200_000) % 8]
            seqs.append(s)
    recs = [np.append(s_, np.uint8(0)) for s_ in seqs]
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    got, inv = run_dense(kmc, cuda, data, idx, 8)
    exp, exp_inv = oracle.count_dense(data, idx, 8)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


def test_k8_hot_half_scans_with_fallback(kmc, oracle, cuda):
    """k = 8, 400 MB: "hot" records (65 % A: AAAAAAAA is 3 % of the windows, > 65 536
    per workgroup piece) are kept exact by the periodic hot-half scans (spill
    entries, no wrap), while "burst" records (a multi-MB poly-A run, > 32 768 adds
    between two scans) wrap and are recounted; workgroups holding both kinds of
    piece keep the scans' spills of the first and drop those of the second."""
    rng = np.random.default_rng(808)
    acgt = np.frombuffer(b"ACGT", np.uint8)

    def hot(n):
        return np.where(rng.random(n) < 0.65, ord("A"), acgt[rng.integers(1, 4, n)]).astype(np.uint8)

    def burst(n, run):
        x = hot(n)
        o = (n - run) // 2
        x[o:o + run] = ord("A")
        return x

    seqs = [hot(100 << 20), burst(5 << 20, 3 << 20), hot(60 << 20), acgt[rng.integers(0, 4, 20 << 20)],
            burst(3 << 20, 1 << 20), hot(150 << 20), burst(7 << 20, 5 << 20), hot(40 << 20)]
    recs = [np.append(x, np.uint8(0)) for x in seqs]
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    got, inv = run_dense(kmc, cuda, data, idx, 8)
    exp, exp_inv = oracle.count_dense(data, idx, 8)
    assert exp[0].max() > 1 << 22
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)


@pytest.mark.parametrize("k", [4, 8])
def test_range_shards_sum_to_full(kmc, oracle, cuda, k):
    """kmc_count_dense_ex over disjoint window ranges, each reading only its
    shard + (k-1)-byte halo, sums to the unsharded histogram."""
    import torch
    rng = np.random.default_rng(5)
    data, idx = random_records(rng, [100_000, 7, 300_000, 123_457], 0.001, 0.001)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    d = dev(data, cuda)
    di = dev(idx, cuda)
    cuts = [0, 4096, 4097, 150_003, 150_016, 400_000, data.size]
    acc = np.zeros_like(exp)
    inv_acc = np.zeros_like(exp_inv)
    for a, b in zip(cuts[:-1], cuts[1:]):
        out = torch.full((1 << (2 * k), idx.size - 1), -7, dtype=torch.int32, device=cuda)
        inv = torch.full((idx.size - 1,), -7, dtype=torch.int32, device=cuda)
        args = kmc.dense_args(d, di, k, out, read=(a, min(b + k - 1, data.size)), win=(a, b), invalid=inv)
        kmc.count_dense_ex(args)
        torch.cuda.synchronize()
        part, pinv = out.cpu().numpy(), inv.cpu().numpy()
        ref_part, ref_pinv = oracle.count_dense(data, idx, k, win=(a, b))
        np.testing.assert_array_equal(part, ref_part)
        np.testing.assert_array_equal(pinv, ref_pinv)
        acc += part
        inv_acc += pinv
    np.testing.assert_array_equal(acc, exp)
    np.testing.assert_array_equal(inv_acc, exp_inv)


@pytest.mark.parametrize("k", [3, 8])
def test_dense_reserved_cus_vs_oracle(kmc, oracle, cuda, k):
    """kmc_set_reserved_cus (bench.py at N > 1 leaves CUs to the overlapped
    all-reduce): fewer workgroups, each with a longer home range -- same counts,
    and a caller workspace sized after the setting."""
    import torch
    rng = np.random.default_rng(4400 + k)
    data, idx = random_records(rng, [3_000_001, 17, 250_000, 1, 4_000_003], 0.002, 0.002, 0.0005)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    d, di = dev(data, cuda), dev(idx, cuda)
    try:
        for reserve in (8, 64):
            kmc.set_reserved_cus(reserve)
            out = torch.full((1 << (2 * k), idx.size - 1), -1, dtype=torch.int32, device=cuda)
            inv = torch.full((idx.size - 1,), -1, dtype=torch.int32, device=cuda)
            args = kmc.dense_args(d, di, k, out, invalid=inv)
            ws = torch.empty(kmc.dense_ex_workspace_size(args), dtype=torch.uint8, device=cuda)
            kmc.count_dense_ex(kmc.dense_args(d, di, k, out, invalid=inv, workspace=ws))
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), exp, err_msg="reserve %d" % reserve)
            np.testing.assert_array_equal(inv.cpu().numpy(), exp_inv, err_msg="reserve %d" % reserve)
        with pytest.raises(kmc.KmcError):
            kmc.set_reserved_cus(65)
    finally:
        kmc.set_reserved_cus(0)


def test_sum_ld_column_block_and_workspace(kmc, oracle, cuda):
    """Writing into columns [off, off+n) of a wider matrix (multi-rank layout),
    with a caller-provided workspace."""
    import torch
    rng = np.random.default_rng(9)
    data, idx = random_records(rng, [5000, 60000, 1], 0.01, 0.0)
    n, k, ld, off = idx.size - 1, 6, 10, 4
    big = torch.full((1 << (2 * k), ld), -1, dtype=torch.int32, device=cuda)
    d, di = dev(data, cuda), dev(idx, cuda)
    flat = big.view(-1)[off:]
    args = kmc.dense_args(d, di, k, flat, ld=ld)
    ws_bytes = kmc.dense_ex_workspace_size(args)
    assert ws_bytes > 0
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    args = kmc.dense_args(d, di, k, flat, ld=ld, workspace=ws)
    kmc.count_dense_ex(args)
    torch.cuda.synchronize()
    got = big.cpu().numpy()
    exp, _ = oracle.count_dense(data, idx, k)
    np.testing.assert_array_equal(got[:, off:off + n], exp)
    assert (got[:, :off] == -1).all() and (got[:, off + n:] == -1).all()
    # too small a workspace is refused
    small = kmc.dense_args(d, di, k, flat, ld=ld, workspace=ws[: ws_bytes // 2])
    with pytest.raises(kmc.KmcError) as e:
        kmc.count_dense_ex(small)
    assert e.value.code == 1004


def test_synthetic_1gbase_k8_full_parity(kmc, oracle, cuda):
    """1 Gbase of the benchmark's own synthetic layout (4 x 250 Mbase), generated
    on the GPU, counted at k = 8 and compared bin for bin with the oracle."""
    import torch
    nrec, L = 4, 250_000_000
    total = nrec * (L + 1)
    buf = torch.empty(total, dtype=torch.uint8, device=cuda)
    kmc.synth_fill(buf, nrec, L, 0x5EED0008)
    idx = kmc.synth_indices(nrec, L)
    out, inv = kmc.count_dense(buf, dev(idx, cuda), 8, invalid=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    host = buf.cpu().numpy()
    exp, exp_inv = oracle.count_dense(host, idx, 8)
    np.testing.assert_array_equal(got, exp)
    assert (inv.cpu().numpy() == 0).all() and (exp_inv == 0).all()
    assert int(got.astype(np.int64).sum()) == nrec * (L - 8 + 1)


@pytest.mark.parametrize("nshards", [2, 7])
def test_gpu_counter_over_planned_shards(kmc, oracle, cuda, nshards):
    """kmc_dist.gpu_counter on each planned shard (only shard + halo on the device)
    sums to the full histogram: the per-rank work of the N-GPU path."""
    import kmc_dist
    rng = np.random.default_rng(21)
    data, idx = random_records(rng, [300_000, 5, 123_457, 64_000], 0.002, 0.002)
    exp, _ = oracle.count_dense(data, idx, 8)
    count = kmc_dist.gpu_counter(cuda)
    acc = np.zeros_like(exp)
    for shard in kmc.plan_shards(idx, 8, nshards):
        acc += count(data, idx, 8, shard).cpu().numpy()
    np.testing.assert_array_equal(acc, exp)


def test_count_multi_single_device(kmc, oracle, cuda):
    """kmc_count_multi (host buffer -> shards -> RCCL all-reduce) on the box's one GPU:
    a first call creates the device set's communicator, later calls (other k, a
    shard larger than one 32 MB pinned staging buffer) reuse it, and after
    kmc_multi_release a call creates it again."""
    rng = np.random.default_rng(22)
    data, idx = random_records(rng, [200_000, 77_777, 3], 0.003, 0.003)
    for k in (5, 8):
        got, inv = kmc.count_multi(data, idx, k, ndev=1, invalid=True)
        exp, exp_inv = oracle.count_dense(data, idx, k)
        np.testing.assert_array_equal(got, exp)
        np.testing.assert_array_equal(inv, exp_inv)
    big, bidx = random_records(rng, [40_000_000, 30_000_001], 0.001, 0.0)  # 70 MB: three staging chunks
    got, _ = kmc.count_multi(big, bidx, 4, ndev=1, devices=[0])
    exp, _ = oracle.count_dense(big, bidx, 4)
    np.testing.assert_array_equal(got, exp)
    # the cached buffers are grow-only: a smaller shard with a larger count matrix
    # (data buffer reused, sum buffer grown) and the invalid vector after a call without it
    many, midx = random_records(rng, [3_000] * 40, 0.01, 0.01)
    got, inv = kmc.count_multi(many, midx, 8, ndev=1, invalid=True)
    exp, exp_inv = oracle.count_dense(many, midx, 8)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(inv, exp_inv)
    got, _ = kmc.count_multi(big, bidx, 4, ndev=1)
    exp, _ = oracle.count_dense(big, bidx, 4)
    np.testing.assert_array_equal(got, exp)
    assert kmc.lib().kmc_multi_release() == 0
    assert kmc.lib().kmc_multi_release() == 0  # idempotent
    got, _ = kmc.count_multi(data, idx, 3, ndev=1)
    exp, _ = oracle.count_dense(data, idx, 3)
    np.testing.assert_array_equal(got, exp)
    with pytest.raises(kmc.KmcError):  # one communicator rank per device
        kmc.count_multi(data, idx, 3, ndev=2, devices=[0, 0])


def test_dense_spill_overflow_raises_status(kmc, oracle, cuda):
    """k = 8 spill lists past their capacity are never silent: with the capacity
    lowered to 1 entry (diagnostic library) a 64 MB poly-A record (every workgroup's
    piece wraps its AAAAAAAA counter ~4 times: several wrap entries each) stores
    KMC_ERR_CAPACITY in the call's status.  Without a status word of its own that is
    the device's host-mapped flag, which kmc_dense_status reports once and clears,
    and which no other call consumes (the next unrelated call used
    to fail in its place); with its own status word (kmc_dense_args::status) the
    call's failure stays in that word and the device flag is untouched.  With the
    capacity restored the counts are the oracle's and nothing is raised."""
    import torch
    rng = np.random.default_rng(404)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    recs = [np.append(np.full(64 << 20, ord("A"), np.uint8), np.uint8(0)),
            np.append(acgt[rng.integers(0, 4, 1_000_000)], np.uint8(0))]
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    exp, exp_inv = oracle.count_dense(data, idx, 8)
    d, di = dev(data, cuda), dev(idx, cuda)
    dv = torch.cuda.current_device()
    small, sidx = random_records(rng, [5000, 70_000])
    ds, dsi = dev(small, cuda), dev(sidx, cuda)
    with kmc.diag() as D:
        assert D.kmc_dense_status(dv) == 0
        assert D.kmc_diag_dense_spill_cap(1) == 0
        kmc.count_dense(d, di, 8, data_bytes=data.size)
        torch.cuda.synchronize()
        assert D.kmc_dense_status(dv) == kmc.KMC_ERR_CAPACITY
        assert D.kmc_dense_status(dv) == 0  # reported once
        kmc.count_dense(d, di, 8, data_bytes=data.size)
        out_s, _ = kmc.count_dense(ds, dsi, 8, data_bytes=small.size)  # an unrelated call: not failed by it
        torch.cuda.synchronize()
        assert D.kmc_dense_status(dv) == kmc.KMC_ERR_CAPACITY
        np.testing.assert_array_equal(out_s.cpu().numpy(), oracle.count_dense(small, sidx, 8)[0])
        # the call's own status word
        st = torch.zeros(1, dtype=torch.int32, device=cuda)
        out = torch.empty((1 << 16, idx.size - 1), dtype=torch.int32, device=cuda)
        kmc.count_dense_ex(kmc.dense_args(d, di, 8, out.view(-1), status=st))
        with pytest.raises(kmc.KmcError) as e:
            kmc.dense_status_check(st)
        assert e.value.code == kmc.KMC_ERR_CAPACITY and D.kmc_dense_status(dv) == 0
        assert D.kmc_diag_dense_spill_cap(0) == 0
        st.zero_()
        kmc.count_dense_ex(kmc.dense_args(d, di, 8, out.view(-1), status=st))
        kmc.dense_status_check(st)
        np.testing.assert_array_equal(out.cpu().numpy(), exp)
        out, inv = kmc.count_dense(d, di, 8, data_bytes=data.size, invalid=True)
        torch.cuda.synchronize()
        assert D.kmc_dense_status(dv) == 0
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    np.testing.assert_array_equal(inv.cpu().numpy(), exp_inv)


@pytest.mark.parametrize("k", [4, 8, 13])
def test_dense_record_of_2p31_windows_reports_error(kmc, cuda, k):
    """int32 counts (the reference's, main.cu:598,637) could wrap for a record of
    2^31 or more windows, which the 64-bit offsets admit: such a call stores
    KMC_ERR_RECORD_TOO_LONG in its status (the device flag, or the call's own word);
    2^31 - 1 windows pass, and the long record counted as two window ranges of the
    same buffer (kmc_count_dense_ex) is exact: the bins sum to its windows in int64.
    A 2.15 GB record: k = 4 and 8 on the LDS path, 13 on the radix path."""
    import torch
    dv = torch.cuda.current_device()
    L = (1 << 31) + k  # windows = L - k + 1 = 2^31 + 1
    buf = torch.empty(L + 1 + 16, dtype=torch.uint8, device=cuda)
    kmc.synth_fill(buf, 1, L, 0x5EED2031 + k)
    nb = 1 << (2 * k)
    out = torch.empty((nb, 1), dtype=torch.int32, device=cuda)
    for n_win, ok in ((L - k + 1, False), ((1 << 31) - 1, True)):
        Lr = n_win + k - 1
        di = dev(np.array([0, Lr + 1], np.int64), cuda)
        saved = buf[Lr].clone()
        buf[Lr] = 0  # the record's terminator
        assert kmc.lib().kmc_dense_status(dv) == 0
        kmc.count_dense(buf, di, k, data_bytes=Lr + 1, out=out)
        torch.cuda.synchronize()
        assert kmc.lib().kmc_dense_status(dv) == (0 if ok else kmc.KMC_ERR_RECORD_TOO_LONG), (k, n_win)
        st = torch.zeros(1, dtype=torch.int32, device=cuda)
        kmc.count_dense_ex(kmc.dense_args(buf[:Lr + 1], di, k, out.view(-1), status=st))
        torch.cuda.synchronize()
        assert int(st.item()) == (0 if ok else kmc.KMC_ERR_RECORD_TOO_LONG)
        if not ok:  # two window ranges of < 2^31 windows each, added in int64
            acc = torch.zeros(nb, dtype=torch.int64, device=cuda)
            cut = 1 << 30
            for lo, hi in ((0, cut), (cut, Lr + 1)):
                st.zero_()
                kmc.count_dense_ex(kmc.dense_args(buf[:Lr + 1], di, k, out.view(-1), read=(lo, min(hi + k - 1, Lr + 1)),
                                                  win=(lo, hi), status=st))
                kmc.dense_status_check(st)
                acc += out[:, 0].to(torch.int64)
            assert int(acc.sum()) == n_win
        else:
            assert int(out.to(torch.int64).sum()) == n_win
        buf[Lr] = saved
    del buf
    torch.cuda.empty_cache()


def test_synth_fill_range_matches_host(kmc, cuda):
    """kmc_synth_fill_range (a rank's byte range of the one global buffer) equals
    the same bytes of the whole-record generator, for unaligned and record-cutting
    ranges."""
    import torch
    L, seed = 4093, 0x5EED0008
    for lo, hi in ((0, 5 * 4094), (1, 4095), (4093, 4094), (4100, 13_000), (3 * 4094 - 5, 5 * 4094)):
        buf = torch.zeros(hi - lo + 64, dtype=torch.uint8, device=cuda)
        kmc.synth_fill_range(buf, lo, hi, L, seed)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(buf[:hi - lo].cpu().numpy(), kmc.synth_host_range(lo, hi, L, seed))
        assert int(buf[hi - lo:].sum()) == 0


@pytest.mark.parametrize("scaling,world,records,L,k", [
    ("strong", 2, 4, 3_000_000, 8),
    ("strong", 8, 3, 2_000_000, 8),
    ("strong", 4, 3, 1_500_000, 11),
    ("strong", 4, 3, 1_000, 8),      # three of the four shards are empty
    ("weak", 4, 2, 1_000_000, 8),
])
def test_bench_rank_counts_sum_to_whole(kmc, oracle, cuda, scaling, world, records, L, k):
    """bench.py's per-rank step on the GPU: each rank holds only its byte range +
    halo (kmc_synth_fill_range) and counts its window range into all columns of
    its matrix; the ranks' matrices sum to the oracle's histogram of the whole
    buffer (the all-reduce is a plain integer sum: tests/test_multi.py)."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    seed = bench.SEED_BASE + k
    acc = None
    for r in range(world):
        p = bench.rank_plan(scaling, world, r, records, L, k)
        base, hold_hi = p["hold"]
        data = torch.empty(max(hold_hi - base, 16), dtype=torch.uint8, device=cuda)
        kmc.synth_fill_range(data, base, hold_hi, L, seed)
        idx = torch.from_numpy(p["indices"]).to(cuda)
        out = torch.full((1 << (2 * k), p["n_tot"]), -5, dtype=torch.int32, device=cuda)
        kmc.count_dense_ex(kmc.dense_args(data, idx, k, out.view(-1), read=p["read"], win=p["win"],
                                          data_offset=base))
        torch.cuda.synchronize()
        part = out.cpu().numpy().astype(np.int64)
        acc = part if acc is None else acc + part
        del out, data
    total = int(p["indices"][-1])
    exp, _ = oracle.count_dense(kmc.synth_host_range(0, total, L, seed), p["indices"], k)
    np.testing.assert_array_equal(acc, exp)


@pytest.mark.parametrize("k,n", [(4, 511), (4, 512), (4, 513), (8, 1023), (8, 1024), (8, 1025)])
def test_first_record_search_at_block_size(kmc, oracle, cuda, k, n):
    """A workgroup finds the record its range starts in by one index load per
    thread when the records fit one block (n <= threads: 512 at k = 4, 1024 at
    k = 8), else by a binary search: record counts either side of that boundary,
    lengths such that workgroup ranges start in records all over the buffer, every
    record against the oracle."""
    import torch
    rng = np.random.default_rng(700 + n)
    lens = rng.integers(0, 9000, size=n)
    lens[::7] = 0
    data, idx = random_records(rng, lens, 0.002, 0.002, 0.0005)
    exp, exp_inv = oracle.count_dense(data, idx, k)
    d, di = dev(data, cuda), dev(idx, cuda)
    out = torch.full((1 << (2 * k), n), -1, dtype=torch.int32, device=cuda)
    inv = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    kmc.count_dense_ex(kmc.dense_args(d, di, k, out, invalid=inv))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    np.testing.assert_array_equal(inv.cpu().numpy(), exp_inv)


@pytest.mark.parametrize("k,n", [(8, 70_000), (9, 65_600)])
def test_many_short_records(kmc, oracle, cuda, k, n):
    """More records than one grid dimension of the per-record helper kernels can
    hold (k = 8: reduce/invalid; k = 9: the per-list histogram, n * 64 lists of
    1024 threads > 2^32): output 18 GB / 69 GB, checked on the device (every
    column sums to the record's valid windows) and on a sample of records against
    the oracle.  A caller workspace keeps the library's cache small afterwards."""
    import torch
    rng = np.random.default_rng(600 + k)
    lens = rng.integers(0, 3 * k, size=n)
    lens[:: 997] = 5000  # a few records cut across workgroups
    data, idx = random_records(rng, lens, 0.01, 0.0)
    d, di = dev(data, cuda), dev(idx, cuda)
    out = torch.empty((1 << (2 * k), n), dtype=torch.int32, device=cuda)
    inv = torch.empty(n, dtype=torch.int32, device=cuda)
    args = kmc.dense_args(d, di, k, out, invalid=inv)
    ws = torch.empty(kmc.dense_ex_workspace_size(args), dtype=torch.uint8, device=cuda)
    kmc.count_dense_ex(kmc.dense_args(d, di, k, out, invalid=inv, workspace=ws))
    torch.cuda.synchronize()
    del ws
    col = torch.zeros(n, dtype=torch.int64, device=cuda)
    for c0 in range(0, 1 << (2 * k), 4096):
        col += out[c0:c0 + 4096].to(torch.int64).sum(dim=0)
    windows = np.maximum(lens - k + 1, 0)
    np.testing.assert_array_equal(col.cpu().numpy() + inv.cpu().numpy(), windows)
    sample = np.unique(np.concatenate([rng.integers(0, n, 40), np.arange(0, n, 997)[:20], [0, n - 1]]))
    for s in sample:
        seg = data[idx[s]:idx[s + 1]]
        exp, exp_inv = oracle.count_dense(seg, np.array([0, seg.size], np.int64), k)
        np.testing.assert_array_equal(out[:, s].cpu().numpy(), exp[:, 0], err_msg="record %d" % s)
        assert int(inv[s]) == int(exp_inv[0])
    del out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [9, 13])
def test_radix_sum_ld_column_block(kmc, oracle, cuda, k):
    """k >= 9 into columns [off, off+n) of a wider matrix (ld > n: the R5 tile
    transpose; ld == n takes the contiguous one), 25 records (not a multiple of
    R5's 16-record tiles), other columns untouched."""
    import torch
    rng = np.random.default_rng(90 + k)
    data, idx = random_records(rng, list(rng.integers(0, 40_000, size=25)), 0.002, 0.0)
    n, ld, off = idx.size - 1, 31, 3
    big = torch.full((1 << (2 * k), ld), -1, dtype=torch.int32, device=cuda)
    d, di = dev(data, cuda), dev(idx, cuda)
    kmc.count_dense_ex(kmc.dense_args(d, di, k, big.view(-1)[off:], ld=ld))
    torch.cuda.synchronize()
    exp, _ = oracle.count_dense(data, idx, k)
    got = big.cpu().numpy()
    np.testing.assert_array_equal(got[:, off:off + n], exp)
    assert (got[:, :off] == -1).all() and (got[:, off + n:] == -1).all()
    del big
    out, _ = run_dense(kmc, cuda, data, idx, k)  # ld == n, 25 records
    np.testing.assert_array_equal(out, exp)
