"""GPU parity of the pairwise k-mer distance (kmc_pair_distances, minKmeres2_hip)
against the oracle (oracle_pair_distances = sequentialKmerCount2, main.cu:604-619;
oracle_min_kmeres2_row = minKmeres2, kernels.h:85-109), the golden fixtures and,
when oracle/_ref is present, the reference's own minKmeres2 kernel.

Float outputs are compared bit for bit (NaN == NaN: records shorter than k give
0/0 in the reference too); the integer sums behind them are exact.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def dev(x, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def same_floats(got, exp, msg=""):
    got = np.asarray(got, dtype=np.float32)
    exp = np.asarray(exp, dtype=np.float32)
    assert got.shape == exp.shape, msg
    both_nan = np.isnan(got) & np.isnan(exp)
    bad = ~both_nan & (got.view(np.uint32) != exp.view(np.uint32)) & ~((got == 0) & (exp == 0))
    assert not bad.any(), "%s: %d mismatches, first at %d: %r vs %r" % (
        msg, int(bad.sum()), int(np.argmax(bad)), got[bad][:3], exp[bad][:3])


def gpu_dist(kmc, cuda, counts, idx, k, ld=0):
    import torch
    out = kmc.pair_distances(dev(counts, cuda), dev(idx.astype(np.int64), cuda), k,
                             num_seqs=idx.size - 1, ld=ld)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name,dialect", G.cases())
def test_count_then_distance_matches_golden(kmc, cuda, name, dialect):
    """Step 1 + step 2 on the GPU == the reference CPU path's CSV values."""
    import torch
    g = G.load(name, dialect)
    idx = G.full_indices(g)
    data = g["data"] if g["data"].size else np.zeros(16, np.uint8)
    d, di = dev(data, cuda), dev(idx, cuda)
    for k in g["ks"]:
        k = int(k)
        counts, _ = kmc.count_dense(d, di, k, data_bytes=g["data"].size)
        out = kmc.pair_distances(counts, di, k)
        torch.cuda.synchronize()
        same_floats(out.cpu().numpy(), g["k%d_dist" % k], "%s/%s k=%d" % (name, dialect, k))


def random_counts(rng, n, k, scale):
    nb = 1 << (2 * k)
    counts = rng.integers(0, scale, size=(nb, n), dtype=np.int64).astype(np.int32)
    lens = counts.astype(np.int64).sum(axis=0) + k - 1 + rng.integers(0, 50, size=n)
    idx = np.concatenate([[0], np.cumsum(lens + 1)]).astype(np.int64)
    return counts, idx


@pytest.mark.parametrize("n,k", [(2, 3), (5, 8), (16, 4), (17, 4), (64, 3), (65, 5), (130, 3), (300, 2),
                                 (200, 8), (3000, 2)])
def test_distances_random_vs_oracle(kmc, oracle, cuda, n, k):
    """Tile edges (16 / 64), split and unsplit bin ranges, k = 2..8."""
    rng = np.random.default_rng(1000 * n + k)
    counts, idx = random_counts(rng, n, k, 40)
    got = gpu_dist(kmc, cuda, counts, idx, k)
    same_floats(got, oracle.pair_distances(counts, np.diff(idx) - 1, k), "n=%d k=%d" % (n, k))


def test_distances_large_counts_exact(kmc, oracle, cuda):
    """Sums far above 2^24: exact integer accumulation, one float rounding."""
    rng = np.random.default_rng(5)
    counts, idx = random_counts(rng, 12, 6, 1 << 22)
    got = gpu_dist(kmc, cuda, counts, idx, 6)
    same_floats(got, oracle.pair_distances(counts, np.diff(idx) - 1, 6))


def test_distances_k13_split(kmc, oracle, cuda):
    """67 M codes per record: the bin axis split over many workgroups."""
    rng = np.random.default_rng(13)
    n, k = 3, 13
    nb = 1 << (2 * k)
    counts = np.zeros((nb, n), dtype=np.int32)
    hot = rng.integers(0, nb, size=200_000)
    for s in range(n):
        np.add.at(counts[:, s], rng.choice(hot, size=300_000), 1)
    lens = counts.astype(np.int64).sum(axis=0) + k - 1
    idx = np.concatenate([[0], np.cumsum(lens + 1)]).astype(np.int64)
    got = gpu_dist(kmc, cuda, counts, idx, k)
    same_floats(got, oracle.pair_distances(counts, lens, k))


def test_distances_sum_ld_column_block(kmc, oracle, cuda):
    """Counts as a column block of a wider matrix (sum_ld > num_seqs)."""
    rng = np.random.default_rng(9)
    n, k, ld = 20, 4, 33
    counts, idx = random_counts(rng, n, k, 100)
    wide = np.full((1 << (2 * k), ld), -7, dtype=np.int32)
    wide[:, :n] = counts
    got = gpu_dist(kmc, cuda, wide, idx, k, ld=ld)
    same_floats(got, oracle.pair_distances(counts, np.diff(idx) - 1, k))


def test_distances_edge_counts(kmc, cuda):
    import torch
    for n in (0, 1):
        out = kmc.pair_distances(torch.zeros((64, max(n, 1)), dtype=torch.int32, device=cuda),
                                 torch.zeros(n + 1, dtype=torch.int64, device=cuda), 3, num_seqs=n)
        torch.cuda.synchronize()
        assert out.numel() == 0
    with pytest.raises(kmc.KmcError):
        kmc.pair_distances(torch.zeros((64, 4), dtype=torch.int32, device=cuda),
                           torch.zeros(5, dtype=torch.int64, device=cuda), 14)


def dropin_all_rows(kmc, cuda, counts, idx32):
    import torch
    n = idx32.size - 1
    sums = dev(counts.reshape(-1), cuda)
    mins = torch.zeros(max(n * (n - 1) // 2, 1), dtype=torch.float32, device=cuda)
    ix = dev(idx32, cuda)
    for cur in range(n):
        kmc.min_kmeres2(sums, mins, n, cur, ix)
    torch.cuda.synchronize()
    return mins.cpu().numpy()[: n * (n - 1) // 2]


@pytest.mark.parametrize("name", ["basic", "maxseqs", "maxseqs_single", "random"])
def test_min_kmeres2_dropin_golden(kmc, cuda, name):
    g = G.load(name, "blank")
    idx = G.full_indices(g).astype(np.int32)
    exp, _ = G.dense_expected(g, 3)
    same_floats(dropin_all_rows(kmc, cuda, exp, idx), g["k3_dist"], name)


def test_min_kmeres2_dropin_float_rounding(kmc, oracle, cuda):
    """Counts large enough that the reference kernel's float running sum rounds:
    the drop-in follows kernels.h:103 (float, code order), not the exact sum."""
    rng = np.random.default_rng(77)
    n = 40
    counts = rng.integers(1 << 20, 1 << 23, size=(64, n), dtype=np.int64).astype(np.int32)
    lens = counts.astype(np.int64).sum(axis=0) + 5
    idx32 = np.concatenate([[0], np.cumsum(lens + 1)]).astype(np.int32)
    exp = np.zeros(n * (n - 1) // 2, dtype=np.float32)
    for cur in range(n):
        oracle.min_kmeres2_row(counts, idx32, cur, 3, exp)
    got = dropin_all_rows(kmc, cuda, counts, idx32)
    same_floats(got, exp)
    if oracle.have_ref_kernel():
        import torch
        L = oracle.ref_kernel()
        sums = dev(counts.reshape(-1), cuda)
        mins = torch.zeros(n * (n - 1) // 2, dtype=torch.float32, device=cuda)
        ix = dev(idx32, cuda)
        for cur in range(n):
            assert L.ref_min_kmeres2_launch(sums.data_ptr(), mins.data_ptr(), n, cur, ix.data_ptr()) == 0
        same_floats(got, mins.cpu().numpy())


def test_min_kmeres2_dropin_vs_reference_kernel(kmc, oracle, cuda):
    """The reference's own minKmeres2 (kernels.h, compiled for gfx950) on counts the
    reference's step 1 produced for random records."""
    if not oracle.have_ref_kernel():
        pytest.skip("oracle/_ref/libref_kernel.so not built")
    import torch
    rng = np.random.default_rng(3)
    n = 70
    lens = rng.integers(1, 5000, size=n)
    recs = [np.append(rng.choice(np.frombuffer(b"ACGTN", dtype=np.uint8), size=int(L),
                                 p=[.245, .245, .245, .245, .02]), np.uint8(0)) for L in lens]
    data = np.concatenate(recs)
    idx32 = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int32)
    counts, _ = oracle.count_dense(data, idx32.astype(np.int64), 3)
    got = dropin_all_rows(kmc, cuda, counts, idx32)
    L = oracle.ref_kernel()
    sums = dev(counts.reshape(-1), cuda)
    mins = torch.zeros(n * (n - 1) // 2, dtype=torch.float32, device=cuda)
    ix = dev(idx32, cuda)
    for cur in range(n):
        assert L.ref_min_kmeres2_launch(sums.data_ptr(), mins.data_ptr(), n, cur, ix.data_ptr()) == 0
    same_floats(got, mins.cpu().numpy())
