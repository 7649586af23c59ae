"""The oracle (C restatement) pinned against the reference's own outputs."""
import os

import numpy as np
import pytest

import golden_util as G


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_bin_order_matches_permutation(oracle, k):
    """Pattern i of the reference's permutation() (utils.h:21-50) has LE code i."""
    pats = np.load(os.path.join(G.GOLDEN, "patterns_k%d.npy" % k))
    for i, row in enumerate(pats):
        assert oracle.lib().oracle_window_code(row.tobytes(), k) == i


@pytest.mark.parametrize("name,dialect", G.cases())
def test_oracle_matches_golden(oracle, name, dialect):
    g = G.load(name, dialect)
    idx = G.full_indices(g)
    for k in g["ks"]:
        k = int(k)
        got, inv = oracle.count_dense(g["data"], idx, k)
        exp, exp_inv = G.dense_expected(g, k)
        np.testing.assert_array_equal(got, exp, err_msg="%s/%s k=%d" % (name, dialect, k))
        np.testing.assert_array_equal(inv, exp_inv)


def _random_records(rng, n, lo, hi, n_frac=0.01, lower_frac=0.01):
    recs = []
    for _ in range(n):
        L = int(rng.integers(lo, hi))
        s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=L)
        s[rng.random(L) < n_frac] = ord("N")
        m = rng.random(L) < lower_frac
        s[m] |= 0x20
        recs.append(np.append(s, np.uint8(0)))
    data = np.concatenate(recs) if recs else np.zeros(0, np.uint8)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    return data, idx


@pytest.mark.parametrize("k", [1, 3, 4, 7])
def test_oracle_matches_python_restatement(oracle, k):
    rng = np.random.default_rng(k)
    data, idx = _random_records(rng, 6, 0, 300)
    got, inv = oracle.count_dense(data, idx, k)
    for s in range(idx.size - 1):
        h = oracle.py_count_record(bytes(data[idx[s]:idx[s + 1]]), k)
        assert h[0] == inv[s]
        np.testing.assert_array_equal(got[:, s], h[1:])


@pytest.mark.parametrize("k", [2, 3, 6, 8, 9])
def test_oracle_matches_reference_live(oracle, k):
    """Against the reference's permutationsCountAll compiled from /root/reference."""
    if not oracle.have_ref_cpu():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(100 + k)
    data, idx = _random_records(rng, 4, 1, 3000, 0.005, 0.005)
    got, inv = oracle.count_dense(data, idx, k)
    for s in range(idx.size - 1):
        h = oracle.ref_count_bytes(data[idx[s]:idx[s + 1]], k)
        assert h[0] == inv[s]
        np.testing.assert_array_equal(got[:, s], h[1:])


_K13_LIVE = r"""
import os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import oracle
rng = np.random.default_rng(113)
recs = []
for L in (0, 12, 13, 14, 40_000, 2_500):
    x = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=L)
    x[rng.random(L) < 0.003] = ord("N")
    recs.append(np.append(x, np.uint8(0)))
data = np.concatenate(recs)
idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
got, inv = oracle.count_dense(data, idx, 13)
bad = 0
for s in range(idx.size - 1):
    h = oracle.ref_count_bytes(data[idx[s]:idx[s + 1]], 13)
    bad += int(h[0] != inv[s]) + int((got[:, s] != h[1:]).sum())
print("mismatches", bad, flush=True)
os._exit(0 if bad == 0 else 1)  # skip the 4^13-entry std::map's destructor (tens of seconds)
"""


def test_oracle_matches_reference_live_k13(oracle):
    """k = 13 (config C3, the largest dense k) against the reference's own
    permutationsCountAll, whose 4^13-entry std::map is built and dropped in a
    child process."""
    import subprocess
    import sys
    if not oracle.have_ref_cpu():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    r = subprocess.run([sys.executable, "-c", _K13_LIVE, os.path.dirname(oracle.__file__)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_oracle_range_partition_sums(oracle):
    """Windowed counting over disjoint start ranges sums to the full count."""
    rng = np.random.default_rng(7)
    data, idx = _random_records(rng, 5, 0, 2000)
    full, _ = oracle.count_dense(data, idx, 5)
    cuts = [0, 100, 1000, 1001, 4096, data.size]
    acc = np.zeros_like(full)
    for a, b in zip(cuts[:-1], cuts[1:]):
        part, _ = oracle.count_dense(data, idx, 5, win=(a, b))
        acc += part
    np.testing.assert_array_equal(acc, full)


# ---------------------------------------------------------------------------
# pairwise distance (step 2)
# ---------------------------------------------------------------------------
def golden_lens(g):
    idx = G.full_indices(g)
    return np.diff(idx) - 1


@pytest.mark.parametrize("name,dialect", G.cases())
def test_oracle_distances_match_golden(oracle, name, dialect):
    """oracle_pair_distances == sequentialKmerCount2 (main.cu:587-621) output."""
    g = G.load(name, dialect)
    for k in g["ks"]:
        k = int(k)
        exp, _ = G.dense_expected(g, k)
        got = oracle.pair_distances(exp, golden_lens(g), k)
        np.testing.assert_array_equal(got, g["k%d_dist" % k], err_msg="%s/%s k=%d" % (name, dialect, k))


@pytest.mark.parametrize("name", ["basic", "maxseqs", "random"])
def test_oracle_gpu_row_semantics_match_golden(oracle, name):
    """The float-accumulating row function (minKmeres2, kernels.h:85-109) equals the
    CPU path whenever its float sum is exact (small records)."""
    g = G.load(name, "blank")
    idx = G.full_indices(g).astype(np.int32)
    exp, _ = G.dense_expected(g, 3)
    n = idx.size - 1
    out = np.zeros(max(n * (n - 1) // 2, 1), dtype=np.float32)
    for cur in range(n):
        oracle.min_kmeres2_row(exp, idx, cur, 3, out)
    np.testing.assert_array_equal(out[: n * (n - 1) // 2], g["k3_dist"])


def test_oracle_distances_match_reference_live(oracle, tmp_path):
    """Random FASTA through the reference's own loader + sequentialKmerCount2."""
    if not oracle.have_ref_cpu():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(31)
    recs = []
    for i in range(9):
        L = int(rng.integers(1, 1500))
        s = rng.choice(np.frombuffer(b"ACGTN", dtype=np.uint8), size=L, p=[.24, .24, .24, .24, .04])
        recs.append(">x%d\n%s\n" % (i, s.tobytes().decode()))
    fa = tmp_path / "d.fa"
    fa.write_text("\n".join(recs).rstrip("\n"))
    n, indexes, data = oracle.ref_import(str(fa))
    idx = indexes if indexes.size == n + 1 else np.append(indexes, data.size)
    for k in (2, 4, 6):
        counts, _ = oracle.count_dense(data, idx, k)
        got = oracle.pair_distances(counts, np.diff(idx) - 1, k)
        np.testing.assert_array_equal(got, oracle.ref_seq_distances(str(fa), k))


# ---------------------------------------------------------------------------
# canonical k-mer self-oracle (no reference counterpart), pinned where the
# reference reaches: for k <= 13 its counts fold from the reference's dense ones
# ---------------------------------------------------------------------------
def le_to_msb(code, k):
    out = 0
    for q in range(k):
        out = (out << 2) | ((code >> (2 * q)) & 3)
    return out


def fold_dense(dense, k, forward):
    """{(record, key): count} from a (4^k, n) dense LE histogram."""
    mask = (1 << (2 * k)) - 1
    res = {}
    codes, recs = np.nonzero(dense)
    for c, s in zip(codes.tolist(), recs.tolist()):
        fw = le_to_msb(c, k)
        key = fw if forward else min(fw, c ^ mask)  # LE code complemented = MSB key of the reverse complement
        res[(s, key)] = res.get((s, key), 0) + int(dense[c, s])
    return res


def canon_dict(keys, counts, off):
    res = {}
    for s in range(off.size - 1):
        for i in range(int(off[s]), int(off[s + 1])):
            res[(s, int(keys[i]))] = int(counts[i])
    return res


@pytest.mark.parametrize("name,dialect", [("basic", "blank"), ("random", "nonl"), ("maxseqs", "blank"),
                                          ("odd", "nonl"), ("crlf", "blank")])
@pytest.mark.parametrize("forward", [False, True])
def test_canonical_oracle_folds_golden_dense(oracle, name, dialect, forward):
    g = G.load(name, dialect)
    idx = G.full_indices(g)
    for k in g["ks"]:
        k = int(k)
        exp, _ = G.dense_expected(g, k)
        keys, counts, off = oracle.count_canonical(g["data"], idx, k, forward=forward)
        assert canon_dict(keys, counts, off) == fold_dense(exp, k, forward), "%s k=%d" % (name, k)
        for s in range(idx.size - 1):  # sorted, distinct within each record
            seg = keys[int(off[s]):int(off[s + 1])]
            assert np.all(seg[1:] > seg[:-1])


def py_canonical(rec, k, soft=False):
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    enc = {"A": 0, "C": 1, "G": 2, "T": 3}
    res = {}
    txt = rec.decode("latin-1")
    for i in range(max(0, len(txt) - k)):  # len includes the terminator
        w = txt[i:i + k]
        if soft:
            w = "".join(ch.upper() if ch in "acgt" else ch for ch in w)
        if any(ch not in enc for ch in w):
            continue
        rc = "".join(comp[ch] for ch in reversed(w))
        key = min(w, rc)
        v = 0
        for ch in key:
            v = (v << 2) | enc[ch]
        res[v] = res.get(v, 0) + 1
    return res


@pytest.mark.parametrize("k", [1, 2, 5, 16, 17, 31])
def test_canonical_oracle_matches_python_strings(oracle, k):
    rng = np.random.default_rng(k)
    recs = []
    for L in (0, 1, k - 1, k, k + 1, 200, 777):
        s = rng.choice(np.frombuffer(b"ACGTNacgt", dtype=np.uint8), size=max(L, 0),
                       p=[.22, .22, .22, .22, .02, .025, .025, .025, .025])
        recs.append(np.append(s, np.uint8(0)))
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    for soft in (False, True):
        keys, counts, off = oracle.count_canonical(data, idx, k, soft=soft)
        got = canon_dict(keys, counts, off)
        exp = {}
        for s in range(len(recs)):
            for key, c in py_canonical(bytes(recs[s]), k, soft).items():
                exp[(s, key)] = c
        assert got == exp


@pytest.mark.parametrize("k", [1, 5, 16, 21, 31])
@pytest.mark.parametrize("sel_bits", [0, 3, 12])
def test_canonical_digest_matches_sort_oracle(oracle, k, sel_bits):
    """oracle_canonical_digest (the rolling, per-record restatement behind the
    full-size canonical check) against oracle_count_canonical (sort + run-length):
    valid windows, the sum of dg_hash(key) * count mod 2^64, and the selected
    subset (top sel_bits of dg_hash(key) == sel_val; 0 bits: every key), on ragged
    records with N runs, lowercase, '\\0' bytes inside a record, repeats."""
    rng = np.random.default_rng(31 * k + sel_bits)
    recs = []
    for L in (0, 1, k - 1, k, k + 1, 200, 5000, 40_000):
        s = rng.choice(np.frombuffer(b"ACGTNacgt\0", dtype=np.uint8), size=max(L, 0),
                       p=[.22, .22, .22, .22, .02, .02, .025, .025, .025, .005])
        recs.append(np.append(s, np.uint8(0)))
    rep = np.frombuffer(b"ACGTTGCAAT" * 300 + b"tttt" * 200, dtype=np.uint8)
    recs.append(np.append(rep, np.uint8(0)))
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    M = (1 << 64) - 1
    for soft, forward in ((False, False), (True, False), (True, True)):
        keys, counts, off = oracle.count_canonical(data, idx, k, soft=soft, forward=forward)
        h = oracle.dg_hash(keys)
        for sel_val in ((0, 5) if sel_bits else (0,)):
            res = oracle.canonical_digest(data, idx, k, soft=soft, forward=forward, sel_val=sel_val,
                                          sel_bits=sel_bits, threads=4)
            for s in range(idx.size - 1):
                a, b = int(off[s]), int(off[s + 1])
                r = res[s]
                assert r["valid"] == int(counts[a:b].astype(np.int64).sum())
                assert r["digest"] == sum(int(x) * int(c) for x, c in zip(h[a:b], counts[a:b])) & M
                sel = (h[a:b] >> np.uint64(64 - sel_bits)) == np.uint64(sel_val) if sel_bits else slice(None)
                np.testing.assert_array_equal(r["keys"], keys[a:b][sel])
                np.testing.assert_array_equal(r["counts"], counts[a:b][sel])
