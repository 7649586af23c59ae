"""FASTA loader (product, C++) against the reference loader's outputs."""
import os

import numpy as np
import pytest

import golden_util as G


@pytest.mark.parametrize("name,dialect", G.cases())
def test_loader_matches_golden(kmc, name, dialect):
    g = G.load(name, dialect)
    path = os.path.join(G.GOLDEN, name + ".fa")
    data, idx, ref_n = kmc.load_fasta(path, kmc.DIALECT_NONL if dialect == "nonl" else kmc.DIALECT_BLANK,
                                      kmc.MAX_SEQS_REFERENCE)
    assert idx.size - 1 == int(g["n_seqs"])
    np.testing.assert_array_equal(data, g["data"])
    np.testing.assert_array_equal(idx, G.full_indices(g))
    assert ref_n == g["indexes"].size  # includes the missing-sentinel quirk


def test_loader_quirks_documented(kmc):
    """Behaviours the survey probed on the reference."""
    gd = lambda n, d: kmc.load_fasta(os.path.join(G.GOLDEN, n + ".fa"), d)  # noqa: E731
    assert gd("maxseqs", 0)[1].size - 1 == 101          # MAX_SEQS=100 keeps 101 records
    assert gd("maxseqs_single", 0)[1].size - 1 == 110   # cap never fires on 1-line records
    assert gd("standard", 0)[1].size - 1 == 1           # importSeqs: one record incl. headers
    assert gd("standard", 1)[1].size - 1 == 4           # importSeqsNoNL splits on '>'
    d, idx, ref_n = gd("trailing_blank", 0)
    assert ref_n == idx.size - 1                        # reference drops the end sentinel
    assert idx[-1] == d.size                            # we always carry it


@pytest.mark.parametrize("seed", range(40))
def test_loader_matches_reference_live(kmc, oracle, tmp_path, seed):
    if not oracle.have_ref_cpu():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(seed)
    path = str(tmp_path / "r.fa")
    G.random_fasta(rng, path)
    for dialect in (0, 1):
        for cap in (kmc.MAX_SEQS_REFERENCE, 3):
            if cap != kmc.MAX_SEQS_REFERENCE:
                continue  # the reference's cap is the compile-time MAX_SEQS
            n, ref_idx, ref_data = oracle.ref_import(path, nonl=bool(dialect))
            data, idx, ref_n = kmc.load_fasta(path, dialect, cap)
            assert idx.size - 1 == n
            np.testing.assert_array_equal(data, ref_data)
            np.testing.assert_array_equal(idx[:ref_idx.size], ref_idx)
            assert ref_n == ref_idx.size


def test_loader_unlimited_and_errors(kmc, tmp_path):
    p = tmp_path / "many.fa"
    p.write_text("".join(">r%d\nACGT\nAC\n\n" % i for i in range(250)).rstrip("\n"))
    _, idx, _ = kmc.load_fasta(str(p), 0, 0)
    assert idx.size - 1 == 250
    _, idx, _ = kmc.load_fasta(str(p), 0, kmc.MAX_SEQS_REFERENCE)
    assert idx.size - 1 == 101
    empty = tmp_path / "empty.fa"
    empty.write_text("")
    d, idx, ref_n = kmc.load_fasta(str(empty), 0)
    assert d.size == 0 and idx.tolist() == [0] and ref_n == 0
    with pytest.raises(kmc.KmcError) as e:
        kmc.load_fasta(str(tmp_path / "missing.fa"))
    assert e.value.code == 1005
