"""GPU FASTA parse (kmc_fasta_parse_device / kmc_fasta_load_device, SURVEY.md §8(f)
F1) against the host loader kmc_fasta_load, which test_loader.py pins to the
reference's importSeqs / importSeqsNoNL (golden fixtures and the live reference).
Bit-exact record bytes and offsets, both dialects, uncapped; the capped path of
kmc_fasta_load_device is the host rule and must equal it too."""
import os

import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def gpu_parse(kmc, cuda, raw_bytes, dialect):
    import torch
    raw = torch.from_numpy(np.frombuffer(raw_bytes, dtype=np.uint8).copy()).to(cuda) if raw_bytes else \
        torch.zeros(0, dtype=torch.uint8, device=cuda)
    data, idx = kmc.parse_fasta_device(raw, dialect)
    torch.cuda.synchronize()
    return data.cpu().numpy(), idx.cpu().numpy()


def same_as_host(kmc, cuda, path, dialect, msg=""):
    with open(path, "rb") as f:
        raw = f.read()
    exp_data, exp_idx, _ = kmc.load_fasta(path, dialect, 0)
    data, idx = gpu_parse(kmc, cuda, raw, dialect)
    np.testing.assert_array_equal(idx, exp_idx, err_msg=msg + " indices")
    np.testing.assert_array_equal(data, exp_data, err_msg=msg + " data")


@pytest.mark.parametrize("name,dialect", G.cases())
def test_golden_files(kmc, cuda, name, dialect):
    same_as_host(kmc, cuda, os.path.join(G.GOLDEN, name + ".fa"), 1 if dialect == "nonl" else 0, name)


@pytest.mark.parametrize("seed", range(60))
def test_random_structures(kmc, cuda, tmp_path, seed):
    rng = np.random.default_rng(1000 + seed)
    path = str(tmp_path / "r.fa")
    G.random_fasta(rng, path, nrec_max=40)
    for dialect in (0, 1):
        same_as_host(kmc, cuda, path, dialect, "seed %d dialect %d" % (seed, dialect))


@pytest.mark.parametrize("text", [
    "", "\n", "\n\n\n", ">", ">h", ">h\n", ">h\nA", ">h\nA\n", "A\nC\n", ">h\n\rAC\nGT\n", ">h\nAC\r\n\r\nGT\n",
    ">a\nAC\n>b\nGT", ">a\nAC\n>b\nGT\n\n", "\r", ">h\n|A|\n\nx", ">h\n>g\nAC\n", ">h\nAC\n\n\n\n>g\n\nTT\n\n",
])
def test_edge_cases(kmc, cuda, tmp_path, text):
    path = str(tmp_path / "e.fa")
    with open(path, "w", newline="") as f:
        f.write(text)
    for dialect in (0, 1):
        same_as_host(kmc, cuda, path, dialect, repr(text))


def test_long_lines_and_many_tiles(kmc, cuda, tmp_path):
    """Lines much longer than a 16 KiB tile, and 40 000 short records over many
    tiles of both the byte and the line scans."""
    rng = np.random.default_rng(7)
    parts = [">big\n", "".join(rng.choice(list("ACGT"), size=200_000)) + "\n", "\n"]
    for i in range(40_000):
        parts.append(">r%d\n%s\n%s\n\n" % (i, "".join(rng.choice(list("ACGTN|"), size=int(rng.integers(1, 30)))),
                                          "A" * int(rng.integers(0, 3))))
    path = str(tmp_path / "m.fa")
    with open(path, "w") as f:
        f.write("".join(parts))
    for dialect in (0, 1):
        same_as_host(kmc, cuda, path, dialect, "dialect %d" % dialect)


def test_load_device_uncapped_and_capped(kmc, cuda):
    import torch
    for name in ("maxseqs", "maxseqs_single", "random", "crlf", "standard"):
        path = os.path.join(G.GOLDEN, name + ".fa")
        for dialect in (0, 1):
            for cap in (0, kmc.MAX_SEQS_REFERENCE, 3):
                exp_data, exp_idx, _ = kmc.load_fasta(path, dialect, cap)
                data, idx = kmc.load_fasta_device(path, dialect, cap)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(idx.cpu().numpy(), exp_idx, err_msg="%s %d %d" % (name, dialect, cap))
                np.testing.assert_array_equal(data.cpu().numpy(), exp_data, err_msg="%s %d %d" % (name, dialect, cap))


def test_synthetic_80col_fasta_then_count(kmc, oracle, cuda, tmp_path):
    """A §8(d)-layout FASTA (80 columns, blank-line separated, no final blank
    line): parsed on the GPU and counted there, equal to the oracle on the host
    loader's buffer."""
    import torch
    rng = np.random.default_rng(3)
    recs = ["".join(rng.choice(list("ACGT"), size=int(L))) for L in (100_000, 80, 81, 250_000, 1)]
    with open(tmp_path / "s.fa", "w") as f:
        f.write("\n".join(">r%04d\n" % i + "\n".join(s[j:j + 80] for j in range(0, len(s), 80)) + "\n"
                          for i, s in enumerate(recs)).rstrip("\n"))
    data, idx = kmc.load_fasta_device(str(tmp_path / "s.fa"), 0, 0)
    exp_data, exp_idx, _ = kmc.load_fasta(str(tmp_path / "s.fa"), 0, 0)
    np.testing.assert_array_equal(idx.cpu().numpy(), exp_idx)
    counts, _ = kmc.count_dense(data, idx, 8)
    torch.cuda.synchronize()
    exp, _ = oracle.count_dense(exp_data, exp_idx, 8)
    np.testing.assert_array_equal(counts.cpu().numpy(), exp)
