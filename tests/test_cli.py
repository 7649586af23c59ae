"""The C++ host driver (dna-kmeres-parallel_amd/bin/kmc, csrc/kmc_main.cpp), the
successor of the reference program's main() (main.cu:120-399).

CPU tests: the binary is built, parses its options like documented and fails
cleanly without a device.  GPU tests: on every golden fixture its
parallel_results.csv equals, line for line, the "%f\\n" text the reference writes
(main.cu:351-358) for the distances of its own sequentialKmerCount2 (golden
kX_dist, both loader dialects), in the default one-launch path and in --dropin
mode (the exact reference launches, k = 3); its --counts dump equals the golden
histograms; its --canonical dump equals the oracle.
"""
import os
import subprocess

import numpy as np
import pytest

import golden_util as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KMC = os.environ.get("KMC_BIN") or os.path.join(REPO, "dna-kmeres-parallel_amd", "bin", "kmc")


def run(args, **kw):
    return subprocess.run([KMC] + [str(a) for a in args], capture_output=True, text=True, timeout=120, **kw)


def test_binary_built_and_links_libkmc():
    assert os.access(KMC, os.X_OK)
    out = subprocess.run(["ldd", KMC], capture_output=True, text=True).stdout
    assert "libkmc.so" in out and "not found" not in out


def test_help_and_option_errors():
    r = run(["--help"])
    assert r.returncode == 0 and "usage: kmc" in r.stdout
    assert run([]).returncode == 2
    assert run(["-k", "14", "x.fa"]).returncode == 2          # dense path stops at k = 13
    assert run(["-k", "32", "--canonical", "x.fa"]).returncode == 2
    assert run(["--dropin", "-k", "4", "x.fa"]).returncode == 2  # the reference launch is k = 3
    assert run(["--bogus", "x.fa"]).returncode == 2
    assert run(["--dialect", "fastq", "x.fa"]).returncode == 2


def test_missing_input_is_an_io_error(tmp_path):
    r = run([tmp_path / "absent.fa"])
    assert r.returncode == 1 and "kmc: " in r.stderr  # no device here, or KMC_ERR_IO on the GPU box


def csv_floats(path):
    with open(path) as f:
        lines = f.read().splitlines()
    return lines, np.array([float(x) for x in lines], dtype=np.float32)


def assert_csv_matches(path, exp, msg):
    """Line for line the reference's "%f" text; NaN lines (records shorter than
    k: 0/0 in the reference too) compare as NaN whatever their sign."""
    lines, got = csv_floats(path)
    exp = np.asarray(exp, dtype=np.float32)
    assert len(lines) == exp.size, msg
    for i, (line, e) in enumerate(zip(lines, exp)):
        if np.isnan(e):
            assert np.isnan(got[i]), "%s line %d: %s vs nan" % (msg, i, line)
        else:
            assert line == "%f" % e, "%s line %d: %s vs %f" % (msg, i, line, e)


def fixture_path(name):
    return os.path.join(G.GOLDEN, name + ".fa")


@pytest.mark.gpu
@pytest.mark.parametrize("name,dialect", G.cases())
def test_cli_distances_equal_reference_csv(cuda, tmp_path, name, dialect):
    g = G.load(name, dialect)
    for k in g["ks"]:
        k = int(k)
        out = tmp_path / ("k%d" % k)
        out.mkdir()
        dump = k <= 11  # k = 12/13 dumps are 16.7 M / 67 M lines: the CSVs are checked only
        r = run(["-q", "-k", k, "--dialect", dialect, "--out", out] + (["--counts", out / "counts.tsv"] if dump else [])
                + [fixture_path(name)])
        assert r.returncode == 0, r.stderr
        assert_csv_matches(out / "parallel_results.csv", g["k%d_dist" % k], "%s/%s k=%d" % (name, dialect, k))
        assert_csv_matches(out / "sequential_results.csv", g["k%d_dist" % k], "%s/%s k=%d seq" % (name, dialect, k))
        if not dump:
            continue
        exp, _ = G.dense_expected(g, k)
        with open(out / "counts.tsv") as f:
            rows = f.read().splitlines()
        assert len(rows) == 1 << (2 * k)
        for code in range(0, 1 << (2 * k), max(1, (1 << (2 * k)) // 64)):
            fields = rows[code].split("\t")
            kmer = "".join("ACGT"[(code >> (2 * p)) & 3] for p in range(k))
            assert fields[0] == kmer
            assert [int(x) for x in fields[1:]] == exp[code].tolist(), "%s k=%d code %d" % (name, k, code)


@pytest.mark.gpu
@pytest.mark.parametrize("name,dialect", G.cases())
def test_cli_dropin_mode_equals_reference_csv(cuda, tmp_path, name, dialect):
    g = G.load(name, dialect)
    r = run(["-q", "--dropin", "--dialect", dialect, "--out", tmp_path, fixture_path(name)])
    assert r.returncode == 0, r.stderr
    assert_csv_matches(tmp_path / "parallel_results.csv", g["k3_dist"], "%s/%s dropin" % (name, dialect))
    assert_csv_matches(tmp_path / "sequential_results.csv", g["k3_dist"], "%s/%s dropin seq" % (name, dialect))


@pytest.mark.gpu
def test_cli_host_loader_same_csv(cuda, tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    for d, extra in ((a, []), (b, ["--host-loader"])):
        r = run(["-q", "-k", 4, "--dialect", "nonl", "--out", d] + extra + [fixture_path("odd")])
        assert r.returncode == 0, r.stderr
    assert (a / "parallel_results.csv").read_text() == (b / "parallel_results.csv").read_text()


@pytest.mark.gpu
def test_cli_prints_the_reference_timers(cuda, tmp_path):
    r = run(["--out", tmp_path, fixture_path("random")])
    assert r.returncode == 0, r.stderr
    for line in ("sequences read .", "Elapsed parallel timer step 1:", "Elapsed parallel step 2 timer:",
                 "Total time elapsed parallel:"):
        assert line in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("k", [5, 31])
def test_cli_canonical_dump_equals_oracle(cuda, oracle, tmp_path, k):
    g = G.load("random", "nonl")
    r = run(["-q", "--canonical", "-k", k, "--dialect", "nonl", "--counts", tmp_path / "c.tsv",
             fixture_path("random")])
    assert r.returncode == 0, r.stderr
    got = {}
    with open(tmp_path / "c.tsv") as f:
        for line in f:
            s, kmer, c = line.split("\t")
            got[(int(s), kmer)] = int(c)
    idx = G.full_indices(g)
    keys, counts, off = oracle.count_canonical(g["data"], idx, k)
    exp = {}
    for s in range(idx.size - 1):
        for i in range(off[s], off[s + 1]):
            key = int(keys[i])
            kmer = "".join("ACGT"[(key >> (2 * (k - 1 - p))) & 3] for p in range(k))
            exp[(s, kmer)] = int(counts[i])
    assert got == exp
