"""Load the golden fixtures of tests/golden (see make_golden.py for the format)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        name, dialect = os.path.basename(f)[:-4].split(".")
        out.append((name, dialect))
    return out


def load(name, dialect):
    z = np.load(os.path.join(GOLDEN, "%s.%s.npz" % (name, dialect)))
    return {key: z[key] for key in z.files}


def dense_expected(g, k):
    """(4^k, n) GPU-layout histogram and bin 0 of the fixture."""
    n = int(g["n_seqs"])
    out = np.zeros((1 << (2 * k), n), dtype=np.int32)
    out[g["k%d_code" % k], g["k%d_rec" % k]] = g["k%d_count" % k]
    return out, g["k%d_invalid" % k]


def full_indices(g):
    """indexes_aux with the end sentinel (absent after a trailing blank line)."""
    idx = g["indexes"].astype(np.int64)
    n = int(g["n_seqs"])
    if idx.size == n:
        idx = np.append(idx, np.int64(g["data"].size))
    return idx


def random_fasta(rng, path, nrec_max=12):
    """A small FASTA with the structures the reference's loader distinguishes:
    blank lines between and inside records, headers, CRLF and '\r'-initial lines,
    lowercase, N, '|', empty sequence lines, optionally no final newline."""
    parts = []
    for i in range(int(rng.integers(1, nrec_max))):
        if rng.random() < 0.1:
            parts.append("\n")
        parts.append(">rec%d %s\n" % (i, "x" * int(rng.integers(0, 5))))
        if rng.random() < 0.1:
            parts.append("\n")
        for _ in range(int(rng.integers(0, 5))):
            L = int(rng.integers(0, 90))
            s = "".join(rng.choice(list("ACGTNacgt|"), size=L, p=[.21, .21, .21, .21, .06, .02, .02, .02, .02, .02]))
            eol = "\r\n" if rng.random() < 0.1 else "\n"
            parts.append(s + eol)
        if rng.random() < 0.7:
            parts.append("\r\n" if rng.random() < 0.2 else "\n")
    txt = "".join(parts)
    if rng.random() < 0.3:
        txt = txt.rstrip("\n")
    with open(path, "w", newline="") as f:
        f.write(txt)
