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
