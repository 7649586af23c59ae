#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the reference itself.

Run in the build container (where /root/reference exists) after
`make -C oracle ref`:

    python tests/golden/make_golden.py

Inputs are small synthetic FASTA files written by this script (seeded, so the
files are reproducible; they are committed next to their outputs).  Outputs are
produced by oracle/_ref/libref_cpu.so, i.e. by the reference's own
importSeqs / importSeqsNoNL (main.cu:474-530 / 401-458) and
permutationsCountAll (main.cu:636-646) compiled from /root/reference.  The
fixtures are data only: each <case>.<dialect>.npz holds

    n_seqs          number of records the loader produced
    indexes         indexes_aux exactly as the loader left it (int64)
    data            the '\\0'-separated device buffer bytes (uint8)
    ks              k values counted
    k{k}_rec/_code/_count   nonzero GPU-layout bins (record, LE code, count)
    k{k}_invalid    CPU bin 0 per record
    k{k}_dist       sequentialKmerCount2's packed upper-triangle distances
                    (main.cu:587-621), float32, n(n-1)/2 entries
and patterns_k{k}.npy holds the bin-order table of permutation() for small k.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(REPO, "oracle", "_ref", "libref_cpu.so")


def wrap80(seq, width=80):
    return [seq[i:i + width] for i in range(0, len(seq), width)] or [""]


def rand_bases(rng, n, n_frac=0.0, lower_frac=0.0):
    s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n)
    if n_frac > 0:
        m = rng.random(n) < n_frac
        s[m] = ord("N")
    if lower_frac > 0:
        m = rng.random(n) < lower_frac
        s[m] = s[m] | 0x20
    return s.tobytes().decode()


def fasta_blank(records, eol="\n", sep_line="", trailing_blank=False):
    """importSeqs dialect: records separated by a blank line, none at the end."""
    out = []
    for i, (hdr, seq) in enumerate(records):
        out.append(">" + hdr + eol)
        for line in wrap80(seq):
            out.append(line + eol)
        if i != len(records) - 1 or trailing_blank:
            out.append(sep_line + "\n")
    return "".join(out)


def fasta_standard(records, final_newline=True):
    out = []
    for hdr, seq in records:
        out.append(">" + hdr + "\n")
        out.extend(line + "\n" for line in wrap80(seq))
    txt = "".join(out)
    return txt if final_newline else txt.rstrip("\n")


def make_cases():
    rng = np.random.default_rng(0x5EED)
    cases = {}
    # 1. mixed content: N runs, lowercase, a '|' byte, records shorter than k
    recs = [
        ("r0 plain", rand_bases(rng, 1500)),
        ("r1 N and lowercase", rand_bases(rng, 333, 0.02, 0.02) + "NNNNNN" + rand_bases(rng, 90)),
        ("r2 eighty", rand_bases(rng, 80)),
        ("r3 bar", rand_bases(rng, 40) + "|" + rand_bases(rng, 41)),
        ("r4 two", "AC"),
        ("r5 three", "GTA"),
        ("r6 polyA", "A" * 300 + "C" * 20 + "A" * 170),
        ("r7 seven", "ACGTTGC"),
    ]
    cases["basic"] = fasta_blank(recs)
    # 2. CRLF file: every line ends in '\r' (kept in the record), separators are "\r"
    recs = [("c%d" % i, rand_bases(rng, 200 + 37 * i)) for i in range(3)]
    cases["crlf"] = fasta_blank(recs, eol="\r\n", sep_line="\r")
    # 3. MAX_SEQS cap with multi-line records: 105 records of 3 lines
    recs = [("m%03d" % i, rand_bases(rng, 200)) for i in range(105)]
    cases["maxseqs"] = fasta_blank(recs)
    # 4. MAX_SEQS with single-line records (the cap is only checked after a second line)
    recs = [("s%03d" % i, rand_bases(rng, 60)) for i in range(110)]
    cases["maxseqs_single"] = fasta_blank(recs)
    # 5. standard FASTA (no blank lines, no final newline): one record under importSeqs
    recs = [("std%d" % i, rand_bases(rng, 170 + 11 * i, 0.01)) for i in range(4)]
    cases["standard"] = fasta_standard(recs, final_newline=False)
    # 6. trailing blank line: the end sentinel is not pushed
    recs = [("t%d" % i, rand_bases(rng, 150)) for i in range(3)]
    cases["trailing_blank"] = fasta_blank(recs, trailing_blank=True)
    # 7. odd structure: blank line after a header, header without sequence,
    #    sequence lines with no header, leading blank lines
    cases["odd"] = (
        "\n\n>h0\n\nACGTACGTAC\nGGTTAACC\n\n>h1 no seq\n>h2\nTTTTGGGGCCCCAAAA\n\n"
        "ACGTNNNN\nACGT\n\n>h3\nacgtACGTacgt\nACGT\n")
    # 8. longer random records for larger k (0.1% N, 0.1% lowercase)
    recs = [("g%d" % i, rand_bases(rng, 6000 + 1000 * i, 0.001, 0.001)) for i in range(3)]
    cases["random"] = fasta_blank(recs)
    return cases


KS_ALL = (1, 2, 3, 4, 5)
KS_BIG = {"basic": (8, 13), "random": (8, 11, 12, 13), "crlf": (8,)}


def main():
    if not os.path.exists(LIB):
        sys.exit("build the reference harness first: make -C oracle ref")
    lib = ctypes.CDLL(LIB)
    lib.ref_import.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.ref_num_indexes.restype = ctypes.c_long
    lib.ref_data_size.restype = ctypes.c_long
    lib.ref_record_size.restype = ctypes.c_long
    lib.ref_seq_distances.argtypes = [ctypes.c_int, ctypes.c_void_p]

    for k in range(1, 6):
        buf = ctypes.create_string_buffer((1 << (2 * k)) * k)
        lib.ref_patterns(k, buf)
        pats = np.frombuffer(buf.raw, dtype=np.uint8).reshape(1 << (2 * k), k)
        np.save(os.path.join(HERE, "patterns_k%d.npy" % k), pats)

    for name, text in make_cases().items():
        fa = os.path.join(HERE, name + ".fa")
        with open(fa, "w", newline="") as f:
            f.write(text)
        for dialect, nonl in (("blank", 0), ("nonl", 1)):
            n = lib.ref_import(fa.encode(), nonl)
            assert n >= 0
            ni = lib.ref_num_indexes()
            idx = (ctypes.c_longlong * max(ni, 1))()
            lib.ref_get_indexes(idx)
            indexes = np.array(idx[:ni], dtype=np.int64)
            dsz = lib.ref_data_size()
            dbuf = ctypes.create_string_buffer(max(dsz, 1))
            lib.ref_get_data(dbuf)
            data = np.frombuffer(dbuf.raw[:dsz], dtype=np.uint8).copy()
            out = {"n_seqs": np.int64(n), "indexes": indexes, "data": data}
            ks = KS_ALL + KS_BIG.get(name, ())
            out["ks"] = np.array(ks, dtype=np.int64)
            for k in ks:
                nb = 1 << (2 * k)
                hist = (ctypes.c_int * (nb + 1))()
                recs, codes, counts, invalid = [], [], [], []
                for s in range(n):
                    lib.ref_count_record(s, k, hist)
                    h = np.frombuffer(hist, dtype=np.int32)
                    nz = np.nonzero(h[1:])[0]
                    recs.append(np.full(nz.size, s, dtype=np.int64))
                    codes.append(nz.astype(np.int64))
                    counts.append(h[1:][nz].astype(np.int32))
                    invalid.append(int(h[0]))
                out["k%d_rec" % k] = np.concatenate(recs) if recs else np.zeros(0, np.int64)
                out["k%d_code" % k] = np.concatenate(codes) if codes else np.zeros(0, np.int64)
                out["k%d_count" % k] = np.concatenate(counts) if counts else np.zeros(0, np.int32)
                out["k%d_invalid" % k] = np.array(invalid, dtype=np.int32)
                dist = np.zeros(max(n * (n - 1) // 2, 1), dtype=np.float32)
                lib.ref_seq_distances(k, dist.ctypes.data)
                out["k%d_dist" % k] = dist[: n * (n - 1) // 2]
            np.savez_compressed(os.path.join(HERE, "%s.%s.npz" % (name, dialect)), **out)
            print("%-15s %-5s n=%3d indexes=%3d bytes=%d ks=%s" % (name, dialect, n, ni, dsz, ks))


if __name__ == "__main__":
    main()
