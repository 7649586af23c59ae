"""oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes bindings for the C restatement (libkmc_oracle.so) and for the reference
build (oracle/_ref/libref_cpu.so, libref_kernel.so), plus a tiny pure-Python
restatement used to cross-check the C one on small inputs.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")

_P = ctypes.c_void_p
_I64 = ctypes.c_int64


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def build(ref=None):
    """Build libkmc_oracle.so (and oracle/_ref when the reference tree exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if ref is None:
        ref = os.path.isdir("/root/reference")
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("KMC_ORACLE_LIB") or os.path.join(HERE, "libkmc_oracle.so")
        if not os.path.exists(path):
            build(ref=False)
        L = ctypes.CDLL(path)
        L.oracle_count_record_cpu.argtypes = [_P, _I64, ctypes.c_int, _P]
        L.oracle_count_dense.argtypes = [_P, _P, _I64, ctypes.c_int, _P, _I64, _P]
        L.oracle_count_dense_range.argtypes = [_P, _P, _I64, ctypes.c_int, _I64, _I64, _P, _I64, _P]
        L.oracle_window_code.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.oracle_window_code.restype = _I64
        L.oracle_pair_distances.argtypes = [_P, _P, _I64, ctypes.c_int, _P]
        L.oracle_count_canonical.restype = _I64
        L.oracle_count_canonical.argtypes = [_P, _P, _I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P]
        L.oracle_min_kmeres2_row.argtypes = [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]
        L.oracle_dg_hash.restype = ctypes.c_uint64
        L.oracle_dg_hash.argtypes = [ctypes.c_uint64]
        L.oracle_canonical_digest.restype = _I64
        L.oracle_canonical_digest.argtypes = [_P, _I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_uint64, _P, _P, _P, _P, _I64]
        _lib = L
    return _lib


def count_dense(data, indices, k, win=None):
    """GPU-layout histogram sum[code, s] (returned as a (4^k, n) int32 array) and
    the CPU path's bin 0 per record.  `data` uint8, `indices` int64 (n+1)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    indices = np.ascontiguousarray(indices, dtype=np.int64)
    n = indices.size - 1
    nb = 1 << (2 * k)
    out = np.zeros((nb, max(n, 0)), dtype=np.int32)
    inv = np.zeros(max(n, 0), dtype=np.int32)
    if n <= 0:
        return out, inv
    dptr = _ptr(data) if data.size else None
    if win is None:
        lib().oracle_count_dense(dptr, _ptr(indices), n, k, _ptr(out), n, _ptr(inv))
    else:
        lib().oracle_count_dense_range(dptr, _ptr(indices), n, k, int(win[0]), int(win[1]),
                                       _ptr(out), n, _ptr(inv))
    return out, inv


def pair_distances(sum_, lens, k):
    sum_ = np.ascontiguousarray(sum_, dtype=np.int32)
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    n = lens.size
    out = np.zeros(max(n * (n - 1) // 2, 1), dtype=np.float32)
    lib().oracle_pair_distances(_ptr(sum_), _ptr(lens), n, k, _ptr(out))
    return out[: n * (n - 1) // 2]


def count_canonical(data, indices, k, soft=False, forward=False):
    """Self-oracle of kmc_count_canonical_hash: (keys u64, counts u32, rec_off u64),
    keys sorted ascending within each record."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    indices = np.ascontiguousarray(indices, dtype=np.int64)
    n = indices.size - 1
    cap = max(int(indices[-1] - indices[0]) if n > 0 else 0, 1)
    keys = np.zeros(cap, dtype=np.uint64)
    counts = np.zeros(cap, dtype=np.uint32)
    off = np.zeros(n + 1, dtype=np.uint64)
    dptr = _ptr(data) if data.size else None
    tot = lib().oracle_count_canonical(dptr, _ptr(indices), n, k, int(soft), int(forward),
                                       _ptr(keys), _ptr(counts), _ptr(off))
    return keys[:tot], counts[:tot], off


DIGEST_SEL_BITS = 12  # the selected subset: top 12 bits of dg_hash(key) == sel_val (1 key in 4 096)


def canonical_digest(data, indices, k, soft=False, forward=False, sel_val=0, sel_bits=DIGEST_SEL_BITS,
                     threads=16):
    """oracle_canonical_digest over every record (records in parallel: ctypes drops
    the GIL).  Returns a list of per-record dicts {valid, digest (uint64 as int),
    keys (uint64, sorted), counts (uint32)}: the full-size check of the canonical
    path (tests/test_canonical_full_size_gpu.py)."""
    from concurrent.futures import ThreadPoolExecutor
    data = np.ascontiguousarray(data, dtype=np.uint8)
    indices = np.ascontiguousarray(indices, dtype=np.int64)
    n = indices.size - 1
    shift = 64 - sel_bits
    base = data.ctypes.data

    def one(s):
        a, E = int(indices[s]), int(indices[s + 1] - indices[s])
        cap = max(E // (1 << sel_bits) * 2 + 4096, 1)
        while True:
            keys = np.zeros(cap, dtype=np.uint64)
            counts = np.zeros(cap, dtype=np.uint32)
            nv, dg = ctypes.c_uint64(0), ctypes.c_uint64(0)
            d = lib().oracle_canonical_digest(ctypes.c_void_p(base + a) if E else None, E, k, int(soft),
                                              int(forward), shift, sel_val, ctypes.byref(nv), ctypes.byref(dg),
                                              _ptr(keys), _ptr(counts), cap)
            if d >= 0:
                return {"valid": nv.value, "digest": dg.value, "keys": keys[:d], "counts": counts[:d]}
            cap *= 4

    order = sorted(range(n), key=lambda s: -int(indices[s + 1] - indices[s]))  # longest first
    with ThreadPoolExecutor(max(1, min(threads, n))) as ex:
        res = dict(zip(order, ex.map(one, order)))
    return [res[s] for s in range(n)]


def dg_hash(x):
    """oracle_dg_hash on a numpy uint64 array (splitmix64's finaliser)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def min_kmeres2_row(sum_, indexes, cur, k, out=None):
    """GPU step-2 semantics (float accumulation) for row `cur`; fills `out`."""
    sum_ = np.ascontiguousarray(sum_, dtype=np.int32)
    indexes = np.ascontiguousarray(indexes, dtype=np.int32)
    n = indexes.size - 1
    if out is None:
        out = np.zeros(max(n * (n - 1) // 2, 1), dtype=np.float32)
    lib().oracle_min_kmeres2_row(_ptr(sum_), _ptr(indexes), n, cur, k, _ptr(out))
    return out


def py_count_record(rec: bytes, k: int):
    """Pure-Python restatement (small inputs only): CPU layout, bin 0 = invalid."""
    code = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}
    hist = [0] * ((1 << (2 * k)) + 1)
    E = len(rec)  # record bytes + terminator
    for i in range(max(0, E - k)):
        c = 0
        for q in range(k):
            b = code.get(rec[i + q])
            if b is None:
                c = -1
                break
            c |= b << (2 * q)
        hist[c + 1 if c >= 0 else 0] += 1
    return hist


# --------------------------------------------------------------------------
# oracle/_ref: the reference's own code, compiled from /root/reference.
# --------------------------------------------------------------------------
_ref_cpu = None


def have_ref_cpu():
    return os.path.exists(os.path.join(REF_DIR, "libref_cpu.so"))


def ref_cpu():
    global _ref_cpu
    if _ref_cpu is None:
        L = ctypes.CDLL(os.path.join(REF_DIR, "libref_cpu.so"))
        L.ref_import.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.ref_num_indexes.restype = ctypes.c_long
        L.ref_data_size.restype = ctypes.c_long
        L.ref_count_bytes.argtypes = [_P, ctypes.c_long, ctypes.c_int, _P]
        L.ref_build_map.argtypes = [ctypes.c_int]
        _ref_cpu = L
    return _ref_cpu


def ref_import(path, nonl=False):
    """Reference loader -> (n_seqs, indexes_aux (raw), data bytes)."""
    L = ref_cpu()
    n = L.ref_import(path.encode(), 1 if nonl else 0)
    if n < 0:
        raise FileNotFoundError(path)
    ni = L.ref_num_indexes()
    idx = (ctypes.c_longlong * max(ni, 1))()
    L.ref_get_indexes(idx)
    dsz = L.ref_data_size()
    buf = ctypes.create_string_buffer(max(dsz, 1))
    L.ref_get_data(buf)
    return n, np.array(idx[:ni], dtype=np.int64), np.frombuffer(buf.raw[:dsz], dtype=np.uint8).copy()


def ref_seq_distances(path, k, nonl=False):
    """sequentialKmerCount2 (main.cu:587-621) on the file's records, as imported by
    the reference loader: packed upper-triangle float32 distances."""
    L = ref_cpu()
    n, _, _ = ref_import(path, nonl)
    out = np.zeros(max(n * (n - 1) // 2, 1), dtype=np.float32)
    L.ref_seq_distances.argtypes = [ctypes.c_int, _P]
    L.ref_seq_distances(k, _ptr(out))
    return out[: n * (n - 1) // 2]


def ref_count_bytes(rec: np.ndarray, k: int):
    """permutationsCountAll on one record (bytes incl. terminator): CPU layout."""
    L = ref_cpu()
    L.ref_build_map(k)
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    out = np.zeros((1 << (2 * k)) + 1, dtype=np.int32)
    L.ref_count_bytes(_ptr(rec), rec.size, k, _ptr(out))
    return out


_ref_kernel = None


def have_ref_kernel():
    return os.path.exists(os.path.join(REF_DIR, "libref_kernel.so"))


def ref_kernel():
    global _ref_kernel
    if _ref_kernel is None:
        import torch  # noqa: F401  (one HIP runtime per process: torch's, see kmc._load)
        L = ctypes.CDLL(os.path.join(REF_DIR, "libref_kernel.so"))
        L.ref_kernel_launch.argtypes = [_P, _P, ctypes.c_uint, _P]
        L.ref_min_kmeres2_launch.argtypes = [_P, _P, ctypes.c_int, ctypes.c_int, _P]
        _ref_kernel = L
    return _ref_kernel
