"""kmc.py — Python binding of libkmc.so (the C ABI in include/kmc.h).

The product is the HIP/C++ library; this module only marshals pointers for the
tests, the benchmark and Python callers.  Device buffers are torch tensors
(PyTorch is the allocator/stream provider here, nothing else).  There is no CPU
fallback: every entry point raises if libkmc.so is missing or a call fails.

Reference interface mirrored (axlwild/dna-kmeres-parallel):
    sumKmereCoincidencesGlobalMemory(data, indices, num_seqs, sum)  kernels.h:113
        -> dropin_count(data, indices_i32, num_seqs)
    permutationsCountAll generalised to any k, GPU layout           main.cu:636-646
        -> count_dense(data, indices, k)
    importSeqs / importSeqsNoNL                                     main.cu:474-545 / 401-473
        -> load_fasta(path, dialect)
"""
import ctypes
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.environ.get("KMC_LIB") or os.path.join(HERE, "lib", "libkmc.so")
# the diagnostic build (test hooks kmc_diag_*, see diag()); never used by the product path
DIAG_LIB_PATH = os.environ.get("KMC_DIAG_LIB") or os.path.join(HERE, "lib", "libkmc_diag.so")
HEADER = os.path.join(REPO, "include", "kmc.h")

DIALECT_BLANK = 0  # importSeqs
DIALECT_NONL = 1   # importSeqsNoNL
MAX_SEQS_REFERENCE = 100
DROPIN_K = 3
KMC_ERR_CAPACITY = 1009
KMC_ERR_RECORD_TOO_LONG = 1010
KMC_ERR_INTERNAL = 1011


class KmcError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__("%s failed: %s (%d)" % (what, error_string(code), code))


_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_I64 = ctypes.c_int64


class DenseArgs(ctypes.Structure):
    _fields_ = [
        ("data", _P), ("indices", _P), ("num_seqs", _U64), ("k", ctypes.c_int),
        ("sum", _P), ("sum_ld", _U64), ("invalid", _P),
        ("read_lo", _U64), ("read_hi", _U64), ("win_lo", _U64), ("win_hi", _U64),
        ("workspace", _P), ("workspace_bytes", ctypes.c_size_t), ("status", _P),
    ]


_lib = None
_diag_lib = None
_active = None  # the diagnostic library while inside diag()


def lib():
    """Load libkmc.so (built in-tree by `make -C dna-kmeres-parallel_amd`)."""
    global _lib
    if _active is not None:
        return _active
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


class diag:
    """Context manager: inside it every binding calls lib/libkmc_diag.so, the same
    library built with the test hooks (kmc_diag_radix_mode, kmc_diag_canon_claim_cap,
    kmc_diag_canon_sort_cap, kmc_diag_dense_spill_cap) that force an algorithm
    choice (kmc_diag_canon_sort_cap_big, kmc_diag_canon_direct too); libkmc.so
    exports none of them.  `with kmc.diag() as D: D.kmc_diag_...`"""

    def __enter__(self):
        global _diag_lib, _active
        if _diag_lib is None:
            _diag_lib = _load(DIAG_LIB_PATH)
            _diag_lib.kmc_diag_radix_mode.argtypes = [ctypes.c_int, ctypes.c_float]
            _diag_lib.kmc_diag_canon_claim_cap.argtypes = [ctypes.c_uint]
            _diag_lib.kmc_diag_canon_sort_cap.argtypes = [ctypes.c_uint]
            _diag_lib.kmc_diag_canon_sort_cap_big.argtypes = [ctypes.c_uint]
            _diag_lib.kmc_diag_canon_direct.argtypes = [ctypes.c_int]
            _diag_lib.kmc_diag_canon_fallback.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)] * 2
            _diag_lib.kmc_diag_canon_fallback_detail.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_uint,
                                                                 ctypes.POINTER(ctypes.c_ulonglong)]
            _diag_lib.kmc_diag_dense_spill_cap.argtypes = [ctypes.c_uint]
            _diag_lib.kmc_diag_canon_stale_queue.argtypes = [ctypes.c_longlong]
        self._prev = _active
        _active = _diag_lib
        return _diag_lib

    def __exit__(self, *exc):
        global _active
        L = _active
        # restore the defaults for the next user of the diagnostic library
        L.kmc_diag_radix_mode(0, 1.0)
        L.kmc_diag_canon_claim_cap(0)
        L.kmc_diag_canon_sort_cap(1 << 30)  # (also restores the big instance's cap)
        L.kmc_diag_canon_direct(1)
        L.kmc_diag_dense_spill_cap(0)
        L.kmc_diag_canon_stale_queue(-1)
        _active = self._prev
        return False


def hip_runtimes():
    """Paths of the HIP runtime libraries (libamdhip64) mapped into this process."""
    with open("/proc/self/maps") as f:
        return sorted(set(line.split()[-1] for line in f if "/libamdhip64.so" in line))


def _load(path):
    """One HIP runtime per process: torch ships its own libamdhip64 (torch/lib),
    libkmc.so names the SONAME libamdhip64.so.7 (found through its RUNPATH in
    /opt/rocm/lib).  The dynamic loader satisfies a NEEDED entry with an already
    loaded library of that SONAME, so torch is imported FIRST (when it is
    installed) and libkmc then binds to torch's runtime; loaded the other way
    round, both runtimes would be mapped and each would initialise the GPU on its
    own.  A second runtime mapped anyway is refused here."""
    if not os.path.exists(path):
        raise RuntimeError("%s not built: run `make -C %s` (no CPU fallback exists)" % (os.path.basename(path), HERE))
    # KMC_NO_TORCH=1: host-only use of the binding (loader, shard planner) without
    # paying torch's import; such a process must then not import torch at all
    if os.environ.get("KMC_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401  (maps torch's HIP runtime before libkmc's NEEDED entry is resolved)
        except ImportError:
            pass
    L = ctypes.CDLL(path)
    rt = hip_runtimes()
    if len(rt) > 1:
        raise RuntimeError("two HIP runtimes are mapped in this process (%s): each would initialise the GPU on its "
                           "own, so %s is refused; import torch before loading it (or set KMC_NO_TORCH=1 only in "
                           "processes that never import torch)" % (", ".join(rt), os.path.basename(path)))
    L.kmc_error_string.restype = ctypes.c_char_p
    L.kmc_error_string.argtypes = [ctypes.c_int]
    L.kmc_version.restype = ctypes.c_int
    L.kmc_version.argtypes = []
    L.sumKmereCoincidencesGlobalMemory_hip.argtypes = [_P, _P, ctypes.c_uint, _P, _P]
    L.kmc_count_dense_workspace_size.restype = ctypes.c_size_t
    L.kmc_count_dense_workspace_size.argtypes = [ctypes.c_int, _U64, _U64, ctypes.c_int]
    L.kmc_count_dense.argtypes = [_P, _P, _U64, _U64, ctypes.c_int, _P, _P, _P, ctypes.c_size_t, _P]
    L.kmc_count_dense_ex.argtypes = [ctypes.POINTER(DenseArgs), _P]
    L.kmc_count_dense_ex_workspace_size.restype = ctypes.c_size_t
    L.kmc_count_dense_ex_workspace_size.argtypes = [ctypes.POINTER(DenseArgs), ctypes.c_int]
    L.kmc_dense_status.argtypes = [ctypes.c_int]
    L.kmc_trace_set_events.argtypes = [_P, _P]
    L.kmc_set_reserved_cus.argtypes = [ctypes.c_int]
    L.kmc_plan_shards.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_int, _U64, _P]
    L.kmc_count_multi.argtypes = [_P, _P, _U64, _U64, ctypes.c_int, ctypes.c_int, _P, _P, _P]
    L.kmc_multi_release.argtypes = []
    L.kmc_synth_fill.argtypes = [_P, _U64, _U64, _U64, _U64, _P]
    L.kmc_synth_fill_range.argtypes = [_P, _U64, _U64, _U64, _U64, _P]
    L.kmc_synth_indices.argtypes = [_P, _U64, _U64]
    L.kmc_synth_indices.restype = None
    L.kmc_fasta_load.argtypes = [ctypes.c_char_p, ctypes.c_int, _I64, ctypes.POINTER(_P)]
    for fn in ("kmc_fasta_num_seqs", "kmc_fasta_data_bytes", "kmc_fasta_reference_num_indexes"):
        getattr(L, fn).restype = _U64
        getattr(L, fn).argtypes = [_P]
    L.kmc_fasta_indices.restype = _P
    L.kmc_fasta_indices.argtypes = [_P]
    L.kmc_fasta_data.restype = _P
    L.kmc_fasta_data.argtypes = [_P]
    L.kmc_fasta_free.argtypes = [_P]
    L.kmc_fasta_free.restype = None
    L.kmc_fasta_parse_device.argtypes = [_P, _U64, ctypes.c_int, _P, _U64, _P, _U64, ctypes.POINTER(_U64),
                                         ctypes.POINTER(_U64), _P]
    L.kmc_fasta_load_device.argtypes = [ctypes.c_char_p, ctypes.c_int, _I64, ctypes.POINTER(_P),
                                        ctypes.POINTER(_U64), ctypes.POINTER(_P), ctypes.POINTER(_U64), _P]
    L.kmc_pair_distances_workspace_size.restype = ctypes.c_size_t
    L.kmc_pair_distances_workspace_size.argtypes = [_U64, ctypes.c_int, ctypes.c_int]
    L.kmc_pair_distances.argtypes = [_P, _U64, _P, _U64, ctypes.c_int, _P, _P, ctypes.c_size_t, _P]
    L.minKmeres2_hip.argtypes = [_P, _P, ctypes.c_int, ctypes.c_int, _P, _P]
    L.kmc_count_canonical_hash.argtypes = [_P, _P, _U64, ctypes.c_int, ctypes.c_uint, _P, _P, _U64, _P,
                                           ctypes.POINTER(_U64), _P]
    L.kmc_count_canonical_hash_ex.argtypes = [_P, _P, _U64, ctypes.c_int, ctypes.c_uint, _P, _P, _U64, _P,
                                              ctypes.POINTER(_U64), _P, ctypes.c_size_t, _P]
    L.kmc_count_canonical_workspace_size.restype = ctypes.c_size_t
    L.kmc_count_canonical_workspace_size.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_int]
    return L


def error_string(code):
    return lib().kmc_error_string(int(code)).decode()


def _check(rc, what):
    if rc != 0:
        raise KmcError(rc, what)


def header_symbols(path=HEADER):
    """Function names declared by include/kmc.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", txt, flags=re.M)
    return sorted(set(n for n in names if n not in ("defined",)))


# ---------------------------------------------------------------------------
# device entry points (torch tensors on cuda)
# ---------------------------------------------------------------------------
def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def dropin_count(data, indices, num_seqs=None, out=None, stream=None):
    """Exact drop-in of the reference launch (k = 3): returns int32 sum[4^3 * n]
    in the reference layout sum[s + n*code] (flat, like the reference)."""
    import torch
    n = int(num_seqs if num_seqs is not None else indices.numel() - 1)
    if out is None:
        out = torch.empty((1 << (2 * DROPIN_K)) * n, dtype=torch.int32, device=data.device)
    rc = lib().sumKmereCoincidencesGlobalMemory_hip(_dptr(data), _dptr(indices), n, _dptr(out), _stream(stream))
    _check(rc, "sumKmereCoincidencesGlobalMemory_hip")
    return out


def dense_workspace_size(k, num_seqs, data_bytes, device=0):
    return int(lib().kmc_count_dense_workspace_size(k, num_seqs, data_bytes, device))


def count_dense(data, indices, k, data_bytes=None, invalid=False, workspace=None, out=None, stream=None):
    """k-mer histogram of every record: returns (sum (4^k, n) int32, invalid (n,) or None)."""
    import torch
    n = indices.numel() - 1
    nb = 1 << (2 * k)
    if data_bytes is None:
        data_bytes = data.numel()
    if out is None:
        out = torch.empty((nb, n), dtype=torch.int32, device=data.device)
    inv = torch.empty(n, dtype=torch.int32, device=data.device) if invalid else None
    ws_ptr, ws_bytes = None, 0
    if workspace is not None:
        ws_ptr, ws_bytes = _dptr(workspace), workspace.numel() * workspace.element_size()
    rc = lib().kmc_count_dense(_dptr(data), _dptr(indices), n, data_bytes, k, _dptr(out), _dptr(inv),
                               ws_ptr, ws_bytes, _stream(stream))
    _check(rc, "kmc_count_dense")
    return out, inv


def dense_args(data, indices, k, out, read=(0, None), win=(0, None), ld=0, invalid=None, workspace=None,
               data_offset=0, status=None):
    """Build a kmc_dense_args.  `data_offset` = global offset of data[0] (the data
    pointer handed to the library is data_ptr - data_offset).  `status`: an int32
    device tensor (zeroed by the caller) that receives this call's deferred status
    (see dense_status_check); None: the device's flag (kmc_dense_status)."""
    a = DenseArgs()
    a.data = ctypes.c_void_p(data.data_ptr() - data_offset)
    a.indices = ctypes.c_void_p(indices.data_ptr())
    a.num_seqs = indices.numel() - 1
    a.k = k
    a.sum = ctypes.c_void_p(out.data_ptr())
    a.sum_ld = ld
    a.invalid = _dptr(invalid)
    a.read_lo = read[0]
    a.read_hi = read[1] if read[1] is not None else data_offset + data.numel()
    a.win_lo = win[0]
    a.win_hi = win[1] if win[1] is not None else data_offset + data.numel()
    if workspace is not None:
        a.workspace = ctypes.c_void_p(workspace.data_ptr())
        a.workspace_bytes = workspace.numel() * workspace.element_size()
    a.status = _dptr(status)
    return a


def dense_status_check(status=None, device=None):
    """Raise KmcError for a failed asynchronous dense call (synchronises first):
    `status` = the call's own int32 status tensor, or None for the device's flag
    (kmc_dense_status, which it clears)."""
    import torch
    torch.cuda.synchronize()
    if status is not None:
        _check(int(status.reshape(-1)[0].item()), "dense count (deferred status)")
    else:
        dv = torch.cuda.current_device() if device is None else device
        _check(lib().kmc_dense_status(dv), "dense count (kmc_dense_status)")


def count_dense_ex(args, stream=None):
    rc = lib().kmc_count_dense_ex(ctypes.byref(args), _stream(stream))
    _check(rc, "kmc_count_dense_ex")


def dense_ex_workspace_size(args, device=0):
    return int(lib().kmc_count_dense_ex_workspace_size(ctypes.byref(args), device))


def pair_distances_workspace_size(num_seqs, k, device=0):
    return int(lib().kmc_pair_distances_workspace_size(num_seqs, k, device))


def pair_distances(counts, indices, k, num_seqs=None, ld=0, out=None, workspace=None, stream=None):
    """All-pairs k-mer distance (kmc_pair_distances): `counts` is the int32 count
    matrix sum[s + ld*code] (e.g. count_dense's (4^k, n) tensor), `indices` the
    device int64 offsets.  Returns float32 [n(n-1)/2], packed upper triangle."""
    import torch
    n = int(num_seqs if num_seqs is not None else indices.numel() - 1)
    if out is None:
        out = torch.empty(max(n * (n - 1) // 2, 0), dtype=torch.float32, device=counts.device)
    ws_ptr, ws_bytes = None, 0
    if workspace is not None:
        ws_ptr, ws_bytes = _dptr(workspace), workspace.numel() * workspace.element_size()
    rc = lib().kmc_pair_distances(_dptr(counts), ld, _dptr(indices), n, k, _dptr(out), ws_ptr, ws_bytes,
                                  _stream(stream))
    _check(rc, "kmc_pair_distances")
    return out


CANON_SOFTMASK = 1
CANON_FORWARD = 2
CANON_MAX_K = 31


def count_canonical(data, indices, k, flags=0, capacity=None, workspace=None, stream=None):
    """Canonical k-mer counts per record (kmc_count_canonical_hash[_ex]): returns
    (keys uint64 as int64 tensor, counts int32 tensor, rec_offsets int64 tensor);
    record s owns [rec_offsets[s], rec_offsets[s+1]), order within it unspecified.
    `workspace`: a caller device buffer of canonical_workspace_size() bytes (None:
    the library's own)."""
    import torch
    n = indices.numel() - 1
    if capacity is None:
        capacity = max(int(data.numel()), 1)
    keys = torch.empty(capacity, dtype=torch.int64, device=data.device)
    counts = torch.empty(capacity, dtype=torch.int32, device=data.device)
    off = torch.zeros(max(n + 1, 1), dtype=torch.int64, device=data.device)
    tot = _U64(0)
    if workspace is None:
        rc = lib().kmc_count_canonical_hash(_dptr(data), _dptr(indices), n, k, flags, _dptr(keys), _dptr(counts),
                                            capacity, _dptr(off), ctypes.byref(tot), _stream(stream))
    else:
        rc = lib().kmc_count_canonical_hash_ex(_dptr(data), _dptr(indices), n, k, flags, _dptr(keys),
                                               _dptr(counts), capacity, _dptr(off), ctypes.byref(tot),
                                               _dptr(workspace), workspace.numel() * workspace.element_size(),
                                               _stream(stream))
    _check(rc, "kmc_count_canonical_hash")
    t = int(tot.value)
    return keys[:t], counts[:t], off


def canonical_workspace_size(indices_host, k, device=0):
    """kmc_count_canonical_workspace_size for host int64 offsets (num_seqs + 1)."""
    idx = np.ascontiguousarray(indices_host, dtype=np.int64)
    return int(lib().kmc_count_canonical_workspace_size(idx.ctypes.data_as(_P), idx.size - 1, k, device))


def min_kmeres2(sums, mins, num_seqs, current_seq, indexes, stream=None):
    """Drop-in of one reference minKmeres2 launch (k = 3, int32 indexes)."""
    rc = lib().minKmeres2_hip(_dptr(sums), _dptr(mins), num_seqs, current_seq, _dptr(indexes), _stream(stream))
    _check(rc, "minKmeres2_hip")


def trace_events(before=None, after=None):
    """Record torch.cuda.Event `before`/`after` around the next dense count kernels."""
    b = ctypes.c_void_p(before._as_parameter_.value) if before is not None else None
    a = ctypes.c_void_p(after._as_parameter_.value) if after is not None else None
    _check(lib().kmc_trace_set_events(b, a), "kmc_trace_set_events")


def set_reserved_cus(n):
    """Leave n CUs out of the dense (k <= 8) grid, for a concurrent kernel (kmc.h)."""
    _check(lib().kmc_set_reserved_cus(int(n)), "kmc_set_reserved_cus")


def synth_fill(data, num_records, record_len, seed, first_base=0, stream=None):
    rc = lib().kmc_synth_fill(_dptr(data), num_records, record_len, seed, first_base, _stream(stream))
    _check(rc, "kmc_synth_fill")


def synth_fill_range(data, lo, hi, record_len, seed, stream=None):
    """Global bytes [lo, hi) of the synthetic record stream into data[0 .. hi-lo)."""
    rc = lib().kmc_synth_fill_range(_dptr(data), lo, hi, record_len, seed, _stream(stream))
    _check(rc, "kmc_synth_fill_range")


def synth_indices(num_records, record_len):
    out = np.zeros(num_records + 1, dtype=np.int64)
    lib().kmc_synth_indices(out.ctypes.data_as(_P), num_records, record_len)
    return out


# ---------------------------------------------------------------------------
# sharding (host planning; device work in kmc_dist.py / kmc_count_multi)
# ---------------------------------------------------------------------------
class Shard(ctypes.Structure):
    _fields_ = [("win_lo", _U64), ("win_hi", _U64), ("read_lo", _U64), ("read_hi", _U64)]


def plan_shards(indices, k, nshards, align=4096):
    """Byte-balanced shards of [indices[0], indices[-1]): list of (win_lo, win_hi, read_lo, read_hi)."""
    idx = np.ascontiguousarray(indices, dtype=np.int64)
    out = (Shard * nshards)()
    _check(lib().kmc_plan_shards(idx.ctypes.data_as(_P), idx.size - 1, k, nshards, align, out), "kmc_plan_shards")
    return [(s.win_lo, s.win_hi, s.read_lo, s.read_hi) for s in out]


def count_multi(data, indices, k, ndev=1, devices=None, invalid=False):
    """Single-process multi-GPU count of a host buffer (kmc_count_multi: shards + RCCL all-reduce)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    idx = np.ascontiguousarray(indices, dtype=np.int64)
    n = idx.size - 1
    out = np.zeros((1 << (2 * k), n), dtype=np.int32)
    inv = np.zeros(n, dtype=np.int32) if invalid else None
    devs = None
    if devices is not None:
        devs = (ctypes.c_int * ndev)(*devices)
    rc = lib().kmc_count_multi(data.ctypes.data_as(_P), idx.ctypes.data_as(_P), n, data.size, k, ndev, devs,
                               out.ctypes.data_as(_P), inv.ctypes.data_as(_P) if inv is not None else None)
    _check(rc, "kmc_count_multi")
    return out, inv


# ---------------------------------------------------------------------------
# host: FASTA loader
# ---------------------------------------------------------------------------
def load_fasta(path, dialect=DIALECT_BLANK, max_seqs=MAX_SEQS_REFERENCE):
    """Returns (data uint8, indices int64 [n+1], reference_num_indexes)."""
    L = lib()
    h = _P()
    _check(L.kmc_fasta_load(os.fsencode(path), dialect, max_seqs, ctypes.byref(h)), "kmc_fasta_load")
    try:
        n = L.kmc_fasta_num_seqs(h)
        nbytes = L.kmc_fasta_data_bytes(h)
        idx = np.ctypeslib.as_array(ctypes.cast(L.kmc_fasta_indices(h), ctypes.POINTER(_I64)), (n + 1,)).copy()
        if nbytes:
            data = np.ctypeslib.as_array(ctypes.cast(L.kmc_fasta_data(h), ctypes.POINTER(ctypes.c_uint8)),
                                         (nbytes,)).copy()
        else:
            data = np.zeros(0, dtype=np.uint8)
        ref_n = L.kmc_fasta_reference_num_indexes(h)
    finally:
        L.kmc_fasta_free(h)
    return data, idx, int(ref_n)


def parse_fasta_device(raw, dialect=DIALECT_BLANK, stream=None):
    """GPU FASTA parse (kmc_fasta_parse_device) of raw file bytes in a uint8 device
    tensor; returns (data uint8 tensor, indices int64 tensor [n+1]) on its device."""
    import torch
    n = int(raw.numel())
    if n % 16 or raw.data_ptr() % 16:  # the kernel reads whole 16-byte pieces of raw
        pad = torch.zeros(n + 16 - n % 16, dtype=torch.uint8, device=raw.device)
        pad[:n] = raw
        raw = pad
    data = torch.empty(n + 16, dtype=torch.uint8, device=raw.device)
    cap = 1024
    while True:
        idx = torch.empty(cap, dtype=torch.int64, device=raw.device)
        ns, nb = _U64(0), _U64(0)
        rc = lib().kmc_fasta_parse_device(_dptr(raw) if n else None, n, dialect, _dptr(data), n + 16, _dptr(idx),
                                          cap, ctypes.byref(ns), ctypes.byref(nb), _stream(stream))
        if rc == KMC_ERR_CAPACITY and ns.value + 1 > cap:
            cap = int(ns.value) + 1
            continue
        _check(rc, "kmc_fasta_parse_device")
        return data[:nb.value], idx[:ns.value + 1]


def load_fasta_device(path, dialect=DIALECT_BLANK, max_seqs=MAX_SEQS_REFERENCE, stream=None):
    """kmc_fasta_load_device: (data uint8 tensor, indices int64 tensor [n+1]) on the
    current device (copies of the library's buffers, which are freed here)."""
    import torch
    L = lib()
    d, ix = _P(), _P()
    nb, ns = _U64(0), _U64(0)
    _check(L.kmc_fasta_load_device(os.fsencode(path), dialect, max_seqs, ctypes.byref(d), ctypes.byref(nb),
                                   ctypes.byref(ix), ctypes.byref(ns), _stream(stream)), "kmc_fasta_load_device")
    dev = torch.device("cuda", torch.cuda.current_device())
    data = torch.empty(nb.value, dtype=torch.uint8, device=dev)
    idx = torch.empty(ns.value + 1, dtype=torch.int64, device=dev)
    hip = _hip()
    if nb.value:
        _check(hip.hipMemcpy(_P(data.data_ptr()), d, nb.value, 3), "hipMemcpy")
    _check(hip.hipMemcpy(_P(idx.data_ptr()), ix, (ns.value + 1) * 8, 3), "hipMemcpy")
    hip.hipFree(d)
    hip.hipFree(ix)
    return data, idx


_hip_lib = None


def _hip():
    global _hip_lib
    if _hip_lib is None:
        _hip_lib = ctypes.CDLL("libamdhip64.so.7")  # by SONAME: the runtime libkmc.so is bound to
        _hip_lib.hipMemcpy.argtypes = [_P, _P, ctypes.c_size_t, ctypes.c_int]
        _hip_lib.hipFree.argtypes = [_P]
    return _hip_lib


# ---------------------------------------------------------------------------
# host reference of the synthetic generator (tests compare the kernel to it)
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def splitmix64_np(seed, n):
    """Outputs n of splitmix64 (numpy uint64 array in, array out)."""
    n = np.asarray(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (n + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_host_range(lo, hi, record_len, seed):
    """Same bytes as kmc_synth_fill_range, on the host (small sizes)."""
    p = np.arange(lo, hi, dtype=np.uint64)
    rb = np.uint64(record_len + 1)
    r, off = p // rb, p % rb
    g = r * np.uint64(record_len) + off
    words = splitmix64_np(seed, g >> np.uint64(5))
    codes = ((words >> (np.uint64(2) * (g & np.uint64(31)))) & np.uint64(3)).astype(np.uint8)
    out = np.frombuffer(b"ACGT", dtype=np.uint8)[codes]
    out[off == np.uint64(record_len)] = 0
    return out


def synth_host(num_records, record_len, seed, first_base=0):
    """Same bytes as kmc_synth_fill, on the host (small sizes)."""
    g = np.arange(num_records * record_len, dtype=np.uint64) + np.uint64(first_base)
    words = splitmix64_np(seed, g >> np.uint64(5))
    codes = ((words >> (np.uint64(2) * (g & np.uint64(31)))) & np.uint64(3)).astype(np.uint8)
    bases = np.frombuffer(b"ACGT", dtype=np.uint8)[codes].reshape(num_records, record_len)
    out = np.zeros((num_records, record_len + 1), dtype=np.uint8)
    out[:, :record_len] = bases
    return out.reshape(-1)
