"""The C-ABI library loads on a CPU-only host and exports what include/kmc.h declares."""
import ctypes
import subprocess

import numpy as np


def test_library_exports_every_header_symbol(kmc):
    names = kmc.header_symbols()
    assert "sumKmereCoincidencesGlobalMemory_hip" in names
    assert "kmc_count_dense" in names and "kmc_fasta_load" in names
    L = kmc.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_binding_declares_every_signature(kmc):
    """kmc.py sets argtypes for every entry point of the header (ctypes would
    otherwise pass Python ints as 32-bit ints: 64-bit sizes silently truncated)."""
    L = kmc.lib()
    assert [n for n in kmc.header_symbols() if getattr(L, n).argtypes is None] == []


def _dynamic_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return sorted(l.split()[-1] for l in out.splitlines() if l.strip())


def test_library_exports_exactly_the_header(kmc):
    """libkmc.so (hidden visibility + libkmc.map) exports exactly kmc.h's entry points:
    no test hook, no internal or C++ symbol that another caller could bind to."""
    assert _dynamic_symbols(kmc.LIB_PATH) == kmc.header_symbols()


def test_diag_library_adds_only_the_test_hooks(kmc):
    """lib/libkmc_diag.so: the same entry points plus the kmc_diag_* hooks."""
    got = _dynamic_symbols(kmc.DIAG_LIB_PATH)
    hooks = [n for n in got if n.startswith("kmc_diag_")]
    assert hooks == ["kmc_diag_canon_claim_cap", "kmc_diag_canon_direct", "kmc_diag_canon_fallback",
                     "kmc_diag_canon_fallback_detail",
                     "kmc_diag_canon_sort_cap",
                     "kmc_diag_canon_sort_cap_big", "kmc_diag_canon_stale_queue", "kmc_diag_dense_spill_cap",
                     "kmc_diag_radix_mode"]
    assert sorted(set(got) - set(hooks)) == kmc.header_symbols()
    assert kmc.lib() is not None
    with kmc.diag() as D:  # inside diag() every binding uses the diagnostic library
        assert kmc.lib() is D and D.kmc_diag_radix_mode(1, 1.0) == 0
    assert not hasattr(kmc.lib(), "kmc_diag_radix_mode")
    assert kmc.lib().kmc_dense_status(0) == 0  # no device touched: nothing raised


def test_error_strings_and_version(kmc):
    assert kmc.error_string(0) == "success"
    assert "aligned" in kmc.error_string(1003)
    # 0.2.0: kmc_dense_args carries `status` (the ctypes mirror must match it)
    assert kmc.lib().kmc_version() == 200
    assert [f[0] for f in kmc.DenseArgs._fields_][-1] == "status"


def test_argument_errors_need_no_device(kmc):
    L = kmc.lib()
    # k outside the dense range, null pointers, zero records
    assert L.kmc_count_dense(None, None, 1, 16, 0, None, None, None, 0, None) == 1002
    assert L.kmc_count_dense(None, None, 1, 16, 99, None, None, None, 0, None) == 1002
    assert L.kmc_count_dense(None, None, 1, 16, 3, None, None, None, 0, None) == 1001
    assert L.kmc_count_dense(None, None, 0, 0, 3, None, None, None, 0, None) == 0
    assert L.sumKmereCoincidencesGlobalMemory_hip(None, None, 0, None, None) == 0
    assert L.sumKmereCoincidencesGlobalMemory_hip(None, None, 3, None, None) == 1001
    # the canonical counter takes any data pointer (since round 4, like the dense
    # entry points): a misaligned one is not refused, null offsets are
    buf = (ctypes.c_char * 64)()
    base = ctypes.addressof(buf)
    mis = ctypes.c_void_p(base + (1 if base % 16 == 0 else 0) + (16 - base % 16) % 16)
    nd = ctypes.c_uint64(0)
    assert L.kmc_count_canonical_hash(mis, None, 1, 21, 0, None, None, 0, ctypes.c_void_p(base),
                                      ctypes.byref(nd), None) == 1001
    assert L.kmc_count_canonical_hash_ex(mis, None, 1, 21, 0, None, None, 0, ctypes.c_void_p(base),
                                         ctypes.byref(nd), None, 0, None) == 1001
    assert L.kmc_count_canonical_hash(mis, None, 1, 32, 0, None, None, 0, None, ctypes.byref(nd), None) == 1002
    # size query: host offsets, bad arguments give 0 (no device needed for those)
    idx = np.array([0, 100, 50], dtype=np.int64)  # decreasing: refused
    assert L.kmc_count_canonical_workspace_size(idx.ctypes.data_as(ctypes.c_void_p), 2, 21, 0) == 0
    assert L.kmc_count_canonical_workspace_size(None, 2, 21, 0) == 0
    assert L.kmc_count_canonical_workspace_size(idx.ctypes.data_as(ctypes.c_void_p), 1, 40, 0) == 0


def test_synth_indices_and_host_generator(kmc):
    idx = kmc.synth_indices(3, 10)
    assert idx.tolist() == [0, 11, 22, 33]
    a = kmc.synth_host(3, 10, seed=0x5EED0008)
    assert a.size == 33 and a[10] == 0 and a[21] == 0 and a[32] == 0
    assert set(np.unique(np.delete(a, [10, 21, 32]))) <= set(b"ACGT")
    # first_base offsets the base stream: record 1 of a 2-record run == record 0 shifted by 10
    b = kmc.synth_host(2, 10, seed=0x5EED0008)
    c = kmc.synth_host(1, 10, seed=0x5EED0008, first_base=10)
    np.testing.assert_array_equal(b[11:22], c)


def _runtimes_in_child(code):
    import json
    import os
    import sys
    pkg = os.path.dirname(os.path.abspath(__import__("kmc").__file__))
    prog = "import sys, json; sys.path.insert(0, %r)\n%s\nimport kmc\nprint(json.dumps(kmc.hip_runtimes()))" % (
        pkg, code)
    out = subprocess.run([sys.executable, "-c", prog], check=True, capture_output=True, text=True, timeout=300)
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_one_hip_runtime_per_process():
    """kmc._load imports torch before libkmc.so, so the library binds to the HIP
    runtime torch ships (the SONAME libamdhip64.so.7 is already loaded) instead of
    mapping /opt/rocm's beside it -- whichever of kmc and torch the caller touches
    first.  Checked in fresh processes through /proc/self/maps (no device needed)."""
    for code in ("import kmc; kmc.lib()\nimport torch",
                 "import torch\nimport kmc; kmc.lib()",
                 "import kmc; kmc.lib(); kmc._hip()\nimport torch"):
        rt = _runtimes_in_child(code)
        assert len(rt) == 1, (code, rt)
