"""The C-ABI library loads on a CPU-only host and exports what include/kmc.h declares."""
import ctypes

import numpy as np


def test_library_exports_every_header_symbol(kmc):
    names = kmc.header_symbols()
    assert "sumKmereCoincidencesGlobalMemory_hip" in names
    assert "kmc_count_dense" in names and "kmc_fasta_load" in names
    L = kmc.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_error_strings_and_version(kmc):
    assert kmc.error_string(0) == "success"
    assert "aligned" in kmc.error_string(1003)
    assert kmc.lib().kmc_version() >= 100


def test_argument_errors_need_no_device(kmc):
    L = kmc.lib()
    # k outside the dense range, null pointers, zero records
    assert L.kmc_count_dense(None, None, 1, 16, 0, None, None, None, 0, None) == 1002
    assert L.kmc_count_dense(None, None, 1, 16, 99, None, None, None, 0, None) == 1002
    assert L.kmc_count_dense(None, None, 1, 16, 3, None, None, None, 0, None) == 1001
    assert L.kmc_count_dense(None, None, 0, 0, 3, None, None, None, 0, None) == 0
    assert L.sumKmereCoincidencesGlobalMemory_hip(None, None, 0, None, None) == 0
    assert L.sumKmereCoincidencesGlobalMemory_hip(None, None, 3, None, None) == 1001
    # the canonical counter still needs a 16-byte aligned data pointer: refused
    # before any device call (the dense entry points take any pointer, like
    # kernels.h:113: tests/test_dense_gpu.py runs them on data + 1 .. 15)
    buf = (ctypes.c_char * 64)()
    base = ctypes.addressof(buf)
    mis = ctypes.c_void_p(base + (1 if base % 16 == 0 else 0) + (16 - base % 16) % 16)
    nd = ctypes.c_uint64(0)
    assert L.kmc_count_canonical_hash(mis, ctypes.c_void_p(base), 1, 21, 0, None, None, 0, ctypes.c_void_p(base),
                                      ctypes.byref(nd), None) == 1003


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
