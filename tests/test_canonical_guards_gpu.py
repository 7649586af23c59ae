"""The round-5 canon_table_kernel fault (gpurun_out/r05e/tests.log): regression
input, workspace hygiene and the device-side bound guards (DESIGN.md §4.4,
"The round-5 memory-aperture fault").

What faulted: canon_table_kernel (512 x 512 threads) aborted its queue with
HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in test_full_size_checks_catch_tampered_output,
the first small call after four 3.1 Gbase calls had filled the library-owned
workspace.  An aperture violation is an address far outside any allocation: a
list id or key range taken from queue entries this call never wrote (a counter
not reset per call, or entries past it).  These tests:

  * run that exact input (repeat_genome(0.03, seed=5, min_len=20_000), k = 31,
    soft-mask) in direct mode through every queue -- both table-kernel launches,
    the big K4s instance, the fallback copy queue -- with the diagnostic caps
    (sort_cap 0: every list to the table kernel's first launch; 1: the big
    instance takes lists of 2..12 288 keys; the shipped split), each time in a
    caller workspace filled with 0xFF bytes, and compare every record with the
    self-oracle: a kernel that read any workspace byte this call did not write
    would read all-ones list ids / ranges (caught by the guards) or wrong keys;
  * reproduce the defect class with a test hook (kmc_diag_canon_stale_queue: the
    second queue's count starts at v instead of 0) and show that the guards turn
    it into KMC_ERR_INTERNAL instead of a fault, and that the next call on the
    same poisoned workspace is exact again.
Canonical counting has no reference counterpart; the oracle is
the definition, /root/reference/main.cu:636-646 generalised to k = 31.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = 31


def _crowded_records(rng):
    """Records of one list each made of a 200-bp unit repeated 20 times: more than
    128 crowded slots, so K4s queues them to the table kernel's second launch."""
    recs = []
    for _ in range(8):
        unit = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=200)
        recs.append(np.append(np.tile(unit, 20), np.uint8(0)))
    return recs


@pytest.fixture(scope="module")
def fault_input(cuda):
    """The r05e input, plus records that reach the second table launch."""
    import torch
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import genome_synth
    g, gi, _, _ = genome_synth.repeat_genome(torch, cuda, 0.03, seed=5, min_len=20_000)
    gh, gih = g.cpu().numpy(), gi.cpu().numpy().astype(np.int64)
    del g, gi
    extra = _crowded_records(np.random.default_rng(55))
    data = np.concatenate([gh] + extra)
    idx = np.concatenate([gih, gih[-1] + np.cumsum([r.size for r in extra])]).astype(np.int64)
    return data, idx


@pytest.fixture(scope="module")
def fault_oracle(oracle, fault_input):
    data, idx = fault_input
    return oracle.count_canonical(data, idx, K, soft=True)


def _poisoned_ws(torch, kmc, cuda, idx):
    wsb = kmc.canonical_workspace_size(idx, K, torch.cuda.current_device())
    assert wsb > 0
    return torch.full((wsb,), 0xFF, dtype=torch.uint8, device=cuda)


def _run(torch, kmc, cuda, data_d, idx_d, ws):
    keys, counts, off = kmc.count_canonical(data_d, idx_d, K, flags=kmc.CANON_SOFTMASK,
                                            capacity=int(data_d.numel()), workspace=ws)
    torch.cuda.synchronize()
    return keys.cpu().numpy().view(np.uint64), counts.cpu().numpy().view(np.uint32), off.cpu().numpy()


def _assert_same(got, exp, msg):
    gk, gc, go = got
    ek, ec, eo = exp
    np.testing.assert_array_equal(go, eo, err_msg=msg + ": record offsets")
    for s in range(go.size - 1):
        a, b = int(go[s]), int(go[s + 1])
        o = np.argsort(gk[a:b], kind="stable")
        p = np.argsort(ek[a:b], kind="stable")
        np.testing.assert_array_equal(gk[a:b][o], ek[a:b][p], err_msg="%s: record %d keys" % (msg, s))
        np.testing.assert_array_equal(gc[a:b][o], ec[a:b][p], err_msg="%s: record %d counts" % (msg, s))


@pytest.mark.parametrize("scap", [0, 1, None])
def test_fault_input_every_queue_poisoned_workspace(kmc, cuda, fault_input, fault_oracle, scap):
    """Direct mode on the r05e input in a 0xFF-filled caller workspace: exact, and
    the queues the fault involved were used (diagnostic counters)."""
    import ctypes
    import torch
    data, idx = fault_input
    data_d = torch.from_numpy(data).to(cuda)
    idx_d = torch.from_numpy(idx).to(cuda)
    with kmc.diag() as D:
        if scap is not None:
            assert D.kmc_diag_canon_sort_cap(scap) == 0
        ws = _poisoned_ws(torch, kmc, cuda, idx)
        got = _run(torch, kmc, cuda, data_d, idx_d, ws)
        ent, pairs = ctypes.c_ulonglong(0), ctypes.c_ulonglong(0)
        assert D.kmc_diag_canon_fallback(ctypes.byref(ent), ctypes.byref(pairs)) == 0
        per = (ctypes.c_ulonglong * 1)()
        q3 = (ctypes.c_ulonglong * 3)()
        assert D.kmc_diag_canon_fallback_detail(per, 0, q3) == 0
    _assert_same(got, fault_oracle, "sort_cap=%s" % scap)
    big, table1, table2 = q3[0], q3[1], q3[2]
    if scap == 0:  # every list through the table kernel's first launch, each a queued copy
        assert table1 > 0 and ent.value >= table1 and pairs.value > 0, (big, table1, table2, ent.value)
    else:  # the crowded records: K4s (common or big instance) -> the second launch
        assert table2 >= 8, (big, table1, table2)
        if scap == 1:
            assert big > 0, (big, table1, table2)
    del ws, data_d, idx_d
    torch.cuda.empty_cache()


@pytest.mark.parametrize("stale", [5, 1 << 40])
def test_stale_queue_count_raises_internal_not_a_fault(kmc, cuda, fault_input, fault_oracle, stale):
    """The defect class of the fault, forced: the second table queue's count starts
    at `stale` in a workspace whose bytes are 0xFF, so its first entries (or its
    count itself) are not this call's.  The guards skip them and the call returns
    KMC_ERR_INTERNAL; the same poisoned workspace then gives the exact result."""
    import torch
    data, idx = fault_input
    data_d = torch.from_numpy(data).to(cuda)
    idx_d = torch.from_numpy(idx).to(cuda)
    with kmc.diag() as D:
        ws = _poisoned_ws(torch, kmc, cuda, idx)
        assert D.kmc_diag_canon_stale_queue(stale) == 0
        with pytest.raises(kmc.KmcError) as ei:
            _run(torch, kmc, cuda, data_d, idx_d, ws)
        assert ei.value.code == kmc.KMC_ERR_INTERNAL
        assert D.kmc_diag_canon_stale_queue(-1) == 0
        ws.fill_(0xFF)
        got = _run(torch, kmc, cuda, data_d, idx_d, ws)
    _assert_same(got, fault_oracle, "after the guarded call, stale=%d" % stale)
    del ws, data_d, idx_d
    torch.cuda.empty_cache()


def test_library_workspace_after_a_larger_call(kmc, cuda, fault_input, fault_oracle):
    """The r05e sequence with the library-owned workspace: a larger call first (the
    workspace grows and keeps its bytes), then the fault input -- exact."""
    import torch
    data, idx = fault_input
    rng = np.random.default_rng(5)
    big = rng.choice(np.frombuffer(b"ACGTacgtN", dtype=np.uint8), size=60_000_000)
    big[-1] = 0
    bd = torch.from_numpy(big).to(cuda)
    bi = torch.tensor([0, 25_000_000, big.size], dtype=torch.int64, device=cuda)
    kmc.count_canonical(bd, bi, K, flags=kmc.CANON_SOFTMASK, capacity=big.size)
    torch.cuda.synchronize()
    del bd, bi
    got = _run(torch, kmc, cuda, torch.from_numpy(data).to(cuda), torch.from_numpy(idx).to(cuda), None)
    _assert_same(got, fault_oracle, "library workspace after a 60 Mbase call")
