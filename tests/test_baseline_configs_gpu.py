"""The BASELINE.json configurations at their full size, in the driver-run GPU suite.

C2 (configs[1], the bench's workload): 10 records x 1 Gbase, k = 8, one
kmc_count_dense call over the 10 Gbase buffer in HBM.
C3 (configs[2]): the same 10 Gbase at k = 13 (67 M bins per record), in the
library's automatic mode -- at this size every (record, bucket) list holds ~1 M
windows, far above the sampled-partition threshold (256 K), so the sampled radix
path (S1 sample, capacity regions, R3 ring scatter, R4 region walk) is what runs.

Reference semantics: kernels.h:113-144 (one histogram per record, k-mer-major
layout sum[s + n*code]) generalised by permutationsCountAll (main.cu:636-646).
At this size the CPU oracle cannot count the whole job in seconds, so the full
results are checked through size-independent properties plus bin-level slices:
  * every record's column sums to its L - k + 1 windows, and invalid == 0;
  * linearity: the counts of 2 and 3 byte-range shards (kmc_count_dense_ex window
    ranges over the same buffer, cuts inside records) sum to the whole, bin for bin;
  * three 1 Mbase slices (k = 8) / one 4 Mbase slice (k = 13) -- a record start, a
    record end, the 2-way shard cut -- counted as window ranges of the full buffer
    equal oracle.count_dense of the same bytes, bin for bin;
  * one whole 1 Gbase record bin for bin against an independent counter
    (torch.bincount of the record's codes, built with plain tensor ops).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NREC, L = 10, 1_000_000_000
SEED_BASE = 0x5EED0000  # bench.py's seeds: 0x5EED0000 + k


@pytest.fixture(scope="module")
def job(kmc, cuda):
    import torch
    buf = torch.empty(NREC * (L + 1) + 16, dtype=torch.uint8, device=cuda)
    state = {"buf": buf, "idx": kmc.synth_indices(NREC, L), "k": None}

    def regen(k):
        if state["k"] != k:
            kmc.synth_fill(buf, NREC, L, SEED_BASE + k)
            torch.cuda.synchronize()
            state["k"] = k
        return buf

    state["regen"] = regen
    yield state
    del state["buf"]
    torch.cuda.empty_cache()


def torch_record_hist(buf, a, e, k, chunk=200_000_000):
    """Histogram of the windows of the all-ACGT record buf[a:e] (e = its terminator)
    with plain torch ops: codes by a lookup + shifted sums, then bincount."""
    import torch
    lut = torch.zeros(256, dtype=torch.int32, device=buf.device)
    for i, ch in enumerate(b"ACGT"):
        lut[ch] = i
    nb = 1 << (2 * k)
    hist = torch.zeros(nb, dtype=torch.int64, device=buf.device)
    nw = e - a - k + 1
    for s in range(0, nw, chunk):
        m = min(chunk, nw - s)
        c = lut[buf[a + s:a + s + m + k - 1].to(torch.int64)]
        code = torch.zeros(m, dtype=torch.int32, device=buf.device)
        for p in range(k):
            code |= c[p:p + m] << (2 * p)
        hist += torch.bincount(code.to(torch.int64), minlength=nb)
        del c, code
    return hist


def slice_vs_oracle(kmc, oracle, buf, di, idx, k, s, lo, hi):
    """Windows [lo, hi) of record s counted by kmc_count_dense_ex over the full
    buffer vs the oracle on the same bytes as a record of their own."""
    import torch
    n = idx.size - 1
    top = min(hi + k - 1, int(idx[s + 1]))
    out = torch.empty((1 << (2 * k), n), dtype=torch.int32, device=buf.device)
    kmc.count_dense_ex(kmc.dense_args(buf, di, k, out.view(-1), read=(lo, top), win=(lo, hi)))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    host = buf[lo:top].cpu().numpy()
    if top < int(idx[s + 1]):
        host = np.append(host, np.uint8(0))  # windows lo .. hi-1 exactly
    exp, _ = oracle.count_dense(host, np.array([0, host.size], dtype=np.int64), k)
    np.testing.assert_array_equal(got[:, s], exp[:, 0], err_msg="slice [%d, %d) of record %d" % (lo, hi, s))
    others = np.delete(got, s, axis=1)
    assert not others.any(), "windows outside the slice were counted"


def check_config(kmc, oracle, job, k, slice_len):
    import torch
    buf = job["regen"](k)
    idx = job["idx"]
    di = torch.from_numpy(idx).to(buf.device)
    data_bytes = int(idx[-1])
    full, inv = kmc.count_dense(buf, di, k, data_bytes=data_bytes, invalid=True)
    torch.cuda.synchronize()
    assert kmc.lib().kmc_dense_status(torch.cuda.current_device()) == 0
    # (1) column sums and invalid windows
    sums = full.sum(dim=0, dtype=torch.int64).cpu().numpy()
    assert (sums == L - k + 1).all(), sums
    assert not inv.cpu().numpy().any()
    # (2) linearity over 2 and 3 byte-range shards (cuts inside records)
    for nsh, align in ((2, 4096), (3, 1)):
        acc = torch.zeros_like(full)
        part = torch.empty_like(full)
        for (a, b, rl, rh) in kmc.plan_shards(idx, k, nsh, align):
            kmc.count_dense_ex(kmc.dense_args(buf, di, k, part.view(-1), read=(rl, rh), win=(a, b)))
            acc += part
        torch.cuda.synchronize()
        assert torch.equal(acc, full), "%d shards do not sum to the whole" % nsh
        del acc, part
    # (3) bin-level slices against the oracle
    cut = kmc.plan_shards(idx, k, 2, 4096)[0][1]
    s_cut = int(np.searchsorted(idx, cut, side="right") - 1)
    slices = [(3, int(idx[3]), int(idx[3]) + slice_len),
              (6, int(idx[7]) - slice_len, int(idx[7])),
              (s_cut, cut - slice_len // 2, cut + slice_len // 2)]
    if slice_len > 1_000_000:
        slices = slices[2:]
    for s, lo, hi in slices:
        slice_vs_oracle(kmc, oracle, buf, di, idx, k, s, lo, hi)
    # (4) one whole record against an independent torch counter
    r = 9
    h = torch_record_hist(buf, int(idx[r]), int(idx[r + 1]) - 1, k)
    assert torch.equal(h, full[:, r].to(torch.int64)), "record %d differs from torch.bincount" % r
    del full, inv, h
    torch.cuda.empty_cache()


def test_c2_10gbase_k8_full_size(kmc, oracle, cuda, job):
    check_config(kmc, oracle, job, 8, 1_000_000)


def test_c3_10gbase_k13_full_size_auto_mode(kmc, oracle, cuda, job):
    check_config(kmc, oracle, job, 13, 4_000_000)
