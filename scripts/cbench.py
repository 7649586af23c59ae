#!/usr/bin/env python3
"""Benchmark of the two non-headline BASELINE.json configurations (diagnostic;
bench.py times configs[1], the headline):
  C3  10 Gbase synthetic, k = 13 dense histogram (radix path), whole call timed
  C4  GRCh38-sized synthetic (3.1 Gbase, 25 chromosome-like records, ~5 % N runs,
      ~50 % soft-masked lowercase), k = 31 canonical counting with KMC_CANON_SOFTMASK
  C4R the same size and k, repeat-rich (scripts/genome_synth.py: interspersed and
      tandem repeats, reverse-complemented copies, soft-masked repeats)
Input resident in HBM; one JSON line per configuration.
Usage: python scripts/cbench.py [--configs c3,c4] [--iters 3] [--gbases-c4 3.1]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-kmeres-parallel_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "?"


def threads_used():
    return min(16, len(os.sched_getaffinity(0)))


def c3_cpu_baseline(data, L, k, sample):
    """The reference's own CPU path (permutationsCountAll via oracle/_ref) at k = 13
    on `threads` disjoint samples of the same records; the std::map of 4^k patterns
    is built once beforehand and timed separately."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "oracle"))
    sys.path.insert(0, repo)
    import numpy as np
    import oracle
    import bench
    if not oracle.have_ref_cpu():
        return None
    t0 = time.perf_counter()
    oracle.ref_cpu().ref_build_map(k)
    build_s = time.perf_counter() - t0
    th = threads_used()
    host = [np.append(data[(t % 10) * (L + 1) + (t // 10) * sample:][:sample].cpu().numpy(), np.uint8(0))
            for t in range(th)]
    rate, kind, dt, kmers = bench.cpu_baseline(host, k, th)
    return {"value": rate, "unit": "k-mers/s", "cores": th, "kind": kind, "map_build_s": build_s,
            "sample": "%d threads x %d bases of the same records (%.1f s wall, %d k-mers), permutationsCountAll "
                      "(main.cu:636-646); the 4^%d-entry std::map built once in %.1f s (not in the rate); CPU: %s"
                      % (th, sample, dt, kmers, k, build_s, cpu_model())}


def c4_cpu_baseline(data, idx, k, sample):
    """No reference counterpart (the reference stops at dense tables): the oracle's
    C restatement (per record: keys, sort, run-length) on `threads` samples."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import threading
    import numpy as np
    import oracle
    th = threads_used()
    bufs = []
    for t in range(th):
        o = int(idx[t % (idx.numel() - 1)].item()) + (t // (idx.numel() - 1)) * sample
        bufs.append(np.append(data[o:o + sample].cpu().numpy(), np.uint8(0)))
    res = [None] * th

    def work(i):
        b = bufs[i]
        res[i] = oracle.count_canonical(b, np.array([0, b.size], dtype=np.int64), k, soft=True)
    ts = [threading.Thread(target=work, args=(i,)) for i in range(th)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    kmers = sum(max(0, b.size - k) for b in bufs)
    return {"value": kmers / dt, "unit": "k-mers/s", "cores": th, "kind": "port",
            "sample": "%d threads x %d bases of the same records (%.1f s wall), oracle_count_canonical "
                      "(oracle/kmc_oracle.c: keys, qsort, run-length; no reference counterpart); CPU: %s"
                      % (th, sample, dt, cpu_model())}


def check_c3(torch, kmc, data, idx, out, recs, L, k, slice_bases=4_000_000):
    """Parity of the timed C3 call: every record's column sums to its L - k + 1
    windows (uniform ACGT, no invalid window), and a 4 Mbase window range of
    record 3 counted through the same radix path equals the oracle's histogram of
    that range."""
    import numpy as np
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "oracle"))
    import oracle
    col = torch.zeros(recs, dtype=torch.int64, device=out.device)
    for c0 in range(0, out.shape[0], 1 << 22):
        col += out[c0:c0 + (1 << 22)].to(torch.int64).sum(dim=0)
    sums = col.cpu().numpy()
    assert (sums == L - k + 1).all(), "C3 column sums %s != %d" % (sums, L - k + 1)
    r = 3 % recs
    lo = r * (L + 1) + 123_457
    hi = lo + slice_bases
    part = torch.zeros_like(out)
    kmc.count_dense_ex(kmc.dense_args(data, idx, k, part, read=(lo, hi + k - 1), win=(lo, hi)))
    torch.cuda.synchronize()
    host = data[lo:hi + k - 1].cpu().numpy()
    exp, _ = oracle.count_dense(np.append(host, np.uint8(0)), np.array([0, host.size + 1], np.int64), k)
    got = part[:, r].cpu().numpy()
    assert (got == exp[:, 0]).all(), "C3 slice histogram differs from the oracle"
    assert int(part.to(torch.int64).sum()) == slice_bases
    return {"column_sums": "all %d == L-k+1" % recs, "slice": "record %d windows [%d, %d) == oracle" % (r, lo, hi)}


def check_c4(torch, kmc, data, idx, k, keys, counts, off, slice_bases=2_000_000):
    """Parity of the timed C4 call: the counts sum to the valid (soft-masked ACGT)
    windows, counted independently on the device, every key is <= its reverse
    complement, and a 2 Mbase slice counted as its own record equals the oracle."""
    import numpy as np
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "oracle"))
    import oracle
    lut = torch.zeros(256, dtype=torch.int32, device=data.device)
    for ch in b"ACGTacgt":
        lut[ch] = 1
    valid = 0
    step = 1 << 28
    n = data.numel()
    for o in range(0, n, step):
        e = min(n, o + step + k - 1)
        v = lut[data[o:e].long()]
        cs = torch.cumsum(torch.nn.functional.pad(v, (1, 0)), 0)
        w = cs[k:] - cs[:-k]  # bases o + i .. o + i + k - 1
        m = min(step, n - o)
        valid += int((w[:m] == k).sum())
    tot = int(counts.to(torch.int64).sum())
    assert tot == valid, "C4 counts sum %d != valid windows %d" % (tot, valid)
    mask = (1 << (2 * k)) - 1
    kk = keys[:: max(1, keys.numel() // 100_000)].cpu().numpy().astype(np.uint64)
    rc = np.zeros_like(kk)
    x = kk.copy()
    for _ in range(k):
        rc = (rc << np.uint64(2)) | (np.uint64(3) - (x & np.uint64(3)))
        x >>= np.uint64(2)
    assert (kk <= rc).all() and (kk <= np.uint64(mask)).all(), "C4 key above its reverse complement"
    lo = int(idx[1].item()) + 5_000_000
    sl = data[lo:lo + slice_bases]
    buf = torch.zeros(slice_bases + 16, dtype=torch.uint8, device=data.device)
    buf[:slice_bases] = sl
    sidx = torch.tensor([0, slice_bases + 1], dtype=torch.int64, device=data.device)
    gk, gc, _ = kmc.count_canonical(buf, sidx, k, flags=kmc.CANON_SOFTMASK)
    host = np.append(sl.cpu().numpy(), np.uint8(0))
    ek, ec, _ = oracle.count_canonical(host, np.array([0, host.size], np.int64), k, soft=True)
    got = dict(zip(gk.cpu().numpy().astype(np.uint64).tolist(), gc.cpu().numpy().tolist()))
    exp = dict(zip(ek.astype(np.uint64).tolist(), ec.tolist()))
    assert got == exp, "C4 slice differs from the oracle"
    return {"sum_counts": "== %d valid windows (independent device count)" % valid,
            "keys_canonical": "sampled keys <= reverse complement",
            "slice": "record 1 bases [%d, %d) as a record == oracle (%d distinct)" % (lo, lo + slice_bases, len(exp))}


def c1_line(torch, kmc, dev, iters, recs=4, L=250_000, k=4, cpu_reps=40):
    """Config C1 (BASELINE configs[0]): 1 Mbase synthetic FASTA (4 records x 250
    kbase, SURVEY.md §8(d) layout), k = 4 (256 bins), the reference's CPU path.
    The reference's own permutationsCountAll (oracle/_ref, main.cu:636-646) counts
    each record on 1 thread and on 16 threads (every thread the whole 1 Mbase
    workload, `cpu_reps` times, so the sample is long enough to time), beside the
    GPU call (kmc_count_dense, median of launches), whose result is checked bin for
    bin against the reference's counts."""
    import numpy as np
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "oracle"), repo]
    import bench
    import oracle
    seed = 0x5EED0000 + k
    host = kmc.synth_host(recs, L, seed)
    idx = kmc.synth_indices(recs, L)
    d = torch.from_numpy(host).to(dev)
    di = torch.from_numpy(idx).to(dev)
    out = torch.empty((1 << (2 * k), recs), dtype=torch.int32, device=dev)
    inv = torch.empty(recs, dtype=torch.int32, device=dev)
    args = kmc.dense_args(d, di, k, out, invalid=inv)
    ws = torch.empty(max(kmc.dense_ex_workspace_size(args), 1), dtype=torch.uint8, device=dev)
    args = kmc.dense_args(d, di, k, out, invalid=inv, workspace=ws)
    med, best = timed(torch, lambda: kmc.count_dense_ex(args), max(iters, 20))
    kmers = recs * (L - k + 1)
    line = {"config": "C1", "k": k, "records": recs, "bases": recs * L, "s_med": med, "s_min": best,
            "kmers_per_s": kmers / med, "note": "1 Mbase is launch-bound on the GPU (a few us of work)"}
    if not oracle.have_ref_cpu():
        line["cpu_baseline"] = None
        return line
    oracle.ref_cpu().ref_build_map(k)
    recs_host = [host[int(idx[r]):int(idx[r + 1])].copy() for r in range(recs)]  # each ends in its '\0'
    ref = np.stack([oracle.ref_count_bytes(b, k) for b in recs_host], axis=1)  # [4^k + 1][recs], bin 0 invalid
    got = out.cpu().numpy()
    assert (got == ref[1:]).all() and (inv.cpu().numpy() == ref[0]).all(), "C1 GPU counts differ from the reference"
    line["parity"] = "GPU counts + invalid == the reference's permutationsCountAll, every bin of every record"
    work = [b for _ in range(cpu_reps) for b in recs_host]
    res = {}
    for th in (1, 16):
        per = [work] * th  # each thread: the whole workload cpu_reps times

        def one(i, out_):
            out_[i] = sum(int(oracle.ref_count_bytes(b, k).astype(np.int64).sum()) for b in per[i])
        import threading
        tot = [0] * th
        ts = [threading.Thread(target=one, args=(i, tot)) for i in range(th)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        res[th] = (sum(tot) / dt, dt, sum(tot))
    line["cpu_baseline"] = {
        "value": res[16][0], "unit": "k-mers/s", "cores": 16, "kind": "reference", "value_1thread": res[1][0],
        "sample": "the whole C1 workload (%d records x %d bases) x %d per thread; 16 threads: %.1f s, 1 thread: "
                  "%.1f s; the reference's permutationsCountAll (main.cu:636-646) built -O2 from /root/reference; "
                  "CPU: %s" % (recs, L, cpu_reps, res[16][1], res[1][1], cpu_model())}
    line["gpu_vs_cpu16"] = line["kmers_per_s"] / res[16][0]
    return line


def timed(torch, fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c3,c4,c4r")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--gbases-c3", type=float, default=10.0)
    ap.add_argument("--gbases-c4", type=float, default=3.1)
    ap.add_argument("--k3", type=int, default=13)
    ap.add_argument("--cpu-sample-c3", type=int, default=2_000_000, help="bases per CPU thread (0 = skip)")
    ap.add_argument("--cpu-sample-c4", type=int, default=16_000_000, help="bases per CPU thread (0 = skip)")
    ap.add_argument("--no-check", dest="check", action="store_false", help="skip the parity checks")
    ap.add_argument("--canon-direct", type=int, default=None,
                    help="A/B of the canonical output path through the diagnostic library: 1 = direct output "
                         "(the default), 0 = pk + place copy (the layout before round 5)")
    a = ap.parse_args()
    import torch
    import kmc
    if a.canon_direct is not None:
        D = kmc.diag().__enter__()  # every binding calls lib/libkmc_diag.so from here on
        assert D.kmc_diag_canon_direct(a.canon_direct) == 0
    dev = torch.device("cuda:0")
    cfgs = a.configs.split(",")
    if "c1" in cfgs:
        print(json.dumps(c1_line(torch, kmc, dev, a.iters)), flush=True)
    if "c3r" in cfgs:  # k = 13 over the repeat-rich genome, uppercased (skewed buckets: the rings' cold path)
        import genome_synth
        data, idx, lens, st = genome_synth.repeat_genome(torch, dev, a.gbases_c4)
        data.sub_(((data >= ord("a")) & (data <= ord("z"))).to(torch.uint8) << 5)  # elementwise (3.1 G bytes)
        k = a.k3
        recs = len(lens)
        out = torch.empty((1 << (2 * k), recs), dtype=torch.int32, device=dev)
        args = kmc.dense_args(data, idx, k, out)
        ws = torch.empty(kmc.dense_ex_workspace_size(args), dtype=torch.uint8, device=dev)
        args = kmc.dense_args(data, idx, k, out, workspace=ws)
        med, best = timed(torch, lambda: kmc.count_dense_ex(args), a.iters)
        inv = torch.empty(recs, dtype=torch.int32, device=dev)
        kmc.count_dense_ex(kmc.dense_args(data, idx, k, out, invalid=inv, workspace=ws))
        col = torch.zeros(recs, dtype=torch.int64, device=dev)
        for c0 in range(0, out.shape[0], 1 << 22):
            col += out[c0:c0 + (1 << 22)].to(torch.int64).sum(dim=0)
        windows = torch.tensor([max(0, L - k + 1) for L in lens], dtype=torch.int64, device=dev)
        assert bool(((col + inv.to(torch.int64)) == windows).all()), "C3R column sums + invalid != windows"
        kmers = int(windows.sum())
        alg = data.numel() + 4 * (1 << (2 * k)) * recs
        line = {"config": "C3R", "k": k, "records": recs, "bases": sum(lens), "s_med": med, "s_min": best,
                "kmers_per_s": kmers / med, "alg_bytes": alg, "GBps": alg / med / 1e9, "frac8TB": alg / med / 8e12,
                "input": "repeat-rich synthetic genome (scripts/genome_synth.py), uppercased", "composition": st,
                "max_bin": int(out.max().item()), "parity": "column sums + invalid == windows for every record"}
        print(json.dumps(line), flush=True)
        del data, out, ws, args, inv
        torch.cuda.empty_cache()
    if "c3" in cfgs:
        recs = 10
        L = int(a.gbases_c3 * 1e9 / recs)
        data = torch.empty(recs * (L + 1), dtype=torch.uint8, device=dev)
        kmc.synth_fill(data, recs, L, 0x5EED0000 + a.k3)
        idx = torch.from_numpy(kmc.synth_indices(recs, L)).to(dev)
        k = a.k3
        out = torch.empty((1 << (2 * k), recs), dtype=torch.int32, device=dev)
        args = kmc.dense_args(data, idx, k, out)
        ws = torch.empty(kmc.dense_ex_workspace_size(args), dtype=torch.uint8, device=dev)
        args = kmc.dense_args(data, idx, k, out, workspace=ws)
        med, best = timed(torch, lambda: kmc.count_dense_ex(args), a.iters)
        kmers = recs * (L - k + 1)
        alg = data.numel() + 4 * (1 << (2 * k)) * recs
        line = {"config": "C3", "k": k, "records": recs, "bases": recs * L, "s_med": med, "s_min": best,
                "kmers_per_s": kmers / med, "alg_bytes": alg, "GBps": alg / med / 1e9, "frac8TB": alg / med / 8e12}
        if a.check:
            line["parity"] = check_c3(torch, kmc, data, idx, out, recs, L, k)
        if a.cpu_sample_c3 > 0:
            line["cpu_baseline"] = c3_cpu_baseline(data, L, k, a.cpu_sample_c3)
        print(json.dumps(line), flush=True)
        del data, out, ws, args
        torch.cuda.empty_cache()
    for cfg in [c for c in cfgs if c in ("c4", "c4r")]:
        if cfg == "c4":
            import genome_synth
            data, idx, lens = genome_synth.grch38_like(torch, dev, a.gbases_c4)
            extra = {"input": "iid ACGT, 5 % N runs, 50 % soft-masked runs (no repeats)"}
        else:  # repeat-rich stand-in (scripts/genome_synth.py)
            import genome_synth
            t0 = time.perf_counter()
            data, idx, lens, st = genome_synth.repeat_genome(torch, dev, a.gbases_c4)
            torch.cuda.synchronize()
            extra = {"input": "repeat-rich synthetic genome (scripts/genome_synth.py)", "composition": st,
                     "gen_s": time.perf_counter() - t0}
        k = 31
        kmers = sum(max(0, L - k + 1) for L in lens)
        res = {}

        def run():
            res.clear()  # the previous result's 12 B/window output freed first (no second allocation)
            res["r"] = kmc.count_canonical(data, idx, k, flags=kmc.CANON_SOFTMASK)
        med, best = timed(torch, run, a.iters)
        keys, counts, off = res["r"]
        tot = int(counts.sum().item())
        alg = 17 * kmers  # 1 B input + 16 B table slot per k-mer
        line = {"config": cfg.upper(), "k": k, "records": len(lens), "bases": sum(lens), "windows": kmers,
                "valid_windows": tot, "distinct": int(keys.numel()), "s_med": med, "s_min": best,
                "kmers_per_s": kmers / med, "alg_bytes": alg, "GBps": alg / med / 1e9, "frac8TB": alg / med / 8e12}
        if a.canon_direct is not None:
            line["canon_direct"] = a.canon_direct
        line.update(extra)
        line["max_count"] = int(counts.max().item())
        line["keys_count_gt1"] = int((counts > 1).sum().item())
        if a.check:
            line["parity"] = check_c4(torch, kmc, data, idx, k, keys, counts, off)
        if a.cpu_sample_c4 > 0:
            line["cpu_baseline"] = c4_cpu_baseline(data, idx, k, a.cpu_sample_c4)
        print(json.dumps(line), flush=True)
        del data, idx, keys, counts, off
        res.clear()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
