#!/usr/bin/env python3
"""bench.py — k-mers/s of the dense k-mer counter on synthetic FASTA in HBM.

Workload (BASELINE.json configs[1]): 10 Gbase per GPU as 10 records of 1 Gbase,
k = 8 (65 536-bin dense histogram), the synthetic layout of SURVEY.md §8(d)
(uniform iid ACGT from splitmix64, seed 0x5EED0000 + k, one '\\0' after each
record).  One step = one full pass of the hot path over the batch: count every
window of every record (kmc_count_dense_ex: histogram kernel + slab reduce +
spill fix-up; it overwrites every entry of the rank's columns), and, for N > 1,
zero the other ranks' columns and the RCCL all-reduce of the int32 count matrix
(records sharded by rank: weak scaling, 10 Gbase per GPU; the N-rank job is one
10N-Gbase FASTA).  Two count matrices alternate between steps, so that a step's
all-reduce (async, on RCCL's stream) overlaps the next step's counting; the timed
region ends after every all-reduce has completed.

Printed (rank 0, one JSON line): metric/value/unit as BASELINE.json, roofline of
the histogram kernel (algorithmic bytes = input ASCII bytes + int32 output,
SURVEY.md §8(d)) timed with HIP events around that kernel on its own stream,
and the reference CPU path (its own permutationsCountAll compiled from
/root/reference into oracle/_ref) timed on a bounded sample of the same bytes.
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dna-kmeres-parallel_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=14)  # the clocks settle over ~10 launches
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--records", type=int, default=10, help="records per GPU")
    ap.add_argument("--record-len", type=int, default=1_000_000_000, help="bases per record")
    ap.add_argument("--cpu-sample", type=int, default=64_000_000,
                    help="bases per CPU thread for the reference CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, available cores)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_dense_k8_10gbase.json"),
                    help="HBM traffic per launch measured by rocprofv3 --pmc (see profiles/)")
    return ap.parse_args()


def cpu_baseline(host_bytes_list, k, threads):
    """Reference CPU path (permutationsCountAll, main.cu:636-646) on `threads`
    disjoint samples in parallel; returns (kmers/s, kind, detail)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle

    if oracle.have_ref_cpu():
        kind = "reference"
        oracle.ref_cpu().ref_build_map(k)  # std::map of 4^k patterns, built once (setup)

        def work(buf, out):
            out[:] = oracle.ref_count_bytes(buf, k)
    else:
        kind = "port"

        def work(buf, out):
            idx = np.array([0, buf.size], dtype=np.int64)
            s, inv = oracle.count_dense(buf, idx, k)
            out[0] = inv[0]
            out[1:] = s[:, 0]
    outs = [np.zeros((1 << (2 * k)) + 1, dtype=np.int32) for _ in host_bytes_list]
    ths = [threading.Thread(target=work, args=(b, o)) for b, o in zip(host_bytes_list, outs)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    kmers = sum(int(o.astype(np.int64).sum()) for o in outs)
    return kmers / dt, kind, dt, kmers


def overlapped_steps(bufs, count, world, all_reduce):
    """step(i) counts into bufs[i % len(bufs)] (count(j): this rank's columns) and,
    for world > 1, zeroes the matrix first and starts its all-reduce without
    waiting for it (all_reduce(t, async_op=True)), so that it overlaps the next
    step, which uses the other matrix; a matrix is reused only after its previous
    all-reduce is done.  drain() waits for every pending all-reduce."""
    nbuf = len(bufs)
    pending = [None] * nbuf  # the all-reduce last issued on each matrix

    def step(i):
        j = i % nbuf
        if world > 1:
            if pending[j] is not None:
                pending[j].wait()  # stream-ordered on RCCL: the previous all-reduce of this matrix
            bufs[j].zero_()  # the other ranks' columns, before the summing all-reduce
        count(j)
        if world > 1:
            pending[j] = all_reduce(bufs[j], async_op=True)
        return j

    def drain():
        for j in range(nbuf):
            if pending[j] is not None:
                pending[j].wait()
                pending[j] = None

    return step, drain


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import kmc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    k = args.k
    nb = 1 << (2 * k)
    n_loc, L = args.records, args.record_len
    n_tot = n_loc * world
    seed = 0x5EED0000 + k
    data_bytes = n_loc * (L + 1)
    # this rank's records are records [rank*n_loc, (rank+1)*n_loc) of one global
    # FASTA whose base stream is continuous across records
    data = torch.empty(data_bytes, dtype=torch.uint8, device=dev)
    kmc.synth_fill(data, n_loc, L, seed, first_base=rank * n_loc * L)
    idx = torch.from_numpy(kmc.synth_indices(n_loc, L)).to(dev)
    # count matrices sum[s_global + n_tot*code]; with N > 1 two of them, so that a
    # step's all-reduce (RCCL, its own stream) overlaps the next step's counting
    nbuf = 2 if world > 1 else 1
    bufs = [torch.zeros((nb, n_tot), dtype=torch.int32, device=dev) for _ in range(nbuf)]
    a0 = kmc.dense_args(data, idx, k, bufs[0].view(-1)[rank * n_loc:], ld=n_tot)
    ws = torch.empty(kmc.dense_ex_workspace_size(a0, local), dtype=torch.uint8, device=dev)
    args_b = [kmc.dense_args(data, idx, k, b.view(-1)[rank * n_loc:], ld=n_tot, workspace=ws) for b in bufs]
    stream = torch.cuda.current_stream()

    def count(j):
        kmc.count_dense_ex(args_b[j], stream)  # overwrites every entry of this rank's columns

    step, drain = overlapped_steps(bufs, count, world, dist.all_reduce if world > 1 else None)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for b, e in ev:  # materialise the events before handing them to the library
        b.record(stream)
        e.record(stream)
    # warm-up: the correctness guard runs on an early warm result, and the last
    # warm-up steps follow it, so that the clocks that dropped while the host
    # checked are back up when the timed steps start (after idling, the GPU ramps
    # its clock over ~10 launches of this kernel: profiles/r01_kernel_launches.json)
    n_after = min(12, max(args.warmup - 1, 0))
    last = 0
    for i in range(args.warmup - n_after):
        last = step(i)
    drain()
    torch.cuda.synchronize()
    if args.warmup > 0:
        # every window of the synthetic input is valid, so each record's column sums to L-k+1
        tot = bufs[last].to(torch.int64).sum(dim=0)
        if not bool((tot == (L - k + 1)).all()):
            raise SystemExit("count check failed: column sums %s" % tot[:4].tolist())
    for i in range(args.warmup - n_after, args.warmup):
        step(i)
    drain()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        kmc.trace_events(ev[i][0], ev[i][1])
        step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    kmc.trace_events(None, None)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    kern_ms = torch.tensor([sum(b.elapsed_time(e) for b, e in ev) / args.steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(kern_ms, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    kern_ms = float(kern_ms.item())

    kmers_per_step = n_tot * (L - k + 1)
    value = kmers_per_step * args.steps / elapsed
    # algorithmic bytes of one histogram launch on one GPU: ASCII input incl.
    # terminators + int32 output of this rank's records
    alg_bytes = data_bytes + 4 * nb * n_loc
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.pmc):
        with open(args.pmc) as f:
            pmc = json.load(f)
        if pmc.get("k") == k and pmc.get("data_bytes") == data_bytes:
            traffic = pmc.get("hbm_bytes_per_launch")

    result = {
        "metric": "k-mers/sec (whole node), 10 Gbase synthetic FASTA, at 1/2/4/8 MI355X",
        "value": value,
        "unit": "k-mers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 uniform ACGT generated in HBM; SURVEY.md 8(d) layout)",
        "config": {
            "workload": "dense k=%d histogram, %d records x %d bases per GPU (%.1f Gbase per GPU)"
                        % (k, n_loc, L, n_loc * L / 1e9),
            "k": k, "records_per_gpu": n_loc, "record_len": L, "total_records": n_tot,
            "bins": nb, "parallelism": "records sharded over %d GPU(s), RCCL all-reduce of int32 counts "
                                       "(overlapping the next step)" % world,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "kernel": "count_dense_kernel<8> (HIP events around the histogram launch)",
            "kernel_ms": kern_ms,
            "alg_bytes_per_launch": alg_bytes,
        },
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        S = args.cpu_sample
        host = []
        for t in range(threads):
            r = t % n_loc
            off = r * (L + 1) + (t // n_loc) * S
            chunk = data[off: off + S].cpu().numpy()
            host.append(np.append(chunk, np.uint8(0)))  # one record of S bases + terminator
        rate, kind, dt, kmers = cpu_baseline(host, k, threads)
        # the same code on one thread (a quarter of one sample)
        one = [np.append(host[0][: max(S // 4, k + 1)], np.uint8(0))]
        rate1, _, dt1, _ = cpu_baseline(one, k, 1)
        import platform
        cpu_model = platform.processor()
        try:
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("model name"):
                        cpu_model = line.split(":", 1)[1].strip()
                        break
        except OSError:
            pass
        result["cpu_baseline"] = {
            "value": rate, "unit": "k-mers/s", "cores": threads, "kind": kind,
            "value_1thread": rate1,
            "sample": "%d threads x %d bases of the same synthetic records (%.0f s wall, %d k-mers), "
                      "k=%d, permutationsCountAll (substr + std::map, main.cu:636-646) -O2; value_1thread: "
                      "1 thread x %d bases (%.1f s); CPU: %s"
                      % (threads, S, dt, kmers, k, one[0].size - 1, dt1, cpu_model),
        }
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
