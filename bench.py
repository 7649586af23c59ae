#!/usr/bin/env python3
"""bench.py — k-mers/s of the dense k-mer counter on synthetic FASTA in HBM.

Workload (BASELINE.json metric and configs[1]): one synthetic FASTA of 10
records x 1 Gbase (10 Gbase), k = 8 (65 536-bin dense histogram), the layout of
SURVEY.md §8(d): uniform iid ACGT from splitmix64 (seed 0x5EED0000 + k), one
'\\0' after each record, one global buffer with record r at bytes
[r*(L+1), (r+1)*(L+1)).

Scaling modes:
  strong (default) — the 10 Gbase job is cut into N byte ranges by kmc_plan_shards
      (4 KiB-aligned cuts, a k-1 byte halo past each), as the reference's one
      launch over the whole buffer (main.cu:290) split N ways; rank r holds only
      its range + halo in HBM;
  weak — every rank holds `--records` whole records of its own (C5: 80 Gbase on 8
      GPUs is `--scaling weak` with 10 records per GPU).
Either way one step = one full pass of the hot path over the job: every rank
counts the windows starting in its byte range (kmc_count_dense_ex over the
global record offsets: histogram kernel + slab reduce + spill fix-up), which
overwrites all N_rec columns of its int32 count matrix (zeros for records it
does not touch), then (N > 1) one RCCL all-reduce (sum) of that matrix over
xGMI.  Two matrices alternate, so a step's async all-reduce overlaps the next
step's counting; the timed region ends after every all-reduce has completed.

Launch: `python bench.py --gpus N` starts N rank processes itself (before any
GPU call) when WORLD_SIZE is not set; under torch.distributed.run (one process
per GPU, WORLD_SIZE/RANK/LOCAL_RANK set) it runs as that rank.

Printed (rank 0, one JSON line): metric/value/unit as BASELINE.json, roofline of
the histogram kernel (algorithmic bytes = the rank's input ASCII bytes + int32
output) timed with HIP events around that kernel on its own
stream, and the reference CPU path (its own permutationsCountAll compiled from
/root/reference into oracle/_ref) on every host core this process may use.
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dna-kmeres-parallel_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SEED_BASE = 0x5EED0000


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=14)  # the clocks settle over ~10 launches (after the guard step)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed: histogram launches back to back for this long (wall) after the correctness "
                         "guard and before the W warm-up steps, so that the GPU clock has ramped up from the "
                         "guard's host-side idle (0 = none); the timed region is unchanged")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: --records records in total, byte-range shards; weak: --records per GPU")
    ap.add_argument("--records", type=int, default=10)
    ap.add_argument("--record-len", type=int, default=1_000_000_000, help="bases per record")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="bases per CPU worker for the reference CPU baseline (0 = sized to ~15 s; -1 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may run on")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_dense_k8_shards.json"),
                    help="HBM traffic per launch measured by rocprofv3 --pmc, per shard size (see profiles/)")
    ap.add_argument("--pmc-lds", default=os.path.join(REPO, "profiles", "pmc_lds_k8_10gbase.json"),
                    help="LDS-array cycles per window of the k = 8 kernel (rocprofv3 --pmc, see profiles/)")
    ap.add_argument("--allreduce-reps", type=int, default=20,
                    help="N > 1: all-reduces timed alone after the timed region")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="CUs left out of the histogram grid for the overlapped all-reduce, whose RCCL "
                         "channels are capped to match (NCCL_MAX_NCHANNELS); -1 = 4 at N > 1, 0 at N = 1")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launch: N rank processes when no launcher started us
# ---------------------------------------------------------------------------
def spawn_ranks(n, argv):
    """Start n copies of this script as ranks 0..n-1 (env as torch.distributed.run
    sets it) and return the worst exit status.  Runs before anything touches the
    GPU: the children are fresh processes, nothing is exec'ed."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    return rc


# ---------------------------------------------------------------------------
# the step driver (also run by tests/test_multi.py with gloo and the oracle)
# ---------------------------------------------------------------------------
def rank_plan(scaling, world, rank, records, L, k, align=4096):
    """What rank `rank` of a `world`-rank job counts and holds.

    Returns a dict: n_tot (records of the job), indices (global int64 offsets,
    n_tot + 1), win = (win_lo, win_hi) (windows starting there are this rank's),
    read = (read_lo, read_hi) (bytes the count reads: the range + its k-1 halo),
    base (global offset of the rank's buffer start, read_lo rounded down to 16 so
    the library's data pointer stays aligned), hold = (base, read_hi)."""
    import numpy as np

    import kmc
    if scaling == "strong":
        n_tot = records
        idx = kmc.synth_indices(n_tot, L)
        win_lo, win_hi, read_lo, read_hi = kmc.plan_shards(idx, k, world, align)[rank]
    elif scaling == "weak":
        n_tot = records * world
        idx = kmc.synth_indices(n_tot, L)
        win_lo, win_hi = int(idx[rank * records]), int(idx[(rank + 1) * records])
        read_lo, read_hi = win_lo, win_hi  # whole records: the last byte is a terminator, no halo
    else:
        raise ValueError(scaling)
    base = int(read_lo) & ~15
    return {"n_tot": n_tot, "indices": np.asarray(idx, dtype=np.int64), "win": (int(win_lo), int(win_hi)),
            "read": (int(read_lo), int(read_hi)), "base": base, "hold": (base, int(read_hi))}


def overlapped_steps(bufs, count, world, all_reduce):
    """step(i) counts into bufs[i % len(bufs)] (count(j) overwrites every entry of
    matrix j: this rank's counts, zeros for records it does not touch) and, for
    world > 1, starts the matrix's all-reduce without waiting for it
    (all_reduce(t, async_op=True)), so that it overlaps the next step, which uses
    the other matrix; a matrix is reused only after its previous all-reduce is
    done.  drain() waits for every pending all-reduce."""
    nbuf = len(bufs)
    pending = [None] * nbuf  # the all-reduce last issued on each matrix

    def step(i):
        j = i % nbuf
        if pending[j] is not None:
            pending[j].wait()  # stream-ordered on RCCL: the previous all-reduce of this matrix
            pending[j] = None
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


def host_kmer_hist(bases, k):
    """numpy histogram of the windows of one all-ACGT byte run (LE bin order:
    the first base is the least significant digit, utils.h:35-47)."""
    import numpy as np
    lut = np.zeros(256, dtype=np.int64)
    lut[np.frombuffer(b"ACGT", dtype=np.uint8)] = np.arange(4)
    c = lut[bases]
    nw = c.size - k + 1
    code = np.zeros(nw, dtype=np.int64)
    for p in range(k):
        code |= c[p:p + nw] << (2 * p)
    return np.bincount(code, minlength=1 << (2 * k))


# ---------------------------------------------------------------------------
# CPU baseline: the reference's permutationsCountAll on the host cores
# ---------------------------------------------------------------------------
def usable_cores():
    """(cores this process may run on: affinity capped by the cgroup CPU quota,
    CPUs of the machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n, os.cpu_count() or n


def cpu_baseline(host_bytes_list, k, threads):
    """Reference CPU path (permutationsCountAll, main.cu:636-646) on `threads`
    disjoint samples in parallel (ctypes drops the GIL); returns (kmers/s, kind,
    seconds, kmers)."""
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


def cpu_model():
    import platform
    m = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return m


def run_cpu_baseline(args, data, k):
    """The reference CPU path on this rank's bytes of the job (the whole buffer at
    N = 1, rank 0's shard otherwise): one worker per usable core, each on its own
    S-base slice (slices spread over the held bytes; they overlap only when the
    shard is smaller than threads x S)."""
    import numpy as np
    threads, node_cpus = usable_cores()
    if args.cpu_threads:
        threads = args.cpu_threads
    held = int(data.numel())
    # one thread first: its rate sizes the per-worker sample to ~15 s of work
    probe = np.append(data[: min(4_000_000, held)].cpu().numpy(), np.uint8(0))
    rate1, kind, dt1, _ = cpu_baseline([probe], k, 1)
    S = args.cpu_sample or int(min(max(rate1 * 15.0, 1e6), 256e6))
    S = max(min(S, held), k)
    step = (held - S) // max(threads - 1, 1) if threads > 1 else 0
    host = [np.append(data[t * step: t * step + S].cpu().numpy(), np.uint8(0)) for t in range(threads)]
    rate, kind, dt, kmers = cpu_baseline(host, k, threads)
    return {
        "value": rate, "unit": "k-mers/s", "cores": threads, "kind": kind,
        "value_1thread": rate1, "node_cpus": node_cpus,
        "sample": "%d workers x %d bases of this rank's synthetic records (%.1f s wall, %d k-mers), k=%d, the "
                  "reference's permutationsCountAll (substr + std::map, main.cu:636-646) built -O2 from "
                  "/root/reference; cores = the CPUs this process may use (affinity and cgroup quota; the "
                  "machine shows %d); value_1thread: 1 worker x %d bases (%.1f s); CPU: %s"
                  % (threads, S, dt, kmers, k, node_cpus, probe.size - 1, dt1, cpu_model()),
    }


# ---------------------------------------------------------------------------
def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, argv))

    import numpy as np
    import torch
    import torch.distributed as dist

    import kmc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    # KMC_BENCH_BACKEND=gloo: rehearsal of the N-rank path with every rank on the
    # one GPU of a test box (RCCL needs one device per rank); never a measurement
    backend = os.environ.get("KMC_BENCH_BACKEND", "nccl")
    local = local % torch.cuda.device_count() if backend != "nccl" else local
    # each step's all-reduce overlaps the next step's counting; the histogram grid is
    # one static workgroup per CU, so a CU held by RCCL delays the launch (+12 % per
    # step at 8-way with 8 CUs held for 50 us, scripts/interfere.py).  Leaving
    # reserve_cus CUs to RCCL, its channels capped to as many, keeps them apart
    # (the same experiment: 0.348-0.351 -> 0.318 ms; 0.311 -> 0.318 ms alone).
    # Round 4 (profiles/r04k_interfere_reserve.log): 4 CUs cost less alone (0.305
    # against 0.311 ms) and held the step at 0.309-0.310 ms in 3 of 4 stand-in runs,
    # where 8 did not (0.349-0.352 ms); 4 RCCL channels carry the 2.6 MB (C2) or
    # 21 MB (C5) all-reduce well inside one step.
    reserve = args.reserve_cus if args.reserve_cus >= 0 else (4 if world > 1 else 0)
    if world > 1 and reserve > 0:
        os.environ.setdefault("NCCL_MAX_NCHANNELS", str(reserve))
    kmc.set_reserved_cus(reserve)
    args.reserve_cus_eff = reserve
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    k = args.k
    nb = 1 << (2 * k)
    L = args.record_len
    seed = SEED_BASE + k
    plan = rank_plan(args.scaling, world, rank, args.records, L, k)
    n_tot = plan["n_tot"]
    base, hold_hi = plan["hold"]
    (win_lo, win_hi), (read_lo, read_hi) = plan["win"], plan["read"]
    # this rank's bytes of the one global buffer (its byte range + halo), generated in HBM
    data = torch.empty(max(hold_hi - base, 16), dtype=torch.uint8, device=dev)
    kmc.synth_fill_range(data, base, hold_hi, L, seed)
    idx = torch.from_numpy(plan["indices"]).to(dev)
    nbuf = 2 if world > 1 else 1
    bufs = [torch.empty((nb, n_tot), dtype=torch.int32, device=dev) for _ in range(nbuf)]

    def dargs(out, ws=None):
        return kmc.dense_args(data, idx, k, out.view(-1), read=(read_lo, read_hi), win=(win_lo, win_hi),
                              workspace=ws, data_offset=base)

    ws = torch.empty(max(kmc.dense_ex_workspace_size(dargs(bufs[0]), local), 1), dtype=torch.uint8, device=dev)
    args_b = [dargs(b, ws) for b in bufs]
    stream = torch.cuda.current_stream()

    def count(j):
        kmc.count_dense_ex(args_b[j], stream)  # overwrites every entry of the matrix

    step, drain = overlapped_steps(bufs, count, world, dist.all_reduce if world > 1 else None)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for b, e in ev:  # materialise the events before handing them to the library
        b.record(stream)
        e.record(stream)
    # the correctness guard runs BEFORE the warm-up (round 6), so that the W warm-up
    # steps run back to back right before the timed region: the host's expected
    # slice histogram is computed first (the GPU idles then anyway), then one step
    # (not one of the W) and the slice are counted and compared.  Until round 5 the
    # guard ran between warm-up steps, and with the driver's --warmup 5 only four
    # steps followed the host's check, while the clock, dropped during it, ramps over
    # ~10 launches of this kernel (profiles/r01_kernel_launches.json): the driver's
    # kernel time then included the ramp (BENCH_r05 2.126 ms, against 2.05-2.07 ms
    # with 14 warm-up steps).
    s_lo = win_lo - base
    s_len = min(1 << 20, L - (win_lo % (L + 1)), max(win_hi - win_lo, 0))
    exp = host_kmer_hist(kmc.synth_host_range(win_lo, win_lo + s_len, L, seed), k) if s_len >= k else None
    last = step(0)
    drain()
    torch.cuda.synchronize()
    # (1) every window of the synthetic input is valid: after the all-reduce each
    # record's column sums to L-k+1; (2) bins, not only totals: a 1 Mbase slice of
    # this rank's bytes counted as a record of its own equals a numpy histogram of
    # the same bytes regenerated on the host
    tot = bufs[last].to(torch.int64).sum(dim=0)
    if not bool((tot == (L - k + 1)).all()):
        raise SystemExit("count check failed: column sums %s" % tot[:4].tolist())
    if exp is not None:
        sl = torch.zeros(s_len + 16, dtype=torch.uint8, device=dev)
        sl[:s_len] = data[s_lo:s_lo + s_len]
        got, _ = kmc.count_dense(sl, torch.tensor([0, s_len + 1], dtype=torch.int64, device=dev), k)
        if not np.array_equal(got.view(-1).cpu().numpy().astype(np.int64), exp):
            raise SystemExit("count check failed: a 1 Mbase slice differs from its host histogram")
    # clock settle (round 6): the guard's host work above idles the GPU, and the clock
    # then ramps over ~10-25 launches of this kernel -- with the driver's --warmup 5
    # the first ~10 timed steps were still ramping (profiles/r06w_bench5.json:
    # 2.36 -> 2.11 ms over the 20 steps).  Untimed histogram launches (this rank's
    # count alone, no collective, so ranks may differ in how many they run) for
    # settle_ms of wall time first; then the W warm-up steps and the K timed steps
    # exactly as before.
    settle_n = 0
    if args.settle_ms > 0:
        t_s = time.perf_counter()
        while (time.perf_counter() - t_s) * 1e3 < args.settle_ms and settle_n < 4096:
            for _ in range(4):
                count(last)
            settle_n += 4
            torch.cuda.synchronize()
    args.settle_launches = settle_n
    for i in range(args.warmup):
        step(i + 1)
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
    if kmc.lib().kmc_dense_status(local) != 0:  # a k = 8 spill list overflowed (never expected)
        raise SystemExit("count check failed: kmc_dense_status reports a spill overflow")
    # algorithmic bytes of one histogram launch on this GPU: its ASCII input bytes +
    # the int32 matrix it writes
    alg_bytes = (win_hi - win_lo) + 4 * nb * n_tot
    step_ms = [b.elapsed_time(e) for b, e in ev]
    kern_ms = sum(step_ms) / args.steps
    result = finalize(args, world, rank, backend, data, bufs[0], L, k, n_tot, (win_lo, win_hi), t1 - t0, kern_ms,
                      alg_bytes, timer="cuda", step_ms=step_ms)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure_allreduce(like, reps, timer):
    """Average time of one all-reduce (SUM) of a matrix shaped like the count
    matrix, alone: not overlapped with counting, on a scratch tensor of zeros (so
    repeated sums cannot overflow).  timer "cuda": HIP events on the current stream
    around each synchronous dist.all_reduce (the collective's own stream joins the
    current one before and after it); "host": wall time (the gloo CPU tests)."""
    import torch
    import torch.distributed as dist
    x = torch.zeros_like(like)
    dist.all_reduce(x)  # first call: communicator/channel setup, not timed
    if timer == "cuda":
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        dist.barrier()
        for b, e in ev:
            b.record(st)
            dist.all_reduce(x)
            e.record(st)
        torch.cuda.synchronize()
        return sum(b.elapsed_time(e) for b, e in ev) / reps
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(x)
    return (time.perf_counter() - t0) / reps * 1e3


def over_ranks(world, vals, device):
    """(max, ...) of per-rank floats over the job: every entry is maxed; pass -x
    for a minimum."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def dense_code_object_id(lib_path=None):
    """Identity of the histogram kernel's build: sha256 (16 hex digits) of the gfx950
    code object that holds count_dense_kernel inside libkmc.so's offload bundles
    (one bundle per translation unit; the same sources and compiler give the same
    bytes).  PMC summaries store the id of the build they measured, and the bench
    line uses only entries whose id matches the library it ran (None: not found)."""
    import hashlib
    import struct
    if lib_path is None:
        import kmc
        lib_path = kmc.LIB_PATH
    try:
        with open(lib_path, "rb") as f:
            b = f.read()
    except OSError:
        return None
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    i = b.find(magic)
    while i >= 0:
        n = struct.unpack_from("<Q", b, i + 24)[0]
        o = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, o)
            o += 24
            triple = b[o:o + tl]
            o += tl
            if b"gfx950" in triple and size:
                co = b[i + off:i + off + size]
                if b"count_dense_kernel" in co:
                    return hashlib.sha256(co).hexdigest()[:16]
        i = b.find(magic, i + len(magic))
    return None


def pmc_traffic(path, k, data_bytes, build_id):
    """HBM bytes per launch of the histogram kernel over a shard of data_bytes
    window bytes, measured by rocprofv3 PMC (profiles/pmc_*.json: one object or a
    list of them, one per shard size) on the build `build_id`; None when no
    measurement of this build matches (a counter of another build is never
    reported as this run's traffic)."""
    if not path or not os.path.exists(path) or build_id is None:
        return None
    with open(path) as f:
        pmc = json.load(f)
    for e in (pmc if isinstance(pmc, list) else [pmc]):
        if e.get("k") == k and e.get("data_bytes") == data_bytes and e.get("build_id") == build_id:
            return e.get("hbm_bytes_per_launch")
    return None


def lds_floor(path, k, build_id):
    """The LDS-array roof of the k = 8 histogram (7 array cycles per
    wave-wide ds_add_u32, 72 % of them bank conflicts of random bins): the share of
    the kernel's shader cycles in which an average CU's LDS array is busy
    (SQ_LDS_IDX_ACTIVE / CUs / (GRBM_GUI_ACTIVE / 8), rocprofv3 PMC of this bench
    command, profiles/pmc_lds_k8_10gbase.json).  None when not measured."""
    if k != 8 or not path or not os.path.exists(path) or build_id is None:
        return None
    with open(path) as f:
        m = json.load(f)
    return m if m.get("k") == k and "lds_busy_frac" in m and m.get("build_id") == build_id else None


def finalize(args, world, rank, backend, data, matrix, L, k, n_tot, win, elapsed, kern_ms, alg_bytes, timer,
             step_ms=None):
    """Everything after the timed region, at every N: the all-reduce timed alone,
    the max-over-ranks statistics, the reference CPU path on rank 0, and the JSON
    line (returned on rank 0, None elsewhere).  tests/test_multi.py runs it with
    gloo at world 2 on CPU tensors (timer "host")."""
    import torch.distributed as dist
    win_lo, win_hi = win
    nb = 1 << (2 * k)
    dev = matrix.device
    ar_ms = measure_allreduce(matrix, args.allreduce_reps, timer) if world > 1 else 0.0
    build_id = dense_code_object_id() if timer == "cuda" else None
    traffic = pmc_traffic(args.pmc, k, win_hi - win_lo, build_id)
    achieved_rank = alg_bytes / (kern_ms * 1e-3) / 1e9
    # per-step histogram kernel times of this rank (HIP events): the spread shows a
    # clock still ramping in the first timed steps
    st = sorted(step_ms) if step_ms else [kern_ms]
    med = st[len(st) // 2] if len(st) % 2 else 0.5 * (st[len(st) // 2 - 1] + st[len(st) // 2])
    # max over ranks of time-likes; min of achieved and of "traffic known" (as -x)
    elapsed, kern_ms, ar_ms, neg_ach, neg_known, traffic_max, k_med, k_min, k_max = over_ranks(
        world, [elapsed, kern_ms, ar_ms, -achieved_rank, -(1.0 if traffic is not None else 0.0),
                float(traffic or 0.0), med, st[0], st[-1]], dev)
    achieved = -neg_ach
    traffic = traffic_max if -neg_known > 0.5 else None  # every rank's shard size was measured

    kmers_per_step = n_tot * (L - k + 1)
    value = kmers_per_step * args.steps / elapsed
    # the whole job's algorithmic bytes per k-mer: every input
    # byte once + the int32 output once, over the windows
    job_bytes = n_tot * (L + 1) + 4 * nb * n_tot
    node_gbps = value * job_bytes / kmers_per_step / 1e9
    if args.scaling == "strong":
        par = ("one %.1f Gbase buffer cut into %d byte-range shard(s) (kmc_plan_shards, 4 KiB cuts, k-1 halo), "
               "RCCL all-reduce of the int32 count matrix overlapping the next step" % (n_tot * L / 1e9, world))
    else:
        par = ("%d records per GPU, RCCL all-reduce of the int32 count matrix overlapping the next step"
               % args.records)
    result = {
        "metric": "k-mers/sec (whole node), 10 Gbase synthetic FASTA, at 1/2/4/8 MI355X",
        "value": value,
        "unit": "k-mers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": {"ms": getattr(args, "settle_ms", 0.0), "launches": getattr(args, "settle_launches", 0),
                   "how": "untimed histogram launches back to back (this rank's count only) after the correctness "
                          "guard and before the W warm-up steps, for settle.ms of wall time, so that the GPU "
                          "clock has ramped up from the guard's host-side idle; the timed region is exactly K "
                          "full steps either way"},
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 uniform ACGT generated in HBM; SURVEY.md 8(d) layout)",
        "config": {
            "workload": "dense k=%d histogram, %d records x %d bases (%.1f Gbase) in total, %s"
                        % (k, n_tot, L, n_tot * L / 1e9,
                           "split over the GPUs" if args.scaling == "strong" else "%d records per GPU" % args.records),
            "k": k, "total_records": n_tot, "record_len": L, "bins": nb, "parallelism": par,
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "reserved_cus": getattr(args, "reserve_cus_eff", None),
            "rccl_max_channels": os.environ.get("NCCL_MAX_NCHANNELS") if world > 1 else None,
            "backend": dist.get_backend() if world > 1 else "none (1 GPU)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "kernel": "count_dense_kernel<%d> (HIP events around the histogram launch; slowest rank)" % k,
            "kernel_ms": kern_ms,
            "kernel_ms_median": k_med,
            "kernel_ms_min": k_min,
            "kernel_ms_max": k_max,
            "kernel_ms_steps": [round(x, 4) for x in (step_ms or [])] if rank == 0 else None,
            "kernel_ms_how": "per timed step, HIP events around the histogram launch; kernel_ms is their mean "
                             "(achieved / frac use it), median / min / max over the steps (each the slowest rank's); "
                             "kernel_ms_steps: rank 0's, in step order (a clock still ramping shows in the first)",
            "alg_bytes_per_launch": alg_bytes,
            "build_id": build_id,
            "traffic_how": ("HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE of this "
                            "shard size, taken on the build whose code-object id is build_id (%s); null when no PMC "
                            "entry of this build exists" % os.path.relpath(args.pmc, REPO)) if args.pmc else None,
            # the whole node: value x algorithmic bytes per k-mer of the job over N x peak
            "node_achieved": node_gbps,
            "node_peak": HBM_PEAK_GBPS * world,
            "node_frac": node_gbps / (HBM_PEAK_GBPS * world),
            "alg_bytes_per_kmer": job_bytes / kmers_per_step,
        },
        "allreduce": {
            "ms": ar_ms,
            "bytes": 4 * nb * n_tot,
            "how": ("%d synchronous all-reduces (SUM, int32) of a matrix shaped like the count matrix, timed alone "
                    "after the timed region with HIP events on the current stream (slowest rank); in the timed "
                    "steps each all-reduce overlaps the next step's counting" % args.allreduce_reps)
                   if world > 1 else "none (1 GPU)",
        },
    }
    # the roof that binds k = 8: the LDS array, not HBM
    m = lds_floor(getattr(args, "pmc_lds", None), k, build_id)
    if m is not None:
        result["roofline"].update({
            "binding": "lds",
            "lds_floor_ms": m["lds_busy_frac"] * kern_ms,
            "lds_floor_frac": m["lds_busy_frac"],
            "lds_how": "the k = 8 kernel is bound by its LDS array, not HBM: an average CU's array is busy "
                       "lds_floor_frac of the kernel's shader cycles (%.2f array cycles per wave-wide ds_add_u32, "
                       "%.0f %% of them bank-conflict cycles of random bins; SQ_LDS_IDX_ACTIVE / %d CUs / "
                       "(GRBM_GUI_ACTIVE / 8) over %d launches of the N = 1 bench command, %s); lds_floor_ms = that share "
                       "of kernel_ms, the time of the LDS work alone"
                       % (m["array_cycles_per_atomic"], 100 * m["conflict_frac"], m["cus"], m["launches"],
                          os.path.relpath(args.pmc_lds, REPO)),
        })
    if world > 1:
        dist.barrier()  # every rank's GPU work is done before rank 0 takes the host cores
    if rank == 0 and args.cpu_sample >= 0:
        result["cpu_baseline"] = run_cpu_baseline(args, data, k)
    if backend != "nccl":
        result["rehearsal"] = "KMC_BENCH_BACKEND=%s, %d ranks sharing device(s): not a measurement" % (backend, world)
    if world > 1:
        dist.barrier()
    return result if rank == 0 else None


if __name__ == "__main__":
    main()
