"""Sharding and the N>1 path on CPU: shard plans, and world_size-2 gloo runs of
the shard + all_reduce driver with the oracle as the per-shard counter (the
checker stands in for the HIP kernel; the GPU tests check the kernel's shards)."""
import os
import socket

import numpy as np
import pytest


def _records(seed, lens):
    rng = np.random.default_rng(seed)
    recs = []
    for L in lens:
        s = rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=L, p=[.24, .24, .24, .24, .04])
        recs.append(np.append(s, np.uint8(0)))
    data = np.concatenate(recs)
    idx = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.int64)
    return data, idx


@pytest.mark.parametrize("n", [1, 2, 3, 8, 13])
def test_plan_shards_cover_disjoint_aligned(kmc, n):
    data, idx = _records(1, [10_000, 1, 70_000, 5000, 123_457])
    k = 5
    plan = kmc.plan_shards(idx, k, n)
    assert len(plan) == n
    assert plan[0][0] == idx[0] and plan[-1][1] == idx[-1]
    for (a, b, rl, rh), nxt in zip(plan, plan[1:] + [None]):
        assert a <= b and rl == a and rh == min(b + k - 1, idx[-1])
        if nxt is not None:
            assert nxt[0] == b and b % 4096 == 0
    sizes = [b - a for a, b, _, _ in plan]
    assert max(sizes) - min(sizes) <= 2 * 4096


def test_plan_shards_sum_to_full_with_oracle(kmc, oracle):
    data, idx = _records(2, [50_000, 3, 30_000])
    full, inv = oracle.count_dense(data, idx, 6)
    for n in (2, 5, 64):
        acc = np.zeros_like(full)
        ainv = np.zeros_like(inv)
        for a, b, rl, rh in kmc.plan_shards(idx, 6, n):
            p, pi = oracle.count_dense(data, idx, 6, win=(a, b))
            acc += p
            ainv += pi
        np.testing.assert_array_equal(acc, full)
        np.testing.assert_array_equal(ainv, inv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, k, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "dna-kmeres-parallel_amd"), os.path.join(repo, "oracle")]
    import torch
    import torch.distributed as dist

    import kmc_dist
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data, idx = _records(3, [40_000, 2, 90_001, 7, 60_000])

    def cpu_counter(d, ix, kk, shard):  # the checker standing in for the HIP kernel
        part, _ = oracle.count_dense(d, ix, kk, win=(shard[0], shard[1]))
        return torch.from_numpy(part)

    out = kmc_dist.count_sharded(data, idx, k, cpu_counter)
    full, _ = oracle.count_dense(data, idx, k)
    q.put((rank, bool(np.array_equal(out.numpy(), full)), int(out.sum())))
    dist.destroy_process_group()


@pytest.mark.parametrize("k", [3, 8])
def test_gloo_world2_shard_allreduce(k):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert res[0][2] == res[1][2]


def _overlap_worker(rank, world, port, steps, q):
    """bench.py's overlapped steps with a CPU stand-in for the count: each step
    writes rank- and step-specific values into this rank's columns; after the
    async gloo all-reduces every matrix must hold the sum over ranks of its last
    step's columns."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import torch
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nb, n_loc = 64, 3
    n_tot = n_loc * world
    bufs = [torch.full((nb, n_tot), -7, dtype=torch.int32) for _ in range(2)]
    last_step = [None, None]

    def count(j):  # this rank's columns only, every entry overwritten
        i = last_step[j]
        cols = torch.arange(n_loc, dtype=torch.int32) + rank * n_loc
        bufs[j][:, rank * n_loc:(rank + 1) * n_loc] = (i * 1000 + cols)[None, :] + torch.arange(nb, dtype=torch.int32)[:, None]

    step, drain = bench.overlapped_steps(bufs, count, world, dist.all_reduce)
    ok = True
    for i in range(steps):
        j = i % 2
        last_step[j] = i
        step(i)
    drain()
    for j in range(2):
        i = last_step[j]
        exp = (i * 1000 + torch.arange(n_tot, dtype=torch.int32))[None, :] + torch.arange(nb, dtype=torch.int32)[:, None]
        ok = ok and bool(torch.equal(bufs[j], exp))
    q.put((rank, ok))
    dist.destroy_process_group()


def test_gloo_world2_bench_overlapped_allreduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, 7, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
