"""kmc_dist.py — one process per GPU: shard, count, all-reduce (torch.distributed).

SURVEY.md §8(e): every rank counts the windows starting in its byte range of
the global record buffer (reading a k-1 byte halo past it, kmc_count_dense_ex)
into the full [4^k][num_seqs] int32 matrix, zeros elsewhere; one all_reduce(SUM)
(RCCL over xGMI on MI355X) makes every rank hold the whole histogram.  Integer
sums: bit-exact and independent of the reduction order.

`counter(data, indices, k, shard)` returns a rank's partial (4^k, n) int32
matrix as a torch tensor on the collective's device; `gpu_counter` is the HIP
one.  Shard = (win_lo, win_hi, read_lo, read_hi) from kmc.plan_shards.
"""
import numpy as np

import kmc


def gpu_counter(device):
    """Partial histogram of one shard on `device` with the HIP kernel: only the
    shard's bytes plus its halo are copied to the device.  The library picks its
    workspace and CU count from the current HIP device, so the call runs with
    `device` current and on that device's stream, whatever the caller's current
    device is."""
    import torch

    device = torch.device(device)

    def count(data, indices, k, shard):
        win_lo, win_hi, read_lo, read_hi = shard
        n = len(indices) - 1
        with torch.cuda.device(device):
            out = torch.zeros((1 << (2 * k), n), dtype=torch.int32, device=device)
            if win_hi <= win_lo:
                return out
            base = read_lo & ~15  # keep (device pointer - base) 16-byte aligned
            chunk = torch.from_numpy(np.ascontiguousarray(data[base:read_hi])).to(device)
            idx = torch.from_numpy(np.ascontiguousarray(indices, dtype=np.int64)).to(device)
            args = kmc.dense_args(chunk, idx, k, out, read=(read_lo, read_hi), win=(win_lo, win_hi),
                                  data_offset=base)
            kmc.count_dense_ex(args, stream=torch.cuda.current_stream(device))
        return out

    return count


def check_record_windows(indices, k):
    """Raise KmcError(KMC_ERR_RECORD_TOO_LONG) when a record has 2^31 or more
    windows: every shard of it has fewer (no rank's device check fires), but the
    all_reduce adds the int32 parts of the whole record, which could wrap."""
    idx = np.asarray(indices, dtype=np.int64)
    if idx.size > 1 and int((np.diff(idx) - k).max()) >= 1 << 31:
        raise kmc.KmcError(kmc.KMC_ERR_RECORD_TOO_LONG, "count_sharded")


def count_sharded(data, indices, k, counter, group=None):
    """Histogram of the whole buffer, computed by this rank's shard + all_reduce."""
    import torch.distributed as dist

    check_record_windows(indices, k)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    shard = kmc.plan_shards(indices, k, world)[rank]
    part = counter(data, indices, k, shard)
    dist.all_reduce(part, op=dist.ReduceOp.SUM, group=group)
    return part
