"""Multi-GPU plumbing: the compiled-table blob is built once on rank 0 and broadcast
to every rank (RCCL over xGMI with the "nccl" backend; gloo on CPU in the tests); each rank then
evaluates its own contiguous request shard, with shard boundaries balanced by work (requests plus
containers); the verdict words are gathered back into disjoint slices of one host array after the
passes. There is no collective on the per-request path."""
import ctypes as C

import numpy as np

from . import EvaluationEnvironment
from . import _native as N


def broadcast_environment(policies, dist, rank, device=-1, tensor_device="cpu", **opts):
    """Rank 0 compiles `policies`; the blob (kw_env_serialize) goes to all ranks in two broadcasts
    (length, bytes); ranks != 0 rebuild it with kw_env_deserialize on `device`."""
    import torch

    if rank == 0:
        env = EvaluationEnvironment(policies, device=device, **opts)
        blob = env.serialize()
        n = torch.tensor([len(blob)], dtype=torch.int64, device=tensor_device)
    else:
        n = torch.zeros(1, dtype=torch.int64, device=tensor_device)
    dist.broadcast(n, 0)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=tensor_device)
    if rank == 0:
        buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    dist.broadcast(buf, 0)
    if rank != 0:
        env = EvaluationEnvironment.from_serialized(bytes(buf.cpu().numpy()), device=device)
    return env


def shard(rows_per_rank, rank):
    """Equal row counts: rank r owns requests [r * rows_per_rank, (r + 1) * rows_per_rank)."""
    return rank * rows_per_rank, rows_per_rank


def weight_bounds(ctr_off, world):
    """Contiguous shards of a batch with equal work, weight(row) = 1 + its containers (ctr_off is
    the batch's container offsets, n + 1 entries): bounds[0] = 0 <= ... <= bounds[world] = n, shard k
    = rows [bounds[k], bounds[k + 1]), each starting at the first row whose weight prefix reaches
    k / world of the total."""
    ctr_off = np.asarray(ctr_off, dtype=np.int64)
    n = len(ctr_off) - 1
    prefix = np.arange(n + 1, dtype=np.int64) + (ctr_off - ctr_off[0])  # weight of rows [0, r)
    total = int(prefix[-1])
    targets = [total * k // world for k in range(1, world)]
    inner = np.searchsorted(prefix, targets, side="left")
    return np.concatenate([[0], inner, [n]]).astype(np.int64)


def synth_bounds(config, total_rows, world, seed):
    """weight_bounds of the synthetic stream rows [0, total_rows) computed from the row shapes alone
    (kws_shard_bounds), so that every rank derives the same bounds without generating the rows."""
    out = (C.c_uint64 * (world + 1))()
    if N.synth().kws_shard_bounds(config, total_rows, seed, world, out) != 0:
        raise ValueError("kws_shard_bounds failed")
    return np.array(out[:], dtype=np.int64)


def balanced_shard(config, rows_per_rank, world, rank, seed):
    """Weak scaling with balanced work: the job is world * rows_per_rank synthetic requests, split by
    synth_bounds; returns (row0, n) of this rank's shard."""
    b = synth_bounds(config, world * rows_per_rank, world, seed)
    return int(b[rank]), int(b[rank + 1] - b[rank])


def gather_verdicts(verdicts, bounds, npol, dist, rank, world, tensor_device="cpu"):
    """Gathers every rank's verdict words (its shard's rows x npol, row-major) into disjoint slices
    of one host array on rank 0 (rows [bounds[k], bounds[k + 1]) from rank k); returns it on rank 0
    and None elsewhere. Shards may differ in size: each sends a zero-padded buffer of the largest
    shard (one gather; RCCL over xGMI when tensor_device is a GPU)."""
    import torch

    sizes = [int(bounds[k + 1] - bounds[k]) * npol for k in range(world)]
    mine = np.asarray(verdicts, dtype=np.uint32).reshape(-1)
    if mine.size != sizes[rank]:
        raise ValueError(f"rank {rank}: {mine.size} verdict words, shard holds {sizes[rank]}")
    cap = max(max(sizes), 1)
    send = torch.zeros(cap, dtype=torch.int32, device=tensor_device)
    send[: mine.size].copy_(torch.from_numpy(mine.view(np.int32)))
    recv = [torch.empty(cap, dtype=torch.int32, device=tensor_device) for _ in range(world)] if rank == 0 else None
    dist.gather(send, recv, dst=0)
    if rank != 0:
        return None
    out = np.empty(int(bounds[world] - bounds[0]) * npol, dtype=np.uint32)
    for k in range(world):
        a = int(bounds[k] - bounds[0]) * npol
        out[a: a + sizes[k]] = recv[k][: sizes[k]].cpu().numpy().view(np.uint32)
    return out.reshape(-1, npol) if npol else out
