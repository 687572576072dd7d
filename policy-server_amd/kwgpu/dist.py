"""Multi-GPU plumbing: the compiled-table blob is built once on rank 0 and broadcast
to every rank (RCCL over xGMI with the "nccl" backend; gloo on CPU in the tests); each rank then
evaluates its own contiguous request shard. There is no collective on the per-request path."""
from . import EvaluationEnvironment


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
    """Weak scaling: rank r owns requests [r * rows_per_rank, (r + 1) * rows_per_rank)."""
    return rank * rows_per_rank, rows_per_rank
