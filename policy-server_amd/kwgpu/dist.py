"""Multi-GPU plumbing: the compiled-table blob is built once on rank 0 and broadcast
to every rank (RCCL over xGMI with the "nccl" backend; gloo on CPU in the tests); each rank then
evaluates its own contiguous request shard, with shard boundaries balanced by work (requests plus
containers); after the passes each rank copies its verdict words D2H into its own disjoint slice of
one shared host array (a file mapping). There is no collective on the per-request path."""
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


def job_bounds(config, world, seed, rows_per_rank=None, total_rows=None):
    """Shard bounds of a bench job (synth_bounds over the job's rows): weak scaling (the default) is
    `rows_per_rank` requests per rank, world * rows_per_rank in all; strong scaling is a fixed job of
    `total_rows` requests whatever the world size (BASELINE C4 "1M requests sharded across 8", C5 10M
    over 1/2/4/8). Returns (bounds, total_rows, scaling)."""
    if (rows_per_rank is None) == (total_rows is None):
        raise ValueError("exactly one of rows_per_rank / total_rows")
    if total_rows is not None:
        if total_rows < 0:
            raise ValueError("total_rows must be >= 0")
        return synth_bounds(config, total_rows, world, seed), int(total_rows), "strong"
    return synth_bounds(config, world * rows_per_rank, world, seed), int(world * rows_per_rank), "weak"


def balanced_shard(config, rows_per_rank, world, rank, seed):
    """Weak scaling with balanced work: the job is world * rows_per_rank synthetic requests, split by
    synth_bounds; returns (row0, n) of this rank's shard."""
    b = synth_bounds(config, world * rows_per_rank, world, seed)
    return int(b[rank]), int(b[rank + 1] - b[rank])


def _gather_dirs():
    import tempfile

    return ("/dev/shm", tempfile.gettempdir())


def _gather_dir(total_bytes):
    """Index into _gather_dirs() of the first file system with room for the job's verdict array:
    /dev/shm (tmpfs, shared pages), else the temp directory (page-cache backed); -1 when neither."""
    import os

    for k, d in enumerate(_gather_dirs()):
        try:
            st = os.statvfs(d)
        except OSError:
            continue
        if st.f_bavail * st.f_frsize >= total_bytes + (256 << 20):
            return k
    return -1


def gather_verdicts(source, bounds, npol, dist, rank, world, tensor_device="cpu", chunk_words=1 << 24):
    """The job's verdict words in one host array on rank 0: rows [bounds[k],
    bounds[k + 1]) come from rank k, which copies its shard (a device Batch after its pass, through
    kw_batch_verdicts' pinned bounce, or a host uint32 array, `chunk_words` at a time) straight
    into its own disjoint slice of one shared file mapping, so no rank holds a second copy and no
    verdict word crosses RCCL or any other collective: two broadcast int64s (the file's token and
    directory), one all-reduce that proves every rank mapped the same file, and one barrier.
    The file is unlinked as soon as every rank has it mapped, so a rank that fails later leaves
    nothing behind in tmpfs. When the ranks do not share one host (a rank could not open the file,
    or opened a different one) the words travel by point-to-point sends to rank 0 instead
    (`_gather_p2p`). Returns the (rows, npol) array on rank 0 and None elsewhere. Raises
    RuntimeError when no file system on rank 0's host has room for the words."""
    import os

    import torch

    total_words = int(bounds[world] - bounds[0]) * npol
    a = int(bounds[rank] - bounds[0]) * npol
    n = int(bounds[rank + 1] - bounds[rank]) * npol
    src = None
    if isinstance(source, np.ndarray):
        src = np.asarray(source, dtype=np.uint32).reshape(-1)
        if src.size != n:
            raise ValueError(f"rank {rank}: {src.size} verdict words, shard holds {n}")
    tok = [0, -1]
    name = None
    try:
        if rank == 0:  # rank 0 names, places and sizes the file (sparse until the ranks write)
            tok = [(os.getpid() << 24) | int.from_bytes(os.urandom(3), "little"), _gather_dir(total_words * 4)]
            if tok[1] >= 0:
                name = os.path.join(_gather_dirs()[tok[1]], f"kwgpu_verdicts_{tok[0]}.u32")
                with open(name, "wb") as f:
                    f.truncate(max(total_words, 1) * 4)
        t = torch.tensor(tok, dtype=torch.int64, device=tensor_device)
        dist.broadcast(t, 0)
        tok = [int(x) for x in t.cpu().tolist()]
        if tok[1] < 0:
            raise RuntimeError(f"no file system has room for {total_words * 4 / 1e9:.1f} GB of verdict words")
        path = os.path.join(_gather_dirs()[tok[1]], f"kwgpu_verdicts_{tok[0]}.u32")
        # every rank must map rank 0's file: same (st_dev, st_ino) everywhere, or nobody uses it
        mm, ident = None, [-1, -1]
        try:
            mm = np.memmap(path, dtype=np.uint32, mode="r+", shape=(max(total_words, 1),))
            st = os.stat(path)
            ident = [int(st.st_dev), int(st.st_ino)]
        except (OSError, ValueError):
            mm = None
        rd = torch.tensor([ident[0], ident[1], -ident[0], -ident[1]], dtype=torch.int64, device=tensor_device)
        dist.all_reduce(rd, op=dist.ReduceOp.MAX)  # max == -max(-x) == min: all equal iff max(x) == min(x)
        lo_hi = [int(x) for x in rd.cpu().tolist()]
        shared = lo_hi[0] >= 0 and lo_hi[0] == -lo_hi[2] and lo_hi[1] == -lo_hi[3]
        if rank == 0 and name is not None:
            os.unlink(name)  # every rank holds its mapping (or gave up on it): the name is no longer needed
            name = None
    finally:
        if rank == 0 and name is not None:
            os.unlink(name)
    if not shared:
        del mm
        return _gather_p2p(source, src, n, bounds, npol, dist, rank, world, tensor_device, chunk_words)
    mine = mm[a:a + n]
    if src is not None:
        for c in range(0, n, chunk_words):
            mine[c:c + chunk_words] = src[c:c + chunk_words]
    elif n:
        source.verdicts(count=n, out=mine)  # one D2H (pinned bounce) into the shared pages
    mm.flush()
    del mine
    dist.barrier()  # every slice written
    if rank != 0:
        del mm
        return None
    out = mm[:total_words]
    return out.reshape(-1, npol) if npol else out


def _gather_p2p(source, src, n, bounds, npol, dist, rank, world, tensor_device, chunk_words):
    """gather_verdicts across hosts: every rank k > 0 sends its shard to rank 0 in `chunk_words`
    pieces (point-to-point, in rank order); rank 0 assembles the whole array in its own memory."""
    import torch

    if src is None:
        src = np.empty(n, dtype=np.uint32)
        if n:
            source.verdicts(count=n, out=src)
    if rank != 0:
        for c in range(0, n, chunk_words):
            piece = torch.from_numpy(src[c:c + chunk_words].view(np.int32).copy()).to(tensor_device)
            dist.send(piece, 0)
        return None
    total_words = int(bounds[world] - bounds[0]) * npol
    out = np.empty(max(total_words, 1), dtype=np.uint32)
    out[:n] = src
    for k in range(1, world):
        a = int(bounds[k] - bounds[0]) * npol
        nk = int(bounds[k + 1] - bounds[k]) * npol
        for c in range(0, nk, chunk_words):
            m = min(chunk_words, nk - c)
            piece = torch.empty(m, dtype=torch.int32, device=tensor_device)
            dist.recv(piece, k)
            out[a + c:a + c + m] = piece.cpu().numpy().view(np.uint32)
    out = out[:total_words]
    return out.reshape(-1, npol) if npol else out
