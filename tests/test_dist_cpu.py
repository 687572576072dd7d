"""CPU, world size 2 over gloo: the multi-GPU plumbing of SURVEY §8(e) without a GPU.

* the compiled-table blob built on rank 0 reaches rank 1 intact (kwgpu.dist.broadcast_environment,
  the same function bench.py runs over RCCL), and the rebuilt environment answers the host-side
  accessors identically (policy ids, modes, allowed_to_mutate, namespace bypass);
* the weak-scaling shards partition the job: concatenating the ranks' synthetic shards gives
  exactly the rows of one batch generated at once (no cross-rank state, no data-path collective).
"""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from helpers import ROOT, config

ROWS = 257


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _strings(col, n):
    return [bytes(col.bytes[col.off[i]:col.off[i + 1]]) for i in range(n)]


def _worker(rank, world, port, out_dir):
    import sys

    for p in (os.path.join(ROOT, "policy-server_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import kwgpu as K
    from kwgpu.dist import broadcast_environment, shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        env = broadcast_environment(config("c5_mixed"), dist, rank, device=-1, continue_on_errors=True,
                                    always_accept_namespace="kubewarden")
        ids = env.policy_ids()
        row0, n = shard(ROWS, rank)
        syn = K.SynthBatch(5, n, seed=11, row0=row0)  # owns the columns the view points at
        soa = syn.soa()
        np.save(os.path.join(out_dir, f"blob{rank}.npy"), np.frombuffer(env.serialize(), dtype=np.uint8))
        facts = [ids, [env.get_policy_mode(i) for i in ids], [env.get_policy_allowed_to_mutate(i) for i in ids],
                 env.should_always_accept_requests_made_inside_of_namespace("kubewarden")]
        with open(os.path.join(out_dir, f"facts{rank}.txt"), "w") as f:
            f.write(repr(facts))
        with open(os.path.join(out_dir, f"uids{rank}.txt"), "wb") as f:
            f.write(b"\n".join(_strings(soa.uid, n)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_blob_broadcast_and_shards(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    b0, b1 = np.load(tmp_path / "blob0.npy"), np.load(tmp_path / "blob1.npy")
    assert b0.size > 0 and np.array_equal(b0, b1)
    assert (tmp_path / "facts0.txt").read_text() == (tmp_path / "facts1.txt").read_text()

    import kwgpu as K

    syn = K.SynthBatch(5, world * ROWS, seed=11)
    whole = syn.soa()
    want = _strings(whole.uid, world * ROWS)
    got = (tmp_path / "uids0.txt").read_bytes().split(b"\n") + (tmp_path / "uids1.txt").read_bytes().split(b"\n")
    assert got == want
