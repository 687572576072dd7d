"""CPU, world size 2 over gloo: the multi-GPU plumbing of SURVEY §8(e) without a GPU.

* the compiled-table blob built on rank 0 reaches rank 1 intact (kwgpu.dist.broadcast_environment,
  the same function bench.py runs over RCCL), and the rebuilt environment answers the host-side
  accessors identically (policy ids, modes, allowed_to_mutate, namespace bypass);
* the shards are balanced by work (requests + containers, kws_shard_bounds on C5's Zipf container
  counts) and partition the job: concatenating the ranks' synthetic shards gives exactly the rows of
  one batch generated at once (no cross-rank state, no data-path collective);
* each rank EVALUATES its shard with its own environment (rank 1: the deserialized blob) through
  the slot compiler's host walk (kw_debug_host_walk: the device kernel's tables and walks on the
  host), each rank copies its verdict words into its own disjoint slice of one shared host array
  (kwgpu.dist.gather_verdicts: a /dev/shm file mapping, written in chunks, no collective carrying
  verdict words), and rank 0's array equals the oracle's verdicts for the whole job.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import ROOT, config

ROWS = 257
SEED = 11


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _strings(col, n):
    return [bytes(col.bytes[col.off[i]:col.off[i + 1]]) for i in range(n)]


def _worker(rank, world, port, out_dir, split=False):
    import sys

    for p in (os.path.join(ROOT, "policy-server_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import kwgpu as K
    import kwgpu.dist as D
    from kwgpu.dist import broadcast_environment, gather_verdicts, synth_bounds

    if split and rank > 0:  # this rank "lives on another host": rank 0's file is not in its directories
        own = os.path.join(out_dir, f"host{rank}")
        os.makedirs(own, exist_ok=True)
        D._gather_dirs = lambda: (own, own)

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        env = broadcast_environment(config("c5_mixed"), dist, rank, device=-1, continue_on_errors=True,
                                    always_accept_namespace="kubewarden")
        ids = env.policy_ids()
        bounds = synth_bounds(5, world * ROWS, world, SEED)
        row0, n = int(bounds[rank]), int(bounds[rank + 1] - bounds[rank])
        syn = K.SynthBatch(5, n, seed=SEED, row0=row0)  # owns the columns the view points at
        soa = syn.soa()
        np.save(os.path.join(out_dir, f"blob{rank}.npy"), np.frombuffer(env.serialize(), dtype=np.uint8))
        facts = [ids, [env.get_policy_mode(i) for i in ids], [env.get_policy_allowed_to_mutate(i) for i in ids],
                 env.should_always_accept_requests_made_inside_of_namespace("kubewarden")]
        with open(os.path.join(out_dir, f"facts{rank}.txt"), "w") as f:
            f.write(repr(facts))
        with open(os.path.join(out_dir, f"uids{rank}.txt"), "wb") as f:
            f.write(b"\n".join(_strings(soa.uid, n)))
        verdicts = syn.batch().debug_host_walk(env, ids)
        # each rank's words go straight into its slice of one shared file mapping, 1000 words a copy
        gathered = gather_verdicts(verdicts, bounds, len(ids), dist, rank, world, chunk_words=1000)
        if rank == 0:
            assert not [f for f in os.listdir("/dev/shm") if f.startswith("kwgpu_verdicts_")]  # name unlinked
            np.save(os.path.join(out_dir, "gathered.npy"), gathered)
            np.save(os.path.join(out_dir, "bounds.npy"), bounds)
        else:
            assert gathered is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,split", [(2, False), (3, False), (3, True)])
def test_blob_broadcast_shards_and_gathered_verdicts(tmp_path, world, split):
    """split: ranks 1.. cannot see rank 0's gather file (as on another host), so gather_verdicts
    must detect it and fall back to point-to-point sends, with the same result."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), split), nprocs=world, join=True)
    if split:
        assert not [f for r in range(1, world) for f in os.listdir(tmp_path / f"host{r}")]
    b0 = np.load(tmp_path / "blob0.npy")
    for r in range(1, world):
        assert b0.size > 0 and np.array_equal(b0, np.load(tmp_path / f"blob{r}.npy"))
        assert (tmp_path / "facts0.txt").read_text() == (tmp_path / f"facts{r}.txt").read_text()

    import kwgpu as K
    import oracle as O

    syn = K.SynthBatch(5, world * ROWS, seed=SEED)
    whole = syn.soa()
    want = _strings(whole.uid, world * ROWS)
    got = []
    for r in range(world):
        got += (tmp_path / f"uids{r}.txt").read_bytes().split(b"\n")
    assert got == want

    # the shards carry equal work (1 + containers per row), within one row's weight
    bounds = np.load(tmp_path / "bounds.npy")
    ctr = np.ctypeslib.as_array(whole.ctr_off, shape=(world * ROWS + 1,)).astype(np.int64)
    w = 1 + np.diff(ctr)
    loads = [int(w[bounds[k]:bounds[k + 1]].sum()) for k in range(world)]
    assert max(loads) - min(loads) <= 2 * int(w.max()), loads

    oe = O.OracleEnv(config("c5_mixed"), continue_on_errors=True, always_accept_namespace="kubewarden")
    ids = [p["id"] for p in oe.pol]
    gathered = np.load(tmp_path / "gathered.npy")
    expect = oe.eval(whole, ids).reshape(world * ROWS, len(ids))
    assert gathered.shape == expect.shape and np.array_equal(gathered, expect)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_job_bounds_weak_and_strong(world):
    """bench.py's shard arithmetic (kwgpu.dist.job_bounds): weak scaling is world x rows requests,
    strong scaling (--total-rows) a fixed job; either way the bounds partition the job's rows in
    order, and every shard's work (1 + containers per row, C5's Zipf counts) is within one row's
    weight of total / world."""
    import kwgpu as K
    from kwgpu.dist import job_bounds
    total = 997
    for kw in ({"total_rows": total}, {"rows_per_rank": total // world}):
        bounds, rows, scaling = job_bounds(5, world, SEED, **kw)
        assert scaling == ("strong" if "total_rows" in kw else "weak")
        assert rows == (total if "total_rows" in kw else world * (total // world))
        assert len(bounds) == world + 1 and bounds[0] == 0 and bounds[-1] == rows
        assert all(bounds[k] <= bounds[k + 1] for k in range(world))
        syn = K.SynthBatch(5, rows, seed=SEED)
        ctr = np.ctypeslib.as_array(syn.soa().ctr_off, shape=(rows + 1,)).astype(np.int64)
        w = 1 + np.diff(ctr)
        loads = [int(w[bounds[k]:bounds[k + 1]].sum()) for k in range(world)]
        assert max(loads) - min(loads) <= 2 * int(w.max()), loads
    with pytest.raises(ValueError):
        job_bounds(5, world, SEED)


def test_bench_multi_gpu_default_is_baselines_strong_job():
    """with WORLD_SIZE > 1 and no size flag, bench.py's `value` is BASELINE's own
    multi-GPU workload — the config's request count as one job sharded across the ranks (strong
    scaling: C4's 1M over N, C5's 10M) — and weak scaling (that many per rank) is measured beside it
    as `weak_scaling`. A 2-process gloo dry run (--dry-run: the host walk, 1/1000 of the rows)
    exercises that argument path and prints both fields."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(root, "bench.py"),
                          "--gpus", "2", "--steps", "2", "--warmup", "1", "--dry-run"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["total_requests"] == 1000  # C4's 1M / 1000 in a dry run, one job over both ranks
    assert sum(d["shards"]["rows"]) == 1000 and "one job sharded across 2 GPU(s)" in d["config"]["workload"]
    w = d["weak_scaling"]
    assert w["scaling"] == "weak" and w["total_requests"] == 2000 and w["value"] > 0
    assert d["value"] > 0 and "weak_scaling" in d["config"]["workload"]
