"""bench.py — batched admission evaluation on MI355X (BASELINE.json metric).

Workload (the configuration the metric "at 64 policies" is quoted on):
1M synthetic Pod AdmissionReviews per GPU x 64 compiled policies (22 psp-capabilities,
21 psp-apparmor, 21 safe-labels; configs/c4_64.yml). A step = one validate pass of the hot path
(string classification kernel + policy evaluation kernel) over the GPU's whole resident batch,
producing 64M verdict words. Inputs are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Multi-GPU: one process per GPU; rank 0 compiles the policy set and broadcasts the compiled-table
blob once over RCCL (torch.distributed "nccl" = RCCL on ROCm); every rank evaluates its own request
shard; no collective on the per-request path. With several GPUs and no size flag, `value` is BASELINE's
own multi-GPU workload, strong scaling: the config's request count as ONE job sharded across the GPUs
(C4: 1M requests over N GPUs; --config c5_mixed: 10M), and the same run then measures weak scaling
(that many requests per GPU) as the `weak_scaling` field. --rows R (per GPU, weak) or --total-rows T
(one job, strong) choose one measurement explicitly. Timing: barrier + synchronize on both sides of
exactly K steps, max over ranks. Rank 0 prints one JSON line.
"""
import hashlib
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "policy-server_amd"))

METRIC = "admission requests evaluated/sec (node) at 64 policies; HBM GB/s vs peak"
SEED = 20250509
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# BASELINE.json configs: policies file, synthetic workload id, default requests per GPU,
# and the workload named in the JSON line. The metric is quoted on C4 (the default); the others are
# measured with --config and committed under profiles/.
CONFIGS = {
    "c1_namespace": (1, 10_000, "C1 namespace_simple: {rows} synthetic Pod AdmissionReviews x namespace-validate "
                                "(valid_namespace kubewarden-approved)"),
    "c2_trusted": (2, 1_000_000, "C2 trusted-repos: {rows} synthetic Pods x trusted-repos (registries.allow "
                                 "[ghcr.io, quay.io, registry.k8s.io], tags.reject [latest])"),
    "c3_group": (3, 1_000_000, "C3 policy group: {rows} synthetic Pods x sigstore_pgp() || (sigstore_gh_action() && "
                               "reject_latest_tag()) (image-glob stand-ins for the sigstore members) + its 3 members"),
    "c4_64": (4, 1_000_000, "C4: {rows} synthetic Pod AdmissionReviews per GPU x {npol} compiled policies (c4_64.yml: "
                            "22 psp-capabilities, 21 psp-apparmor, 21 safe-labels)"),
    "c5_mixed": (5, 10_000_000, "C5 mixed-resource stream: {rows} synthetic Pods 70% / Deployments 20% / Namespaces "
                                "10%, containers Zipf(1.3) over 1..64, x the {npol} C4 policies"),
    "c6_256": (6, 1_000_000, "C6 (VERDICT r01 #3): {rows} synthetic Pods x {npol} columns (c6_256.yml: 256 policies "
                             "over 240 registries, 230 image globs, 150 label keys, a 40-member group, + members)"),
}


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=None, help="requests per GPU, weak scaling (default: the config's)")
    ap.add_argument("--total-rows", type=int, default=None,
                    help="a fixed job of this many requests sharded across the GPUs (strong scaling)")
    ap.add_argument("--config", default="c4_64", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (rank 0), about 10-30 s")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-modes", action="store_true", help="skip the end-to-end / flatten timings")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo, the host walk (kw_debug_host_walk) as the step over a 1/1000 sample of "
                         "the config's rows; exercises the argument path and the JSON fields only (tests)")
    args = ap.parse_args()
    dry = args.dry_run
    args.synth, default_rows, workload = CONFIGS[args.config]
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    also_weak = False
    if dry:
        default_rows = max(100, default_rows // 1000)
    if args.rows is None and args.total_rows is None:
        if world_env > 1:  # BASELINE's multi-GPU configs are fixed jobs: strong first, weak beside it
            args.total_rows = default_rows
            also_weak = True
        else:
            args.rows = default_rows

    import numpy as np
    import torch
    import yaml

    import kwgpu as K

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    dist = None
    if world > 1:
        import torch.distributed as dist
        if not dry:
            torch.cuda.set_device(local)
        dist.init_process_group("gloo" if dry else "nccl")
    device = -1 if dry else local
    sync = (lambda: None) if dry else torch.cuda.synchronize

    with open(os.path.join(ROOT, "configs", f"{args.config}.yml")) as f:
        policies = yaml.safe_load(f)

    # compiled tables: built once on rank 0, broadcast over RCCL to the other GPUs
    if world > 1:
        from kwgpu.dist import broadcast_environment

        env = broadcast_environment(policies, dist, rank, device=device, tensor_device="cpu" if dry else "cuda")
    else:
        env = K.EvaluationEnvironment(policies, device=device)
    ids = env.policy_ids()
    npol = len(ids)

    from kwgpu.dist import job_bounds

    def measure(total_rows=None, rows_per_rank=None):
        """One job (world x rows_per_rank requests, weak; or total_rows, strong) split into shards of
        equal work (1 + containers per request): generate this rank's shard resident in HBM, W warmup
        steps, then exactly K timed steps between barriers; the time is the max over ranks."""
        t0 = time.time()
        bounds, job_rows, scaling = job_bounds(args.synth, world, SEED, total_rows=total_rows, rows_per_rank=rows_per_rank)
        row0, nrows = int(bounds[rank]), int(bounds[rank + 1] - bounds[rank])
        syn = K.SynthBatch(args.synth, nrows, seed=SEED, row0=row0)
        batch = syn.batch() if dry else syn.batch().to_device(device)
        step = (lambda: batch.debug_host_walk(env, ids)) if dry else (lambda: batch.validate(env, ids))
        log(f"rank {rank}: {nrows} requests generated + resident in {time.time() - t0:.1f}s; {npol} policies ({scaling})")
        for _ in range(args.warmup):
            step()
        sync()
        if dist:
            dist.barrier()
        sync()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if dry else "cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return syn, batch, bounds, job_rows, scaling, nrows, elapsed

    weak = None
    if also_weak:  # the weak-scaling field first (its batch is released before the primary job's)
        wsyn, wbatch, _, wjob, _, wrows, welapsed = measure(rows_per_rank=default_rows)
        weak = {"value": wjob * args.steps / welapsed, "unit": "requests/s", "ms_per_step": welapsed * 1e3 / args.steps,
                "requests_per_gpu": wrows, "total_requests": wjob, "scaling": "weak",
                "workload": workload.format(rows=default_rows, npol=npol)}
        wbatch.close()
        del wsyn, wbatch
    syn, batch, bounds, job_rows, scaling, nrows, elapsed = measure(total_rows=args.total_rows, rows_per_rank=args.rows)
    ms_per_step = elapsed * 1e3 / args.steps
    value = job_rows * args.steps / elapsed

    # per-kernel device time with HIP events on the launch stream
    if dry:
        from types import SimpleNamespace
        tm = SimpleNamespace(classify_ms=0.0, evaluate_ms=ms_per_step, total_ms=ms_per_step, classify_bytes=0.0,
                             evaluate_bytes=0.0)
        args.no_cpu_baseline = args.no_host_modes = True
    else:
        tm = batch.timed(env, ids, warmup=2, reps=max(5, args.steps))
    kernels = {"classify": (tm.classify_ms, tm.classify_bytes), "evaluate": (tm.evaluate_ms, tm.evaluate_bytes)}
    dom = max(kernels, key=lambda k: kernels[k][0])
    ms, nbytes = kernels[dom]
    achieved = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    gather = None
    if dry:
        frac_allowed = None
    elif dist:
        # verdict words back to the host after the timed region: each rank copies its shard D2H into
        # its own disjoint slice of one shared host array (kwgpu.dist.gather_verdicts), rank 0 holds it
        from kwgpu.dist import gather_verdicts
        t = time.perf_counter()
        allv = gather_verdicts(batch, bounds, npol, dist, rank, world, tensor_device="cuda")
        if rank == 0:
            dt = time.perf_counter() - t
            flat = allv.reshape(-1)
            frac_allowed = sum(int(np.count_nonzero(flat[c:c + (1 << 26)] & K._native.KW_F_ALLOWED))
                               for c in range(0, flat.size, 1 << 26)) / max(flat.size, 1)
            gather = {"rows": int(allv.shape[0]), "bytes": int(allv.nbytes), "s": dt, "GB_per_s": allv.nbytes / dt / 1e9,
                      "how": "per-rank D2H into disjoint slices of one shared host file mapping"}
            del allv
    else:
        v = batch.verdicts()
        frac_allowed = float(((v & K._native.KW_F_ALLOWED) != 0).mean())
        del v

    result = None
    if rank == 0:
        traffic_bytes, traffic_src = (None, "dry run") if dry else traffic(args, nrows)
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(policies, ids, args)
        modes = None if args.no_host_modes else host_modes(env, ids, syn, device, args, nbytes)
        result = {
            "metric": METRIC, "value": value, "unit": "requests/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "u8", "data": "synthetic" + (" (dry run: host walk, no GPU)" if dry else ""),
            "config": {"workload": (workload.format(rows=args.rows, npol=npol) if scaling == "weak" else
                                    workload.format(rows=job_rows, npol=npol).replace(" per GPU", "")
                                    + f", one job sharded across {world} GPU(s)"
                                    + (f" (strong scaling; weak_scaling: {default_rows} per GPU)" if weak else "")),
                       "config": args.config, "requests_per_gpu": job_rows / world, "total_requests": job_rows,
                       "policies": npol, "parallelism": f"dp{world} (request shards)"},
            "evaluations_per_s": value * npol,
            "kernel_ms": {"classify": tm.classify_ms, "evaluate": tm.evaluate_ms, "total": tm.total_ms},
            "roofline": {"kernel": "evaluate_tiles_kernel",
                         "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_bytes,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": nbytes, "algorithmic_bytes_per_request": nbytes / nrows},
            "weak_scaling": weak,
            "cpu_baseline": cpu,
            "timing_modes": modes,
            "verdicts_final_allowed_fraction": frac_allowed,
            "shards": {"rows": [int(bounds[k + 1] - bounds[k]) for k in range(world)], "balance": "1 + containers"},
            "gather": gather,
        }
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


def pcie_rates(nbytes, reps=5):
    """Pinned host <-> HBM copy rates (GB/s, best of `reps`) of one `nbytes` buffer each way: the
    PCIe ceiling of the bulk path, which moves the pass's input columns in and its verdict words out."""
    import torch

    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    out = {}
    for name, fn in (("h2d", lambda: dev.copy_(host, non_blocking=True)), ("d2h", lambda: host.copy_(dev, non_blocking=True))):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        out[name] = nbytes / best / 1e9
    # both directions at once on two streams, in 16 interleaved pieces each way like the bulk path's
    # chunks (one whole buffer each way measured 57 or 97 GB/s from run to run): aggregate GB/s
    dev2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    host2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    cuts = [nbytes * i // 16 for i in range(17)]
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for a, b in zip(cuts, cuts[1:]):
            with torch.cuda.stream(s_in):
                dev[a:b].copy_(host[a:b], non_blocking=True)
            with torch.cuda.stream(s_out):
                host2[a:b].copy_(dev2[a:b], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    out["bidir"] = 2 * nbytes / best / 1e9
    del dev, host, dev2, host2
    return out


def host_modes(env, ids, syn, device, args, alg_bytes=None):
    """SURVEY §8(d) timing modes 2 and 3 beside the HBM-resident `value` (mode 1): the end-to-end
    batch rate (host SoA -> H2D -> kernel -> D2H of the verdicts; pageable host buffers, device
    allocation included) and the host JSON -> SoA flatten rate (kw_batch_from_json, 1 and N
    threads) on a sample of the same synthetic requests."""
    import torch

    import kwgpu as K
    out = {}
    import numpy as np
    npol = len(ids)

    def best_of(fn, reps=3, prep=None):
        best = None
        for _ in range(reps):
            hb = syn.batch()  # fresh host columns each time (nothing resident)
            if prep:
                prep(hb)
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn(hb)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
            hb.close()
        return best

    # two HBM-resident passes in flight (serving-like: kwhost's pipeline workers run theirs on separate
    # streams). Two device copies of the batch, each on its own stream, steps alternating between
    # them: the second pass's workgroups take the CUs the first one's last tile round leaves idle.
    # Reported beside `value` (one pass at a time), not as it.
    if device >= 0:
        ba, bb = syn.batch().to_device(device), syn.batch().to_device(device)
        try:
            for _ in range(2):
                ba.validate(env, ids)
                bb.validate(env, ids)
            torch.cuda.synchronize()
            k = max(10, args.steps)
            t = time.perf_counter()
            for i in range(k):
                (ba if i % 2 == 0 else bb).validate(env, ids)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            out["two_in_flight"] = {"value": syn.n * k / dt, "unit": "requests/s", "steps": k, "ms_per_step": dt * 1e3 / k,
                                    "what": "HBM-resident passes over two device copies of the batch, each on its own "
                                            "stream, alternating: two passes in flight"}
        finally:
            ba.close()
            bb.close()
    # the PCIe ceiling of the bulk path: its input columns in and its verdict words out, each at the
    # measured pinned copy rate of that direction (the two directions overlap)
    out_bytes = syn.n * npol * 4
    rates = pcie_rates(out_bytes)
    in_bytes = max(0.0, (alg_bytes or 0.0) - out_bytes)
    bound_s = max(in_bytes / (rates["h2d"] * 1e9), out_bytes / (rates["d2h"] * 1e9))
    bidir_s = (in_bytes + out_bytes) / (rates["bidir"] * 1e9)
    out["pcie"] = {"h2d_GB_per_s": rates["h2d"], "d2h_GB_per_s": rates["d2h"], "bidir_GB_per_s": rates["bidir"],
                   "bytes_in": in_bytes, "bytes_out": out_bytes,
                   "bulk_bound_requests_per_s": syn.n / bound_s if bound_s > 0 else None,
                   "bulk_bound_bidir_requests_per_s": syn.n / max(bound_s, bidir_s) if bound_s > 0 else None,
                   "what": "pinned copies of one verdict-array-sized buffer each way (best of 5); bound = rows / "
                           "max(input columns / H2D rate, verdict words / D2H rate); bidir: one buffer each way at "
                           "once on two streams in 16 interleaved pieces (aggregate rate), its bound = rows / "
                           "max(that, (in + out) / bidir)"}
    # pipelined bulk path (kw_validate_host): row chunks whose staging fill, H2D, kernel and D2H overlap
    pin = K.PinnedWords(syn.n * npol, device=device)
    try:
        dt = best_of(lambda hb: hb.validate_host(env, ids, out=pin.array, device=device))
        out["end_to_end"] = {"value": syn.n / dt, "unit": "requests/s", "rows": syn.n, "ms": dt * 1e3,
                             "what": "kw_validate_host: host SoA -> pinned staging (host workers) -> H2D -> evaluate -> "
                                     "D2H straight into a pinned verdict buffer the caller keeps, in overlapped "
                                     "262144-row chunks on three streams; plan and tile descriptors included, best of 3"}
        # the same with the batch's columns page-locked in place beforehand (kw_batch_pin_host, untimed;
        # its own cost reported beside): no staging fill on the host workers
        reg = []

        def pin_cols(hb):
            t = time.perf_counter()
            hb.pin_host(device)
            reg.append(time.perf_counter() - t)
        dt = best_of(lambda hb: hb.validate_host(env, ids, out=pin.array, device=device), prep=pin_cols)
        out["end_to_end_pinned_columns"] = {
            "value": syn.n / dt, "unit": "requests/s", "rows": syn.n, "ms": dt * 1e3, "pin_host_ms": min(reg) * 1e3,
            "what": "kw_validate_host as end_to_end, the batch's large columns page-locked in place before the "
                    "timed call (kw_batch_pin_host, pin_host_ms, not timed): H2D by DMA from the columns, no "
                    "staging fill; for a caller that keeps its batches or runs several passes over one"}
    finally:
        pin.close()
    vout = np.empty(syn.n * npol, dtype=np.uint32)  # a pageable verdict buffer, reused as a server would
    vout.fill(0)
    dt = best_of(lambda hb: hb.validate_host(env, ids, out=vout, device=device))
    out["end_to_end_pageable"] = {"value": syn.n / dt, "unit": "requests/s", "rows": syn.n, "ms": dt * 1e3,
                                  "what": "the same into a pageable verdict buffer (pinned bounce blocks, copy-out "
                                          "on the host workers overlapped with the next chunk)"}

    def serial(hb):
        hb.to_device(device)
        hb.validate(env, ids)
        hb.verdicts(out=vout)
    dt = best_of(serial)
    out["end_to_end_serial"] = {"value": syn.n / dt, "unit": "requests/s", "rows": syn.n, "ms": dt * 1e3,
                                "what": "unpipelined: kw_batch_to_device (every column) -> kw_validate_batch -> "
                                        "kw_batch_verdicts into the pageable buffer, best of 3"}
    import ctypes as C
    n = min(100_000, syn.n)
    docs = [syn.json(i).encode() for i in range(n)]
    nbytes = sum(len(d) for d in docs)
    arr = (C.c_char_p * n)(*docs)  # the C ABI call alone is timed
    lens = (C.c_size_t * n)(*[len(d) for d in docs])
    L = K._native.lib()
    threads = max(1, min(16, len(cpu_threads())))
    fl = {}
    for th in sorted({1, threads}):
        os.environ["KW_FLATTEN_THREADS"] = str(th)
        best = None
        for _ in range(3):  # best of three calls (the first also warms the flattener's per-thread buffers)
            h, bad, err = C.c_void_p(), C.c_int64(-1), C.create_string_buffer(512)
            t = time.perf_counter()
            rc = L.kw_batch_from_json(arr, lens, n, K._native.KW_DOC_ADMISSION_REVIEW, C.byref(h), C.byref(bad), err,
                                      len(err))
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
            if rc == 0:
                L.kw_batch_destroy(h)
        fl[str(th)] = n / best
    os.environ.pop("KW_FLATTEN_THREADS", None)
    out["flatten"] = {"unit": "requests/s", "by_threads": fl, "rows": n, "mean_doc_bytes": nbytes / n,
                      "what": "kw_batch_from_json: AdmissionReview JSON -> SoA columns"}
    return out


def library_sha256():
    """sha256 of the libkwgpu.so this process evaluates with (KWGPU_LIB or the in-tree build)."""
    import kwgpu._native as N
    h = hashlib.sha256()
    with open(N.LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def traffic(args, rows):
    """(HBM bytes per launch of the tiled kernel, provenance) from the committed PMC summary
    (profiles/traffic.json, written by scripts/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench, FETCH_SIZE doubled per the gfx950 calibration). The bytes are
    None when the file is absent, was measured on another workload or shard size, or on another build
    of the library (its sha256 differs from the running one's): a kernel change must not keep printing
    an old measurement."""
    # profiles/traffic.json holds the metric's config (C4); profiles/traffic_<config>.json the others
    # (written by scripts/pmc.sh, copied from the GPU box)
    t, name = None, None
    for name in ("traffic.json", f"traffic_{args.config}.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                t = json.load(f)
        except (OSError, ValueError):
            t = None
            continue
        if t.get("config") == args.config:
            break
    if t is None:
        return None, f"no profiles/traffic.json or traffic_{args.config}.json"
    if t.get("config") != args.config or t.get("rows") != rows:
        return None, f"profiles/{name} is for {t.get('config')} x {t.get('rows')} rows, not this workload"
    if t.get("lib_sha256") != library_sha256():
        return None, f"profiles/{name} was measured on another build of libkwgpu.so (sha256 differs)"
    return t.get("bytes_per_launch"), (f"profiles/{name}: {t.get('source')}; round {t.get('round')}; "
                                       f"lib sha256 {t.get('lib_sha256')[:16]}")


def cpu_threads():
    """The host cores this process may use: its affinity set, capped by the box's CPU share
    (OMP_NUM_THREADS, which gpurun boxes set to 16)."""
    cpus = sorted(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return cpus[:share] if share > 0 else cpus


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(policies, ids, args):
    """The oracle (C restatement of EvaluationEnvironment::validate, oracle/kworacle.c) on the host
    cores, one thread pinned per core, on a bounded sample of the same workload. The reference's own
    wasmtime path cannot run here (no Rust toolchain, policy modules are remote OCI artifacts:
    SURVEY §8(c))."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    import kwgpu as K
    cpus = cpu_threads()
    threads = len(cpus)
    oe = O.OracleEnv(policies)
    probe_rows = 2000
    syn = K.SynthBatch(args.synth, probe_rows, seed=SEED)
    t = time.perf_counter()
    oe.eval(syn.soa(), ids, threads=threads, cpus=cpus)
    per_row = (time.perf_counter() - t) / probe_rows
    # a sample of up to 2M requests, evaluated in repeated passes until the CPU budget is spent
    rows = int(min(2_000_000, max(probe_rows, args.cpu_seconds / 4 / max(per_row, 1e-9))))
    syn = K.SynthBatch(args.synth, rows, seed=SEED)
    soa = syn.soa()
    passes = 0
    t = time.perf_counter()
    while True:
        oe.eval(soa, ids, threads=threads, cpus=cpus)
        passes += 1
        dt = time.perf_counter() - t
        if dt >= args.cpu_seconds:
            break
    # the JSON-in variant: AdmissionReview documents -> SoA (the host flattener, same
    # threads) -> the restated validate, on a 100k-document sample
    import ctypes as C
    nj = min(100_000, rows)
    jsyn = K.SynthBatch(args.synth, nj, seed=SEED)
    docs = [jsyn.json(i).encode() for i in range(nj)]
    arr = (C.c_char_p * nj)(*docs)
    lens = (C.c_size_t * nj)(*[len(d) for d in docs])
    L = K._native.lib()
    os.environ["KW_FLATTEN_THREADS"] = str(threads)
    jpass, jt = 0, time.perf_counter()
    while True:
        h, bad, err = C.c_void_p(), C.c_int64(-1), C.create_string_buffer(512)
        rc = L.kw_batch_from_json(arr, lens, nj, K._native.KW_DOC_ADMISSION_REVIEW, C.byref(h), C.byref(bad), err, len(err))
        if rc != 0:
            raise RuntimeError(err.value)
        hb = K.Batch(h.value, None)
        oe.eval(hb.view(), ids, threads=threads, cpus=cpus)
        jpass += 1
        jdt = time.perf_counter() - jt
        if jdt >= args.cpu_seconds / 3:
            break
    os.environ.pop("KW_FLATTEN_THREADS", None)
    return {"value": rows * passes / dt, "unit": "requests/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{rows} synthetic {args.config} requests x {len(ids)} policies, {passes} passes ({dt:.1f}s, "
                      f"oracle/kworacle.c, {threads} threads pinned one per core)",
            "json_in": {"value": nj * jpass / jdt, "unit": "requests/s",
                        "sample": f"{nj} AdmissionReview documents, {jpass} passes ({jdt:.1f}s): kw_batch_from_json + "
                                  f"the restated validate, {threads} threads"}}


if __name__ == "__main__":
    main()
