"""GPU parity: verdict words from the HIP path (through the C ABI) == the oracle's, bit-exact.

Oracle: oracle/kworacle.c + oracle/oracle.py (CPU restatement; families parity-unpinned, service /
group semantics pinned by tests/golden). Inputs: seeded synthetic AdmissionReviews
(policy-server_amd/csrc/synth.cpp) at sizes the oracle finishes in seconds; full-size batches are
checked through size-independent properties (sub-batch invariance, determinism, row-mode ==
all-pairs mode).
"""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts, golden, many_policies_config, reference_doc, wide_docs, wide_entity_case

pytestmark = pytest.mark.gpu
NS = "kubewarden"


@pytest.fixture(autouse=True)
def _poisoned_verdicts(monkeypatch):
    """Every pass in this module starts from verdict words filled with a sentinel no verdict word
    equals (KW_POISON_VERDICTS, capi.cpp run_pass): a tile the schedule skipped cannot pass by
    keeping an earlier pass's words (the failure signature of r02's s45 build)."""
    monkeypatch.setenv("KW_POISON_VERDICTS", "1")

CASES = [  # (policies file, synth config, rows)
    ("parity", 0, 20000),
    ("c1_namespace", 1, 20000),
    ("c2_trusted", 2, 20000),
    ("c3_group", 3, 20000),
    ("c4_64", 4, 4000),
    ("c5_mixed", 5, 2000),
    ("c6_256", 6, 3000),
]


def _envs(name):
    doc = config(name)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    assert env.policy_ids() == [p["id"] for p in oe.pol]
    return env, oe


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
@pytest.mark.parametrize("name,scfg,rows", CASES)
def test_all_pairs_match_oracle(name, scfg, rows, origin):
    env, oe = _envs(name)
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=1000 + scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids, origin)
    gpu = b.verdicts()
    ora = oe.eval(syn.soa(), ids, origin)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)


def _check_responses(env, oe, b, soa, docs, ids, origin, rows):
    """kw_format_response_doc of every (row, column) == the oracle's response derived from the
    document itself (OracleEnv.response_doc: its own evaluation, full entity indices, its own
    short-circuit causes), never from the product's verdict word."""
    v = b.verdicts().reshape(len(docs), len(ids))
    checked = 0
    for r in rows:
        for j, pid in enumerate(ids):
            members = env.group_members(j) if env.is_group(j) else []
            mv = [int(v[r, m]) for m in members] if members else None
            try:
                want = oe.response_doc(soa, r, j, origin, doc=docs[r])
            except KeyError as e:
                with pytest.raises(K.PolicyNotFound):
                    b.format_response(env, r, j, int(v[r, j]), mv, doc=docs[r])
                assert str(e).strip("'").startswith("unknown policy")
                continue
            got = b.format_response(env, r, j, int(v[r, j]), mv, doc=docs[r])
            assert got == want, (r, pid, got, want)
            checked += 1
    return checked


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
@pytest.mark.parametrize("name,scfg,rows", CASES[:4] + CASES[6:])
def test_responses_match_oracle(name, scfg, rows, origin):
    env, oe = _envs(name)
    ids = env.policy_ids()
    n = 300
    syn = K.SynthBatch(scfg, n, seed=77 + scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids, origin)
    docs = [syn.json(r) for r in range(n)]
    checked = _check_responses(env, oe, b, syn.soa(), docs, ids, origin, range(n))
    assert checked >= min(1000, n * len(ids) // 2)


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_messages_exact_past_255(origin):
    """VERDICT r01 repro: 300 containers / 300 labels, the only violators at index 299 (and 270 /
    280): the GPU path names exactly them."""
    doc, pols = wide_entity_case()
    env = K.EvaluationEnvironment(pols, device=0)
    oe = O.OracleEnv(pols)
    ids = env.policy_ids()
    b = K.Batch.from_json([doc] * 3).to_device(0)
    b.validate(env, ids, origin)
    assert np.array_equal(b.verdicts(), oe.eval(b.view(), ids, origin))
    _check_responses(env, oe, b, b.view(), [doc] * 3, ids, origin, range(3))
    v = b.verdicts()
    got = b.format_response(env, 0, ids.index("caps"), int(v[ids.index("caps")]), doc=doc)
    assert got["status"]["message"] == "container 'c299' adds capability 'NET_ADMIN', which is not allowed"


def test_entity_indices_past_16_bits():
    """A request with 70,000 labels and another whose single container adds 70,000 capabilities:
    the violating entity's index does not fit ARG (KW_ARG_WIDE); the overflow path records it in
    the pass's side data and the response names the right entity."""
    n = 70_000
    labels = {f"k{i}": ("bad" if i == n - 1 else "ok") for i in range(n)}
    caps = ["CHOWN"] * (n - 1) + ["NET_ADMIN"]
    mk = lambda uid, meta, ctrs: {"request": {  # noqa: E731
        "uid": uid, "kind": {"group": "", "version": "v1", "kind": "Pod"},
        "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE", "userInfo": {},
        "object": {"kind": "Pod", "metadata": meta, "spec": {"containers": ctrs}}}}
    import json
    docs = [json.dumps(mk("labels", {"labels": labels}, [{"name": "a", "image": "nginx"}])),
            json.dumps(mk("caps", {}, [{"name": "big", "image": "nginx", "securityContext": {"capabilities": {"add": caps}}}])),
            json.dumps(mk("small", {"labels": {"k1": "bad"}}, [{"name": "s", "image": "nginx"}]))]
    mod = "registry://ghcr.io/kubewarden/policies/"
    pols = {"caps": {"module": mod + "psp-capabilities:v0.1.7", "settings": {"allowed_capabilities": ["CHOWN"]}},
            "labels": {"module": mod + "safe-labels:v0.1.14",
                       "settings": {"constrained_labels": {f"k{n - 1}": "^ok$", "k1": "^ok$"}}}}
    env = K.EvaluationEnvironment(pols, device=0)
    oe = O.OracleEnv(pols)
    ids = env.policy_ids()
    b = K.Batch.from_json(docs).to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        v = b.verdicts()
        assert np.array_equal(v, oe.eval(b.view(), ids, origin))
        assert v[0 * 2 + 1] >> 16 == K._native.KW_ARG_WIDE and v[1 * 2 + 0] >> 16 == K._native.KW_ARG_WIDE
        assert b.wide_arg(0, ids.index("labels")) == n - 1
        assert b.wide_arg(1, ids.index("caps")) == n - 1
        _check_responses(env, oe, b, b.view(), docs, ids, origin, range(3))
    got = b.format_response(env, 1, 0, int(v[2]), doc=docs[1])
    assert got["status"]["message"] == "container 'big' adds capability 'NET_ADMIN', which is not allowed"


@pytest.mark.parametrize("case", golden("reference_cases.json")["groups"], ids=lambda c: c["ref"])
def test_group_short_circuit_vectors_on_gpu(case):
    """evaluation_environment.rs:979-1042 through the HIP path: the reference's happy / unhappy OPA
    fixtures are stood in for by declarative members on its privileged-pod fixture (unhappy:
    pod-privileged, "Privileged container is not allowed"; happy: psp-capabilities allowing "*").
    Accepted or rejected as pinned, and the causes are exactly the pinned members (as a set)."""
    mod = "registry://ghcr.io/kubewarden/"
    members = {m: ({"module": mod + "tests/pod-privileged:v0.2.1"} if kind == "unhappy"
                   else {"module": mod + "policies/psp-capabilities:v0.1.7", "settings": {"allowed_capabilities": ["*"]}})
               for m, kind in case["members"].items()}
    pols = {"group": {"policies": members, "expression": case["expression"], "message": "group message"}}
    env = K.EvaluationEnvironment(pols, device=0)
    resp = env.evaluate("group", reference_doc("pod_with_privileged_containers.json"))
    assert resp["allowed"] is case["allowed"]
    if case["allowed"]:
        assert "status" not in resp and "warnings" not in resp
    else:
        causes = resp["status"]["details"]["causes"]
        assert sorted(c["field"] for c in causes) == sorted(c["field"] for c in case["causes"])
        assert all(c["message"] == "Privileged container is not allowed" for c in causes)
        assert resp["status"]["message"] == "group message"


@pytest.mark.parametrize("name,scfg", [("parity", 0), ("c6_256", 6)])
def test_row_mode_equals_all_pairs(name, scfg):
    """kw_validate_rows (one policy per row, the micro-batcher shape) agrees with the all-pairs pass
    (c6: the rows' distinct policies span several slot-plan chunks of one launch)."""
    env, _ = _envs(name)
    ids = env.policy_ids()
    n = 30000
    syn = K.SynthBatch(scfg, n, seed=5)
    b = syn.batch().to_device(0)
    b.validate(env, ids, K.VALIDATE)
    full = b.verdicts().reshape(n, len(ids))
    rng = np.random.default_rng(3)
    pick = rng.integers(0, len(ids), n)
    b.validate_rows(env, [int(x) for x in pick], K.VALIDATE)
    rows = b.verdicts(n)
    assert np.array_equal(rows, full[np.arange(n), pick])


def _oracle_threads():
    import os
    return max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.mark.parametrize("name,scfg,n", [("c4_64", 4, 1_000_000), ("c5_mixed", 5, 10_000_000), ("c2_trusted", 2, 1_000_000),
                                         ("c3_group", 3, 1_000_000), ("c1_namespace", 1, 1_000_000)])
def test_full_size_matches_oracle(name, scfg, n):
    """BASELINE sizes: C4 at 1M requests x 64 policies, C5 (mixed kinds, skewed container counts)
    at its 10M requests x 64 policies (640M verdict words), and C1-C3 at 1M (128-row tiles: the
    planner's taller layout), every verdict word against the oracle (C restatement, 16 threads);
    plus determinism across launches."""
    env, oe = _envs(name)
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, n, seed=scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids)
    v1 = b.verdicts()
    ora = oe.eval(syn.soa(), ids, threads=_oracle_threads())
    assert np.array_equal(v1, ora), diff_verdicts(v1, ora, len(ids), ids)
    b.validate(env, ids)
    assert np.array_equal(b.verdicts(), v1)
    allowed = (v1 & K._native.KW_F_ALLOWED) != 0
    assert allowed.any() and (~allowed).any()


def test_edge_batches():
    """Empty rows, no containers, huge container counts, long strings, empty batch."""
    doc = config("parity")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    long_img = "ghcr.io/" + "/".join(["seg%03d" % i for i in range(300)]) + ":v" + "9" * 500
    ctrs = [{"name": f"c{i}", "image": long_img if i % 7 == 0 else f"quay.io/x/y{i}:latest",
             "securityContext": {"privileged": i == 299, "capabilities": {"add": ["CHOWN"] * (i % 3)}}}
            for i in range(300)]
    docs = [
        {"request": {"uid": "a", "kind": {"group": "", "version": "v1", "kind": "Pod"},
                     "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE",
                     "userInfo": {}, "object": {"kind": "Pod", "metadata": {"labels": {"app": "x" * 5000}},
                                                "spec": {"containers": ctrs}}}},
        {"request": {"uid": "b", "kind": {"group": "", "version": "v1", "kind": "Pod"},
                     "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "DELETE",
                     "userInfo": {}, "object": None}},
        {"request": {"uid": "c", "kind": {"group": "", "version": "v1", "kind": "Pod"}, "namespace": NS,
                     "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE",
                     "userInfo": {}, "object": {"kind": "Pod", "spec": {"containers": []}}}},
    ]
    b = K.Batch.from_json(docs).to_device(0)
    b.validate(env, ids)
    gpu = b.verdicts()
    ora = oe.eval(b.view(), ids)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
    raw = K.Batch.from_json(['{"request": {"user": "tonio", "namespace": "kubewarden"}}', '{"request": null}'],
                            raw=True).to_device(0)
    raw.validate(env, ids)
    gpu = raw.verdicts()
    ora = oe.eval(raw.view(), ids)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
    empty = K.Batch.from_json([]).to_device(0)
    empty.validate(env, ids)
    assert len(empty.verdicts()) == 0


@pytest.mark.parametrize("q", ["0.5", "0.05"])
@pytest.mark.parametrize("name,scfg,rows", [CASES[0], CASES[4]])
def test_split_tiles_match_oracle(monkeypatch, name, scfg, rows, q):
    """Capacities forced below most tiles' needs (KW_TILE_QUANTILE): tiles run as halved request
    runs and single requests beyond the capacities take the overflow kernels; verdicts unchanged."""
    monkeypatch.setenv("KW_TILE_QUANTILE", q)
    env, oe = _envs(name)
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=4242 + scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids, K.VALIDATE)
    gpu = b.verdicts()
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)


@pytest.mark.parametrize("name,scfg,rows", [CASES[0], CASES[4], CASES[6]])
def test_global_tables_match_oracle(monkeypatch, name, scfg, rows):
    """Classifiers and slot records read from global memory (the path of policy sets whose tables
    exceed the per-workgroup LDS budget; forced here with KW_GLOBAL_TABLES)."""
    monkeypatch.setenv("KW_GLOBAL_TABLES", "1")
    env, oe = _envs(name)
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=99 + scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids, K.VALIDATE)
    gpu = b.verdicts()
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)


def test_caller_stream():
    """kw_validate_batch runs on the caller's hipStream_t (kwgpu.h): a pass on a torch stream, then
    one on the batch's own stream, both equal to the oracle."""
    import torch
    env, oe = _envs("c4_64")
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 20000, seed=5)
    b = syn.batch().to_device(0)
    s = torch.cuda.Stream(device=0)
    b.validate(env, ids, K.VALIDATE, stream=s.cuda_stream)
    v1 = b.verdicts()
    b.validate(env, ids[::-1], K.AUDIT)
    v2 = b.verdicts()
    assert np.array_equal(v1, oe.eval(syn.soa(), ids, K.VALIDATE))
    assert np.array_equal(v2, oe.eval(syn.soa(), ids[::-1], K.AUDIT))


def test_wide_requests():
    """Requests with more than 64 containers / labels (entity indices past one byte of the reason
    argument) among ordinary ones, C4 policies."""
    doc = config("c4_64")
    env = K.EvaluationEnvironment(doc, device=0)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    docs = wide_docs()
    b = K.Batch.from_json(docs).to_device(0)
    b.validate(env, ids)
    gpu = b.verdicts()
    ora = oe.eval(b.view(), ids)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_shared_slots_match_oracle(origin):
    """Copies of plain policies under other modes / allowedToMutate share one evaluation slot on the
    device (slotplan.cpp); each column still answers with its own mode."""
    from test_slots import dup_config
    doc = dup_config()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    syn = K.SynthBatch(0, 6000, seed=4242)
    b = syn.batch().to_device(0)
    b.validate(env, ids, origin)
    gpu = b.verdicts()
    ora = oe.eval(syn.soa(), ids, origin)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)


def test_repeated_passes_on_one_batch():
    """The dynamic tile schedule's per-XCD counters are zeroed by each launch's last workgroups:
    back-to-back passes over one resident batch (other policy lists and origins in between) all
    cover every tile."""
    env, oe = _envs("c4_64")
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 30000, seed=99)
    b = syn.batch().to_device(0)
    soa = syn.soa()
    for k, (cols, origin) in enumerate([(ids, K.VALIDATE), (ids[:20], K.AUDIT), (ids, K.VALIDATE),
                                        (ids[::-1], K.AUDIT), (ids, K.VALIDATE)]):
        b.validate(env, cols, origin)
        gpu = b.verdicts()
        ora = oe.eval(soa, cols, origin)
        assert np.array_equal(gpu, ora), f"pass {k}: " + diff_verdicts(gpu, ora, len(cols), cols)


@pytest.mark.parametrize("name,scfg,n,world", [("c4_64", 4, 1_000_000, 4), ("c5_mixed", 5, 2_000_000, 8)])
def test_serialized_blob_on_device_shards_match_oracle(name, scfg, n, world):
    """The multi-GPU path of SURVEY §8(e) on one device: the environment is compiled on the host
    (no device), its blob goes through kw_env_serialize -> kw_env_deserialize(device=0) (what every
    rank >= 1 runs after the RCCL broadcast), the job is cut into `world` shards by weight_bounds
    (1 + containers per request; equal to the synthetic stream's kws_shard_bounds), each shard is
    generated alone and validated on the GPU with the deserialized tables, and the concatenated
    verdict words equal the oracle's for the whole job, bit-exact."""
    from kwgpu.dist import synth_bounds, weight_bounds

    doc = config(name)
    host = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    env = K.EvaluationEnvironment.from_serialized(host.serialize(), device=0)
    ids = env.policy_ids()
    assert ids == host.policy_ids()
    seed = 31 + scfg
    whole = K.SynthBatch(scfg, n, seed=seed)
    soa = whole.soa()
    bounds = weight_bounds(np.ctypeslib.as_array(soa.ctr_off, shape=(n + 1,)), world)
    assert np.array_equal(bounds, synth_bounds(scfg, n, world, seed))
    parts = []
    for k in range(world):
        syn = K.SynthBatch(scfg, int(bounds[k + 1] - bounds[k]), seed=seed, row0=int(bounds[k]))
        b = syn.batch().to_device(0)
        b.validate(env, ids)
        parts.append(b.verdicts())
        b.close()
    got = np.concatenate(parts)
    ora = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS).eval(soa, ids, threads=_oracle_threads())
    assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)


@pytest.mark.parametrize("tile_rows", ["8", "24"])
def test_dynamic_schedule_covers_every_tile(monkeypatch, tile_rows):
    """Stress of the two-ahead per-XCD tile schedule (kernels.hip: the descriptor of the next tile
    copied into the LDS slot the previous tile used, the counter fetch for the tile after next read
    after the staging barrier, the XCD's last workgroup zeroing its counter): tiles forced down to
    8 / 24 requests (tens of thousands of tiles, a dozen per workgroup and XCD range), back-to-back
    passes over batches of very different sizes (1 to 300k rows: ranges of 0..4.7k tiles per XCD,
    so counters must restart from zero every launch), origins and policy lists alternating, every
    pass starting from poisoned verdict words, each compared with the oracle."""
    monkeypatch.setenv("KW_SLOT_ROWS", tile_rows)
    for name, scfg in (("c2_trusted", 2), ("c4_64", 4)):
        env, oe = _envs(name)
        ids = env.policy_ids()
        for k, n in enumerate([300_000, 1, 77, 5_003, 300_000 if scfg == 2 else 60_000]):
            syn = K.SynthBatch(scfg, n, seed=900 + k)
            b = syn.batch().to_device(0)
            for cols, origin in ((ids, K.VALIDATE), (ids[::-1], K.AUDIT)):
                b.validate(env, cols, origin)
                gpu = b.verdicts()
                ora = oe.eval(syn.soa(), cols, origin, threads=_oracle_threads())
                assert np.array_equal(gpu, ora), f"{name} rows {n}: " + diff_verdicts(gpu, ora, len(cols), cols)
            b.close()


def test_container_ranges_path_matches_oracle(monkeypatch):
    """The P2 form that ORs a container's predecessor ranges four loads a round (TileArgs::ctr_ranges,
    chosen when a tile's container capacity exceeds 4 x its rows): C5's Zipf container counts in
    8-row tiles are known to select it (asserted through the host plan), verdicts unchanged."""
    monkeypatch.setenv("KW_SLOT_ROWS", "8")
    env, oe = _envs("c5_mixed")
    ids = env.policy_ids()
    syn = K.SynthBatch(5, 20000, seed=515)
    b = syn.batch().to_device(0)
    plan = b.debug_plan(env, ids)
    assert plan["rows"] == 8 and plan["cmax"] > 4 * plan["rows"], plan
    b.validate(env, ids)
    gpu = b.verdicts()
    ora = oe.eval(syn.soa(), ids)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)


def test_wide_groups_match_oracle():
    """Groups past the jump-code limits (a 100-member group, a 100-deep == nest) on the GPU: the
    members' pass, the placeholder columns of the main pass and the combine kernel, against the
    oracle bit-exact in both origins and in row mode; causes (kw_batch_group_causes, the pass's
    multi-word side data) equal the oracle's as sets; responses equal the oracle's."""
    from test_wide_groups import wide_config
    doc = wide_config()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    n = 3000
    syn = K.SynthBatch(0, n, seed=41)
    b = syn.batch().to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        gpu = b.verdicts()
        ora = oe.eval(syn.soa(), ids, origin)
        assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
    v = gpu.reshape(n, len(ids))
    checked = 0
    for g in ("big", "deep"):
        j = ids.index(g)
        members = env.group_members(j)
        for r in range(n):
            if (int(v[r, j]) >> 8) & 0xFF != O.R_GROUP:
                continue
            want = oe.detail(syn.soa(), r, j, K.AUDIT)["causes"]
            assert b.group_causes(r, j, int(v[r, j])) == sorted(want), (g, r)
            if checked < 40:
                resp = b.format_response(env, r, j, int(v[r, j]), [int(v[r, m]) for m in members], doc=syn.json(r))
                assert resp == oe.response_doc(syn.soa(), r, j, K.AUDIT, doc=syn.json(r)), (g, r)
                checked += 1
    assert checked >= 40
    rng = np.random.default_rng(9)
    pick = rng.integers(0, len(ids), n)
    b.validate(env, ids, K.VALIDATE)
    full = b.verdicts().reshape(n, len(ids))
    b.validate_rows(env, [int(x) for x in pick], K.VALIDATE)
    assert np.array_equal(b.verdicts(n), full[np.arange(n), pick])
