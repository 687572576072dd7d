"""CPU: the slot compiler (slotplan.cpp) and the bit-parallel entity walks (slots.hpp) that the
device's evaluate_slots_kernel runs agree with the oracle, bit-exact, on every configuration.

kw_debug_host_walk runs the sequential form of the slot walks (slots.hpp walk_*) on the host with
the blob's column automata; the device computes the same first violations entity-parallel. It is
a diagnostic of the slot compiler only (the product path is the GPU: kw_validate_* never calls it);
the GPU parity tests (test_parity_gpu.py) check the kernel itself against the oracle.
Covers: every family, monitor mode, allowedToMutate, groups with short-circuit causes, init errors,
the namespace bypass, raw requests, both origins, policy lists with repeats and > 64 slots (several
column chunks), and the edge documents of the GPU edge test.
"""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts, many_policies_config, wide_docs, wide_entity_case

NS = "kubewarden"
CASES = [("parity", 0, 3000), ("c1_namespace", 1, 2000), ("c2_trusted", 2, 3000), ("c3_group", 3, 3000),
         ("c4_64", 4, 1500), ("c5_mixed", 5, 800)]


def _envs(name):
    doc = config(name)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    return env, oe


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
@pytest.mark.parametrize("name,scfg,rows", CASES)
def test_host_walk_matches_oracle(name, scfg, rows, origin):
    env, oe = _envs(name)
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=500 + scfg)
    b = syn.batch()
    got = b.debug_host_walk(env, ids, origin)
    want = oe.eval(syn.soa(), ids, origin)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


def test_chunked_policy_lists():
    """Repeated columns, groups split across chunk boundaries, > 64 slots and unaligned chunks."""
    env, oe = _envs("parity")
    ids = env.policy_ids()
    rng = np.random.default_rng(7)
    cols = [ids[int(i)] for i in rng.integers(0, len(ids), 150)]
    syn = K.SynthBatch(0, 700, seed=9)
    b = syn.batch()
    got = b.debug_host_walk(env, cols)
    want = oe.eval(syn.soa(), cols)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(cols), cols)
    c4, o4 = _envs("c4_64")
    ids4 = c4.policy_ids()
    cols = ids4 + ids4[:37]  # 101 columns: one full chunk and one unaligned
    syn = K.SynthBatch(4, 500, seed=10)
    got = syn.batch().debug_host_walk(c4, cols)
    want = o4.eval(syn.soa(), cols)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(cols), cols)


def test_edge_documents():
    env, oe = _envs("parity")
    ids = env.policy_ids()
    ctrs = [{"name": f"c{i}", "image": f"quay.io/x/y{i}:latest",
             "securityContext": {"privileged": i == 99, "capabilities": {"add": ["CHOWN"] * (i % 3), "drop": ["ALL"]}}}
            for i in range(100)]
    docs = [
        {"request": {"uid": "a", "kind": {"group": "", "version": "v1", "kind": "Pod"},
                     "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE",
                     "userInfo": {}, "object": {"kind": "Pod", "metadata": {"labels": {"app": "x" * 500, "debug": "1"}},
                                                "spec": {"containers": ctrs}}}},
        {"request": {"uid": "b", "kind": {"group": "", "version": "v1", "kind": "Pod"},
                     "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "DELETE",
                     "userInfo": {}, "object": None}},
        {"request": {"uid": "c", "kind": {"group": "", "version": "v1", "kind": "Pod"}, "namespace": NS,
                     "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE", "userInfo": {}, "object": {"kind": "Pod", "spec": {"containers": []}}}},
    ]
    b = K.Batch.from_json(docs)
    got = b.debug_host_walk(env, ids)
    want = oe.eval(b.view(), ids)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    raw = K.Batch.from_json(['{"request": {"user": "tonio", "namespace": "kubewarden"}}', '{"request": null}'], raw=True)
    got = raw.debug_host_walk(env, ids)
    want = oe.eval(raw.view(), ids)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


def test_wide_documents():
    doc = config("c4_64")
    env, oe = K.EvaluationEnvironment(doc), O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(wide_docs())
    got = b.debug_host_walk(env, ids)
    want = oe.eval(b.view(), ids)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


def dup_config():
    """parity.yml plus copies of its plain policies under other names, modes and allowedToMutate:
    equal compiled settings share one slot (slotplan.cpp build_slot_chunks), the column words keep
    each copy's own mode / mutation constraint."""
    import copy
    doc = config("parity")
    out = dict(doc)
    for name, e in doc.items():
        if "module" not in e:
            continue
        for k, (mode, a2m) in enumerate([("monitor", False), ("protect", True), ("monitor", True)]):
            c = copy.deepcopy(e)
            c["policyMode"] = mode
            c["allowedToMutate"] = a2m
            out[f"{name}-dup{k}"] = c
    return out


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_shared_slots_keep_column_modes(origin):
    doc = dup_config()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    assert len(ids) > 64  # several chunks, duplicates within and across them
    syn = K.SynthBatch(0, 1200, seed=77)
    got = syn.batch().debug_host_walk(env, ids, origin)
    want = oe.eval(syn.soa(), ids, origin)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


def test_many_policies_host_walk():
    """configs/c6_256.yml: 256 policies (+ a 40-member group's members as columns), hundreds of
    patterns per column, several slot chunks in one list; the group's causes beyond the 16-bit ARG."""
    doc = many_policies_config()
    env, oe = K.EvaluationEnvironment(doc), O.OracleEnv(doc)
    ids = env.policy_ids()
    assert len(ids) >= 256 + 40
    syn = K.SynthBatch(6, 600, seed=66)
    got = syn.batch().debug_host_walk(env, ids)
    want = oe.eval(syn.soa(), ids)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    g = ids.index("group-40")
    v = got.reshape(600, len(ids))[:, g]
    rejected = (v & K._native.KW_F_ALLOWED) == 0
    assert rejected.any() and (~rejected).any()
    assert all(((w >> 16) == K._native.KW_ARG_WIDE) for w in v[rejected])  # causes live in the side data


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_messages_exact_past_255(origin):
    """A request with 300 containers and 300 labels where only container c299 adds a capability the
    policy does not allow and only label k299 fails its constraint: the responses name exactly them
    (the verdict word carries full entity indices; the oracle derives its response from the
    document, not from the word)."""
    doc, pols = wide_entity_case()
    env, oe = K.EvaluationEnvironment(pols), O.OracleEnv(pols)
    ids = env.policy_ids()
    b = K.Batch.from_json([doc])
    v = b.debug_host_walk(env, ids, origin)
    assert np.array_equal(v, oe.eval(b.view(), ids, origin))
    got = {pid: b.format_response(env, 0, j, int(v[j]), doc=doc) for j, pid in enumerate(ids)}
    for j, pid in enumerate(ids):
        assert got[pid] == oe.response_doc(b.view(), 0, j, origin, doc=doc), pid
    assert got["caps"]["status"]["message"] == "container 'c299' adds capability 'NET_ADMIN', which is not allowed"
    assert got["labels"]["status"]["message"] == "label 'k299' value 'bad' does not match the constraint '^ok$'"
    assert got["labels-denied"]["status"]["message"] == "label 'k280' is denied"
    assert got["apparmor"]["status"]["message"] == ("container 'c270' uses AppArmor profile 'localhost/evil', "
                                                    "which is not allowed")


def test_planner_budget():
    """The tile kernel's plan on the host (kw_debug_plan): C4 fits four 256-thread workgroups per CU
    (<= 40 KB of LDS each, the occupancy the bench is measured at), and the 256-policy set runs all
    its slot-plan chunks in one launch (each request staged and classified once)."""
    c4 = K.EvaluationEnvironment(config("c4_64"))
    p = K.SynthBatch(4, 50000, seed=1).batch().debug_plan(c4, c4.policy_ids())
    assert p["lds_bytes"] <= 160 * 1024 // 4 and p["lds_tables"] == 1 and p["chunks"] == 1, p
    c6 = K.EvaluationEnvironment(many_policies_config())
    p = K.SynthBatch(6, 5000, seed=1).batch().debug_plan(c6, c6.policy_ids())
    assert p["chunks"] >= 5 and p["launches"] == 1, p


def test_planner_tile_height():
    """Tile height (kw_debug_plan rows): 64 requests for small batches and for layouts whose
    per-request LDS needs them for four workgroups per CU (C4); for large batches with small
    per-request LDS (C2 trusted-repos, C3 group) the tallest of 128..96 rows that keeps four or more
    workgroups per CU and sends at most 2 % of its tiles' image segments past one round of the
    workgroup's 256 lanes (synth containers 1+Geom(0.5): 112 rows, 1.9 % of tiles over 256)."""
    import numpy as np
    c4 = K.EvaluationEnvironment(config("c4_64"))
    p = K.SynthBatch(4, 600_000, seed=1).batch().debug_plan(c4, c4.policy_ids())
    assert p["rows"] == 64, p
    for name, scfg in (("c2_trusted", 2), ("c3_group", 3)):
        env = K.EvaluationEnvironment(config(name))
        small = K.SynthBatch(scfg, 50_000, seed=1).batch().debug_plan(env, env.policy_ids())
        assert small["rows"] == 64, (name, small)
        bb = K.SynthBatch(scfg, 600_000, seed=1).batch()
        big = bb.debug_plan(env, env.policy_ids())
        assert 96 <= big["rows"] <= 128 and big["lds_bytes"] <= 160 * 1024 // 4, (name, big)
        v = bb.view()
        co = np.ctypeslib.as_array(v.ctr_off, (v.n_requests + 1,)).astype(np.int64)
        per_tile = np.diff(co[::big["rows"]])
        assert (per_tile > 256).mean() <= 0.02, (name, big["rows"], (per_tile > 256).mean())
        if big["rows"] < 128:  # the next taller candidate would have sent more than 2 % past one round
            taller = np.diff(co[::big["rows"] + 8])
            assert (taller > 256).mean() > 0.02, (name, big["rows"])


def test_planner_host_workers_back_to_back():
    """The planner's host parallel-fors (tile needs, capacity quantiles, descriptors) run back to back
    with different task counts (small and large batches alternating, from two Python threads) and
    always return the same plan: a parallel-for never runs another call's tasks (r03: a worker late
    for one call could take an index of the next, past its task count, and hang it)."""
    import threading
    c4 = K.EvaluationEnvironment(config("c4_64"))
    ids = c4.policy_ids()
    sizes = (300_000, 90, 70_000, 1)
    mine = [[K.SynthBatch(4, n, seed=3).batch() for n in sizes] for _ in range(2)]  # a batch per thread
    want = [b.debug_plan(c4, ids) for b in mine[0]]
    errors = []

    def hammer(k):
        try:
            for it in range(60):
                j = (it + k) % len(sizes)
                assert mine[k][j].debug_plan(c4, ids) == want[j]
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)
    th = [threading.Thread(target=hammer, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "planner parallel-for hung"
    assert not errors, errors
