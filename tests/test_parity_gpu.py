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
from helpers import config, diff_verdicts, wide_docs

pytestmark = pytest.mark.gpu
NS = "kubewarden"

CASES = [  # (policies file, synth config, rows)
    ("parity", 0, 20000),
    ("c1_namespace", 1, 20000),
    ("c2_trusted", 2, 20000),
    ("c3_group", 3, 20000),
    ("c4_64", 4, 4000),
    ("c5_mixed", 5, 2000),
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


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
@pytest.mark.parametrize("name,scfg,rows", CASES[:4])
def test_responses_match_oracle(name, scfg, rows, origin):
    """kw_format_response_doc (service epilogue, JSONPatch of accepted mutations included) == the
    oracle's restated AdmissionResponse."""
    env, oe = _envs(name)
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, 600, seed=77 + scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids, origin)
    v = b.verdicts().reshape(600, len(ids))
    soa = syn.soa()
    docs = [syn.json(r) for r in range(600)]
    checked = 0
    for r in range(600):
        for j, pid in enumerate(ids):
            members = env.group_members(j) if env.is_group(j) else []
            mv = [int(v[r, m]) for m in members] if members else None
            try:
                want = oe.response(soa, r, j, int(v[r, j]), mv, doc=docs[r])
            except KeyError as e:
                with pytest.raises(K.PolicyNotFound):
                    b.format_response(env, r, j, int(v[r, j]), mv, doc=docs[r])
                assert str(e).strip("'").startswith("unknown policy")
                continue
            got = b.format_response(env, r, j, int(v[r, j]), mv, doc=docs[r])
            assert got == want, (r, pid, got, want)
            checked += 1
    assert checked >= min(1000, 600 * len(ids) // 2)


def test_row_mode_equals_all_pairs():
    """kw_validate_rows (one policy per row, the micro-batcher shape) agrees with the all-pairs pass."""
    env, _ = _envs("parity")
    ids = env.policy_ids()
    n = 30000
    syn = K.SynthBatch(0, n, seed=5)
    b = syn.batch().to_device(0)
    b.validate(env, ids, K.VALIDATE)
    full = b.verdicts().reshape(n, len(ids))
    rng = np.random.default_rng(3)
    pick = rng.integers(0, len(ids), n)
    b.validate_rows(env, [int(x) for x in pick], K.VALIDATE)
    rows = b.verdicts(n)
    assert np.array_equal(rows, full[np.arange(n), pick])


def test_full_size_properties():
    """1M-request C4 batch: deterministic across launches, and every 4096-row slice evaluated as its
    own batch reproduces the full batch's verdicts (no cross-request state)."""
    env, oe = _envs("c4_64")
    ids = env.policy_ids()
    n = 1_000_000
    syn = K.SynthBatch(4, n, seed=4)
    b = syn.batch().to_device(0)
    b.validate(env, ids)
    v1 = b.verdicts()
    b.validate(env, ids)
    v2 = b.verdicts()
    assert np.array_equal(v1, v2)
    v1 = v1.reshape(n, len(ids))
    for start in (0, 123_456, n - 4096):
        sub = K.SynthBatch(4, 4096, seed=4, row0=start)
        sb = sub.batch().to_device(0)
        sb.validate(env, ids)
        assert np.array_equal(sb.verdicts().reshape(4096, len(ids)), v1[start:start + 4096])
        # and the oracle agrees on the slice
        assert np.array_equal(oe.eval(sub.soa(), ids).reshape(4096, len(ids)), v1[start:start + 4096])
    # sanity of the workload: both outcomes occur for every family
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
