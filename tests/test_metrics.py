"""Batched metrics (kw_metrics_*): the reference's series and attribute sets, recorded from verdict
words. The expected samples are restated here from src/metrics.rs:49-140 and the recording sites of
service::evaluate (src/api/service.rs:40-71 namespace bypass, :78-84 initialization error,
:118-150 evaluated); the verdict words come from the oracle (CPU), so no device is needed."""
import json

import numpy as np

import kwgpu as K
import oracle as O
from helpers import config

BOUNDS = [0, 5, 10, 25, 50, 75, 100, 250, 500, 750, 1000, 2500, 5000, 7500, 10000]


def _docs(n):
    syn = K.SynthBatch(0, n, seed=11)
    docs = []
    for i in range(n):
        d = json.loads(syn.json(i))
        r = d["request"]
        if i % 3 == 0:
            r["requestKind"] = {"group": "apps" if i % 2 else "", "version": "v1", "kind": "Deployment" if i % 2 else "Pod"}
        if i % 7 == 0:
            r["namespace"] = "kubewarden"  # the always-accept namespace: bypass
        if i % 11 == 0:
            r.pop("namespace", None)
        if i % 5 == 0:
            r["operation"] = "UPDATE"
        docs.append(d)
    return docs


def _expected(env, docs, pols, verdicts, lat, origin, raw):
    """{(metric, labels): value} as the reference would record them, one call per (row, policy)."""
    out = {}

    def add(key, v=1):
        out[key] = out.get(key, 0) + v

    for d, p, v, ms in zip(docs, pols, verdicts, lat):
        v = int(v)
        pid = env.policy_id(p)
        fst = (v & K._native.KW_F_STATUS_MASK) >> K._native.KW_F_STATUS_SHIFT
        if fst == K._native.KW_FST_INIT_ERROR:  # PolicyInitializationError: counter only
            labels = frozenset({("policy_name", pid), ("initialization_error", env.policy_initialization_error(p))})
            add(("kubewarden_policy_evaluations_total", labels))
            continue
        mode = "monitor" if env.get_policy_mode(p) == K.PolicyMode.Monitor else "protect"
        if v & K._native.KW_BYPASS:
            accepted, mutated, code = True, False, None
        else:
            accepted, mutated = bool(v & K._native.KW_V_ALLOWED), bool(v & K._native.KW_V_MUTATED)
            code = 500 if ((v >> 8) & 0xff) == 14 else None  # KW_R_GROUP_EXPR
        kv = {("policy_name", pid), ("policy_mode", mode), ("accepted", str(accepted).lower()),
              ("mutated", str(mutated).lower())}
        if not raw:
            r = d["request"]
            kv |= {("resource_kind", (r.get("requestKind") or {}).get("kind", "")),
                   ("resource_request_operation", r["operation"]),
                   ("request_origin", "audit" if origin == K.AUDIT else "validate")}
            if isinstance(r.get("namespace"), str):
                kv.add(("resource_namespace", r["namespace"]))
        if code is not None:
            kv.add(("error_code", str(code)))
        labels = frozenset(kv)
        add(("kubewarden_policy_evaluations_total", labels))
        for b in BOUNDS:
            add(("kubewarden_policy_evaluation_latency_milliseconds_bucket", labels | {("le", str(b))}),
                1 if ms <= b else 0)
        add(("kubewarden_policy_evaluation_latency_milliseconds_bucket", labels | {("le", "+Inf")}))
        add(("kubewarden_policy_evaluation_latency_milliseconds_sum", labels), ms)
        add(("kubewarden_policy_evaluation_latency_milliseconds_count", labels))
    return out


def _run(origin, raw):
    doc = config("parity")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden", device=-1)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    ids = env.policy_ids()
    assert ids == [oe.pol[i]["id"] for i in range(len(ids))]
    n = 96
    docs = _docs(n)
    batch = K.Batch.from_json([{"request": d["request"]["object"]} if raw else d for d in docs], raw=raw)
    top = [i for i in range(len(ids)) if "/" not in ids[i]]  # the addressed policies (not group members)
    pols = [top[i % len(top)] for i in range(n)]
    full = oe.eval(batch.view(), list(range(len(ids))), origin).reshape(n, len(ids))
    verdicts = [int(full[i, pols[i]]) for i in range(n)]
    lat = [(0, 3, 7, 60, 260, 20000)[i % 6] for i in range(n)]
    m = K.Metrics()
    m.record(env, batch, list(range(n)), pols, verdicts, lat, origin)
    got = m.samples()
    want = _expected(env, docs, pols, verdicts, lat, origin, raw)
    assert got == want
    return m, verdicts


def test_metrics_validate_match_the_reference_attribute_sets():
    m, v = _run(K.VALIDATE, raw=False)
    text = m.render()
    assert "# TYPE kubewarden_policy_evaluations_total counter" in text
    assert "# TYPE kubewarden_policy_evaluation_latency_milliseconds histogram" in text
    flags = np.array(v, dtype=np.uint32)
    assert (flags & K._native.KW_BYPASS).any()  # the always-accept namespace was exercised
    assert 'error_code="500"' in text  # group-int: non-bool expression
    assert "initialization_error=" in text  # bad-settings / group-invalid
    assert 'resource_kind="Deployment"' in text and 'resource_kind=""' in text


def test_metrics_audit_and_raw():
    m, _ = _run(K.AUDIT, raw=False)
    assert 'request_origin="audit"' in m.render()
    m, _ = _run(K.VALIDATE, raw=True)
    text = m.render()
    assert "resource_kind" not in text and "request_origin" not in text


def test_metrics_accumulate_and_reset():
    doc = config("parity")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden", device=-1)
    batch = K.Batch.from_json(_docs(2))
    p = env.lookup("pod-privileged")
    m = K.Metrics()
    for _ in range(3):
        m.record(env, batch, [0, 1], [p, p], [K._native.KW_V_ALLOWED | K._native.KW_F_ALLOWED] * 2, [1, 1])
    tot = [v for (name, _), v in m.samples().items() if name == "kubewarden_policy_evaluations_total"]
    assert sum(tot) == 6
    m.reset()
    assert not m.samples()
    try:
        m.record(env, batch, [5], [p], [0], [0])  # row out of range: KW_E_ARG, nothing recorded
        raise AssertionError("expected an error")
    except K.EvaluationError:
        pass
    assert not m.samples()
