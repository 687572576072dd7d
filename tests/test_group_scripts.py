"""CPU: policy-group scripts beyond the bool-only subset (expr.hpp: let bindings, if / else
expressions, statement sequences, integers, strings, rhai's mixed-type comparisons, checked
arithmetic, evaluation errors on some paths). The product's parser, validator and device forms
(truth table) against the oracle's independent interpreter (oracle.py parse_script / run_script):
validity and messages at load, verdict words through the slot compiler's host walk
(kw_debug_host_walk), and the response texts of rejections and evaluation errors.
Reference: evaluation_environment.rs:496-506 (validation), :596-611 (evaluation); the language
itself is upstream rhai 1.21.0 and parity beyond the pinned vectors is unpinned."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import diff_verdicts

MEMBERS = {  # members whose results vary over the parity mix (config 0)
    "ns": {"module": "registry://ghcr.io/kubewarden/policies/namespace-validate-policy:v0.1.0",
           "settings": {"valid_namespace": "kubewarden-approved"}},
    "priv": {"module": "registry://ghcr.io/kubewarden/policies/pod-privileged:v0.2.0"},
    "reg": {"module": "registry://ghcr.io/kubewarden/policies/trusted-repos-policy:v0.1.12",
            "settings": {"registries": {"allow": ["ghcr.io", "quay.io"]}}},
    "latest": {"module": "registry://ghcr.io/kubewarden/policies/trusted-repos-policy:v0.1.12",
               "settings": {"tags": {"reject": ["latest"]}}},
}

VALID = [
    "let a = ns(); let b = priv(); a || b",
    "let x = reg(); if x { latest() } else { ns() && priv() }",
    "if ns() { true } else if priv() { latest() } else { false }",
    "let n = if reg() { 1 } else { 2 }; n * 3 > 4 || latest()",
    '"ab" + "c" == "abc" && priv()',
    '"abc" < "abd" && (reg() | latest())',
    "ns() == 1 || priv()",             # mixed types compare unequal (rhai built-in)
    "ns() != 1 && priv() ^ reg()",
    "({ let y = 3; y * 2 }) > 5 && latest()",    # a block as an operand (a statement expression)
    "for x in [1] { } [ns()].contains(true)",     # two statements: a loop, then an array
    "let z = 5; let z = z + 1; z == 6 && reg()",
    "if priv() { true } else { ns() + 1 == 2 }",  # an evaluation error on one path only
    "if reg() { 1 } else { true }",               # not a bool on one path
    "latest(); ns() || priv()",                    # a discarded statement still calls its member
    "if reg() { ns() } else { priv() }; latest()",
]
INVALID = [
    "let = 1; ns()",
    "let a = ns() a",
    "ns() + 1",                 # fails when validated with every member true
    "if 1 { ns() } else { priv() }",
    "unknown_member() || ns()",
    'let s = "x; ns()',
    "x || ns()",
    "9223372036854775807 + 1 == 0 || ns()",
    "1 / 0 == 1",
    "{ let y = 3; y * 2 } > 5 && latest()",  # a block statement ends at its brace (rhai's parse_stmt)
]


def _doc(expr):
    return {"g": {"policies": MEMBERS, "expression": expr, "message": "group rejected"}}


@pytest.mark.parametrize("expr", VALID + INVALID)
def test_validity_and_messages_match_oracle(expr):
    doc = _doc(expr)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    P = oe.pol[oe.ids["g"]]
    assert P["valid"] is (expr in VALID), (expr, P["expr_error"])
    if expr in VALID:
        env.validate_settings("g")
    else:
        with pytest.raises(K.PolicyInitialization) as e:
            env.validate_settings("g")
        assert str(e.value) == P["expr_error"]


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_script_groups_host_walk_and_responses(origin):
    doc = {}
    for k, e in enumerate(VALID):
        doc.update({f"g{k}": dict(_doc(e)["g"], message=f"group {k} rejected")})
    env = K.EvaluationEnvironment(doc, continue_on_errors=True)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    ids = env.policy_ids()
    assert ids == [p["id"] for p in oe.pol]
    syn = K.SynthBatch(0, 400, seed=77)
    b = syn.batch()
    got = b.debug_host_walk(env, ids, origin)
    want = oe.eval(syn.soa(), ids, origin)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    v = got.reshape(400, len(ids))
    seen = set()
    for j, pid in enumerate(ids):
        if not env.is_group(j):
            continue
        members = env.group_members(j)
        for r in range(400):
            reason = (int(v[r, j]) >> 8) & 0xFF
            if reason not in (O.R_GROUP, O.R_GROUP_EXPR):
                continue
            seen.add(reason)
            resp = b.format_response(env, r, j, int(v[r, j]), [int(v[r, m]) for m in members], doc=syn.json(r))
            assert resp == oe.response_doc(syn.soa(), r, j, origin, doc=syn.json(r)), (pid, r)
    assert seen == {O.R_GROUP, O.R_GROUP_EXPR}
