"""GPU: the extended group-expression language on the device, in both device forms a non-bool
script takes (the truth table read in the tile kernel, and with KW_GROUP_FORM=script the typed
bytecode run by wide_groups_kernel), against the oracle's independent interpreter and the
hand-written rhai expectations (tests/rhai_cases.py). Verdict words poisoned first, so a skipped
pair cannot pass; responses formatted from the device words must equal the oracle's."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import diff_verdicts
from rhai_cases import VALID
from test_rhai_forms import MEMBERS, VECTORS, check_expected, groups_doc, review

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("form", ["table", "script"])
def test_forms_on_device_match_oracle(monkeypatch, form):
    monkeypatch.setenv("KW_POISON_VERDICTS", "1")
    if form == "script":
        monkeypatch.setenv("KW_GROUP_FORM", "script")
    else:
        monkeypatch.delenv("KW_GROUP_FORM", raising=False)
    doc = groups_doc(VALID)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    ids = env.policy_ids()
    # every member vector, repeated so that the combine kernel's grid strides over many pairs
    docs = [review(VECTORS[k % len(VECTORS)], f"uid-{k}") for k in range(8 * 64)]
    b = K.Batch.from_json(docs).to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(b.view(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    v = got.reshape(len(docs), len(ids))
    for k, (expr, cases) in enumerate(VALID):
        j = ids.index(f"g{k}")
        members = env.group_members(j)
        for acc, exp in cases:
            r = VECTORS.index(acc)
            resp = b.format_response(env, r, j, int(v[r, j]), [int(v[r, m]) for m in members], doc=docs[r])
            assert resp == oe.response_doc(b.view(), r, j, K.AUDIT, doc=docs[r]), (expr, acc)
    b.validate(env, ids, K.VALIDATE)
    v = b.verdicts().reshape(len(docs), len(ids))
    for k, (expr, cases) in enumerate(VALID):
        j = ids.index(f"g{k}")
        members = env.group_members(j)
        for acc, exp in cases:
            r = VECTORS.index(acc)
            resp = b.format_response(env, r, j, int(v[r, j]), [int(v[r, m]) for m in members], doc=docs[r])
            check_expected(resp, exp, (form, expr, acc))


@pytest.mark.parametrize("form", ["table", "script"])
def test_groups_without_members_on_device(monkeypatch, form):
    """a group with no members (evaluation_environment.rs:793-799, "2 > 1" with an empty
    policies map) next to wide script groups; its verdict and the script groups' causes must equal
    the oracle's (the combine kernel reads a group's cause words only when it has some)."""
    monkeypatch.setenv("KW_POISON_VERDICTS", "1")
    if form == "script":
        monkeypatch.setenv("KW_GROUP_FORM", "script")
    else:
        monkeypatch.delenv("KW_GROUP_FORM", raising=False)
    doc = {"empty_true": {"policies": {}, "expression": "2 > 1", "message": "m"},
           "empty_false": {"policies": {}, "expression": "let v = [1]; v.pop(); v.len() > 0", "message": "m"},
           "scripted": {"policies": MEMBERS, "expression": 'let s = "a"; s.make_upper(); s == "A" && a() && b()',
                        "message": "m"}}
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    ids = env.policy_ids()
    docs = [review(VECTORS[k % len(VECTORS)], f"uid-{k}") for k in range(256)]
    b = K.Batch.from_json(docs).to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(b.view(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


# KW_SCRIPT_SEEDS widens the sweep for a deep run (r06: profiles/r06_script_fuzz_deep.log)
@pytest.mark.parametrize("seed", range(int(__import__("os").environ.get("KW_SCRIPT_SEEDS", "3"))))
def test_random_scripts_on_device(monkeypatch, seed):
    """tests/fuzz.py's script generator (r06: with the standard-package functions and `&mut` method
    calls) in the typed-bytecode form run by wide_groups_kernel: 60 random groups per seed, every
    member vector, verdict words and formatted responses against the oracle's interpreter."""
    import random

    from fuzz import _script
    monkeypatch.setenv("KW_POISON_VERDICTS", "1")
    monkeypatch.setenv("KW_GROUP_FORM", "script")
    rng = random.Random(8000 + seed)
    rows = [(_script(rng, ["a", "b", "c"]), []) for _ in range(60)]
    doc = groups_doc(rows)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    ids = env.policy_ids()
    docs = [review(VECTORS[k % len(VECTORS)], f"uid-{k}") for k in range(len(VECTORS) * 16)]
    b = K.Batch.from_json(docs).to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(b.view(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    v = got.reshape(len(docs), len(ids))
    for k in range(len(rows)):
        j = ids.index(f"g{k}")
        members = env.group_members(j)
        for r in range(len(VECTORS)):
            resp = b.format_response(env, r, j, int(v[r, j]), [int(v[r, m]) for m in members], doc=docs[r])
            assert resp == oe.response_doc(b.view(), r, j, K.AUDIT, doc=docs[r]), (rows[k][0], VECTORS[r])
