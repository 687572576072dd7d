"""Group scripts beyond the bool-only subset with more than 16 members (VERDICT r03 "What's
missing" 3): `let` / `if` / integers / strings over 40 members compile to typed bytecode (kwdev.hpp
SOp) that the wide path's combine kernel runs per row (slots.hpp run_script_prog); the oracle
evaluates them with its own interpreter (oracle.py run_script) over the members' own results.
CPU: the product's host walk of that bytecode against the oracle, words and responses."""
import random

import numpy as np
import pytest

import kwgpu as K
import oracle as O
from fuzz import MOD, _script, _settings
from helpers import diff_verdicts

NS = "kubewarden"


def big_script_policies(seed, nmem=40, ngroups=3):
    rng = random.Random(seed)
    doc = {}
    for g in range(ngroups):
        names = [f"m{j}" for j in range(nmem)]
        members = {}
        for nm in names:
            fam = rng.choice(["caps", "aa", "labels", "trusted", "ns", "priv"])
            while True:  # settings the schema accepts (a broken member would make the group answer 404)
                st = _settings(rng, fam)
                probe = O.OracleEnv({"p": {"module": MOD[fam], "settings": st}}, continue_on_errors=True)
                if not probe.pol[0]["init_error"]:
                    break
            members[nm] = {"module": MOD[fam], "settings": st}
        expr = _script(rng, names)
        if g == 0:  # every construct at least once: let, if / else, ints, strings, member calls
            expr = ('let n = if m0() { 1 } else { 2 }; let s = if m1() { "a" } else { "b" }; '
                    'let t = s + "x"; (n * 3 - 1 >= 2 && t != "ax") || (m2() && m3()) || m39() || '
                    '(if m7() { m8() == m9() } else { m10() ^ m11() }) && (n % 2 == 0 || m12())')
        doc[f"big-{g}"] = {"policies": members, "expression": expr, "message": f"big group {g} rejected"}
        if g == 2:
            doc[f"big-{g}"]["policyMode"] = "monitor"
    doc["plain"] = {"module": MOD["ns"], "settings": {"valid_namespace": "kubewarden-approved"}}
    return doc


def _envs(doc, device=-1):
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=device)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    assert env.policy_ids() == [p["id"] for p in oe.pol]
    return env, oe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_big_scripts_compile_and_host_walk_matches_oracle(seed):
    doc = big_script_policies(seed)
    env, oe = _envs(doc)
    for g in range(3):
        env.validate_settings(f"big-{g}")  # no engine-limit init error any more
    ids = env.policy_ids()
    for scfg in (4, 5):
        syn = K.SynthBatch(scfg, 1500, seed=seed * 10 + scfg)
        for origin in (K.VALIDATE, K.AUDIT):
            got = syn.batch().debug_host_walk(env, ids, origin)
            want = oe.eval(syn.soa(), ids, origin)
            assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    # not vacuous: the groups accept, reject and (some rows) fail to evaluate
    reasons = {(int(w) >> 8) & 0xFF for w in want.reshape(-1, len(ids))[:, :3].reshape(-1)}
    assert 0 in reasons and O.R_GROUP in reasons


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_big_scripts_on_gpu(seed):
    """The same through the HIP path: member pass, then the combine kernel's bytecode VM; words in
    both origins and in row mode, and responses (messages, cause lists of the big groups from the
    pass's side data) equal the oracle's derived ones."""
    from test_parity_gpu import _check_responses
    doc = big_script_policies(seed)
    env, oe = _envs(doc, device=0)
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 4000, seed=seed)
    b = syn.batch().to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(syn.soa(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, len(ids), syn.n)
    b.validate_rows(env, [ids[int(j)] for j in pick], K.AUDIT)
    assert np.array_equal(b.verdicts(count=syn.n), want.reshape(syn.n, len(ids))[np.arange(syn.n), pick])
    docs = [syn.json(i) for i in range(300)]
    hb = K.Batch.from_json(docs).to_device(0)
    hb.validate(env, ids, K.VALIDATE)
    assert _check_responses(env, oe, hb, hb.view(), docs, ids, K.VALIDATE, range(0, 300, 11)) > 0
