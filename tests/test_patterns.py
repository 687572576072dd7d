"""CPU: the pattern-dialect and automaton-size cases (tests/pattern_cases.py) through the product's
host walk (kw_debug_host_walk: the blob's tables, NFA elements run by the host Pike VM) against the
oracle, and the environment-level behaviour VERDICT r03 asked for: a valid pattern never fails the
environment, whatever its automaton size; refused constructs are init errors on both sides with the
same message."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import diff_verdicts
from pattern_cases import policies, reviews

VALID = ["labels-dialect", "labels-unicode", "labels-blowup", "images-blowup", "registries-blowup", "images-mixed", "images-utf8"]


def test_blowup_patterns_never_fail_the_environment():
    """Without continue_on_errors, a set of only valid patterns builds (no BootstrapFailure), and no
    policy carries an init error: the blow-up patterns became NFA elements."""
    doc = {k: v for k, v in policies().items() if k in VALID}
    env = K.EvaluationEnvironment(doc, continue_on_errors=False)
    O.OracleEnv(doc, continue_on_errors=False)
    for pid in VALID:
        assert env.policy_initialization_error(pid) is None
        env.validate_settings(pid)


def test_refused_constructs_are_init_errors_on_both_sides():
    doc = policies()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    for pid in ("labels-refused", "labels-lookaround"):
        msg = env.policy_initialization_error(pid)
        assert msg and msg.startswith("Policy settings are invalid:")
        assert msg == oe.pol[oe.lookup(pid)]["init_error"]
    with pytest.raises(K.PolicyInitialization):  # settings validation fails the build (evaluation_environment.rs:216-225)
        K.EvaluationEnvironment(doc, continue_on_errors=False)
    with pytest.raises(O.ConfigError):
        O.OracleEnv(doc, continue_on_errors=False)


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_host_walk_matches_oracle(origin):
    doc = policies()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    ids = env.policy_ids()
    docs = reviews()
    b = K.Batch.from_json(docs)
    got = b.debug_host_walk(env, ids, origin)
    want = oe.eval(b.view(), ids, origin)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    # the cases are not vacuous: every valid policy both accepts and rejects some rows
    v = want.reshape(len(docs), len(ids))
    for j, pid in enumerate(ids):
        if pid in VALID:
            allowed = v[:, j] & 1
            assert allowed.any() and not allowed.all(), pid
