"""CPU: policy groups past the jump-code limits: more than 64 members, and
value stacks deeper than 64 (== / != nesting). Such a group's members run as a separate pass and
its expression runs over their verdict words (expr.hpp "wide"; kernels.hip wide_groups_kernel).
Here: the slot compiler's host walk (kw_debug_host_walk, the same jump code on the host) against
the oracle's recursive evaluation, bit-exact, in both origins. The reference builds a group over
any number of members (evaluation_environment.rs:613-648, config.rs:386-388). The GPU twin, with
causes compared as sets and responses, is in tests/test_parity_gpu.py."""
import random

import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import diff_verdicts

NS_MOD = "registry://ghcr.io/kubewarden/policies/namespace-validate-policy:v0.1.0"
TR_MOD = "registry://ghcr.io/kubewarden/policies/trusted-repos-policy:v0.1.12"
PRIV_MOD = "registry://ghcr.io/kubewarden/policies/pod-privileged:v0.2.0"
CAPS_MOD = "registry://ghcr.io/kubewarden/policies/psp-capabilities:v0.1.7"


def member(rng, k):
    f = k % 4
    if f == 0:
        return {"module": NS_MOD, "settings": {"valid_namespace": rng.choice(["ns-001", "ns-002", "kubewarden-approved"])}}
    if f == 1:
        return {"module": TR_MOD, "settings": {"registries": {"allow": rng.sample(["ghcr.io", "quay.io", "gcr.io",
                                                                                   "registry.k8s.io"], 2)}}}
    if f == 2:
        return {"module": PRIV_MOD}
    return {"module": CAPS_MOD, "settings": {"allowed_capabilities": rng.sample(["NET_ADMIN", "CHOWN", "KILL", "SETUID",
                                                                                  "SYS_TIME"], 3)}}


def tree(rng, names, depth):
    if depth <= 0 or rng.random() < 0.15:
        return f"{rng.choice(names)}()"
    op = rng.choice(["||", "&&", "||", "&&", "==", "!="])
    t = f"({tree(rng, names, depth - 1)} {op} {tree(rng, names, depth - 1)})"
    return f"!{t}" if rng.random() < 0.1 else t


def wide_config(seed=7, nmem=100):
    rng = random.Random(seed)
    names = [f"m{k:03d}" for k in range(nmem)]
    members = {n: member(rng, k) for k, n in enumerate(names)}
    # every member appears at least once: a chain over all of them, mixed with a random tree
    chain = " || ".join(f"({names[k]}() && {names[k + 1]}())" for k in range(0, nmem - 1, 2))
    big = {"policies": members, "expression": f"({chain}) && {tree(rng, names, 6)}", "message": "big group rejected"}
    # a value stack deeper than 64: == nested 100 deep on the right over 20 members
    d_names = names[:20]
    deep_expr = "true"
    for k in range(100):
        deep_expr = f"({d_names[k % 20]}() == {deep_expr})"
    deep = {"policies": {n: members[n] for n in d_names}, "expression": deep_expr, "message": "deep group rejected"}
    plain = {"plain-ns": {"module": NS_MOD, "settings": {"valid_namespace": "ns-001"}}}
    return {**plain, "big": big, "deep": deep, "small": {"policies": {n: members[n] for n in names[:3]},
                                                         "expression": f"{names[0]}() || {names[1]}() && {names[2]}()",
                                                         "message": "small"}}


def test_wide_groups_compile_as_wide():
    env = K.EvaluationEnvironment(wide_config(), continue_on_errors=True)
    oe = O.OracleEnv(wide_config(), continue_on_errors=True)
    for g in ("big", "deep", "small"):
        env.validate_settings(g)
        assert oe.pol[oe.ids[g]]["valid"]
    assert len(env.group_members(env.lookup("big"))) == 100
    assert O.expr_depth(oe.pol[oe.ids["deep"]]["ast"]) > 64


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_wide_groups_host_walk_matches_oracle(origin):
    doc = wide_config()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    ids = env.policy_ids()
    assert ids == [p["id"] for p in oe.pol]
    syn = K.SynthBatch(0, 500, seed=31)
    got = syn.batch().debug_host_walk(env, ids, origin)
    want = oe.eval(syn.soa(), ids, origin)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    v = got.reshape(500, len(ids))
    for g in ("big", "deep"):
        col = v[:, ids.index(g)]
        reasons = set(int(x) >> 8 & 0xFF for x in col)
        assert O.R_GROUP in reasons and 0 in reasons, (g, reasons)  # both outcomes occur
