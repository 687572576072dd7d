"""Containers' predecessor sets by a segmented wave OR-scan (kernels.hip seg_or_scan_excl, the
kFeatRng instantiation). Where tiles carry many containers per request
(TileArgs::ctr_ranges: C5's heavy region) P2 takes the union of a container's predecessors in its
request — the sets that decide which container is a slot's first violation
(service.rs validation_response_with_constraints: the first offending entity in object order) —
from a scan over the wave's lanes instead of per-lane loops; a request that began before the
wave's first container adds that part from LDS in lane 0.

The documents below put many violating containers in one request (so the first-violation index
depends on every predecessor), requests of 0 to 150 containers (segments that start before a
wave, span one or several waves, or end at its last lane), and requests with no pod spec among
them. CPU: the planner launches such a batch as the scan instantiation and C4's as the plain
one. GPU: verdict words against the oracle, both origins."""
import random

import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts

NS = "kubewarden"
CAPS = ["AUDIT_WRITE", "CHOWN", "SETGID", "SETUID", "SYS_ADMIN", "SYS_TIME", "NET_ADMIN", "KILL", "DAC_OVERRIDE",
        "MKNOD", "NET_RAW", "FOWNER", "SYS_PTRACE", "NET_BIND_SERVICE"]
PROFILES = ["runtime/default", "localhost/custom", "unconfined", "localhost/evil"]
KEYS = ["app", "tier", "env", "team", "owner"]


def scan_docs(n=700, seed=3):
    rng = random.Random(seed)
    docs = []
    for r in range(n):
        u = rng.random()
        n_ctr = 0 if u < 0.04 else rng.randint(65, 150) if u < 0.12 else rng.randint(1, 5) if u < 0.2 else rng.randint(6, 40)
        ctrs, ann = [], {}
        for i in range(n_ctr):
            sc = {}
            if rng.random() < 0.7:
                sc["capabilities"] = {"add": rng.sample(CAPS, rng.randint(0, 3)),
                                      "drop": rng.sample(CAPS, rng.randint(0, 2))}
            if rng.random() < 0.05:
                sc["privileged"] = True
            ctrs.append({"name": f"c{i}", "image": "nginx", "securityContext": sc})
            if rng.random() < 0.3:
                ann[f"container.apparmor.security.beta.kubernetes.io/c{i}"] = rng.choice(PROFILES)
        meta = {"labels": {k: rng.choice(["a", "b", "prod", "x" * 9]) for k in rng.sample(KEYS, rng.randint(0, 3))},
                "annotations": ann}
        pod = rng.random() >= 0.06
        obj = {"kind": "Pod", "metadata": meta, "spec": {"containers": ctrs}} if pod else \
              {"kind": "ConfigMap", "metadata": meta, "data": {"k": "v"}}
        kind = "Pod" if pod else "ConfigMap"
        docs.append({"request": {"uid": str(r), "kind": {"group": "", "version": "v1", "kind": kind},
                                 "resource": {"group": "", "version": "v1", "resource": kind.lower() + "s"},
                                 "operation": "CREATE", "userInfo": {}, "namespace": "default", "object": obj}})
    return docs


def test_scan_instantiation_planned():
    doc = config("c5_mixed")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    b = K.Batch.from_json(scan_docs())
    p = b.debug_plan(env, ids)
    assert p["cmax"] > 4 * p["rows"] and p["scan_regions"] == 1, p
    c4 = K.EvaluationEnvironment(config("c4_64"))
    p4 = K.SynthBatch(4, 5000, seed=1).batch().debug_plan(c4, c4.policy_ids())
    assert p4["scan_regions"] == 0, p4


def test_host_walk_matches_oracle():
    """The documents through the host walk (the slot compiler's sequential form) against the oracle."""
    doc = config("c5_mixed")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    b = K.Batch.from_json(scan_docs(300, seed=4))
    got = b.debug_host_walk(env, ids).reshape(-1)
    want = oe.eval(b.view(), ids).reshape(-1)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


@pytest.mark.gpu
@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_scan_matches_oracle(origin):
    doc = config("c5_mixed")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    b = K.Batch.from_json(scan_docs()).to_device(0)
    assert b.debug_plan(env, ids, origin)["scan_regions"] == 1
    b.validate(env, ids, origin)
    gpu = b.verdicts()
    ora = oe.eval(b.view(), ids, origin)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
