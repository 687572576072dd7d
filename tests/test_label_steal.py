"""A fifth label block's labels taken by idle lanes of the first four (kernels.hip P1 label items,
`steal_ok`). A 64-row tile holding 257-320 labels has a fifth label block. In a
label-pair pass, lanes of the first four blocks whose own key has no value constraint classify the
remainder labels. The first block r % 4 takes remainder label r, on its (r / 4)-th free lane. The
fifth block classifies what they did not take.

The batches give every request four or five labels (tiles of 256-320 labels), with the share of
unconstrained keys from none to most:
- none: nothing is taken, and the fifth block classifies every remainder label;
- few: some are taken, the rest fall to the fifth block;
- most: all are taken.
Value-constrained keys include C4's `env` (a chain of two DFAs: the pair helpers share the free
lanes). CPU: the host walk against the oracle. GPU: verdict words against the oracle, both
origins."""
import random

import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts

CONSTRAINED = ["app", "app.kubernetes.io/instance", "app.kubernetes.io/name", "app.kubernetes.io/version", "component",
               "cost-center", "critical", "debug", "env", "experimental", "legacy", "managed-by", "owner", "part-of",
               "region", "tier"]
FREE = [f"free{j}" for j in range(12)] + ["unconstrained", "k8s.io/other"]
VALUES = ["", "prod", "dev", "backend", "cache", "true", "x", "abcdefgh", "abcdefghi", "A_b.c-9", "v1.2.3", "1234",
          "us-west-1", "team-a", "frontend", "Z" * 40, "a" * 8 + "1234", "web", "é", "abc def", "eu-east-3"]
MIXES = {"none": 0.0, "few": 0.15, "most": 0.8}


def steal_docs(free_share, n=640, seed=0, five=0.6):
    rng = random.Random(seed)
    docs = []
    for r in range(n):
        count = 5 if rng.random() < five else 4
        keys = set()
        while len(keys) < count:
            keys.add(rng.choice(FREE) if rng.random() < free_share else rng.choice(CONSTRAINED))
        labels = {k: rng.choice(VALUES) for k in sorted(keys)}
        docs.append({"request": {"uid": str(r), "kind": {"group": "", "version": "v1", "kind": "Pod"},
                                 "resource": {"group": "", "version": "v1", "resource": "pods"},
                                 "operation": "CREATE", "userInfo": {}, "namespace": "default",
                                 "object": {"kind": "Pod", "metadata": {"labels": labels},
                                            "spec": {"containers": [{"name": "c", "image": "nginx"}]}}}})
    return docs


@pytest.mark.parametrize("mix", sorted(MIXES))
def test_host_walk_matches_oracle(mix):
    doc = config("c4_64")
    env = K.EvaluationEnvironment(doc)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(steal_docs(MIXES[mix], n=256, seed=3))
    got = b.debug_host_walk(env, ids).reshape(-1)
    want = oe.eval(b.view(), ids).reshape(-1)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


@pytest.mark.gpu
@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
@pytest.mark.parametrize("five", [0.6, 1.0])
@pytest.mark.parametrize("mix", sorted(MIXES))
def test_steal_matches_oracle(mix, five, origin):
    doc = config("c4_64")
    env = K.EvaluationEnvironment(doc, device=0)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(steal_docs(MIXES[mix], seed=11, five=five)).to_device(0)
    plan = b.debug_plan(env, ids, origin)
    assert plan["chunks"] == 1 and plan["rows"] == 64 and 256 < plan["lmax"] <= 320, plan
    b.validate(env, ids, origin)
    gpu = b.verdicts()
    ora = oe.eval(b.view(), ids, origin)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
