"""Second label-value DFAs on idle lanes (kernels.hip P1 label items, `label_pairs`).
C4's policies constrain the key `env` with five patterns that compile into a chain of two DFAs
(every other key: one DFA or none). In a single-chunk pass a label whose chain has a second DFA
hands that walk to a lane of its wave with nothing to walk; labels left without such a lane walk
it themselves.

The batches below vary the share of `env` labels per wave from none to all of them (all: no idle
lane but the tile's tail, so nearly every second walk falls back to its own lane), with values
from 0 to 40 bytes (one to six 8-byte windows) that match none, some or all of the patterns, and
unconstrained keys as the idle lanes. CPU: the host walk against the oracle. GPU: verdict words
against the oracle, both origins."""
import random

import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts

ENV_VALUES = ["", "prod", "dev", "backend", "cache", "true", "x", "abcdefgh", "abcdefghi", "A_b.c-9",
              "v1.2.3", "1234", "us-west-1", "team-a", "frontend", "Z" * 40, "a" * 8 + "1234", "web",
              "é", "abc def"]
OTHER_KEYS = ["app", "tier", "owner", "region", "legacy", "debug", "unconstrained", "k8s.io/other"]


def pair_docs(env_share, n=500, seed=0):
    """Keys are unique within a request, so the share of `env` labels is set by how many other
    labels a request carries: 1.0 = `env` alone, 0.5 = `env` plus one other, 0.05 = `env` in 30 %
    of requests among 1-12 others, 0.0 = never."""
    rng = random.Random(seed)
    docs = []
    for r in range(n):
        labels = {}
        if env_share >= 1.0 or env_share >= 0.5 or (env_share > 0.0 and rng.random() < 0.3):
            labels["env"] = rng.choice(ENV_VALUES)
        others = 0 if env_share >= 1.0 else 1 if env_share >= 0.5 else rng.randint(1, 12)
        for key in rng.sample(OTHER_KEYS + [f"x{j}" for j in range(8)], others):
            labels[key] = rng.choice(ENV_VALUES)
        docs.append({"request": {"uid": str(r), "kind": {"group": "", "version": "v1", "kind": "Pod"},
                                 "resource": {"group": "", "version": "v1", "resource": "pods"},
                                 "operation": "CREATE", "userInfo": {}, "namespace": "default",
                                 "object": {"kind": "Pod", "metadata": {"labels": labels},
                                            "spec": {"containers": [{"name": "c", "image": "nginx"}]}}}})
    return docs


SHARES = [0.0, 0.05, 0.5, 1.0]


@pytest.mark.parametrize("share", SHARES)
def test_host_walk_matches_oracle(share):
    doc = config("c4_64")
    env = K.EvaluationEnvironment(doc)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(pair_docs(share, n=200, seed=7))
    got = b.debug_host_walk(env, ids).reshape(-1)
    want = oe.eval(b.view(), ids).reshape(-1)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


@pytest.mark.gpu
@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
@pytest.mark.parametrize("share", SHARES)
def test_pairs_match_oracle(share, origin):
    doc = config("c4_64")
    env = K.EvaluationEnvironment(doc, device=0)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(pair_docs(share)).to_device(0)
    assert b.debug_plan(env, ids, origin)["chunks"] == 1
    b.validate(env, ids, origin)
    gpu = b.verdicts()
    ora = oe.eval(b.view(), ids, origin)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
