"""GPU: random policy sets (tests/fuzz.py) through the HIP path — all-pairs verdict words equal the
oracle's bit-exact in both origins, and row mode (one random policy per row, the serving path)
equals the all-pairs words it selects."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from fuzz import random_policies
from helpers import diff_verdicts

pytestmark = pytest.mark.gpu
NS = "kubewarden"


@pytest.mark.parametrize("seed", range(100, 108))
def test_random_policy_sets_on_gpu(seed):
    doc = random_policies(seed)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    scfg = (0, 4, 5)[seed % 3]
    syn = K.SynthBatch(scfg, 3000, seed=1700 + seed)
    b = syn.batch().to_device(0)
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(syn.soa(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    # row mode: one policy per row (groups included), against the all-pairs words of the last pass
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, len(ids), syn.n)
    b.validate_rows(env, [ids[int(j)] for j in pick], K.AUDIT)
    rows = b.verdicts(count=syn.n)
    full = want.reshape(syn.n, len(ids))
    assert np.array_equal(rows, full[np.arange(syn.n), pick])
