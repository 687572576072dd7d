"""CPU: random policy sets (tests/fuzz.py) — the slot compiler's host walk (the device kernel's
tables and walks on the host, kw_debug_host_walk) equals the oracle's verdicts, bit-exact, in both
origins; and the environment's init-error rows agree with the oracle's. The GPU twin is
tests/test_fuzz_gpu.py."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from fuzz import random_policies
from helpers import diff_verdicts

NS = "kubewarden"


@pytest.mark.parametrize("seed", range(40))
def test_random_policy_sets_host_walk(seed):
    doc = random_policies(seed)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    assert ids == [p["id"] for p in oe.pol]
    for i in ids:
        assert bool(env.policy_initialization_error(i)) == bool(oe.pol[oe.ids[i]].get("init_error")), i
    scfg = (0, 4, 5)[seed % 3]
    syn = K.SynthBatch(scfg, 600, seed=900 + seed)
    b = syn.batch()
    for origin in (K.VALIDATE, K.AUDIT):
        got = b.debug_host_walk(env, ids, origin)
        want = oe.eval(syn.soa(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
