"""GPU: random policy sets (tests/fuzz.py) through the HIP path — all-pairs verdict words equal the
oracle's bit-exact in both origins, and row mode (one random policy per row, the serving path)
equals the all-pairs words it selects."""
import os

import numpy as np
import pytest

import kwgpu as K
import oracle as O
from fuzz import random_policies
from helpers import diff_verdicts

pytestmark = pytest.mark.gpu
NS = "kubewarden"


# KW_FUZZ_SEEDS widens the sweep for a deep run (profiles/r03_fuzz_deep.log: 200 seeds)
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("KW_FUZZ_SEEDS", "8"))))
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
    # the bulk host -> host path on a fresh copy of the rows, in chunks of a few tiles
    bulk = syn.batch().validate_host(env, ids, origin=K.AUDIT, chunk_rows=448)
    assert np.array_equal(bulk, want), diff_verdicts(bulk, want, len(ids), ids)


@pytest.mark.parametrize("raw", [False, True])
def test_odd_documents_on_gpu(raw):
    """Randomly shaped documents (tests/test_flatten_fuzz.py: mistyped and missing members, escapes,
    duplicate keys) through the flattener and the HIP path: all-pairs words equal the oracle's on the
    same rows in both origins, and for AdmissionReviews every response of a row sample (JSONPatches of
    odd securityContexts included) equals the oracle's, derived from the document itself."""
    import random

    from helpers import config
    from test_flatten_fuzz import _doc
    from test_parity_gpu import _check_responses
    doc = config("parity")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    rng = random.Random(77 + raw)
    docs = [d for d in (_doc(rng, raw) for _ in range(800)) if O.flatten_doc(d, raw=raw) is not None]
    assert len(docs) > 400
    b = K.Batch.from_json(docs, raw=raw).to_device(0)
    soa = b.view()
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(soa, ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
        if not raw:
            assert _check_responses(env, oe, b, soa, docs, ids, origin, range(0, len(docs), 7)) > 0
