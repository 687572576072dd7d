"""GPU: the pattern-dialect and automaton-size cases (tests/pattern_cases.py) through the HIP path.
Label constraints in the Rust `regex` dialect and patterns beyond the DFA state budget (NFA elements:
nfa_classify_kernel, then the tile kernel's NFA instantiation) give the oracle's verdict words in
both origins, in row mode, through the bulk host path, and for synthetic batches; responses of a row
sample equal the oracle's (messages name the constraint)."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from fuzz import random_policies
from helpers import diff_verdicts
from pattern_cases import policies, reviews

pytestmark = pytest.mark.gpu
NS = "kubewarden"


@pytest.fixture(autouse=True)
def _poisoned_verdicts(monkeypatch):
    monkeypatch.setenv("KW_POISON_VERDICTS", "1")


def _envs(doc):
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    assert env.policy_ids() == [p["id"] for p in oe.pol]
    return env, oe


def test_pattern_cases_on_gpu():
    from test_parity_gpu import _check_responses
    env, oe = _envs(policies())
    ids = env.policy_ids()
    docs = reviews(600)
    b = K.Batch.from_json(docs).to_device(0)
    soa = b.view()
    for origin in (K.VALIDATE, K.AUDIT):
        b.validate(env, ids, origin)
        got = b.verdicts()
        want = oe.eval(soa, ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
        assert _check_responses(env, oe, b, soa, docs, ids, origin, range(0, 600, 37)) > 0
    rng = np.random.default_rng(5)
    pick = rng.integers(0, len(ids), len(docs))
    b.validate_rows(env, [ids[int(j)] for j in pick], K.AUDIT)
    full = want.reshape(len(docs), len(ids))
    assert np.array_equal(b.verdicts(count=len(docs)), full[np.arange(len(docs)), pick])
    bulk = K.Batch.from_json(docs).validate_host(env, ids, origin=K.AUDIT, chunk_rows=128)
    assert np.array_equal(bulk, want), diff_verdicts(bulk, want, len(ids), ids)


@pytest.mark.parametrize("scfg,rows", [(4, 20000), (5, 6000), (2, 20000)])
def test_pattern_cases_on_synthetic_batches(scfg, rows):
    """Synthetic Pods (labels from the C4 vocabulary, images of every shape) against the same set:
    tens of thousands of label values and image references through the NFA pre-pass."""
    env, oe = _envs(policies())
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=4242 + scfg)
    b = syn.batch().to_device(0)
    b.validate(env, ids, K.VALIDATE)
    got = b.verdicts()
    want = oe.eval(syn.soa(), ids, K.VALIDATE)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)


def test_fuzz_sets_with_nfa_elements_on_gpu():
    """Random policy sets (tests/fuzz.py: the dialect regexes and blow-up patterns are in its
    vocabulary) whose classifiers hold NFA elements, over skewed C5 rows."""
    checked = 0
    for seed in range(300, 340):
        doc = random_policies(seed)
        env, oe = _envs(doc)
        ids = env.policy_ids()
        syn = K.SynthBatch(5, 1500, seed=seed)
        b = syn.batch().to_device(0)
        b.validate(env, ids, K.VALIDATE)
        got, want = b.verdicts(), oe.eval(syn.soa(), ids, K.VALIDATE)
        assert np.array_equal(got, want), (seed, diff_verdicts(got, want, len(ids), ids))
        checked += 1
        if checked == 10:
            break
    assert checked == 10
