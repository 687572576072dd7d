"""The Unicode classes of the regex dialect on the device, code point by code point. The device walks
label values through its own per-key tables (kernels.hip kv_walk: 129-entry or full byte-class
maps, u8 / u16 transitions, 8-byte windows, the second-DFA helper lanes). This test compares it
with the oracle over every code point of the BMP and a sample of plane 1, one code point per label
value. The pattern set covers `\\p{..}`, `\\w \\d \\s`, case folding and word boundaries
(tests/test_unicode_tables.py checks the host matcher the same way, against definitions outside
the generator).

CPU: the host walk against the oracle on a sample. GPU: every verdict word against the oracle."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import diff_verdicts

MODULE = "registry://ghcr.io/kubewarden/policies/safe-labels:v0.1.14"
PATTERNS = {
    "upper": r"^\p{Lu}$",
    "letter_or_mark": r"^[\p{L}\p{M}]$",
    "not_number": r"^\P{N}$",
    "word": r"^\w$",
    "digit": r"^\d$",
    "space": r"^\s$",
    "fold": r"(?i)^[a-zß-ÿσ]$",
    "boundary": r"\b.\b",
    "symbol_or_punct": r"^[\p{S}\p{P}]+$",
    "cased_letter": r"^\p{LC}$",
}


def _policies():
    pols = {}
    for name, rx in PATTERNS.items():
        pols[f"labels-{name}"] = {"module": MODULE, "settings": {"constrained_labels": {"k": rx}}}
    return pols


def _code_points(stride_bmp=1, stride_smp=7):
    cps = [cp for cp in range(0x20, 0x10000, stride_bmp) if not 0xD800 <= cp < 0xE000]
    cps += list(range(0x10000, 0x20000, stride_smp))
    return cps


def _docs(cps):
    return [{"request": {"uid": str(i), "kind": {"group": "", "version": "v1", "kind": "Pod"},
                         "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE",
                         "userInfo": {}, "namespace": "default",
                         "object": {"kind": "Pod", "metadata": {"labels": {"k": chr(cp)}},
                                    "spec": {"containers": [{"name": "c", "image": "nginx"}]}}}}
            for i, cp in enumerate(cps)]


def test_host_walk_matches_oracle_on_a_sample():
    doc = _policies()
    env = K.EvaluationEnvironment(doc)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(_docs(_code_points(stride_bmp=37, stride_smp=101)))
    got = b.debug_host_walk(env, ids).reshape(-1)
    want = oe.eval(b.view(), ids).reshape(-1)
    assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
    # the sample is not trivial: every pattern accepts some code points and rejects others
    ok = (want.reshape(-1, len(ids)) & K._native.KW_F_ALLOWED) != 0
    assert ok.any(axis=0).all() and (~ok).any(axis=0).all()


@pytest.mark.gpu
def test_device_matches_oracle_per_code_point():
    doc = _policies()
    env = K.EvaluationEnvironment(doc, device=0)
    oe = O.OracleEnv(doc)
    ids = env.policy_ids()
    b = K.Batch.from_json(_docs(_code_points())).to_device(0)
    b.validate(env, ids)
    gpu = b.verdicts()
    ora = oe.eval(b.view(), ids)
    assert np.array_equal(gpu, ora), diff_verdicts(gpu, ora, len(ids), ids)
