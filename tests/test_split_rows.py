"""Light / heavy split at upload (capi.cpp split_rows / permute_batch):
a batch whose heavy requests (more than 5 containers) are 1-50 % of the rows and hold >= 30 % of
the containers goes to the device with its light rows first and its heavy rows after them, each
region with its own tile geometry; verdict words and side data are scattered back to batch rows at
read-back. KW_SPLIT=1 forces the split at any size (tests), KW_SPLIT=0 turns it off.

CPU: the reordered batch holds every row's columns unchanged (row by row against the source
batch), the host walk over it is the source's walk permuted, the auto thresholds, and the planner's
two region geometries. GPU: a forced split at small sizes against the oracle and against the
unsplit upload — all-pairs words, partial read-backs, rows mode, groups with side data (> 15 and
> 64 members, split policies) and formatted responses. The full C5 size (10M, auto split) is
test_parity_gpu.py::test_full_size_matches_oracle[c5_mixed]."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts, wide_docs

NS = "kubewarden"


def _strs(col, lo, hi):
    return [bytes(col.bytes[col.off[i]:col.off[i + 1]]) for i in range(lo, hi)]


def _row(v, r):
    """Every column of request r of a kw_soa view, as plain values."""
    c0, c1 = v.ctr_off[r], v.ctr_off[r + 1]
    l0, l1 = v.lbl_off[r], v.lbl_off[r + 1]
    ctrs = []
    for c in range(c0, c1):
        ctrs.append((v.ctr_flags[c], _strs(v.ctr_name, c, c + 1), _strs(v.ctr_image, c, c + 1),
                     _strs(v.ctr_apparmor, c, c + 1), _strs(v.cap_add, v.capadd_off[c], v.capadd_off[c + 1]),
                     _strs(v.cap_drop, v.capdrop_off[c], v.capdrop_off[c + 1])))
    return (v.req_flags[r], _strs(v.uid, r, r + 1), _strs(v.ns, r, r + 1), _strs(v.op, r, r + 1),
            _strs(v.kind, r, r + 1), ctrs, _strs(v.lbl_key, l0, l1), _strs(v.lbl_val, l0, l1))


def _check_reorder(b, expect_split=True):
    rb, perm, split = b.debug_reorder()
    n = b.n
    assert rb.n == n and sorted(perm.tolist()) == list(range(n))
    v, rv = b.view(), rb.view()
    ctrs = np.array([v.ctr_off[r + 1] - v.ctr_off[r] for r in range(n)])
    if expect_split:
        assert 0 < split < n
        assert (ctrs[perm[:split]] <= 5).all() and (ctrs[perm[split:]] > 5).all()
        # batch order within each region
        assert (np.diff(perm[:split].astype(np.int64)) > 0).all() and (np.diff(perm[split:].astype(np.int64)) > 0).all()
    for d in range(n):
        assert _row(rv, d) == _row(v, int(perm[d])), d
    return rb, perm, split


def test_reorder_keeps_every_row(monkeypatch):
    monkeypatch.setenv("KW_SPLIT", "1")
    syn = K.SynthBatch(5, 3000, seed=11)
    b = syn.batch()
    rb, perm, split = _check_reorder(b)
    doc = config("c5_mixed")
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    got = rb.debug_host_walk(env, ids).reshape(b.n, len(ids))
    want = b.debug_host_walk(env, ids).reshape(b.n, len(ids))
    assert np.array_equal(got, want[perm])


def test_reorder_json_rows(monkeypatch):
    """Documents with 80-container rows, labels, annotations and absent fields."""
    monkeypatch.setenv("KW_SPLIT", "1")
    b = K.Batch.from_json(wide_docs())
    _check_reorder(b)


def test_no_split_cases(monkeypatch):
    syn = K.SynthBatch(5, 3000, seed=12)
    b = syn.batch()
    monkeypatch.setenv("KW_SPLIT", "0")
    _, perm, split = b.debug_reorder()
    assert split == 0 and (perm == np.arange(b.n)).all()
    monkeypatch.delenv("KW_SPLIT")
    assert b.debug_reorder()[2] == 0  # auto: below 2^18 rows
    monkeypatch.setenv("KW_SPLIT", "1")
    from test_split_policies import tail_docs
    light = K.Batch.from_json(tail_docs(300))  # one container a request: no heavy rows
    assert light.debug_reorder()[2] == 0


def _per_cu(lds):
    """Workgroups per CU of a layout: 1280-byte LDS granules, 128 per CU (kernels.hpp)."""
    return 128 // ((lds + 1279) // 1280)


def test_auto_split_and_region_geometry(monkeypatch):
    """Auto mode at C5's shape (2^18 + rows): two regions, each at a higher occupancy than the
    unsplit layout (C5's tiles hold two workgroups per CU; the light region's 64-row tiles and the
    heavy region's shorter ones four); C4 at the same size stays one region."""
    monkeypatch.delenv("KW_SPLIT", raising=False)
    n = (1 << 18) + 4096
    b5 = K.SynthBatch(5, n, seed=5).batch()
    _, perm, split = b5.debug_reorder()
    assert 0.5 * n < split < 0.95 * n
    env = K.EvaluationEnvironment(config("c5_mixed"), continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    p = b5.debug_plan(env, ids)
    assert p["regions"] == 2 and p["split"] == split
    monkeypatch.setenv("KW_SPLIT", "0")
    u = b5.debug_plan(env, ids)
    monkeypatch.delenv("KW_SPLIT")
    assert u["regions"] == 1 and _per_cu(u["lds_bytes"]) == 2, u
    assert _per_cu(p["lds_bytes"]) == 4 and _per_cu(p["heavy_lds_bytes"]) == 4, p
    assert p["rows"] == 64 and 8 <= p["heavy_rows"] < 64 and p["heavy_cmax"] > p["cmax"], p
    assert p["grid"] == 1024 and p["heavy_grid"] == 1024
    b4 = K.SynthBatch(4, n, seed=4).batch()
    assert b4.debug_reorder()[2] == 0
    p4 = b4.debug_plan(env, ids)
    assert p4["regions"] == 1 and p4["split"] == 0


def _split_policies():
    from test_split_policies import split_policies
    return split_policies()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c5_mixed", "c6_256", "parity", "split"])
def test_forced_split_matches_oracle_and_unsplit(monkeypatch, name):
    """C5-generator rows (Zipf containers, so both regions are populated) against policy sets with
    every kind of side data; the split upload against the oracle and the unsplit upload."""
    doc = _split_policies() if name == "split" else config(name)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = env.policy_ids()
    n = 2500
    syn = K.SynthBatch(5, n, seed=21)
    docs = [syn.json(r) for r in range(n)]
    monkeypatch.setenv("KW_SPLIT", "1")
    bs = syn.batch().to_device(0)
    assert 0 < syn.batch().debug_reorder()[2] < n
    monkeypatch.setenv("KW_SPLIT", "0")
    bu = syn.batch().to_device(0)
    from test_parity_gpu import _check_responses
    for origin in (K.VALIDATE, K.AUDIT):
        bs.validate(env, ids, origin)
        got = bs.verdicts()
        want = oe.eval(syn.soa(), ids, origin)
        assert np.array_equal(got, want), diff_verdicts(got, want, len(ids), ids)
        assert np.array_equal(bs.verdicts(count=7 * len(ids) + 3), got[:7 * len(ids) + 3])  # partial read-back
        bu.validate(env, ids, origin)
        assert np.array_equal(bu.verdicts(), got)
        rows = range(0, n, 37)
        assert _check_responses(env, oe, bs, syn.soa(), docs, ids, origin, rows) > 0
        for r in rows:  # side data (wide arguments, > 15-member group causes) per batch row
            for j in range(len(ids)):
                w = int(got[r * len(ids) + j])
                if w >> 16 == 0xFFFF:  # (defined for words whose ARG is KW_ARG_WIDE)
                    assert bs.wide_arg(r, j) == bu.wide_arg(r, j), (r, ids[j])
                if env.is_group(j) and (w >> 8) & 0xFF == O.R_GROUP:
                    assert bs.group_causes(r, j, w) == bu.group_causes(r, j, w), (r, ids[j])
    rng = np.random.default_rng(5)
    pick = rng.integers(0, len(ids), n)
    bs.validate_rows(env, [ids[int(j)] for j in pick], K.AUDIT)
    rows_words = bs.verdicts(count=n)
    assert np.array_equal(rows_words, want.reshape(n, len(ids))[np.arange(n), pick])
