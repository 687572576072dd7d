"""Bulk host -> host path (kw_validate_host): row chunks whose upload, evaluation and read-back
overlap on three streams must give exactly the oracle's verdict words, for pageable and pinned
output buffers, chunk sizes down to a few tiles, and passes that fall back to the unchunked form
(overflow requests, wide group side data). Columns the bulk upload left out are refused by a later
pass instead of being read from unset device memory."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O
from helpers import config, diff_verdicts, many_policies_config

pytestmark = pytest.mark.gpu
NS = "kubewarden"


@pytest.fixture(autouse=True)
def _poisoned_verdicts(monkeypatch):
    monkeypatch.setenv("KW_POISON_VERDICTS", "1")


def _envs(doc):
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace=NS, device=0)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    return env, oe


@pytest.mark.parametrize("name,scfg,rows,chunk", [
    ("c4_64", 4, 30000, 2048),     # 15 chunks of 32 tiles
    ("c4_64", 4, 30000, 0),        # the default chunk size: one chunk
    ("c2_trusted", 2, 50000, 777),  # chunk sizes that cut mid-tile-range (rounded to descriptors)
    ("c3_group", 3, 20000, 4096),
    ("parity", 0, 20000, 1500),
])
def test_bulk_matches_oracle(name, scfg, rows, chunk):
    env, oe = _envs(config(name))
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=4400 + scfg)
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    b = syn.batch()
    got = b.validate_host(env, ids, chunk_rows=chunk)
    assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)
    # pinned output: direct DMA into the caller's buffer, same words
    pin = K.PinnedWords(rows * len(ids))
    try:
        pin.array.fill(0xA5A5A5A5)
        b2 = syn.batch()
        got2 = b2.validate_host(env, ids, out=pin.array, chunk_rows=chunk)
        assert np.array_equal(got2, ora), diff_verdicts(got2, ora, len(ids), ids)
    finally:
        pin.close()


def test_bulk_more_than_256_chunks_pageable_output():
    """past 256 chunks the last chunk takes every remaining tile, so it is
    larger than one full chunk. The pageable output's bounce blocks must be sized for it.
    64-row C4 tiles, chunk_rows=128 (two tiles a chunk after the ramp) on 100k rows: the last of
    the 256 chunks holds about 1,100 tiles."""
    env, oe = _envs(config("c4_64"))
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 100000, seed=4257)
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    got = syn.batch().validate_host(env, ids, chunk_rows=128)
    assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)


def test_pinned_words_outlive_their_wrapper():
    """the page-locked memory lives as long as any view of it, not as long as the
    PinnedWords wrapper. Drop the wrapper, keep only a slice, DMA into the array again."""
    import gc
    env, oe = _envs(config("c4_64"))
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 3000, seed=91)
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    pin = K.PinnedWords(3000 * len(ids))
    arr, fin = pin.array, pin._free
    del pin
    gc.collect()
    assert fin.alive  # `arr` still references the buffer
    arr.fill(0xA5A5A5A5)
    got = syn.batch().validate_host(env, ids, out=arr, chunk_rows=1024)
    tail = got[len(got) // 2:]
    del arr, got
    gc.collect()
    assert fin.alive  # the slice alone keeps it
    assert np.array_equal(tail, ora[len(ora) // 2:])
    del tail
    gc.collect()
    assert not fin.alive  # freed with the last view


def test_bulk_audit_origin_and_reuse():
    """The same batch object through the bulk path twice (the second upload replaces the first),
    in the audit origin, then a device pass over the resident columns."""
    env, oe = _envs(config("c4_64"))
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 9000, seed=77)
    b = syn.batch()
    for origin in (K.VALIDATE, K.AUDIT):
        got = b.validate_host(env, ids, origin=origin, chunk_rows=1024)
        ora = oe.eval(syn.soa(), ids, origin)
        assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)
    b.validate(env, ids)  # the C4 columns are resident: an ordinary pass may reuse them
    assert np.array_equal(b.verdicts(), oe.eval(syn.soa(), ids, K.VALIDATE))


def test_bulk_upload_refuses_missing_columns():
    """kw_validate_host uploads only the string columns its pass reads: a later pass on the same
    device batch that needs image references fails loudly (KW_E_ARG) until the batch is uploaded
    again."""
    env4, _ = _envs(config("c4_64"))
    env2, oe2 = _envs(config("c2_trusted"))
    syn = K.SynthBatch(4, 3000, seed=5)
    b = syn.batch()
    b.validate_host(env4, env4.policy_ids())
    with pytest.raises(K.EvaluationError):
        b.validate(env2, env2.policy_ids())
    b.to_device(0)
    b.validate(env2, env2.policy_ids())
    ids = env2.policy_ids()
    assert np.array_equal(b.verdicts(), oe2.eval(syn.soa(), ids, K.VALIDATE))


def test_bulk_unchunked_forms_match_oracle():
    """C6's 40-member group (wide side data) runs unchunked through the same call; C5's requests
    beyond the tile capacities run on the overflow kernels inside their chunks."""
    env, oe = _envs(many_policies_config())
    ids = env.policy_ids()
    syn = K.SynthBatch(6, 3000, seed=6)
    got = syn.batch().validate_host(env, ids, chunk_rows=512)
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)

    env5, oe5 = _envs(config("c5_mixed"))
    ids5 = env5.policy_ids()
    syn5 = K.SynthBatch(5, 4000, seed=55)
    got5 = syn5.batch().validate_host(env5, ids5, chunk_rows=256)
    ora5 = oe5.eval(syn5.soa(), ids5, K.VALIDATE)
    assert np.array_equal(got5, ora5), diff_verdicts(got5, ora5, len(ids5), ids5)


@pytest.mark.parametrize("q", ["0.5", "0.05"])
def test_bulk_split_and_overflow_tiles(monkeypatch, q):
    """Capacities forced low (KW_TILE_QUANTILE): halved request runs inside chunks and, at 0.05,
    single requests on the overflow kernels right after their chunk's launch."""
    monkeypatch.setenv("KW_TILE_QUANTILE", q)
    env, oe = _envs(config("c4_64"))
    ids = env.policy_ids()
    syn = K.SynthBatch(4, 6000, seed=4804)
    got = syn.batch().validate_host(env, ids, chunk_rows=640)
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)


def test_bulk_overflow_wide_arguments_across_chunks():
    """Two requests beyond every tile capacity (70,000 labels; one container adding 70,000
    capabilities) in different chunks of a chunked bulk pass: the overflow kernels run per chunk,
    the second chunk's side data grows the record buffer without losing the first's, and the
    verdicts, KW_ARG_WIDE arguments and kw_batch_wide_arg values match the oracle."""
    import json
    n = 70_000
    mk = lambda uid, meta, ctrs: json.dumps({"request": {  # noqa: E731
        "uid": uid, "kind": {"group": "", "version": "v1", "kind": "Pod"},
        "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE", "userInfo": {},
        "object": {"kind": "Pod", "metadata": meta, "spec": {"containers": ctrs}}}})
    big_l = mk("labels", {"labels": {f"k{i}": ("bad" if i == n - 1 else "ok") for i in range(n)}},
               [{"name": "a", "image": "nginx"}])
    big_c = mk("caps", {}, [{"name": "big", "image": "nginx",
                             "securityContext": {"capabilities": {"add": ["CHOWN"] * (n - 1) + ["NET_ADMIN"]}}}])
    small = [mk(f"s{i}", {"labels": {"k1": "bad" if i % 3 == 0 else "ok"}},
                [{"name": "s", "image": "nginx", "securityContext": {"capabilities": {"add": ["NET_ADMIN"] if i % 5 == 0 else []}}}])
             for i in range(1500)]
    docs = small[:600] + [big_l] + small[600:1200] + [big_c] + small[1200:]
    rl, rc = 600, 1201
    mod = "registry://ghcr.io/kubewarden/policies/"
    pols = {"caps": {"module": mod + "psp-capabilities:v0.1.7", "settings": {"allowed_capabilities": ["CHOWN"]}},
            "labels": {"module": mod + "safe-labels:v0.1.14",
                       "settings": {"constrained_labels": {f"k{n - 1}": "^ok$", "k1": "^ok$"}}}}
    env = K.EvaluationEnvironment(pols, device=0)
    oe = O.OracleEnv(pols)
    ids = env.policy_ids()
    b = K.Batch.from_json(docs)
    got = b.validate_host(env, ids, chunk_rows=256)
    ora = oe.eval(b.view(), ids, K.VALIDATE).reshape(len(docs), len(ids))
    assert np.array_equal(got.reshape(len(docs), len(ids)), ora)
    li, ci = ids.index("labels"), ids.index("caps")
    assert int(got.reshape(len(docs), len(ids))[rl, li]) >> 16 == K._native.KW_ARG_WIDE
    assert int(got.reshape(len(docs), len(ids))[rc, ci]) >> 16 == K._native.KW_ARG_WIDE
    assert b.wide_arg(rl, li) == n - 1
    assert b.wide_arg(rc, ci) == n - 1


@pytest.mark.parametrize("name,scfg,rows,chunk", [
    ("c4_64", 4, 200000, 8192),   # chunked: the big columns DMA'd in place, the small ones staged
    ("c4_64", 4, 200000, 0),
    ("c2_trusted", 2, 120000, 3000),
    ("many", 6, 20000, 512),      # C6's wide group: the unchunked form with in-place columns
])
def test_bulk_pinned_columns_match_oracle(name, scfg, rows, chunk):
    """kw_batch_pin_host: the batch's large columns page-locked in place and sent by DMA from where
    they lie; the same verdict words as the staged path, pass after pass, into pageable and pinned
    output, and the batch is destroyed with its registration."""
    env, oe = _envs(many_policies_config() if name == "many" else config(name))
    ids = env.policy_ids()
    syn = K.SynthBatch(scfg, rows, seed=5100 + scfg)
    ora = oe.eval(syn.soa(), ids, K.VALIDATE)
    b = syn.batch().pin_host(0)
    b.pin_host(0)  # idempotent
    got = b.validate_host(env, ids, chunk_rows=chunk)
    assert np.array_equal(got, ora), diff_verdicts(got, ora, len(ids), ids)
    pin = K.PinnedWords(rows * len(ids))
    try:
        for origin in (K.AUDIT, K.VALIDATE):
            pin.array.fill(0xA5A5A5A5)
            got2 = b.validate_host(env, ids, out=pin.array, origin=origin, chunk_rows=chunk)
            ora2 = ora if origin == K.VALIDATE else oe.eval(syn.soa(), ids, origin)
            assert np.array_equal(got2, ora2), diff_verdicts(got2, ora2, len(ids), ids)
    finally:
        pin.close()
    b.close()


def test_bulk_concurrent_callers_share_the_pools():
    """Four host threads run bulk passes at once on their own batches (the ctypes call releases the
    GIL): the pooled streams, events, staging and device blocks are handed out under their locks, and
    every thread's verdict words match the oracle, pass after pass."""
    import threading
    env, oe = _envs(config("c4_64"))
    ids = env.policy_ids()
    syns = [K.SynthBatch(4, 20000 + 1000 * i, seed=6100 + i) for i in range(4)]
    oras = [oe.eval(s.soa(), ids, K.VALIDATE) for s in syns]
    errors = []

    def run(i):
        try:
            for rep in range(3):
                b = syns[i].batch()
                if (i + rep) % 2:
                    b.pin_host(0)
                got = b.validate_host(env, ids, chunk_rows=4096)
                if not np.array_equal(got, oras[i]):
                    errors.append((i, rep, diff_verdicts(got, oras[i], len(ids), ids)))
                b.close()
        except Exception as e:  # noqa: BLE001 (reported below with its thread)
            errors.append((i, "raised", repr(e)))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:2]
