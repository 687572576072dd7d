"""CPU: the JSON -> SoA flattener (kw_batch_from_json). Multi-threaded flattening (contiguous
document ranges, concatenated in order) yields exactly the single-threaded columns, and a bad
document is reported at its own row index (the first bad row), as the reference's JsonExtractor
rejects the one body it parses (handlers.rs:29-39)."""
import numpy as np
import pytest

import kwgpu as K

STR_COLS = ["uid", "ns", "op", "kind", "ctr_name", "ctr_image", "ctr_apparmor", "cap_add", "cap_drop",
            "lbl_key", "lbl_val"]


def columns(b):
    v = b.view()
    n = v.n_requests
    arr = lambda p, k: np.ctypeslib.as_array(p, shape=(k,)).copy() if k else np.zeros(0)
    out = {"req_flags": arr(v.req_flags, n), "ctr_off": arr(v.ctr_off, n + 1), "lbl_off": arr(v.lbl_off, n + 1)}
    nc = int(out["ctr_off"][-1])
    out["ctr_flags"] = arr(v.ctr_flags, nc)
    out["capadd_off"] = arr(v.capadd_off, nc + 1)
    out["capdrop_off"] = arr(v.capdrop_off, nc + 1)
    for name in STR_COLS:
        c = getattr(v, name)
        off = arr(c.off, c.n + 1)
        out[name + ".off"] = off
        out[name + ".bytes"] = arr(c.bytes, int(off[-1]))
    return out


def docs(cfg, n, seed):
    syn = K.SynthBatch(cfg, n, seed=seed)
    return [syn.json(i) for i in range(n)]


@pytest.mark.parametrize("cfg", [4, 5])
def test_threaded_flatten_equals_serial(monkeypatch, cfg):
    d = docs(cfg, 9000, 31 + cfg)
    monkeypatch.setenv("KW_FLATTEN_THREADS", "1")
    one = columns(K.Batch.from_json(d))
    monkeypatch.setenv("KW_FLATTEN_THREADS", "4")
    four = columns(K.Batch.from_json(d))
    assert one.keys() == four.keys()
    for k in one:
        assert np.array_equal(one[k], four[k]), k


def test_threaded_flatten_matches_generator_columns(monkeypatch):
    syn = K.SynthBatch(4, 5000, seed=99)
    monkeypatch.setenv("KW_FLATTEN_THREADS", "3")
    got = columns(K.Batch.from_json([syn.json(i) for i in range(5000)]))
    want = columns(syn.batch())
    for k in ["req_flags", "ctr_off", "lbl_off", "ctr_flags", "capadd_off", "capdrop_off"] + \
             [c + s for c in ["ns", "ctr_image", "ctr_apparmor", "cap_add", "cap_drop", "lbl_key", "lbl_val"]
              for s in (".off", ".bytes")]:
        assert np.array_equal(got[k], want[k]), k


@pytest.mark.parametrize("threads", ["1", "4"])
def test_bad_row_reported(monkeypatch, threads):
    d = docs(4, 8000, 5)
    d[5000] = '{"request": {"uid": 7}}'
    d[7000] = "not json"
    monkeypatch.setenv("KW_FLATTEN_THREADS", threads)
    with pytest.raises(K.PayloadError) as e:
        K.Batch.from_json(d)
    assert e.value.row == 5000
