"""CPU: the JSON -> SoA flattener (kw_batch_from_json). Multi-threaded flattening (contiguous
document ranges, concatenated in order) yields exactly the single-threaded columns, and a bad
document is reported at its own row index (the first bad row), as the reference's JsonExtractor
rejects the one body it parses (handlers.rs:29-39)."""
import numpy as np
import pytest

import kwgpu as K
import oracle as O

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


def _one(doc):
    try:
        b = K.Batch.from_json([doc])
    except K.PayloadError as e:
        return str(e)
    return columns(b)


@pytest.mark.parametrize("text,ok", [
    ("0", True), ("-0", True), ("12", True), ("1.5e3", True), ("-2E-2", True), ("1e400", False), ("01", False),
    ("1.", False), (".5", False), ("-", False), ("1e", False), ("1e+", False), ("+1", False), ("0x1", False),
    ("123456789012345678901234567890", True), ("true", True), ("tru", False), ("null", True), ('"a\\u00e9\\ud83d\\ude00"', True),
    ('"\\ud83d"', False), ('"\\x"', False), ('"a\tb"', False), ("[1,]", False), ("{\"a\":1,}", False), ("[1 2]", False),
])
def test_json_grammar(text, ok):
    """RFC 8259 values inside an otherwise valid AdmissionReview (as serde_json reads them): number
    grammar (no leading zeros, digits after '.' and 'e', f64 overflow is an error), escapes and
    surrogate pairs, raw control characters, trailing commas."""
    doc = docs(4, 1, 3)[0]
    doc = doc.replace('"dryRun":false', '"dryRun":false,"extra":' + text)
    got = _one(doc)
    if ok:
        assert isinstance(got, dict), got
    else:
        assert isinstance(got, str) and got.startswith("Failed to parse the request body as JSON"), got


def test_json_recursion_limit():
    """serde_json's recursion limit: 127 nested arrays/objects parse (the document's own nesting
    included), one more is 'recursion limit exceeded' (a 400, not a 422)."""
    doc = docs(4, 1, 3)[0]
    base = 2  # the document and request objects enclose "extra"
    ok = '"extra":' + "[" * (127 - base) + "]" * (127 - base)
    bad = '"extra":' + "[" * (128 - base) + "]" * (128 - base)
    assert isinstance(_one(doc.replace('"dryRun":false', '"dryRun":false,' + ok)), dict)
    got = _one(doc.replace('"dryRun":false', '"dryRun":false,' + bad))
    assert isinstance(got, str) and "recursion limit exceeded" in got


def test_escaped_strings_and_duplicate_keys():
    """Escaped keys and values are unescaped (the arena path) and match their plain spelling. A
    repeated field of a typed object (AdmissionRequest, its kind / resource / userInfo, the review
    envelope) is a deserialize error, 422, as serde's derived structs answer ("duplicate field"); a
    repeated key inside `object` (a serde_json::Value) keeps its last value."""
    doc = docs(4, 1, 3)[0]
    plain = columns(K.Batch.from_json([doc]))
    esc = doc.replace('"namespace":"', '"n\\u0061mespace":"', 1).replace('"operation":"CREATE"', '"operation":"CR\\u0045\\u0041TE"')
    got = _one(esc)
    assert isinstance(got, dict)
    for k in ("ns.bytes", "ns.off", "op.bytes"):
        assert np.array_equal(got[k], plain[k]), k
    for dup, field in ((doc.replace('"operation":"CREATE"', '"operation":"DELETE","operation":"CREATE"'), "operation"),
                       (doc.replace('"request":{', '"request":{"uid":"x",', 1), "uid"),
                       (doc.replace('"userInfo":{', '"userInfo":{"username":"a",', 1), "username"),
                       (doc.replace('"kind":{"group"', '"kind":{"kind":"Pod","group"', 1), "kind"),
                       ('{"request":{},' + doc[1:], "request")):
        got = _one(dup)
        assert isinstance(got, str) and f"duplicate field `{field}`" in got, (field, got)
        assert O.flatten_doc(dup) is None
    i = doc.index('"labels":{') + len('"labels":{')
    dup = doc[:i] + '"app":"first",' + doc[i:]  # inside object: serde_json::Value, the last one wins
    assert O.flatten_doc(dup) is not None
    got = _one(dup)
    assert isinstance(got, dict)
