"""CPU: the compiled classifiers (kwdev.hpp: literal perfect hash, DFA chains with accept classes,
per-key label-value DFAs) match exactly the patterns each string matches one pattern at a time.

kw_env_classify runs the blob's tables on the host (the same tables and algorithms the kernels run)
and returns the matched pattern ids; the expectation comes from kw_pattern_match on every pattern of
the column separately (a one-pattern automaton each). Strings: every pattern named in the configs,
edits of them (prefix / suffix / truncation / case / one-byte change, which also cover equal-length
near misses), the synthetic workload's own strings, and edge strings (empty, long, NUL and high
bytes). Covers literal columns above the single-bucket perfect hash (hash-and-displace tables) and
columns with hundreds of patterns: no column is bounded by a pattern count.
"""
import random

import pytest

import kwgpu as K
from helpers import config, many_policies_config

COL_NS, COL_REG, COL_TAG, COL_IMG, COL_CAP, COL_AA, COL_LK, COL_LV = range(8)
CONFIGS = [("parity", 0), ("c1_namespace", 1), ("c2_trusted", 2), ("c3_group", 3), ("c4_64", 4)]


def _edits(w, rng):
    b = w.encode() if isinstance(w, str) else w
    yield b
    yield b + b"x"
    yield b"x" + b
    yield b[:-1]
    yield b.upper()
    if b:
        i = rng.randrange(len(b))
        yield b[:i] + bytes([(b[i] + 1) % 256]) + b[i + 1:]


def _strings(col, n):
    return [bytes(col.bytes[col.off[i]:col.off[i + 1]]) for i in range(n)]


def _expected(pats, s):
    return [i for i, (kind, text) in enumerate(pats)
            if (text.encode() == s if kind == 0 else K.pattern_match(kind, text, s) == 1)]


def _check_columns(env, syn_cfg, rng, cols=(COL_NS, COL_REG, COL_TAG, COL_IMG, COL_CAP, COL_AA, COL_LK), sample=None):
    syn = K.SynthBatch(syn_cfg, 300, seed=3)
    soa = syn.soa()
    images = _strings(soa.ctr_image, soa.ctr_image.n)
    pool = {COL_NS: _strings(soa.ns, soa.ns.n), COL_CAP: _strings(soa.cap_add, soa.cap_add.n) + _strings(soa.cap_drop, soa.cap_drop.n),
            COL_AA: _strings(soa.ctr_apparmor, soa.ctr_apparmor.n), COL_LK: _strings(soa.lbl_key, soa.lbl_key.n),
            COL_REG: [i.split(b"/")[0] for i in images] + [b"docker.io"],
            COL_TAG: [i.rsplit(b":", 1)[-1] for i in images] + [b"latest"],
            COL_IMG: [b"docker.io/library/" + i + b":latest" for i in images[:80]] + images[:80]}
    edge = [b"", b"\x00", b"\xff" * 3, b"a" * 4097, bytes(range(1, 40))]
    checked = hits = 0
    for col in cols:
        pats = env.patterns(col)
        strs = set(pool[col]) | set(edge)
        for _, text in pats:
            strs.update(_edits(text, rng))
        strs = sorted(strs)
        if sample and len(strs) > sample:
            strs = rng.sample(strs, sample)
        for s in strs:
            got = env.classify(col, s)
            assert got == _expected(pats, s), (col, s)
            checked += 1
            hits += bool(got)
        for i, (kind, text) in enumerate(pats):
            if kind == 0:
                assert i in env.classify(col, text.encode()), (col, text)  # every literal finds itself
    return checked, hits


@pytest.mark.parametrize("name,scfg", CONFIGS)
def test_classifiers_match_patterns(name, scfg):
    env = K.EvaluationEnvironment(config(name), continue_on_errors=True, always_accept_namespace="kubewarden")
    checked, hits = _check_columns(env, scfg, random.Random(7))
    assert checked > 100 and hits > 0


def test_many_patterns_per_column():
    """Hundreds of registries, image globs, label keys, capabilities, profiles and namespaces in one
    policy set: hash-and-displace literal tables and large DFA chains, still exact."""
    doc = many_policies_config()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    for col, at_least in ((COL_REG, 200), (COL_IMG, 200), (COL_LK, 100), (COL_AA, 65), (COL_NS, 25)):
        assert len(env.patterns(col)) >= at_least, col
    checked, hits = _check_columns(env, 6, random.Random(11), sample=400)
    assert checked > 1000 and hits > 100


@pytest.mark.parametrize("name,scfg", [("parity", 0), ("c4_64", 4), (None, 6)])
def test_per_key_value_dfas(name, scfg):
    doc = config(name) if name else many_policies_config()
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    rng = random.Random(11)
    lv = env.patterns(COL_LV)
    by_key = {}
    entries = list(doc.values())
    for e in list(entries):
        entries += list((e.get("policies") or {}).values())
    for e in entries:
        for k, r in ((e.get("settings") or {}).get("constrained_labels") or {}).items():
            by_key.setdefault(k, set()).add(lv.index((2, r)))
    assert by_key
    syn = K.SynthBatch(scfg, 300, seed=5)
    soa = syn.soa()
    values = _strings(soa.lbl_val, soa.lbl_val.n) + [b"", b"v1", b"v1.2.3", b"prod", b"abcdefgh", b"abcdefghi", b"X_Y",
                                                      b"0" * 300]
    checked = hits = 0
    keys = sorted(by_key)
    if len(keys) > 24:
        keys = rng.sample(keys, 24)
    for key in keys + ["not-a-key"]:
        allowed = by_key.get(key, set())
        for v in set(values) | {bytes(e) for e in _edits(rng.choice(["frontend", "v2.0", "eu-west-1"]), rng)}:
            got = env.classify(COL_LV, v, key=key)
            want = [i for i in _expected(lv, v) if i in allowed]
            assert got == want, (name, key, v)
            checked += 1
            hits += bool(got)
    assert checked > 500 and hits > 0
