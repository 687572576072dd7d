"""CPU: the fused kernel's fast classification tables agree with the column DFAs they replace.

* literal columns (namespace, capabilities, AppArmor profiles, label keys): the perfect-hash table
  (kwdev.hpp DevLit, env.cpp build_literal_table) returns exactly the DFA's mask for every string;
* label values: the per-key value DFA returns the LV-chain mask restricted to the regexes constrained
  on the label's key.
Strings: every pattern named in the configs, edits of them (prefix / suffix / truncation / case /
one-byte change, which also cover equal-length near misses), the synthetic workload's own strings,
and edge strings (empty, long, NUL and high bytes). The kernel-side lookup is the same algorithm and
is checked against the oracle by the GPU parity tests.
"""
import random

import pytest

import kwgpu as K
from helpers import config

COL_NS, COL_CAP, COL_AA, COL_LK, COL_LV = 0, 4, 5, 6, 7
CONFIGS = [("parity", 0), ("c1_namespace", 1), ("c4_64", 4), ("c5_mixed", 5)]


def _names(doc):
    """Strings each literal column's patterns are made of, from the policy settings."""
    out = {COL_NS: {"kubewarden"}, COL_CAP: {"ALL"}, COL_AA: set(), COL_LK: set()}
    constrained = []
    entries = list(doc.values())
    for e in entries:
        entries += list((e.get("policies") or {}).values())
    for e in entries:
        s = e.get("settings") or {}
        if "valid_namespace" in s:
            out[COL_NS].add(s["valid_namespace"])
        for k in ("allowed_capabilities", "required_drop_capabilities", "default_add_capabilities"):
            out[COL_CAP].update(c for c in s.get(k) or [] if c != "*")
        out[COL_AA].update(s.get("allowed_profiles") or [])
        out[COL_LK].update(s.get("denied_labels") or [])
        out[COL_LK].update(s.get("mandatory_labels") or [])
        out[COL_LK].update((s.get("constrained_labels") or {}).keys())
        constrained += list((s.get("constrained_labels") or {}).items())
    return out, constrained


def _edits(w, rng):
    b = w.encode()
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


@pytest.mark.parametrize("name,scfg", CONFIGS)
def test_literal_tables_match_dfa(name, scfg):
    doc = config(name)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    rng = random.Random(7)
    names, _ = _names(doc)
    syn = K.SynthBatch(scfg, 400, seed=3)
    soa = syn.soa()
    pool = {COL_NS: _strings(soa.ns, soa.ns.n), COL_CAP: _strings(soa.cap_add, soa.cap_add.n) + _strings(soa.cap_drop, soa.cap_drop.n),
            COL_AA: _strings(soa.ctr_apparmor, soa.ctr_apparmor.n), COL_LK: _strings(soa.lbl_key, soa.lbl_key.n)}
    edge = [b"", b"\x00", b"\xff" * 3, b"a" * 4097, bytes(range(1, 40))]
    checked = 0
    for col in (COL_NS, COL_CAP, COL_AA, COL_LK):
        strs = set(pool[col]) | set(edge)
        for w in names[col]:
            strs.update(_edits(w, rng))
        for s in strs:
            has, dm, fm = env.classify_check(col, s)
            if not has:
                break  # column without patterns or with non-literal patterns: the DFA is used
            assert fm == dm, (name, col, s, hex(dm), hex(fm))
            assert bin(fm).count("1") <= 1
            checked += 1
        for w in names[col] if has else ():
            assert env.classify_check(col, w)[2] != 0, (name, col, w)  # every pattern finds itself
    assert checked > 0


@pytest.mark.parametrize("name,scfg", [("parity", 0), ("c4_64", 4)])
def test_per_key_value_dfas_match_chain(name, scfg):
    doc = config(name)
    env = K.EvaluationEnvironment(doc, continue_on_errors=True, always_accept_namespace="kubewarden")
    rng = random.Random(11)
    names, constrained = _names(doc)
    assert constrained
    syn = K.SynthBatch(scfg, 400, seed=5)
    soa = syn.soa()
    pairs = list(zip(_strings(soa.lbl_key, soa.lbl_key.n), _strings(soa.lbl_val, soa.lbl_val.n)))
    values = [v for _, v in pairs] + [b"", b"v1", b"v1.2.3", b"prod", b"abcdefgh", b"abcdefghi", b"X_Y", b"0" * 300]
    checked = hits = 0
    for key in sorted(names[COL_LK]) + [b"not-a-key".decode()]:
        for v in values + [bytes(e) for e in _edits(rng.choice(["frontend", "v2.0", "eu-west-1"]), rng)]:
            has, dm, fm = env.classify_check(COL_LV, v, key=key)
            assert has
            assert fm == dm, (name, key, v, hex(dm), hex(fm))
            checked += 1
            hits += fm != 0
    assert checked > 1000 and hits > 0
