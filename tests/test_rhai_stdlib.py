"""CPU: every function name of rhai 1.21's standard packages answers a value or a named refusal
(VERDICT r05 #1). The product restates rhai's `Engine::new()`: the functions of
its packages over the engine's values (i64, bool, string, array, ()) are implemented; every other
name of the packages — functions over floats, characters, maps, blobs, timestamps or function
pointers — is refused at load as "unsupported by this engine: <name>", never answered with rhai's
own "Function not found" (which rhai gives only for a name it does not have, or for argument types
no overload takes).

The name list below is written from rhai's package documentation (CorePackage, BitFieldPackage,
BasicMathPackage, BasicArrayPackage, BasicBlobPackage, BasicMapPackage, BasicTimePackage,
MoreStringPackage and the language keywords), not read from either implementation, so a name the
product or the oracle forgot shows up here. Each implemented name carries a probe: a script that
must validate and accept (evaluated through the host walk in both device forms, product and oracle
alike). Reference: rhai 1.21.0 (Cargo.lock:5116-5118), run by evaluation_environment.rs:587-651."""
import pytest

import kwgpu as K
import oracle as O
from test_rhai_forms import MEMBERS, VECTORS, review

IMPLEMENTED = {
    "len": '"ab".len() == 2 && [1].len() == 1',
    "is_empty": '"".is_empty() && ![1].is_empty()',
    "contains": '"abc".contains("b") && [1, 2].contains(2)',
    "to_string": '(5).to_string() == "5"',
    "type_of": 'type_of(1) == "i64"',
    "starts_with": '"abc".starts_with("ab")',
    "ends_with": '"abc".ends_with("bc")',
    "push": "let v = [1]; v.push(2); v == [1, 2]",
    "abs": "abs(-2) == 2",
    "sign": "sign(-2) == -1",
    "is_zero": "(0).is_zero()",
    "is_odd": "(3).is_odd()",
    "is_even": "(2).is_even()",
    "max": "max(1, 2) == 2",
    "min": "min(1, 2) == 1",
    "to_hex": '(255).to_hex() == "ff"',
    "to_octal": '(8).to_octal() == "10"',
    "to_binary": '(2).to_binary() == "10"',
    "parse_int": 'parse_int("12") == 12 && parse_int("z", 36) == 35',
    "to_upper": '"a".to_upper() == "A"',
    "to_lower": '"A".to_lower() == "a"',
    "make_upper": 'let s = "a"; s.make_upper(); s == "A"',
    "make_lower": 'let s = "A"; s.make_lower(); s == "a"',
    "trim": 'let s = " a "; s.trim(); s == "a"',
    "sub_string": '"abc".sub_string(1, 1) == "b"',
    "crop": 'let s = "abc"; s.crop(1); s == "bc"',
    "index_of": '"abc".index_of("c") == 2 && [1, 2].index_of(2) == 1',
    "replace": 'let s = "aba"; s.replace("a", "c"); s == "cbc"',
    "split": '"a,b".split(",") == ["a", "b"]',
    "split_rev": '"a,b".split_rev(",") == ["b", "a"]',
    "bytes": '"ab".bytes() == 2',
    "append": "let v = [1]; v.append([2]); v == [1, 2]",
    "insert": "let v = [2]; v.insert(0, 1); v == [1, 2]",
    "pop": "let v = [1, 2]; v.pop() == 2 && v == [1]",
    "shift": "let v = [1, 2]; v.shift() == 1 && v == [2]",
    "remove": "let v = [1, 2]; v.remove(0) == 1 && v == [2]",
    "reverse": "let v = [1, 2]; v.reverse(); v == [2, 1]",
    "sort": "let v = [2, 1]; v.sort(); v == [1, 2]",
    "clear": "let v = [1]; v.clear(); v == []",
    "truncate": "let v = [1, 2]; v.truncate(1); v == [1]",
    "chop": "let v = [1, 2]; v.chop(1); v == [2]",
    "get": "[1, 2].get(1) == 2",
    "set": "let v = [1, 2]; v.set(1, 3); v == [1, 3]",
    "extract": "[1, 2, 3].extract(1, 1) == [2]",
    "drain": "let v = [1, 2, 3]; v.drain(0, 1) == [1] && v == [2, 3]",
    "retain": "let v = [1, 2, 3]; v.retain(0, 1) == [2, 3] && v == [1]",
    "splice": "let v = [1, 2]; v.splice(0, 1, [9]); v == [9, 2]",
    "dedup": "let v = [1, 1]; v.dedup(); v == [1]",
    "pad": "let v = [1]; v.pad(2, 0); v == [1, 0]",
    "range": "let s = 0; for i in range(0, 3) { s += i; } s == 3",
}

REFUSED = [
    # CorePackage (language core, functions, debugging) and the keyword functions
    "tag", "set_tag", "take", "sleep", "name", "is_anonymous", "to_debug", "print", "debug", "eval", "Fn", "call",
    "curry", "is_def_var", "is_def_fn", "is_shared",
    # BitFieldPackage
    "get_bit", "set_bit", "get_bits", "set_bits", "bits",
    # BasicMathPackage: floating point and conversions
    "to_int", "to_float", "parse_float", "sqrt", "exp", "ln", "log", "floor", "ceiling", "round", "int", "fraction",
    "is_nan", "is_finite", "is_infinite", "sin", "cos", "tan", "sinh", "cosh", "tanh", "asin", "acos", "atan",
    "asinh", "acosh", "atanh", "hypot", "to_degrees", "to_radians", "PI", "E",
    # MoreStringPackage: characters
    "chars", "to_chars",
    # BasicArrayPackage: function pointers
    "map", "filter", "reduce", "reduce_rev", "some", "all", "find", "find_map", "for_each", "zip", "sort_desc",
    # BasicBlobPackage
    "blob", "to_blob", "as_string", "write_ascii", "write_utf8", "write_le", "write_be", "parse_le_int",
    "parse_be_int", "parse_le_float", "parse_be_float",
    # BasicMapPackage
    "keys", "values", "mixin", "fill_with", "to_json",
    # BasicTimePackage
    "timestamp", "elapsed",
]


def _group(expr):
    return {"g": {"policies": MEMBERS, "expression": expr, "message": "m"}}


def test_lists_are_disjoint():
    assert not set(IMPLEMENTED) & set(REFUSED)


@pytest.mark.parametrize("form", ["table", "script"])
def test_every_implemented_name_evaluates(monkeypatch, form):
    if form == "script":
        monkeypatch.setenv("KW_GROUP_FORM", "script")
    else:
        monkeypatch.delenv("KW_GROUP_FORM", raising=False)
    names = sorted(IMPLEMENTED)
    doc = {f"g{k}": {"policies": MEMBERS, "expression": f"({{ {IMPLEMENTED[n]} }}) && a()", "message": "m"}
           for k, n in enumerate(names)}
    env = K.EvaluationEnvironment(doc, continue_on_errors=True)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    ids = env.policy_ids()
    docs = [review(v, f"uid-{v or 'none'}") for v in VECTORS]
    b = K.Batch.from_json(docs)
    got = b.debug_host_walk(env, ids).reshape(len(docs), len(ids))
    want = oe.eval(b.view(), ids).reshape(len(docs), len(ids))
    r = VECTORS.index("a")
    for k, n in enumerate(names):
        env.validate_settings(f"g{k}")
        j = ids.index(f"g{k}")
        assert got[r, j] == want[r, j], n
        members = env.group_members(j)
        resp = b.format_response(env, r, j, int(got[r, j]), [int(got[r, m]) for m in members], doc=docs[r])
        assert resp["allowed"] is True, (n, IMPLEMENTED[n], resp)


@pytest.mark.parametrize("name", REFUSED)
def test_every_other_name_is_refused_by_name(name):
    expr = f"{name}(1) == 1 || a()"
    env = K.EvaluationEnvironment(_group(expr), continue_on_errors=True)
    oe = O.OracleEnv(_group(expr), continue_on_errors=True)
    P = oe.pol[oe.ids["g"]]
    assert P["valid"] is False and P["expr_error"].startswith("unsupported by this engine: "), (name, P["expr_error"])
    with pytest.raises(K.PolicyInitialization) as e:
        env.validate_settings("g")
    assert str(e.value) == P["expr_error"]
    assert "Function not found" not in str(e.value)
    # method style too
    expr = f"(1).{name}() == 1 || a()"
    env = K.EvaluationEnvironment(_group(expr), continue_on_errors=True)
    with pytest.raises(K.PolicyInitialization) as e:
        env.validate_settings("g")
    assert str(e.value).startswith("unsupported by this engine: "), (name, str(e.value))


def test_a_script_function_or_member_of_a_refused_name_still_runs():
    """Refusal is by resolution, as rhai resolves calls: a script function or a member named like a
    package function takes the call."""
    doc = {"g": {"policies": {"sqrt": MEMBERS["a"]}, "expression": "fn map(x) { x } map(sqrt())", "message": "m"}}
    env = K.EvaluationEnvironment(doc, continue_on_errors=True)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    env.validate_settings("g")
    assert oe.pol[oe.ids["g"]]["valid"]
