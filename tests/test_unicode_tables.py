"""The Unicode tables behind the regex dialect (scripts/gen_unicode.py ->
policy-server_amd/csrc/unicode_data.hpp and oracle/unicode_data.h), checked over whole code-point
ranges instead of regex_gen.ALPHA's sample (VERDICT r05 "What's weak" #1: the generator is a single
point of truth for product and oracle).

Each check compares the product's compiled matcher (kw_pattern_match_many: the automaton.cpp DFA the
device tables are built from, and its NFA form) with a definition that does not go through the
generator's tables:

* `\\p{X}` for every General_Category value and group: Python's `unicodedata.category`, per code
  point. This is the database the generator reads. The check covers the generator's run
  compaction and the compiler's UTF-8 range splitting, for every code point of the BMP and plane 1,
  and a stride sample of the rest.
* `\\d`: Rust defines it as `\\p{Nd}`, so it is checked against the category, and against
  `str.isdecimal`.
* `\\s`: Rust defines it as the White_Space property. The 25 code points of PropList.txt
  (Unicode 13.0) are written out below by hand.
* `\\w`: Alphabetic + M + Nd + Pc + Join_Control (UTS #18 Annex C). Alphabetic is L + Nl +
  Other_Alphabetic. The part of Other_Alphabetic outside L and M is derived here from the
  characters' names, not from the generator's list.
* `(?i)`: Rust folds by simple case folding (CaseFolding.txt C + S). Every orbit of characters whose
  Python `casefold` is one character (status C, where full and simple folding agree) must match as
  one class, over the BMP and plane 1. Characters that a lower / upper mapping links to an orbit
  without folding into it must stay outside: U+0131 against {I, i}.

The oracle (oracle/kwregex.c: its own parser and Pike VM over the same generated tables) is checked
on a smaller stride sample of the same code points. Parity with Rust's own tables (Unicode 15.0 in
regex 1.x) is unpinned for characters added after Unicode 13.0: DESIGN.md §6."""
import ctypes as C
import unicodedata

import pytest

import kwgpu as K
import oracle as O
from kwgpu import _native as N

REGEX = 2
FORCE_NFA = 0x100


def _sample():
    cps = []
    for cp in range(0x110000):
        if 0xD800 <= cp < 0xE000:
            continue  # surrogates are not scalar values (a label value is UTF-8)
        plane = cp >> 16
        stride = 1 if plane <= 1 else 4 if plane in (2, 3, 14) else 64
        if cp % stride == 0 or (cp & 0xFFFF) in (0xFFFE, 0xFFFF):
            cps.append(cp)
    return cps


CPS = _sample()
_SUBJ = None


def _subjects():
    global _SUBJ
    if _SUBJ is None:
        bs = [chr(cp).encode() for cp in CPS]
        arr = (C.c_char_p * len(bs))(*bs)
        lens = (C.c_size_t * len(bs))(*[len(x) for x in bs])
        _SUBJ = (bs, arr, lens)
    return _SUBJ


def product(pattern, kind=REGEX):
    """1/0 per code point of CPS: one compilation, one call."""
    bs, arr, lens = _subjects()
    out = (C.c_int32 * len(bs))()
    rc = N.lib().kw_pattern_match_many(kind, pattern.encode(), arr, lens, len(bs), out)
    assert rc == 0, f"product refuses {pattern!r}"
    return bytes(memoryview(out).cast("B"))[::4]


def mismatches(got, want_fn, limit=8):
    bad = []
    for cp, g in zip(CPS, got):
        if g != (1 if want_fn(cp) else 0):
            bad.append(f"U+{cp:04X}")
            if len(bad) >= limit:
                break
    return bad


CATS = ["Lu", "Ll", "Lt", "Lm", "Lo", "Mn", "Mc", "Me", "Nd", "Nl", "No", "Pc", "Pd", "Ps", "Pe", "Pi", "Pf",
        "Po", "Sm", "Sc", "Sk", "So", "Zs", "Zl", "Zp", "Cc", "Cf", "Co", "Cn"]
GROUPS = {"L": "L", "M": "M", "N": "N", "P": "P", "S": "S", "Z": "Z", "C": "C"}


def cat(cp):
    return unicodedata.category(chr(cp))


def test_sample_covers_the_tables():
    assert unicodedata.unidata_version == "13.0.0"  # the generator's database
    assert len(CPS) > 150000 and CPS[0] == 0 and CPS[-1] == 0x10FFFF


@pytest.mark.parametrize("gc", CATS)
def test_general_category(gc):
    got = product(f"^\\p{{{gc}}}$")
    assert not mismatches(got, lambda cp: cat(cp) == gc), gc
    neg = product(f"^\\P{{{gc}}}$")
    assert all(a + b == 1 for a, b in zip(got, neg)), f"\\P{{{gc}}} is not the complement"


@pytest.mark.parametrize("group", sorted(GROUPS))
def test_general_category_groups(group):
    got = product(f"^\\p{{{group}}}$")
    # C includes Cs (surrogates), which no UTF-8 subject holds
    assert not mismatches(got, lambda cp: cat(cp)[0] == group), group


def test_cased_letter_and_nfa_form():
    got = product("^\\p{LC}$")
    assert not mismatches(got, lambda cp: cat(cp) in ("Lu", "Ll", "Lt"))
    for gc in ("Lu", "Nd", "Mn"):  # the NFA form (patterns beyond the DFA budget) reads the same tables
        assert product(f"^\\p{{{gc}}}$", REGEX | FORCE_NFA) == product(f"^\\p{{{gc}}}$"), gc


def test_digit_is_nd():
    got = product("^\\d$")
    assert not mismatches(got, lambda cp: cat(cp) == "Nd")
    assert not mismatches(got, lambda cp: chr(cp).isdecimal())


# White_Space (PropList.txt, Unicode 13.0), written out by hand
WHITE_SPACE = set(range(0x09, 0x0E)) | {0x20, 0x85, 0xA0, 0x1680} | set(range(0x2000, 0x200B)) | {
    0x2028, 0x2029, 0x202F, 0x205F, 0x3000}


def test_space_is_white_space():
    assert len(WHITE_SPACE) == 25
    got = product("^\\s$")
    assert not mismatches(got, lambda cp: cp in WHITE_SPACE)


def other_alphabetic_outside_lm(cp):
    """The Other_Alphabetic code points that are neither letters nor marks: the circled, squared,
    negative circled and negative squared Latin letters (So), named as such."""
    if cat(cp) != "So":
        return False
    name = unicodedata.name(chr(cp), "")
    return any(name.startswith(p) for p in ("CIRCLED LATIN CAPITAL LETTER ", "CIRCLED LATIN SMALL LETTER ",
                                            "SQUARED LATIN CAPITAL LETTER ", "NEGATIVE CIRCLED LATIN CAPITAL LETTER ",
                                            "NEGATIVE SQUARED LATIN CAPITAL LETTER "))


def test_word_class_composition():
    def word(cp):
        c = cat(cp)
        return (c[0] in "LM" or c in ("Nd", "Nl", "Pc") or cp in (0x200C, 0x200D)  # Join_Control
                or other_alphabetic_outside_lm(cp))
    got = product("^\\w$")
    assert not mismatches(got, word)
    # the name-derived part is the four ranges of 26 or 52 letters PropList lists
    assert sum(1 for cp in range(0x110000) if not 0xD800 <= cp < 0xE000 and other_alphabetic_outside_lm(cp)) == 130


@pytest.mark.parametrize("pattern", ["^\\p{Lu}$", "^\\p{Mn}$", "^\\p{Cn}$", "^\\w$", "^\\s$", "^\\d$"])
def test_oracle_agrees_on_a_sample(pattern):
    got = product(pattern)
    for k in range(0, len(CPS), 97):
        cp = CPS[k]
        assert O.regex_match(pattern, chr(cp)) == got[k], (pattern, f"U+{cp:04X}")


def _orbits():
    """Simple case-folding orbits over the BMP and plane 1, from Python's casefold where it yields a
    single character (there full and simple folding coincide: CaseFolding.txt status C). Code points
    whose full folding is longer (status F, with or without an S alternative) are left out, as are
    their orbits' unknown simple members."""
    fold, orbits = {}, {}
    for cp in range(0x20000):
        if 0xD800 <= cp < 0xE000:
            continue
        f = chr(cp).casefold()
        if len(f) == 1:
            fold[cp] = ord(f)
            orbits.setdefault(ord(f), []).append(cp)
    return fold, {k: v for k, v in orbits.items() if len(v) > 1}


def test_case_folding_orbits():
    fold, orbits = _orbits()
    assert len(orbits) > 1300
    checked = 0
    for f, members in sorted(orbits.items()):
        # the characters a lower / upper mapping connects to the orbit without folding into it
        # (U+0131 dotless i against {I, i}): they must stay outside
        near = set()
        for cp in members:
            for m in (chr(cp).lower(), chr(cp).upper()):
                if len(m) == 1 and ord(m) in fold and fold[ord(m)] != f:
                    near.add(ord(m))
        subjects = [chr(cp) for cp in members] + [chr(cp) for cp in sorted(near)]
        for first in members[:2]:
            got = K.pattern_match_many(REGEX, f"(?i)^\\x{{{first:X}}}$", subjects)
            want = [1] * len(members) + [0] * len(near)
            assert got == want, (f"U+{first:04X}", [f"U+{ord(s):04X}" for s in subjects], got)
            checked += 1
    assert checked > 2600
