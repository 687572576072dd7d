"""The label-constraint regex dialect (Rust `regex` syntax and is_match search
semantics, Unicode \\d \\w \\s, word boundaries and simple case folding — ASCII under (?-u) —
matching over code points), three ways:

* the product: automaton.cpp's byte-level DFA (kw_pattern_match, the same compiler that builds the
  device tables);
* the oracle: oracle/kwregex.c, an independent parser and a Pike VM over code points;
* Python's `re` WITHOUT re.ASCII (its own Unicode tables and folding) on a rendering of the same
  tree (tests/regex_gen.py), for random patterns over the characters where Rust and Python agree;
  and a hand table of the constructs VERDICT r03 / r04 named (`(?:)`, `(?i)`, `\\b`, `\\A`/`\\z`,
  Unicode classes and folding, `(?-u)`, `\\p{..}` General_Category classes, Script and other
  properties refused) with Rust's answers written down.

All three must agree on every (pattern, subject). -1 = the pattern is refused (an init error)."""
import re

import pytest

import kwgpu as K
import oracle as O
from regex_gen import Gen

REGEX = 2

# (pattern, subject, expected): 1 match, 0 no match, -1 refused
TABLE = [
    (r"(?:ab)+c", "xababc", 1), (r"(?:ab)+c", "xabc", 1), (r"^(?:ab)+$", "aba", 0),
    (r"(?i)ABC", "xabcx", 1), (r"(?i)^web$", "WeB", 1), (r"(?i:w)eb", "Web", 1), (r"(?i:w)eb", "WEB", 0),
    (r"a(?i)b|c", "aB", 1), (r"a(?i)b|c", "C", 1), (r"(a(?i)b)c", "aBC", 0), (r"(?i)k", "\u212a", 1),
    (r"\bweb\b", "a web b", 1), (r"\bweb\b", "aweb", 0), (r"\bweb\b", "web", 1), (r"\Bb", "ab", 1),
    (r"\bé", "é", 1), (r"\<ab\>", "x ab y", 1), (r"\<ab", "xab", 0), (r"ab\>", "abc", 0),
    (r"\b{start}ab", "xab", 0), (r"\b{end-half}", "", 1), (r"\b{start-half}a", "ba", 0),
    (r"\Aweb\z", "web", 1), (r"\Aweb\z", "web\n", 0), (r"^web$", "web", 1), (r"web$", "web\n", 0),
    (r"(?m)^web$", "a\nweb\nb", 1), (r"^web$", "a\nweb\nb", 0), (r"(?m)^$", "a\n", 1),
    (r"^.$", "é", 1), (r"^[^a]$", "é", 1), (r"^..$", "é", 0), (r"^.$", "\U0001D11E", 1), (r".", "\n", 0),
    (r"(?s).", "\n", 1), (r"^\W$", "é", 0), (r"\d", "٣", 1), (r"\w", "é", 1),
    # Unicode classes, folding and word boundaries (VERDICT r04 probes first); (?-u) keeps ASCII
    (r"^\w+$", "é", 1), (r"^\d$", "٣", 1), (r"^\s$", "\u00a0", 1), (r"(?i)^k$", "\u212a", 1),
    (r"(?-u:\w)", "é", 0), (r"(?-u:\d)", "٣", 0), (r"(?-u:\s)", "\u00a0", 0), (r"(?i-u)^k$", "\u212a", 0),
    (r"^\w+$", "naïve", 1), (r"^\w+$", "e\u0301", 1), (r"^\w$", "\u24b6", 1), (r"^\w$", "\u203f", 1),
    (r"^\w$", "\u200d", 1), (r"^\w$", "²", 0), (r"^\d$", "²", 0), (r"^\s$", "\x1c", 0),
    (r"(?i)^ß$", "ẞ", 1), (r"(?i)^σ$", "ς", 1), (r"(?i)^s$", "ſ", 1), (r"(?i)^i$", "ı", 0),
    (r"(?i)^i$", "İ", 0), (r"(?i)^[a-z]$", "\u212a", 1), (r"(?i)[[:lower:]]", "\u212a", 1),
    (r"[[:alpha:]]", "é", 0), (r"é\b", "é x", 1), (r"a\b", "aé", 0), (r"\Bé", "aé", 1),
    (r"\b{start}é", "-é", 1), (r"\b{end}", "中", 1), (r"^\W+$", "\U0001D11E", 1),
    (r"[[:alpha:]]+\d", "ab1", 1), (r"[:alpha:]", "h", 1), (r"[[:^digit:]]", "5", 0),
    (r"[a-z&&[^aeiou]]", "e", 0), (r"[a-z&&[^aeiou]]", "b", 1), (r"[a-z--b]", "b", 0), (r"[a-c~~b-d]", "b", 0),
    (r"[a-c~~b-d]", "d", 1), (r"[]a]", "]", 1), (r"[^]a]", "]", 0), (r"[a-]", "-", 1), (r"[\]]", "]", 1),
    (r"(?P<x>a)(?<y>b)", "ab", 1), (r"(?P<x>a)(?P<x>b)", "ab", -1), (r"(?x) a b # c", "ab", 1),
    (r"(?x)[a b]", " ", 0), (r"(?x)a\ b", "a b", 1), (r"\x41B\U00000043", "ABC", 1), (r"\x{1D11E}", "\U0001D11E", 1),
    (r"é", "é", 1), (r"(?i)\x41", "a", 1), (r"a{2}{3}", "aaaaaa", 1), (r"a{,3}", "a", -1), (r"a{3,1}", "a", -1),
    (r"a{1001}", "a" * 1001, 1), (r"\-\ \#\&\~", "- #&~", 1), (r"a*?b", "aab", 1), (r"(|a)b", "b", 1), (r"()", "", 1),
    (r"", "", 1), (r"a|", "x", 1),
    # \p{..} General_Category classes (r06): Rust's regex answers, by hand
    (r"\p{L}", "a", 1), (r"\pL", "a", 1), (r"\pL", "1", 0), (r"^\p{Lu}+$", "ÀB", 1), (r"^\p{Lu}+$", "Ab", 0),
    (r"(?i)^\p{Lu}+$", "Ab", 1), (r"(?i)^\P{Lu}$", "a", 0), (r"^\P{Lu}$", "a", 1), (r"^\P{L}$", "é", 0),
    (r"^\p{Ll}$", "ß", 1), (r"^\p{Lt}$", "ǅ", 1), (r"^\p{LC}$", "ǅ", 1), (r"^\p{Lo}$", "中", 1),
    (r"^\p{Lm}$", "ʰ", 1), (r"^\p{Nd}$", "٣", 1), (r"^\p{Nl}$", "ⅻ", 1), (r"^\p{No}$", "²", 1),
    (r"^\p{N}+$", "1²ⅻ", 1), (r"^\p{Mn}$", "\u0301", 1), (r"^\p{M}$", "a", 0), (r"^\p{Pc}$", "_", 1),
    (r"^\p{Pd}$", "-", 1), (r"^\p{Ps}\p{Pe}$", "()", 1), (r"^\p{Pi}\p{Pf}$", "«»", 1), (r"^\p{Po}$", "!", 1),
    (r"^\p{Sm}$", "+", 1), (r"^\p{Sc}$", "€", 1), (r"^\p{Sk}$", "^", 1), (r"^\p{So}$", "©", 1),
    (r"^\p{Zs}$", "\u00a0", 1), (r"^\p{Zl}$", "\u2028", 1), (r"^\p{Zp}$", "\u2029", 1), (r"^\p{Cc}$", "\x1f", 1),
    (r"^\p{Cf}$", "\u200d", 1), (r"^\p{Co}$", "\ue000", 1), (r"^\p{Cn}$", "\U000e0080", 1), (r"^\p{Cs}$", "a", 0),
    (r"^\p{C}$", "\x00", 1), (r"^\p{Z}$", " ", 1), (r"^\p{S}$", "a", 0), (r"^\p{P}$", "a", 0),
    (r"^\p{Uppercase_Letter}$", "A", 1), (r"^\p{uppercaseletter}$", "A", 1), (r"^\p{ Upper-Case_letter }$", "A", 1),
    (r"^\p{isLu}$", "A", 1), (r"^\p{gc=Lu}$", "A", 1), (r"^\p{General_Category:Lu}$", "A", 1),
    (r"^\p{gc!=Lu}$", "A", 0), (r"^\P{gc!=Lu}$", "A", 1), (r"^\p{digit}$", "٣", 1), (r"^\p{punct}$", "!", 1),
    (r"^\p{cntrl}$", "\x7f", 1), (r"^\p{Combining_Mark}$", "\u0301", 1), (r"^\p{Any}$", "\U0010FFFD", 1),
    (r"^\p{ASCII}$", "é", 0), (r"^\p{Assigned}$", "\U000e0080", 0), (r"^\p{White_Space}$", "\u3000", 1),
    (r"^[\p{L}\d]+$", "a1é", 1), (r"^[\p{L}&&\p{Ll}]$", "A", 0), (r"^[\p{L}--\p{Lu}]$", "a", 1),
    (r"^[^\p{L}]$", "1", 1), (r"^[\P{L}]$", "1", 1), (r"\pN\pL", "1a", 1),
    # no assertion holds inside a UTF-8 sequence (r06: the product's \B matched between the bytes of
    # U+2003; Rust never reports an empty match that splits a code point)
    (r"\B", "a\u2003b", 0), (r"\B", "é", 0), (r"\B", "\u2003", 1), (r"a\b{end-half}", "a\u00a0", 1),
    (r"\b{start-half}b", "\u2003b", 1), (r"(?-u)\b{start-half}\b{end-half}", "\u2003", 1),
    (r"(?-u)\B", "ab", -1), (r"(?-u:\B)a", "a", -1),
    # refused by both (as by Rust's parser, or by this dialect: DESIGN.md §2)
    (r"\P{Greek}", "a", -1), (r"\p{Greek}", "a", -1), (r"\p{sc=Latin}", "a", -1), (r"\p{Alphabetic}", "a", -1),
    (r"\p{IsC}", "\x01", -1), (r"\p{L", "a", -1), (r"(?-u)\pL", "a", -1), (r"\p", "a", -1),
    (r"(?-u).", "a", -1), (r"(?-u)[^a]", "b", -1),
    (r"(?-u)\W", "b", -1), (r"(?-u)\xFF", "b", -1), (r"(?-u)a\w", "ab", 1), (r"(?-u)é", "é", 1),
    (r"a\Z", "a", -1), (r"(?R)a", "a", -1), (r"\1", "a", -1), (r"(a)\1", "aa", -1), (r"(?=a)", "a", -1),
    (r"(?<=a)b", "ab", -1), (r"(?!a)", "b", -1), (r"(a", "a", -1), (r"a)", "a", -1), (r"\y", "y", -1),
    (r"[a", "a", -1), (r"[]", "a", -1), (r"[z-a]", "a", -1), (r"*a", "a", -1), (r"a{2", "aa", -1),
    (r"(?i-)a", "a", -1), (r"(?)a", "a", -1), (r"(?ii)a", "a", -1), (r"\0", "\0", -1), (r"[\b]", "b", -1),
    (r"(?#c)a", "a", -1), (r"\e", "e", -1),
]


def product(p, s):
    return K.pattern_match(REGEX, p, s)


@pytest.mark.parametrize("pat,subj,want", TABLE)
def test_dialect_table(pat, subj, want):
    assert product(pat, subj) == want, "product"
    assert O.regex_match(pat, subj) == want, "oracle"
    nfa = K.pattern_match_many(REGEX | 0x100, pat, [subj])
    assert (nfa[0] if nfa is not None else -1) == want, "product NFA form"


def test_common_alphabet_properties():
    """The characters random subjects are drawn from (regex_gen.ALPHA) have the same \\w / \\d / \\s
    membership and case-folding partners in Rust's regex (written here by hand from the Unicode
    properties UTS #18 Annex C names) and in Python's re, and the product and oracle answer them."""
    from regex_gen import ALPHA
    nonword = {"-", ".", " ", "\n", "#", "&", "~", "\U0001D11E", "\u00a0", "\u2003"}
    digits = {"0", "1", "9", "٣", "۵"}
    spaces = {" ", "\n", "\u00a0", "\u2003"}
    for c in ALPHA:
        for cls, members in (("\\w", set(ALPHA) - nonword), ("\\d", digits), ("\\s", spaces)):
            want = 1 if c in members else 0
            assert (1 if re.fullmatch(cls, c) else 0) == want, ("python", cls, c)
            assert product(f"^{cls}$", c) == want, ("product", cls, c)
            assert O.regex_match(f"^{cls}$", c) == want, ("oracle", cls, c)


@pytest.mark.parametrize("block", range(8))
def test_random_patterns_three_ways(block):
    """product == oracle == Python re on random (pattern, subject) pairs of the dialect."""
    checked = 0
    for seed in range(block * 250, (block + 1) * 250):
        g = Gen(seed)
        rust, py = g.pattern()
        pyre = re.compile(py)
        subjects = [g.subject(rust) for _ in range(6)] + [""]
        prod = K.pattern_match_many(REGEX, rust, subjects)
        assert prod is not None, f"product refuses {rust!r}"
        # the product's NFA form (what a pattern beyond the DFA state budget runs as) agrees too
        assert K.pattern_match_many(REGEX | 0x100, rust, subjects) == prod, f"product NFA vs DFA: {rust!r}"
        for s, got_p in zip(subjects, prod):
            want = 1 if pyre.search(s) else 0
            got_o = O.regex_match(rust, s)
            assert got_o == want, f"oracle: {rust!r} on {s!r}: {got_o}, Python {want} ({py!r})"
            assert got_p == want, f"product: {rust!r} on {s!r}: {got_p}, Python {want} ({py!r})"
            checked += 1
    assert checked == 250 * 7
