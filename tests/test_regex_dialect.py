"""The label-constraint regex dialect (Rust `regex` syntax and is_match search
semantics, ASCII \\d \\w \\s \\b and case folding, matching over code points), three ways:

* the product: automaton.cpp's byte-level DFA (kw_pattern_match, the same compiler that builds the
  device tables);
* the oracle: oracle/kwregex.c, an independent parser and a Pike VM over code points;
* Python's `re`, on an explicit rendering of the same tree (tests/regex_gen.py), for random
  patterns; and a hand table of the constructs VERDICT r03 named (`(?:)`, `(?i)`, `\\b`, `\\A`/`\\z`,
  `\\p` refused) with the expected answers written down.

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
    (r"a(?i)b|c", "aB", 1), (r"a(?i)b|c", "C", 1), (r"(a(?i)b)c", "aBC", 0), (r"(?i)k", "K", 0),
    (r"\bweb\b", "a web b", 1), (r"\bweb\b", "aweb", 0), (r"\bweb\b", "web", 1), (r"\Bb", "ab", 1),
    (r"\bé", "é", 0), (r"\<ab\>", "x ab y", 1), (r"\<ab", "xab", 0), (r"ab\>", "abc", 0),
    (r"\b{start}ab", "xab", 0), (r"\b{end-half}", "", 1), (r"\b{start-half}a", "ba", 0),
    (r"\Aweb\z", "web", 1), (r"\Aweb\z", "web\n", 0), (r"^web$", "web", 1), (r"web$", "web\n", 0),
    (r"(?m)^web$", "a\nweb\nb", 1), (r"^web$", "a\nweb\nb", 0), (r"(?m)^$", "a\n", 1),
    (r"^.$", "é", 1), (r"^[^a]$", "é", 1), (r"^..$", "é", 0), (r"^.$", "\U0001D11E", 1), (r".", "\n", 0),
    (r"(?s).", "\n", 1), (r"^\W$", "é", 1), (r"\d", "٣", 0), (r"\w", "é", 0),
    (r"[[:alpha:]]+\d", "ab1", 1), (r"[:alpha:]", "h", 1), (r"[[:^digit:]]", "5", 0),
    (r"[a-z&&[^aeiou]]", "e", 0), (r"[a-z&&[^aeiou]]", "b", 1), (r"[a-z--b]", "b", 0), (r"[a-c~~b-d]", "b", 0),
    (r"[a-c~~b-d]", "d", 1), (r"[]a]", "]", 1), (r"[^]a]", "]", 0), (r"[a-]", "-", 1), (r"[\]]", "]", 1),
    (r"(?P<x>a)(?<y>b)", "ab", 1), (r"(?P<x>a)(?P<x>b)", "ab", -1), (r"(?x) a b # c", "ab", 1),
    (r"(?x)[a b]", " ", 0), (r"(?x)a\ b", "a b", 1), (r"\x41B\U00000043", "ABC", 1), (r"\x{1D11E}", "\U0001D11E", 1),
    (r"é", "é", 1), (r"(?i)\x41", "a", 1), (r"a{2}{3}", "aaaaaa", 1), (r"a{,3}", "a", -1), (r"a{3,1}", "a", -1),
    (r"a{1001}", "a" * 1001, 1), (r"\-\ \#\&\~", "- #&~", 1), (r"a*?b", "aab", 1), (r"(|a)b", "b", 1), (r"()", "", 1),
    (r"", "", 1), (r"a|", "x", 1),
    # refused by both (as by Rust's parser, or by this dialect: DESIGN.md §2)
    (r"\p{L}", "a", -1), (r"\pL", "a", -1), (r"\P{Greek}", "a", -1), (r"(?-u).", "a", -1), (r"(?-u)[^a]", "b", -1),
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


def _py(pt, subj):
    return 1 if re.search(pt, subj, re.ASCII) else 0


@pytest.mark.parametrize("block", range(8))
def test_random_patterns_three_ways(block):
    """product == oracle == Python re on random (pattern, subject) pairs of the dialect."""
    checked = 0
    for seed in range(block * 250, (block + 1) * 250):
        g = Gen(seed)
        rust, py = g.pattern()
        pyre = re.compile(py, re.ASCII)
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
