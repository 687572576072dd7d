"""The trusted-repos glob dialect (fnmatch(3) with flags 0 in a UTF-8 locale, matching
over characters), checked four ways:

* the product: automaton.cpp parse_glob -> the byte-level automaton the device tables are built
  from (kw_pattern_match_many, DFA and forced-NFA forms);
* the oracle: oracle/kwregex.c orc_glob_match, its own parser and a star-restart matcher over code
  points, independent of the process locale;
* glibc's fnmatch(3) itself through ctypes, on ASCII patterns and subjects: glibc 2.35 under this
  image's C.UTF-8 gives both the byte and the character reading on multibyte input (`?` and `??`
  both match "é", measured), so it pins the ASCII syntax rules (escapes, classes, odd brackets) only;
* Python's fnmatch.fnmatchcase, which matches str characters, on the subset both read alike (no
  `\\`, no `[^`, no `[:`): the independent pin of the character reading.

Plus a hand table of the odd cases with the answers written down. -1 = refused (an init error)."""
import ctypes
import fnmatch
import random

import pytest

import kwgpu as K
import oracle as O

GLOB = 1

TABLE = [
    ("*", "", 1), ("*", "a/b", 1), ("a*b", "a/x/b", 1), ("?", "é", 1), ("?", "\U0001F600", 1), ("??", "é", 0),
    ("[!a]", "é", 1), ("[^a]", "é", 1), ("[^a]", "a", 0), ("[é]", "é", 1), ("[à-ê]", "é", 1), ("[à-ê]", "ë", 0),
    ("[!é]", "e", 1), ("[!é]", "é", 0), ("*é?", "xéy", 1), ("*é?", "xé", 0), ("[]a]", "]", 1), ("[!]a]", "]", 0),
    ("[!]a]", "b", 1), ("[a-]", "-", 1), ("[a-]", "b", 0), ("[z-a]", "m", 0), ("[z-a]x", "x", 0),
    ("\\*", "*", 1), ("\\*", "a", 0), ("a\\", "a", 0), ("a\\", "a\\", 0), ("[a", "[a", 1), ("[a", "a", 0),
    ("[\\]]", "]", 1), ("[a\\-z]", "-", 1), ("[a\\-z]", "m", 0), ("[a-\\z]", "m", 1), ("[\\!a]", "!", 1),
    ("[a-", "[a-", 0), ("x[a-", "xb", 0), ("[a-\\", "a", 0), ("[\\", "[\\", 0),
    ("[[:alpha:]]", "q", 1), ("[[:alpha:]]", "1", 0), ("[![:digit:]]", "a", 1), ("[[:digit:][:upper:]]", "Q", 1),
    ("[[:alpha:]]", "é", 0), ("[[:Alpha:]]", "A", 0), ("[[:Alpha:]]", ":", 0), ("[[:Alpha:]]", ":]", 1),
    ("[[:zz:]]", "z]", 1), ("[[:zz:]]", "z", 0),
    ("[[:alpha]", "[", 1), ("[[:alpha]", "a", 1),
    ("[[:word:]]", "a", -1), ("[[:ascii:]]", "a", -1), ("[[:foo:]]", "a", -1), ("[[::]]", "a", -1),
    ("[[.a.]]", "a", -1), ("[[=a=]]", "a", -1),
    ("ghcr.io/*", "ghcr.io/kubewarden/policy", 1), ("*.io", "ghcr.io", 1), ("reg?stry", "regístry", 1),
]


def libc_fnmatch():
    """glibc fnmatch(p, s, 0) -> 1 / 0, or None where it does not pin the dialect (non-ASCII)."""
    f = ctypes.CDLL(None).fnmatch
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    return lambda p, s: (1 if f(p.encode(), s.encode(), 0) == 0 else 0) if (p + s).isascii() else None


@pytest.mark.parametrize("pat,subj,want", TABLE)
def test_glob_table(pat, subj, want):
    assert K.pattern_match(GLOB, pat, subj) == want, "product"
    assert O.glob_match(pat, subj) == want, "oracle"
    if want >= 0 and libc_fnmatch()(pat, subj) is not None:
        assert libc_fnmatch()(pat, subj) == want, "glibc fnmatch"


CHARS = ["a", "b", "é", "/", ".", "-", "]", "!", "\U0001F600", "z"]


def rand_glob(r):
    out = []
    for _ in range(r.randint(0, 6)):
        k = r.random()
        if k < 0.2:
            out.append("*")
        elif k < 0.35:
            out.append("?")
        elif k < 0.6:
            body = []
            for _ in range(r.randint(1, 3)):
                c = r.choice(CHARS)
                if r.random() < 0.3:
                    body.append(c + "-" + r.choice(CHARS))
                elif r.random() < 0.1:
                    body.append(r.choice(["[:alpha:]", "[:digit:]", "[:punct:]", "[:lower:]"]))
                else:
                    body.append(c)
            neg = r.choice(["", "", "!", "^"])
            out.append("[" + neg + "".join(body) + ("]" if r.random() < 0.9 else ""))
        elif k < 0.65:
            out.append("\\" + r.choice(CHARS + ["*", "?", "["]))
        else:
            out.append(r.choice(CHARS))
    if r.random() < 0.03:
        out.append("\\")
    return "".join(out)


def python_reads_alike(p):
    return "\\" not in p and "[^" not in p and "[:" not in p and "[!]" not in p and "[]" not in p


@pytest.mark.parametrize("seed", range(6))
def test_glob_random_four_ways(seed):
    r = random.Random(1000 + seed)
    g = libc_fnmatch()
    checked = 0
    for _ in range(150):
        p = rand_glob(r)
        subs = ["".join(r.choice(CHARS) for _ in range(r.randint(0, 6))) for _ in range(40)]
        want = K.pattern_match_many(GLOB, p, subs)
        nfa = K.pattern_match_many(GLOB | 0x100, p, subs)
        if want is None:
            assert all(O.glob_match(p, s) == -1 for s in subs[:1]), p
            continue
        assert nfa == want, ("forced NFA", p)
        for s, w in zip(subs, want):
            assert O.glob_match(p, s) == w, ("oracle", p, s)
            if g(p, s) is not None:
                assert g(p, s) == w, ("glibc", p, s)
            if python_reads_alike(p):
                assert int(fnmatch.fnmatchcase(s, p)) == w, ("python", p, s)
            checked += 1
    assert checked > 3000
