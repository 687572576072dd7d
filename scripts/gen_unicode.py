"""Generates the Unicode tables of the label-constraint regex dialect from Python's
unicodedata (this image: Python 3.10, Unicode 13.0.0):

  policy-server_amd/csrc/unicode_data.hpp   product (automaton.cpp, kwdev.hpp nfa_run)
  oracle/unicode_data.h                     oracle (kwregex.c), its own layout

The definitions are the Rust `regex` crate's (regex-syntax, UTS #18 Annex C):
  \\w  Alphabetic + M + Nd + Pc + Join_Control. Alphabetic = L + Nl + Other_Alphabetic; the
      Other_Alphabetic code points outside M are the circled / squared Latin letters listed below
      (PropList.txt; unicodedata has no property lookup).
  \\d  Nd.
  \\s  White_Space (a fixed list in the sources, not generated).
  (?i) simple case folding (CaseFolding.txt statuses C + S): a code point folds to casefold() when
      that is one code point, else to lower() when that is one, else to itself; code points with
      the same fold match each other.
  \\p{..} General_Category (r06): one sorted run table (lo, hi, category) covering every assigned
      code point; a code point in no run is Cn. The categories are unicodedata.category's.

and, for the product only, the tables of the group-expression string functions (r06, expr.cpp /
slots.hpp; rhai's to_upper / to_lower / trim / split are Rust's str methods):
  full case mappings   str.upper() / str.lower() of each single code point where it differs (the
                       SpecialCasing unconditional mappings included: ß -> SS, İ -> i̇); Σ's
                       final-sigma context is applied by the caller
  Cased, Case_Ignorable the two properties of the Final_Sigma context (Unicode 3.13), read back from
                       CPython's own implementation of that rule: for a code point c, lower() of
                       "A" + c + "Σ" ends in ς iff c is case-ignorable or cased, and lower() of
                       c + "Σ" ends in ς iff c is cased and not case-ignorable (only that
                       combination matters to the rule)
Rust's regex 1.x / std carry Unicode 15.0 tables; characters added after 13.0 are parity unpinned.
Run: python scripts/gen_unicode.py (the outputs are committed)."""
import os
import sys
import unicodedata

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OTHER_ALPHA_SO = [(0x24B6, 0x24E9), (0x1F130, 0x1F149), (0x1F150, 0x1F169), (0x1F170, 0x1F189)]
JOIN_CONTROL = [(0x200C, 0x200D)]


def ranges(pred):
    out, start = [], None
    for cp in range(0x110000 + 1):
        ok = cp < 0x110000 and not (0xD800 <= cp <= 0xDFFF) and pred(cp)
        if ok and start is None:
            start = cp
        elif not ok and start is not None:
            out.append((start, cp - 1))
            start = None
    return out


def in_ranges(cp, rs):
    return any(lo <= cp <= hi for lo, hi in rs)


def is_word(cp):
    cat = unicodedata.category(chr(cp))
    return (cat[0] in "LM" or cat in ("Nd", "Nl", "Pc") or in_ranges(cp, OTHER_ALPHA_SO)
            or in_ranges(cp, JOIN_CONTROL))


def is_digit(cp):
    return unicodedata.category(chr(cp)) == "Nd"


def simple_fold(cp):
    c = chr(cp)
    f = c.casefold()
    if len(f) == 1:
        return ord(f)
    lo = c.lower()
    if len(lo) == 1:
        return ord(lo)
    return cp


GC_NAMES = ["Cn", "Lu", "Ll", "Lt", "Lm", "Lo", "Mn", "Mc", "Me", "Nd", "Nl", "No", "Pc", "Pd", "Ps", "Pe", "Pi",
            "Pf", "Po", "Sm", "Sc", "Sk", "So", "Zs", "Zl", "Zp", "Cc", "Cf", "Cs", "Co"]


def gc_runs():
    out, prev, start = [], None, 0
    for cp in range(0x110001):
        g = unicodedata.category(chr(cp)) if cp < 0x110000 else None
        if g != prev:
            if prev is not None and prev != "Cn":
                out.append((start, cp - 1, GC_NAMES.index(prev)))
            prev, start = g, cp
    return out


def case_props():
    ign, cased = [], []
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = chr(cp)
        a = ("A" + c + "\u03a3").lower()[-1] == "\u03c2"
        b = (c + "\u03a3").lower()[-1] == "\u03c2"
        if a and not b:
            ign.append(cp)
        if b:
            cased.append(cp)
    return ign, cased


def to_ranges(cps):
    out = []
    for cp in cps:
        if out and out[-1][1] == cp - 1:
            out[-1] = (out[-1][0], cp)
        else:
            out.append((cp, cp))
    return out


def case_maps(fn):
    out = []
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        m = fn(chr(cp))
        if m != chr(cp):
            assert len(m) <= 3
            ms = [ord(x) for x in m] + [0] * (3 - len(m))
            out.append((cp, len(m), ms[0], ms[1], ms[2]))
    return out


def main():
    word = ranges(is_word)
    digit = ranges(is_digit)
    folds = {}
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        f = simple_fold(cp)
        folds.setdefault(f, set()).add(cp)
    orbits = [sorted(s | {f}) for f, s in folds.items() if len(s | {f}) > 1]
    # product: every orbit member -> the next member (a cycle), sorted by code point
    nxt = {}
    for o in orbits:
        for k, cp in enumerate(o):
            nxt[cp] = o[(k + 1) % len(o)]
    cyc = sorted(nxt.items())
    # oracle: (code point, its fold) for every code point whose orbit is not trivial
    pairs = sorted((cp, simple_fold(cp)) for o in orbits for cp in o)
    ver = unicodedata.unidata_version
    gcs = gc_runs()
    ign_cps, cased_cps = case_props()
    ign, cased = to_ranges(ign_cps), to_ranges(cased_cps)
    lows, ups = case_maps(str.lower), case_maps(str.upper)

    def arr(name, items, fmt, per=6, typ="UniRange"):
        lines = [f"inline constexpr {typ} {name}[] = {{"]
        for k in range(0, len(items), per):
            lines.append("    " + " ".join(fmt(x) for x in items[k:k + per]))
        lines.append("};")
        return "\n".join(lines)

    hx = lambda v: f"0x{v:X}"  # noqa: E731
    hpp = [
        "// unicode_data.hpp — GENERATED by scripts/gen_unicode.py from Python's unicodedata "
        f"(Unicode {ver}); do not edit.",
        "// The Unicode classes of the label-constraint regex dialect (DESIGN.md §2): \\w and \\d as the",
        "// Rust regex crate defines them, and simple case folding as cycles over each fold orbit.",
        "#pragma once",
        "#include <cstdint>",
        "",
        "namespace kw {",
        "",
        "struct UniRange {",
        "  uint32_t lo, hi;",
        "};",
        "struct UniFold {",
        "  uint32_t cp, next;  // the next code point of cp's simple case folding orbit (a cycle)",
        "};",
        f'inline constexpr const char* kUnicodeVersion = "{ver}";',
        arr("kUniWord", word, lambda r: f"{{{hx(r[0])}, {hx(r[1])}}},"),
        f"inline constexpr uint32_t kUniWordN = {len(word)};",
        arr("kUniDigit", digit, lambda r: f"{{{hx(r[0])}, {hx(r[1])}}},"),
        f"inline constexpr uint32_t kUniDigitN = {len(digit)};",
        arr("kUniFold", cyc, lambda r: f"{{{hx(r[0])}, {hx(r[1])}}},", typ="UniFold"),
        f"inline constexpr uint32_t kUniFoldN = {len(cyc)};",
        "// General_Category runs (\\p{..}): every assigned code point, sorted; category = kUniGcNames index",
        "struct UniGcRun {",
        "  uint32_t lo, hi, gc;",
        "};",
        "inline constexpr const char* kUniGcNames[] = {" + ", ".join(f'"{g}"' for g in GC_NAMES) + "};",
        arr("kUniGc", gcs, lambda r: f"{{{hx(r[0])}, {hx(r[1])}, {r[2]}}},", per=5, typ="UniGcRun"),
        f"inline constexpr uint32_t kUniGcN = {len(gcs)};",
        "// Full case mappings of single code points (str.lower / str.upper), sorted by code point:",
        "// (cp, n, mapping[3]); Case_Ignorable and Cased-but-not-Case_Ignorable as ranges (Final_Sigma)",
        "struct UniCaseMap {",
        "  uint32_t cp, n, m[3];",
        "};",
        arr("kUniLower", lows, lambda r: f"{{{hx(r[0])}, {r[1]}, {{{hx(r[2])}, {hx(r[3])}, {hx(r[4])}}}}},", per=4,
            typ="UniCaseMap"),
        f"inline constexpr uint32_t kUniLowerN = {len(lows)};",
        arr("kUniUpper", ups, lambda r: f"{{{hx(r[0])}, {r[1]}, {{{hx(r[2])}, {hx(r[3])}, {hx(r[4])}}}}},", per=4,
            typ="UniCaseMap"),
        f"inline constexpr uint32_t kUniUpperN = {len(ups)};",
        arr("kUniCaseIgnorable", ign, lambda r: f"{{{hx(r[0])}, {hx(r[1])}}},"),
        f"inline constexpr uint32_t kUniCaseIgnorableN = {len(ign)};",
        arr("kUniCased", cased, lambda r: f"{{{hx(r[0])}, {hx(r[1])}}},"),
        f"inline constexpr uint32_t kUniCasedN = {len(cased)};",
        "",
        "}  // namespace kw",
        "",
    ]
    with open(os.path.join(ROOT, "policy-server_amd", "csrc", "unicode_data.hpp"), "w") as f:
        f.write("\n".join(hpp))

    def carr(name, items, per=8):
        lines = [f"static const uint32_t {name}[] = {{"]
        flat = [v for it in items for v in it]
        for k in range(0, len(flat), per):
            lines.append("    " + " ".join(f"{hx(v)}," for v in flat[k:k + per]))
        lines.append("};")
        return "\n".join(lines)

    h = [
        "/* unicode_data.h — GENERATED by scripts/gen_unicode.py from Python's unicodedata "
        f"(Unicode {ver}); do not edit.",
        "   TEST INFRASTRUCTURE ONLY (the oracle's regex matcher). Flat u32 arrays: word / digit ranges",
        "   as (lo, hi) pairs; case folding as (code point, simple fold) pairs of every code point whose",
        "   fold orbit is not trivial, sorted by code point; General_Category as (lo, hi, category) runs. */",
        "#ifndef ORC_UNICODE_DATA_H",
        "#define ORC_UNICODE_DATA_H",
        "#include <stdint.h>",
        carr("orc_uni_word", word),
        f"#define ORC_UNI_WORD_N {len(word)}",
        carr("orc_uni_digit", digit),
        f"#define ORC_UNI_DIGIT_N {len(digit)}",
        carr("orc_uni_fold", pairs),
        f"#define ORC_UNI_FOLD_N {len(pairs)}",
        "/* General_Category runs: (lo, hi, category) triples, sorted; category indexes ORC_GC_NAMES",
        "   (unassigned code points are in no run: Cn) */",
        "static const char* const ORC_GC_NAMES[] = {" + ", ".join(f'"{g}"' for g in GC_NAMES) + "};",
        carr("orc_uni_gc", gcs, per=9),
        f"#define ORC_UNI_GC_N {len(gcs)}",
        "#endif",
        "",
    ]
    with open(os.path.join(ROOT, "oracle", "unicode_data.h"), "w") as f:
        f.write("\n".join(h))
    print(f"Unicode {ver}: word {len(word)} ranges, digit {len(digit)}, fold {len(cyc)} orbit members",
          file=sys.stderr)


if __name__ == "__main__":
    main()
