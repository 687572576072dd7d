"""Random label-constraint regexes in the dialect of DESIGN.md §2, each rendered twice from one
tree: as Rust `regex` source (what a policies.yml holds, fed to the product and to the oracle's
kwregex.c) and as a Python `re` pattern matched WITHOUT re.ASCII, so that Python's own Unicode
engine — its \\w \\d \\s, word boundaries and case folding, built from its own Unicode tables — is a
third, independent statement of the semantics (Unicode is the Rust default).

The two engines agree only on a common subset of Unicode (DESIGN.md §2 lists where they differ:
marks, Other_Alphabetic symbols, Pc / Join_Control, No digits, \\x1c-\\x1f, dotted / dotless i).
Subjects are therefore drawn from ALPHA, characters on which Rust's and Python's definitions
agree (tests/test_regex_dialect.py pins each one's properties by hand), and a class is the set of
ALPHA characters Python puts in it:

  Rust construct                 Python rendering
  x under (?i)                   the ALPHA characters Python's (?i)x matches
  .  /  (?s).                    [^\\n]  /  [\\s\\S]
  [...] with &&, --, ~~, nesting  the ALPHA characters of the set (each item's members asked of
                                 Python's engine), (?!) when empty
  \\d \\w \\s \\D \\W \\S           \\d \\w \\s \\D \\W \\S (Unicode)
  \\p{gc} \\P{gc} \\pX             the ALPHA characters of those categories (unicodedata), folded under
                                 (?i) before a \\P negates them
  [:name:]                       its ASCII members (Rust's ASCII classes stay ASCII)
  ^ $ \\A \\z  (?m)^ (?m)$        \\A \\Z \\A \\Z (?<![^\\n]) (?![^\\n])
  \\b \\< \\> \\b{start-half} \\b{end-half}   \\b \\b(?=\\w) \\b(?<=\\w) (?<!\\w) (?!\\w) (Unicode \\w)
  \\B                            (?<=\\w)(?=\\w)|(?<!\\w)(?!\\w)  (Python's \\B never matches an empty string)
  (?flags) mid-group             applied by the generator to the rest of the group (no Python flag)
  (?x) white space, # comments   dropped
"""
import random
import re

META = set("\\.+*?()|[]{}^$#")
CLASS_META = set("\\[]^-&~")
# characters whose \\w / \\d / \\s membership and simple case folding are the same in Rust's regex
# (UTS #18 Annex C) and Python's re: ASCII, Latin / Greek / CJK letters, Nd digits of two scripts,
# an Nl numeral, Lt titlecase, Zs spaces, and the multi-member fold orbits k / K / KELVIN SIGN,
# s / S / LONG S, ß / ẞ, σ / ς / Σ, µ / μ / Μ, θ / ϑ / Θ / ϴ, å / Å / ANGSTROM SIGN
ALPHA = ["a", "b", "c", "k", "z", "A", "B", "K", "Z", "0", "1", "9", "_", "-", ".", " ", "\n", "#", "&", "~",
         "s", "S", "é", "É", "ÿ", "Ω", "ω", "中", "\U0001D11E", "ǅ", "ǈ", "ǉ", "Ǉ", "ª", "ⅻ", "٣", "۵",
         "\u00a0", "\u2003", "ß", "ẞ", "σ", "ς", "Σ", "\u212a", "ſ", "µ", "μ", "Μ", "θ", "ϑ", "Θ", "ϴ",
         "Å", "å", "\u212b"]
UNIVERSE = frozenset(ALPHA)
NAMED = {"alnum": [(48, 57), (65, 90), (97, 122)], "alpha": [(65, 90), (97, 122)], "digit": [(48, 57)],
         "lower": [(97, 122)], "upper": [(65, 90)], "space": [(9, 13), (32, 32)], "word": [(48, 57), (65, 90),
         (95, 95), (97, 122)], "xdigit": [(48, 57), (65, 70), (97, 102)],
         "punct": [(33, 47), (58, 64), (91, 96), (123, 126)], "blank": [(9, 9), (32, 32)], "ascii": [(0, 127)]}


# \p{..} General_Category values (r06): (Rust spelling, categories) — short and long names, aliases,
# loose spellings (case, ' ', '_', '-', an "is" prefix) and gc= forms; Python has no \p, so the
# rendering is the set of ALPHA characters whose unicodedata.category is one of the categories
GC_VALUES = [("L", "Lu Ll Lt Lm Lo"), ("Letter", "Lu Ll Lt Lm Lo"), ("Lu", "Lu"), ("Uppercase_Letter", "Lu"),
             ("lowercase letter", "Ll"), ("Ll", "Ll"), ("Lt", "Lt"), ("LC", "Lu Ll Lt"), ("Cased-Letter", "Lu Ll Lt"),
             ("Lo", "Lo"), ("isLm", "Lm"), ("N", "Nd Nl No"), ("Nd", "Nd"), ("digit", "Nd"), ("Nl", "Nl"),
             ("No", "No"), ("P", "Pc Pd Ps Pe Pi Pf Po"), ("punct", "Pc Pd Ps Pe Pi Pf Po"), ("Pc", "Pc"),
             ("Pd", "Pd"), ("Po", "Po"), ("S", "Sm Sc Sk So"), ("So", "So"), ("Z", "Zs Zl Zp"), ("Zs", "Zs"),
             ("space_separator", "Zs"), ("C", "Cc Cf Cs Co Cn"), ("Cc", "Cc"), ("M", "Mn Mc Me"),
             ("gc=Lu", "Lu"), ("General_Category=Nd", "Nd"), ("gc:L", "Lu Ll Lt Lm Lo")]


def gc_members(cats):
    import unicodedata
    return frozenset(c for c in ALPHA if unicodedata.category(c) in cats.split())


def py_members(py_item):
    """The ALPHA characters Python's engine puts in a one-character pattern."""
    rx = re.compile(py_item)
    return frozenset(c for c in ALPHA if rx.fullmatch(c))


def named(nm):
    return frozenset(c for c in ALPHA if any(lo <= ord(c) <= hi for lo, hi in NAMED[nm]))


def neg(a):
    return UNIVERSE - a


def fold(a):
    """(?i): every ALPHA character that Python's case-insensitive match of a member accepts"""
    out = set(a)
    for c in a:
        out |= py_members("(?i)" + re.escape(c))
    return frozenset(out)


def py_class(chars):
    if not chars:
        return "(?!)"
    return "[" + "".join(f"\\U{ord(c):08x}" for c in sorted(chars)) + "]"


class Flags:
    def __init__(self, i=False, m=False, s=False, x=False):
        self.i, self.m, self.s, self.x = i, m, s, x

    def copy(self):
        return Flags(self.i, self.m, self.s, self.x)


class Gen:
    def __init__(self, seed):
        self.r = random.Random(seed)
        self.names = 0

    def ws(self, f):
        """verbose mode: white space or a comment between items (Rust side only)"""
        if f.x and self.r.random() < 0.3:
            return self.r.choice([" ", "  ", "\t", " # note\n"])
        return ""

    def lit_rust(self, ch, f):
        r = self.r.random()
        cp = ord(ch)
        if f.x and ch.isspace() and cp >= 0x80:  # verbose mode skips Unicode white space too
            return f"\\x{{{cp:x}}}"
        if ch in META or (f.x and ch in " \t\n"):
            return "\\" + ch if ch not in "\n\t" else ("\\n" if ch == "\n" else "\\t")
        if ch == "\n":
            return "\\n"
        if r < 0.1:
            return f"\\x{{{cp:x}}}"
        if r < 0.15 and cp < 0x10000:
            return f"\\u{cp:04x}"
        if r < 0.2 and cp < 0x80:
            return f"\\x{cp:02x}"
        return ch

    def cls_char_rust(self, ch, f):
        if f.x and ch.isspace() and ord(ch) >= 0x80:
            return f"\\x{{{ord(ch):x}}}"
        if ch in CLASS_META or (f.x and ch in " \t\n#"):
            return "\\" + ch if ch not in "\n\t" else ("\\n" if ch == "\n" else "\\t")
        if ch == "\n":
            return "\\n"
        return ch

    def cls_item(self, f, depth):
        """(rust text, set) of one item: char, range, escape class, [:name:], nested class"""
        r = self.r.random()
        if r < 0.35:
            ch = self.r.choice(ALPHA)
            s = frozenset([ch])
            return self.cls_char_rust(ch, f), fold(s) if f.i else s
        if r < 0.55:
            a, b = sorted(self.r.sample(ALPHA, 2), key=ord)
            s = frozenset(c for c in ALPHA if ord(a) <= ord(c) <= ord(b))
            return f"{self.cls_char_rust(a, f)}-{self.cls_char_rust(b, f)}", fold(s) if f.i else s
        if r < 0.7:
            e = self.r.choice("dDwWsS")
            return "\\" + e, py_members("\\" + e)
        if r < 0.76:  # \p{..} / \P{..} / \pX: regex-syntax folds before it negates
            return self.gc_class(f)
        if r < 0.82:
            nm = self.r.choice(sorted(NAMED))
            s = fold(named(nm)) if f.i else named(nm)
            if self.r.random() < 0.25:
                return f"[:^{nm}:]", neg(s)
            return f"[:{nm}:]", s
        if depth < 2:
            return self.cls(f, depth + 1)
        ch = self.r.choice(ALPHA)
        return self.cls_char_rust(ch, f), frozenset([ch])

    def gc_class(self, f):
        name, cats = self.r.choice(GC_VALUES)
        s = gc_members(cats)
        if f.i:
            s = fold(s)
        negate = self.r.random() < 0.3
        if len(name) == 1 and self.r.random() < 0.5:
            txt = ("\\P" if negate else "\\p") + name
        else:
            txt = ("\\P{" if negate else "\\p{") + name + "}"
        if f.x and " " in txt:
            txt = txt.replace(" ", "_")
        return txt, neg(s) if negate else s

    def cls(self, f, depth=0):
        """(rust text '[...]', set)"""
        negate = self.r.random() < 0.25
        parts = []

        def union_part():
            txt, s = "", frozenset()
            for _ in range(self.r.randint(1, 3)):
                t, x = self.cls_item(f, depth)
                if txt and txt[-1] == "-" and t.startswith("-"):
                    t = "\\" + t
                txt += t + self.ws(f).replace("#", "").replace(" note\n", "")
                s = s | x
            return txt, s
        txt, s = union_part()
        if txt.startswith("]") or txt.startswith("^"):
            txt = "\\" + txt
        parts.append(txt)
        while self.r.random() < 0.2:
            op = self.r.choice(["&&", "--", "~~"])
            t2, s2 = union_part()
            if t2.startswith(op[0]):
                t2 = "\\" + t2
            parts.append(op + t2)
            if op == "&&":
                s = s & s2
            elif op == "--":
                s = s - s2
            else:
                s = s ^ s2
        body = "".join(parts)
        if negate:
            return "[^" + body + "]", neg(s)
        return "[" + body + "]", s

    def atom(self, f, depth):
        r = self.r.random()
        if r < 0.38:
            ch = self.r.choice(ALPHA)
            return self.lit_rust(ch, f), py_class(fold(frozenset([ch])) if f.i else frozenset([ch]))
        if r < 0.46:
            return ".", "[\\s\\S]" if f.s else "[^\\n]"
        if r < 0.6:
            t, s = self.cls(f)
            return t, py_class(s)
        if r < 0.64:
            e = self.r.choice("dDwWsS")
            return "\\" + e, "\\" + e
        if r < 0.68:
            t, s = self.gc_class(f)
            return t, py_class(s)
        if r < 0.8:
            k = self.r.choice(["^", "$", "\\A", "\\z", "\\b", "\\B", "\\<", "\\>", "\\b{start}", "\\b{end}",
                               "\\b{start-half}", "\\b{end-half}"])
            py = {"\\A": "\\A", "\\z": "\\Z", "\\b": "\\b", "\\B": "(?<=\\w)(?=\\w)|(?<!\\w)(?!\\w)", "\\<": "\\b(?=\\w)", "\\>": "\\b(?<=\\w)",
                  "\\b{start}": "\\b(?=\\w)", "\\b{end}": "\\b(?<=\\w)", "\\b{start-half}": "(?<!\\w)",
                  "\\b{end-half}": "(?!\\w)"}
            if k == "^":
                return k, "(?<![^\\n])" if f.m else "\\A"
            if k == "$":
                return k, "(?![^\\n])" if f.m else "\\Z"
            return k, "(?:" + py[k] + ")"
        if depth < 3:
            return self.group(f, depth + 1)
        return "a", "a"

    def group(self, f, depth):
        r = self.r.random()
        inner = f.copy()
        if r < 0.3:
            open_ = "("
        elif r < 0.55:
            open_ = "(?:"
        elif r < 0.7:
            self.names += 1
            open_ = self.r.choice(["(?P<g", "(?<g"]) + f"{self.names}>"
        else:
            on, off = "", ""
            for name in "imsx":
                if self.r.random() < 0.4:
                    val = self.r.random() < 0.6
                    setattr(inner, name, val)
                    if val:
                        on += name
                    else:
                        off += name
            if not on and not off:
                inner.i = True
                on = "i"
            open_ = "(?" + on + ("-" + off if off else "") + ":"
        rt, pt = self.alt(inner, depth)
        return open_ + rt + ")", "(?:" + pt + ")"

    def rep(self, f, depth):
        rt, pt = self.atom(f, depth)
        r = self.r.random()
        if r < 0.65:
            return rt, pt
        q = self.r.choice(["*", "+", "?", "{2}", "{1,3}", "{0,2}", "{2,}", "{3}"])
        lazy = "?" if self.r.random() < 0.2 else ""
        return "(?:" + rt + ")" + self.ws(f) + q + lazy, "(?:" + pt + ")" + q + lazy

    def cat(self, f, depth):
        rt, pt = self.ws(f), ""
        for _ in range(self.r.randint(0, 4)):
            if self.r.random() < 0.07:  # a flag directive: the rest of the group
                name = self.r.choice("imsx")
                val = self.r.random() < 0.6
                setattr(f, name, val)
                rt += "(?" + ("" if val else "-") + name + ")" + self.ws(f)
                continue
            a, b = self.rep(f, depth)
            rt += a + self.ws(f)
            pt += b
        return rt, pt

    def alt(self, f, depth):
        rs, ps = [], []
        for _ in range(1 if self.r.random() < 0.7 else self.r.randint(2, 3)):
            a, b = self.cat(f, depth)  # a directive in one branch carries into the next (same group)
            rs.append(a)
            ps.append(b)
        return "|".join(rs), "|".join(ps)

    def pattern(self):
        f = Flags()
        pre = ""
        if self.r.random() < 0.25:
            for name in "imsx":
                if self.r.random() < 0.35:
                    setattr(f, name, True)
                    pre += name
            pre = "(?" + pre + ")" if pre else ""
        rt, pt = self.alt(f, 0)
        return pre + rt, pt

    def subject(self, rust):
        n = self.r.randint(0, 10)
        pool = ALPHA + [c for c in rust if c in UNIVERSE][:12]
        return "".join(self.r.choice(pool) for _ in range(n))
