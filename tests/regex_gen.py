"""Random label-constraint regexes in the dialect of DESIGN.md §2, each rendered twice from one
tree: as Rust `regex` source (what a policies.yml holds, fed to the product and to the oracle's
kwregex.c) and as an equivalent Python `re` pattern whose every construct is explicit (case folding
as classes, classes as code point ranges, ^ $ \\b and friends as ASCII look-arounds), so that
Python's own engine is a third, independent statement of the semantics:

  Rust construct                 Python rendering
  x under (?i)                   [xX]                       (ASCII folding only)
  .  /  (?s).                    [^\\n]  /  [\\s\\S]
  [...] with &&, --, ~~, nesting  [\\uXXXX-\\uYYYY...] (the set computed here), (?!) when empty
  \\d \\w \\s \\D \\W \\S           the ASCII sets / their complements over code points
  ^ $ \\A \\z  (?m)^ (?m)$        \\A \\Z \\A \\Z (?<![^\\n]) (?![^\\n])
  \\b \\< \\> \\b{start-half} \\b{end-half}   with re.ASCII: \\b \\b(?=\\w) \\b(?<=\\w) (?<!\\w) (?!\\w)
  \\B                            (?<=\\w)(?=\\w)|(?<!\\w)(?!\\w)  (Python's \\B never matches an empty string)
  (?flags) mid-group             applied by the generator to the rest of the group (no Python flag)
  (?x) white space, # comments   dropped
"""
import random

META = set("\\.+*?()|[]{}^$#")
CLASS_META = set("\\[]^-&~")
ALPHA = ["a", "b", "c", "k", "z", "A", "B", "K", "Z", "0", "1", "9", "_", "-", ".", " ", "\n", "#", "&", "~",
         "é", "É", "ÿ", "Ω", "中", "\U0001D11E"]
WORD = [(48, 57), (65, 90), (95, 95), (97, 122)]
NAMED = {"alnum": [(48, 57), (65, 90), (97, 122)], "alpha": [(65, 90), (97, 122)], "digit": [(48, 57)],
         "lower": [(97, 122)], "upper": [(65, 90)], "space": [(9, 13), (32, 32)], "word": WORD,
         "xdigit": [(48, 57), (65, 70), (97, 102)], "punct": [(33, 47), (58, 64), (91, 96), (123, 126)],
         "blank": [(9, 9), (32, 32)], "ascii": [(0, 127)]}
VALID = [(0, 0xD7FF), (0xE000, 0x10FFFF)]


def norm(rs):
    out = []
    for lo, hi in sorted(rs):
        if out and lo <= out[-1][1] + 1:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def inter(a, b):
    return norm([(max(x, u), min(y, v)) for x, y in a for u, v in b if max(x, u) <= min(y, v)])


def neg(a):
    out, at = [], 0
    for lo, hi in norm(a):
        if lo > at:
            out.append((at, lo - 1))
        at = hi + 1
    if at <= 0x10FFFF:
        out.append((at, 0x10FFFF))
    return inter(out, VALID)


def union(a, b):
    return norm(list(a) + list(b))


def fold(a):
    add = []
    for lo, hi in a:
        for c in range(max(lo, 65), min(hi, 90) + 1):
            add.append((c + 32, c + 32))
        for c in range(max(lo, 97), min(hi, 122) + 1):
            add.append((c - 32, c - 32))
    return union(a, add)


def py_class(rs):
    rs = norm(rs)
    if not rs:
        return "(?!)"

    def e(c):
        return f"\\U{c:08x}"
    return "[" + "".join(e(lo) if lo == hi else f"{e(lo)}-{e(hi)}" for lo, hi in rs) + "]"


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
            s = [(ord(ch), ord(ch))]
            return self.cls_char_rust(ch, f), fold(s) if f.i else s
        if r < 0.55:
            a, b = sorted(self.r.sample(ALPHA, 2), key=ord)
            s = [(ord(a), ord(b))]
            return f"{self.cls_char_rust(a, f)}-{self.cls_char_rust(b, f)}", fold(s) if f.i else s
        if r < 0.7:
            e = self.r.choice("dDwWsS")
            base = {"d": [(48, 57)], "w": WORD, "s": [(9, 13), (32, 32)]}[e.lower()]
            return "\\" + e, neg(base) if e.isupper() else base
        if r < 0.82:
            nm = self.r.choice(sorted(NAMED))
            s = fold(NAMED[nm]) if f.i else NAMED[nm]
            if self.r.random() < 0.25:
                return f"[:^{nm}:]", neg(s)
            return f"[:{nm}:]", s
        if depth < 2:
            return self.cls(f, depth + 1)
        ch = self.r.choice(ALPHA)
        return self.cls_char_rust(ch, f), [(ord(ch), ord(ch))]

    def cls(self, f, depth=0):
        """(rust text '[...]', set)"""
        negate = self.r.random() < 0.25
        parts = []

        def union_part():
            txt, s = "", []
            for _ in range(self.r.randint(1, 3)):
                t, x = self.cls_item(f, depth)
                if txt and txt[-1] == "-" and t.startswith("-"):
                    t = "\\" + t
                txt += t + self.ws(f).replace("#", "").replace(" note\n", "")
                s = union(s, x)
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
                s = inter(s, s2)
            elif op == "--":
                s = inter(s, neg(s2))
            else:
                s = union(inter(s, neg(s2)), inter(s2, neg(s)))
        body = "".join(parts)
        if negate:
            return "[^" + body + "]", neg(s)
        return "[" + body + "]", s

    def atom(self, f, depth):
        r = self.r.random()
        if r < 0.38:
            ch = self.r.choice(ALPHA)
            s = [(ord(ch), ord(ch))]
            return self.lit_rust(ch, f), py_class(fold(s) if f.i else s)
        if r < 0.46:
            return ".", "[\\s\\S]" if f.s else "[^\\n]"
        if r < 0.6:
            t, s = self.cls(f)
            return t, py_class(inter(s, VALID))
        if r < 0.68:
            e = self.r.choice("dDwWsS")
            base = {"d": [(48, 57)], "w": WORD, "s": [(9, 13), (32, 32)]}[e.lower()]
            return "\\" + e, py_class(neg(base) if e.isupper() else base)
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
        pool = ALPHA + [c for c in rust if c.isalnum()][:12]
        return "".join(self.r.choice(pool) for _ in range(n))
