"""rhaisub.py — the policy-group expression language, restated for the oracle. TEST INFRASTRUCTURE ONLY.

Imported by oracle.py (and through it by tests/, smoke() and bench.py's cpu_baseline leg); never by
the product. The language is the rhai 1.21.0 subset a PolicyGroupEvaluator script may use
(upstream policy-evaluator v0.24.0 / rhai 1.21.0, Cargo.lock:5116-5118, absent from the reference
tree; run by src/evaluation/evaluation_environment.rs:587-651, pinned only by
evaluation_environment.rs:979-1112 and DESIGN.md §2). Written independently of the product's
expr.cpp: a tokenizer over regular expressions, a Pratt parser into tagged tuples, and a tree
walker whose control flow (break / continue / return) travels as Python exceptions.

Values: None is (), bool, int (i64), str, list (array). Supported: let / const, assignment and
`op=`, blocks, if / else, switch (literal, alternative, range and guarded cases, `_`), while, loop,
do-while / do-until, for over arrays and ranges (with a counter), break [value], continue, return,
fn definitions (top level, overloaded by arity, no access to the caller's variables), array
literals, indexing, `in` / `!in`, `??`, `a..b` / `a..=b` / range(a, b) as for-iterables and `in`
operands, string `-`, and the functions of rhai's standard packages (Engine::new(), DESIGN.md
§2.1) over these values: len is_empty contains to_string type_of starts_with ends_with push, abs
sign is_zero is_odd is_even max min to_hex to_octal to_binary parse_int, to_upper to_lower
make_upper make_lower trim sub_string crop index_of replace split split_rev bytes, append insert
pop shift remove reverse sort clear truncate chop get set extract drain retain splice dedup pad.
The packages' other names (_STD_REFUSED) and the constructs the engine leaves out are refused by
name at load ("unsupported by this engine: ..."); an overload whose result type the engine lacks
(a string's pop / get: characters; a string's pad) is refused by name when it runs. The engine
limits of kwdev.hpp (16384 bytes built, 100000 loop iterations + calls, 64 nested calls, arrays 16
deep in a comparison) are applied exactly as the product applies them.
"""
import re
import sys

sys.setrecursionlimit(max(sys.getrecursionlimit(), 8000))  # 64 nested script calls, deep trees

I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1
U64_MAX = (1 << 64) - 1
MAX_ALLOC, MAX_OPS, MAX_CALLS, MAX_CMP = 16384, 100000, 64, 16
UNSUP = "unsupported by this engine: "


class ExprError(Exception):
    pass


class _Break(Exception):
    def __init__(self, value):
        self.value = value


class _Continue(Exception):
    pass


class _Return(Exception):
    def __init__(self, value):
        self.value = value


# ----------------------------------------------------------------------------- tokens
_KEYWORDS = {"let", "const", "if", "else", "true", "false", "switch", "while", "loop", "do", "until", "for", "in",
             "break", "continue", "return", "fn"}
_REFUSED = {"import": "modules (import)", "export": "modules (export)", "as": "modules (as)",
            "private": "private functions", "try": "try / catch", "catch": "try / catch", "throw": "throw",
            "this": "this", "global": "the global namespace", "Fn": "function pointers", "call": "function pointers",
            "curry": "function pointers", "eval": "eval", "print": "print", "debug": "debug",
            "is_def_var": "is_def_var", "is_def_fn": "is_def_fn", "is_shared": "shared values", "static": "static",
            "exit": "exit"}
_BAD_OPS = [("#{", "object maps"),
            ("::", "modules and namespaces"), ("?.", "the ?. operator"), ("?[", "the ?[ operator")]
_OPS = ["..=", "**=", "<<=", ">>=", "=>", "??", "..", "**", "<<", ">>", "||", "&&", "==", "!=", "<=", ">=", "+=", "-=", "*=", "/=", "%=", "|=", "&=", "^="] + \
    list("<>+-*/%!|&^(){}[];=,.")
_IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")
_NUMBODY = re.compile(r"[A-Za-z0-9_]*")
_ESC = {"n": "\n", "t": "\t", "r": "\r", "0": "\0", "\\": "\\", '"': '"', "'": "'"}


def tokenize(s):
    out, i, n = [], 0, len(s)
    while i < n:
        c = s[i]
        if c in " \t\n\r\f\v":  # (ASCII white space only, as the C locale's isspace)
            i += 1
            continue
        if s.startswith("//", i):
            j = s.find("\n", i)
            i = n if j < 0 else j
            continue
        if s.startswith("/*", i):
            depth = 0
            while True:
                if s.startswith("/*", i):
                    depth, i = depth + 1, i + 2
                elif s.startswith("*/", i):
                    depth, i = depth - 1, i + 2
                else:
                    i += 1
                if depth == 0 or i >= n:
                    break
            if depth > 0:
                raise ExprError("Syntax error: unterminated block comment")
            continue
        if c.isascii() and (c.isalpha() or c == "_"):
            m = _IDENT.match(s, i)
            out.append(("id", m.group()))
            i = m.end()
            continue
        if c.isascii() and c.isdigit():
            start = i
            base = 10
            if c == "0" and s[i + 1:i + 2] in ("x", "o", "b"):
                base = {"x": 16, "o": 8, "b": 2}[s[i + 1]]
                i += 2
            m = _NUMBODY.match(s, i)
            i = m.end()
            digits = m.group().replace("_", "")
            if base == 10 and i + 1 < n and s[i] == "." and s[i + 1].isascii() and s[i + 1].isdigit():
                raise ExprError(UNSUP + "floating-point numbers")
            if base == 10 and ("e" in digits or "E" in digits):
                raise ExprError(UNSUP + "floating-point numbers")
            try:
                if not digits:
                    raise ValueError
                v = int(digits, base)
            except ValueError:
                raise ExprError("Syntax error: invalid number: " + s[start:i]) from None
            if (base == 10 and v > I64_MAX) or v > U64_MAX:
                raise ExprError("Syntax error: integer literal too large")
            out.append(("int", v - (1 << 64) if v > I64_MAX else v))
            continue
        if c == '"':
            i += 1
            buf = []
            while True:
                if i >= n:
                    raise ExprError("Syntax error: unterminated string literal")
                ch = s[i]
                i += 1
                if ch == '"':
                    break
                if ch != "\\":
                    buf.append(ch)
                    continue
                if i >= n:
                    raise ExprError("Syntax error: unterminated string literal")
                e = s[i]
                i += 1
                if e in _ESC:
                    buf.append(_ESC[e])
                elif e == "\n":
                    while i < n and s[i] in " \t":
                        i += 1
                elif e in "xuU":
                    w = {"x": 2, "u": 4, "U": 8}[e]
                    h = s[i:i + w]
                    if len(h) != w or any(x not in "0123456789abcdefABCDEF" for x in h):
                        raise ExprError("Syntax error: invalid escape sequence \\" + e)
                    cp = int(h, 16)
                    if cp > 0x10FFFF or 0xD800 <= cp <= 0xDFFF:
                        raise ExprError("Syntax error: invalid escape sequence \\" + e)
                    buf.append(chr(cp))
                    i += w
                else:
                    raise ExprError("Syntax error: invalid escape sequence \\" + e)
            out.append(("str", "".join(buf)))
            continue
        if c == "'":
            raise ExprError(UNSUP + "character literals")
        if c == "`":
            raise ExprError(UNSUP + "back-tick strings and string interpolation")
        if s.startswith("!in", i) and not (i + 3 < n and (s[i + 3].isascii() and (s[i + 3].isalnum() or s[i + 3] == "_"))):
            out.append(("op", "!in"))
            i += 3
            continue
        for b, what in _BAD_OPS:
            if s.startswith(b, i):
                raise ExprError(UNSUP + what)
        for o in _OPS:
            if s.startswith(o, i):
                out.append(("op", o))
                i += len(o)
                break
        else:
            raise ExprError(f"Syntax error: unexpected character '{c}'")
    out.append(("end", None))
    return out


# ----------------------------------------------------------------------------- parser
# binding powers (rhai 1.x): || | ^ 30, && & 60, == != 90, in !in 110, < <= > >= 130, ?? 135,
# .. ..= 140, + - 150, * / % 180, ** 190 (right-associative), << >> 210
_BP = {"||": 30, "|": 30, "^": 30, "&&": 60, "&": 60, "==": 90, "!=": 90, "!in": 110, "<": 130, "<=": 130, ">": 130,
       ">=": 130, "??": 135, "..": 140, "..=": 140, "+": 150, "-": 150, "*": 180, "/": 180, "%": 180, "**": 190,
       "<<": 210, ">>": 210}
_ASSIGN = ["=", "+=", "-=", "*=", "/=", "%=", "|=", "&=", "^=", "**=", "<<=", ">>="]
_BLOCKLIKE = {"if", "switch", "while", "loop", "for", "block"}


class Program:
    def __init__(self, root, fns):
        self.root = root    # ("block", statements, tail)
        self.fns = fns      # {(name, arity): (params, body)}


class _Parser:
    def __init__(self, toks):
        self.t, self.p = toks, 0
        self.loops = 0
        self.in_fn = False
        self.scopes = [[]]
        self.fns = {}

    def peek(self, d=0):
        return self.t[min(self.p + d, len(self.t) - 1)]

    def at_op(self, o, d=0):
        return self.peek(d) == ("op", o)

    def at_id(self, w):
        return self.peek() == ("id", w)

    def near(self):
        k, v = self.peek()
        if k == "end":
            return "end of script"
        if k == "int":
            return str(v)
        if k == "str":
            return f'"{v}"'
        return f"'{v}'"

    def err(self, m):
        raise ExprError(m)

    def expect(self, o, what):
        if not self.at_op(o):
            self.err(f"Syntax error: expecting '{o}' {what}, found {self.near()}")
        self.p += 1

    def is_const(self, name):
        for scope in reversed(self.scopes):
            for n, c in reversed(scope):
                if n == name:
                    return c
        return False

    def block(self, top):
        stmts, tail = [], False
        self.scopes.append([])
        while True:
            if (self.peek()[0] == "end") if top else self.at_op("}"):
                break
            if self.peek()[0] == "end":
                self.err("Syntax error: expecting '}' to close the block")
            if self.at_op(";"):
                self.p += 1
                continue
            if self.at_id("fn"):
                if not top or self.in_fn:
                    self.err("Syntax error: functions can only be defined at global level")
                self.fn_def()
                continue
            st = self.statement()
            decl = st[0] in ("let", "assign", "setidx")
            stmts.append(st)
            if self.at_op(";"):
                self.p += 1
                tail = False
                continue
            if (self.peek()[0] == "end") if top else self.at_op("}"):
                tail = not decl
                break
            if st[0] not in _BLOCKLIKE:
                self.err(f"Syntax error: expecting ';' to terminate this statement, found {self.near()}")
            tail = False
        self.scopes.pop()
        return ("block", stmts, tail)

    def fn_def(self):
        self.p += 1
        k, name = self.peek()
        if k != "id" or name in _KEYWORDS:
            self.err("Syntax error: expecting a function name after 'fn'")
        self.p += 1
        self.expect("(", "after the function name")
        params = []
        while not self.at_op(")"):
            k, v = self.peek()
            if k != "id" or v in _KEYWORDS:
                self.err(f"Syntax error: expecting a parameter name, found {self.near()}")
            if v in params:
                self.err(f"Syntax error: duplicated parameter '{v}' in function '{name}'")
            params.append(v)
            self.p += 1
            if self.at_op(","):
                self.p += 1
            elif not self.at_op(")"):
                self.err(f"Syntax error: expecting ',' or ')' in the parameter list, found {self.near()}")
        self.p += 1
        if (name, len(params)) in self.fns:
            self.err(f"Syntax error: function '{name}' with {len(params)} parameters is defined more than once")
        self.expect("{", "to start the function body")
        saved = (self.loops, self.scopes)
        self.loops, self.scopes, self.in_fn = 0, [[(q, False) for q in params]], True
        body = self.block(False)
        self.loops, self.scopes = saved
        self.in_fn = False
        self.p += 1
        self.fns[(name, len(params))] = (params, body)

    def statement(self):
        if self.at_id("let") or self.at_id("const"):
            const = self.at_id("const")
            self.p += 1
            k, name = self.peek()
            if k != "id" or name in _KEYWORDS:
                self.err("Syntax error: expecting a variable name after 'let'")
            self.p += 1
            init = None
            if self.at_op("="):
                self.p += 1
                init = self.expr(0)
            elif const:
                self.err("Syntax error: expecting '=' after the constant name")
            self.scopes[-1].append((name, const))
            return ("let", name, init)
        for w in ("break", "continue", "return"):
            if self.at_id(w):
                self.p += 1
                if w != "return" and self.loops == 0:
                    self.err(f"Syntax error: {w} should only be used inside a loop")
                val = None
                if w != "continue" and not (self.at_op(";") or self.at_op("}") or self.peek()[0] == "end"
                                            or self.at_op(",")):
                    val = self.expr(0)
                return (w, val)
        if any(self.at_id(w) for w in ("if", "switch", "while", "loop", "do", "for")) or self.at_op("{"):
            return self.primary()  # a statement of its own: nothing continues it (rhai's parse_stmt)
        e = self.expr(0)
        for a in _ASSIGN:
            if self.at_op(a):
                self.p += 1
                rhs = self.expr(0)
                op = "" if a == "=" else a[:-1]
                if e[0] == "var":
                    node, name = ("assign", e[1], op, rhs), e[1]
                elif e[0] == "index" and e[1][0] == "var":
                    node, name = ("setidx", e[1][1], op, e[2], rhs), e[1][1]
                elif e[0] == "index":
                    self.err(UNSUP + "assigning to a nested index or to an element of a temporary value")
                else:
                    self.err("Syntax error: cannot assign to this expression")
                if self.is_const(name):
                    self.err(f"Syntax error: cannot assign to the constant '{name}'")
                return node
        return e

    def binding(self):
        k, v = self.peek()
        if k == "id":
            return 110 if v == "in" else None
        if k != "op":
            return None
        return _BP.get(v)

    def expr(self, min_bp):
        left = self.unary()
        while True:
            bp = self.binding()
            if bp is None or bp < min_bp:
                return left
            op = self.peek()[1]
            self.p += 1
            right = self.expr(bp if op == "**" else bp + 1)
            if op in ("in", "!in"):
                left = ("in", op == "!in", left, right)
            elif op == "??":
                left = ("coalesce", left, right)
            elif op in ("..", "..="):
                left = ("range", op == "..=", op, left, right)
            else:
                left = ("bin", op, left, right)

    def unary(self):
        k, v = self.peek()
        if k == "op" and v in ("!", "-", "+"):
            self.p += 1
            return ("un", v, self.unary())
        return self.postfix()

    def arglist(self):
        args = []
        while not self.at_op(")"):
            args.append(self.expr(0))
            if self.at_op(","):
                self.p += 1
            elif not self.at_op(")"):
                self.err(f"Syntax error: expecting ',' or ')' in the argument list, found {self.near()}")
        self.p += 1
        return args

    def postfix(self):
        e = self.primary()
        while True:
            if self.at_op("."):
                self.p += 1
                k, m = self.peek()
                if k != "id":
                    self.err(f"Syntax error: expecting a method name after '.', found {self.near()}")
                self.p += 1
                if not self.at_op("("):  # property getters of the packages: len, is_empty, bytes
                    if m not in ("len", "is_empty", "bytes"):
                        self.err(UNSUP + f"property access (.{m})")
                    e = ("call", m, [e], True)
                    continue
                self.p += 1
                args = [e] + self.arglist()
                if m in _ALWAYS_MUT and e[0] == "index":
                    self.err(UNSUP + f"mutating an element in place (x[i].{m}(..))")
                if m in _ALWAYS_MUT and e[0] == "var" and self.is_const(e[1]):
                    self.err(f"Syntax error: cannot assign to the constant '{e[1]}'")
                e = ("call", m, args, True)
            elif self.at_op("["):
                self.p += 1
                ix = self.expr(0)
                self.expect("]", "to close the index")
                e = ("index", e, ix)
            else:
                return e

    def braced(self, what):
        if not self.at_op("{"):
            self.err(f"Syntax error: expecting '{{' {what}, found {self.near()}")
        self.p += 1
        b = self.block(False)
        self.p += 1
        return b

    def loop_body(self):
        if not self.at_op("{"):
            self.err(f"Syntax error: expecting '{{' to start the loop body, found {self.near()}")
        self.p += 1
        self.loops += 1
        b = self.block(False)
        self.loops -= 1
        self.p += 1
        return b

    def case_value(self):
        """-> (True, value) or (False, None); a '-' is consumed either way, as the product does."""
        neg = False
        if self.at_op("-"):
            neg = True
            self.p += 1
        k, v = self.peek()
        if k == "int":
            self.p += 1
            return True, (-v if neg else v)
        if neg:
            return False, None
        if k == "str":
            self.p += 1
            return True, v
        if k == "id" and v in ("true", "false"):
            self.p += 1
            return True, v == "true"
        if self.at_op("(") and self.at_op(")", 1):
            self.p += 2
            return True, None
        return False, None

    def switch(self):
        scrut = self.expr(0)
        self.expect("{", "after the switch value")
        cases, seen_wild, plain = [], False, []
        while not self.at_op("}"):
            if seen_wild:
                self.err("Syntax error: the wildcard case '_' must be the last case")
            case = {"vals": [], "range": None, "wild": False, "guard": None}
            if self.at_id("_"):
                self.p += 1
                case["wild"] = seen_wild = True
            else:
                while True:
                    ok, v = self.case_value()
                    if not ok:
                        self.err(f"Syntax error: a switch case must be a constant value, found {self.near()}")
                    if self.at_op("..") or self.at_op("..="):
                        incl = self.at_op("..=")
                        self.p += 1
                        if not _is_int(v):
                            self.err("Syntax error: a switch range case needs integer bounds")
                        ok, h = self.case_value()
                        if not ok or not _is_int(h):
                            self.err("Syntax error: a switch range case needs integer bounds")
                        case["range"] = (v, h, incl)
                        break
                    case["vals"].append(v)
                    if not self.at_op("|"):
                        break
                    self.p += 1
            if self.at_id("if"):
                if case["wild"]:
                    self.err("Syntax error: the wildcard case '_' cannot have a condition")
                self.p += 1
                case["guard"] = self.expr(0)
            self.expect("=>", "after the switch case")
            if case["range"] is None and not case["wild"] and case["guard"] is None:
                for v in case["vals"]:
                    if any(_same(u, v) for u in plain):
                        self.err("Syntax error: duplicated switch case")
                    plain.append(v)
            braced = self.at_op("{")
            if braced:
                case["body"] = self.braced("")
            else:
                case["body"] = self.statement()
                if case["body"][0] in ("let", "assign", "setidx"):
                    self.err("Syntax error: a switch case body must be an expression or a block")
            cases.append(case)
            if self.at_op(","):
                self.p += 1
            elif not self.at_op("}") and not braced:
                self.err(f"Syntax error: expecting ',' between switch cases, found {self.near()}")
        self.p += 1
        return ("switch", scrut, cases)

    def primary(self):
        k, v = self.peek()
        if k in ("int", "str"):
            self.p += 1
            return ("lit", v)
        if self.at_op("("):
            self.p += 1
            if self.at_op(")"):
                self.p += 1
                return ("lit", None)
            e = self.expr(0)
            if not self.at_op(")"):
                self.err(f"Syntax error: expecting ')', found {self.near()}")
            self.p += 1
            return e
        if self.at_op("["):
            self.p += 1
            items = []
            while not self.at_op("]"):
                items.append(self.expr(0))
                if self.at_op(","):
                    self.p += 1
                elif not self.at_op("]"):
                    self.err(f"Syntax error: expecting ',' or ']' in the array literal, found {self.near()}")
            self.p += 1
            return ("array", items)
        if self.at_op("{"):
            self.p += 1
            b = self.block(False)
            self.p += 1
            return b
        if self.at_op("|") or self.at_op("||"):
            self.err(UNSUP + "closures")
        if k == "id":
            if v in _REFUSED:
                self.err(UNSUP + _REFUSED[v])
            self.p += 1
            if v in ("true", "false"):
                return ("lit", v == "true")
            if v == "if":
                c = self.expr(0)
                then = self.braced("after the if condition")
                other = None
                if self.at_id("else"):
                    self.p += 1
                    other = self.primary() if self.at_id("if") else self.braced("or 'if' after 'else'")
                return ("if", c, then, other)
            if v == "switch":
                return self.switch()
            if v == "while":
                c = self.expr(0)
                return ("while", c, self.loop_body())
            if v == "loop":
                return ("loop", self.loop_body())
            if v == "do":
                body = self.loop_body()
                if not (self.at_id("while") or self.at_id("until")):
                    self.err("Syntax error: expecting 'while' or 'until' after the do block")
                until = self.at_id("until")
                self.p += 1
                return ("do", body, until, self.expr(0))
            if v == "for":
                paren = self.at_op("(")
                if paren:
                    self.p += 1
                k2, var = self.peek()
                if k2 != "id" or var in _KEYWORDS:
                    self.err("Syntax error: expecting a loop variable after 'for'")
                self.p += 1
                counter = None
                if paren:
                    self.expect(",", "after the loop variable")
                    k3, counter = self.peek()
                    if k3 != "id" or counter in _KEYWORDS:
                        self.err("Syntax error: expecting the counter variable")
                    self.p += 1
                    self.expect(")", "after the counter variable")
                if not self.at_id("in"):
                    self.err(f"Syntax error: expecting 'in' after the loop variable, found {self.near()}")
                self.p += 1
                it = self.expr(0)
                if it[0] == "call" and not it[3] and it[1] == "range":
                    if len(it[2]) != 2:
                        self.err(UNSUP + "range() with a step")
                    it = ("range", False, "range", it[2][0], it[2][1])
                self.scopes.append([(var, False)] + ([(counter, False)] if counter else []))
                body = self.loop_body()
                self.scopes.pop()
                return ("for", var, counter, it, body)
            if v in ("let", "const", "else", "fn", "in", "until", "break", "continue", "return"):
                self.err(f"Syntax error: unexpected '{v}'")
            if not self.at_op("("):
                return ("var", v)
            self.p += 1
            return ("call", v, self.arglist(), False)
        if k == "end":
            self.err("Syntax error: expecting an expression, found end of script")
        self.err(f"Syntax error: unexpected {self.near()}")


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, bool)


def _same(a, b):
    return type(a) is type(b) and a == b


def _children(n):
    """Sub-nodes of a tagged tuple, with their positions' range permission (for / in)."""
    tag = n[0]
    if tag == "in":
        return [(n[2], False), (n[3], True)]
    if tag == "for":
        return [(n[3], True), (n[4], False)]
    if tag == "block":
        return [(x, False) for x in n[1]]
    if tag == "array":
        return [(x, False) for x in n[1]]
    if tag == "call":
        return [(x, False) for x in n[2]]
    if tag == "switch":
        out = [(n[1], False)]
        for c in n[2]:
            if c["guard"] is not None:
                out.append((c["guard"], False))
            out.append((c["body"], False))
        return out
    return [(x, False) for x in n[1:] if isinstance(x, tuple)]


def _walk_ranges(n, allowed):
    if n[0] == "range" and not allowed:
        raise ExprError(UNSUP + "range values outside `for` and `in`")
    for c, ok in _children(n):
        _walk_ranges(c, ok)


def _stray_range(n, fns, members):
    if n[0] == "call" and n[1] == "range" and not _resolves(n, fns, members):
        return True
    return any(_stray_range(c, fns, members) for c, _ in _children(n))


# rhai 1.21's standard packages (Engine::new()) over the engine's values: (name, arity) of every
# function implemented here, those rhai gives a `&mut` first parameter (a method call on a variable
# changes it), and the rest of the packages' names, refused by name at load
_BUILTINS = {("len", 1), ("is_empty", 1), ("contains", 2), ("to_string", 1), ("type_of", 1), ("starts_with", 2),
             ("ends_with", 2), ("push", 2),
             ("abs", 1), ("sign", 1), ("is_zero", 1), ("is_odd", 1), ("is_even", 1), ("max", 2), ("min", 2),
             ("to_hex", 1), ("to_octal", 1), ("to_binary", 1), ("parse_int", 1), ("parse_int", 2),
             ("to_upper", 1), ("to_lower", 1), ("make_upper", 1), ("make_lower", 1), ("trim", 1), ("sub_string", 2),
             ("sub_string", 3), ("crop", 2), ("crop", 3), ("index_of", 2), ("index_of", 3), ("replace", 3),
             ("split", 1), ("split", 2), ("split", 3), ("split_rev", 2), ("split_rev", 3), ("bytes", 1),
             ("append", 2), ("insert", 3), ("pop", 1), ("shift", 1), ("remove", 2), ("reverse", 1), ("sort", 1),
             ("clear", 1), ("truncate", 2), ("chop", 2), ("get", 2), ("set", 3), ("extract", 2), ("extract", 3),
             ("drain", 3), ("retain", 3), ("splice", 4), ("dedup", 1), ("pad", 3)}
_MUT = {("push", 2), ("make_upper", 1), ("make_lower", 1), ("trim", 1), ("crop", 2), ("crop", 3), ("replace", 3),
        ("split", 2), ("append", 2), ("insert", 3), ("pop", 1), ("shift", 1), ("remove", 2), ("reverse", 1),
        ("sort", 1), ("clear", 1), ("truncate", 2), ("chop", 2), ("set", 3), ("drain", 3), ("retain", 3),
        ("splice", 4), ("dedup", 1), ("pad", 3)}
_ALWAYS_MUT = {n for n, _ in _MUT} - {"split"}  # (split changes arrays only)
_STD_REFUSED = {
    "tag", "set_tag", "take", "sleep", "name", "is_anonymous", "to_debug",
    "print", "debug", "eval", "Fn", "call", "curry", "is_def_var", "is_def_fn", "is_shared",
    "get_bit", "set_bit", "get_bits", "set_bits", "bits",
    "to_int", "to_float", "parse_float", "sqrt", "exp", "ln", "log", "floor", "ceiling", "round", "int", "fraction",
    "is_nan", "is_finite", "is_infinite", "sin", "cos", "tan", "sinh", "cosh", "tanh", "asin", "acos", "atan",
    "asinh", "acosh", "atanh", "hypot", "to_degrees", "to_radians", "PI", "E",
    "chars", "to_chars",
    "map", "filter", "reduce", "reduce_rev", "some", "all", "find", "find_map", "for_each", "zip", "sort_desc",
    "blob", "to_blob", "as_string", "write_ascii", "write_utf8", "write_le", "write_be", "parse_le_int",
    "parse_be_int", "parse_le_float", "parse_be_float",
    "keys", "values", "mixin", "fill_with", "to_json",
    "timestamp", "elapsed"}
# White_Space (PropList.txt): Rust's char::is_whitespace, for trim / split() / parse_int
_WS = "".join(map(chr, [9, 10, 11, 12, 13, 0x20, 0x85, 0xA0, 0x1680] + list(range(0x2000, 0x200B)) +
                  [0x2028, 0x2029, 0x202F, 0x205F, 0x3000]))


def _resolves(n, fns, members):
    _, name, args, method = n
    if not method and (name, len(args)) in fns:
        return True
    if not method and not args and name in members:
        return True
    return (name, len(args)) in _BUILTINS


def parse(s, members):
    """Script -> Program; raises ExprError (syntax, or a construct outside the engine)."""
    ps = _Parser(tokenize(s))
    root = ps.block(True)
    _walk_ranges(root, False)
    for _, body in ps.fns.values():
        _walk_ranges(body, False)
    if _stray_range(root, ps.fns, members) or any(_stray_range(b, ps.fns, members) for _, b in ps.fns.values()):
        raise ExprError(UNSUP + "range values outside `for` and `in`")
    for body in [root] + [b for _, b in ps.fns.values()]:
        name = _refused(body, ps.fns, members)
        if name:
            raise ExprError(UNSUP + name)
    return Program(root, ps.fns)


def _refused(n, fns, members):
    """The first call of a standard-package function outside the engine (_STD_REFUSED), or None."""
    if n[0] == "call" and n[1] in _STD_REFUSED and not _resolves(n, fns, members):
        return n[1]
    for c, _ in _children(n):
        r = _refused(c, fns, members)
        if r:
            return r
    return None


# ----------------------------------------------------------------------------- evaluation
def type_name(v):
    if v is None:
        return "()"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "i64"
    if isinstance(v, str):
        return "string"
    return "array"


def _kind(v):
    return type_name(v)


def _int_pow_shift(op, x, y):
    """rhai's checked ** << >> on i64 (ArithmeticPackage power / shift_left / shift_right): a negative
    shift shifts the other way; 64 or more bits is an error, as is an exponent outside [0, u32::MAX]
    or a power that overflows i64; >> is arithmetic."""
    if op == "**":
        if y > 0xFFFFFFFF:
            raise ExprError(f"Integer raised to too large an index: {x} ** {y}")
        if y < 0:
            raise ExprError(f"Integer raised to a negative index: {x} ** {y}")
        r = x ** y if abs(x) < 2 or y < 64 else None  # (|x| >= 2 overflows i64 within 63 steps)
        if r is None or not I64_MIN <= r <= I64_MAX:
            raise ExprError(f"Exponential overflow: {x} ** {y}")
        return r
    left = op == "<<"
    name = "Left-shift" if left else "Right-shift"
    if y > 0xFFFFFFFF:
        raise ExprError(f"{name} by too many bits: {x} {op} {y}")
    if y < 0:
        if y == I64_MIN:
            raise ExprError(f"{name} by too many bits: {x} {op} {y}")
        return _int_pow_shift(">>" if left else "<<", x, -y)
    if y >= 64:
        raise ExprError(f"{name} by too many bits: {x} {op} {y}")
    if left:
        r = (x << y) & U64_MAX
        return r - (1 << 64) if r > I64_MAX else r
    return x >> y


def _offset_len(n, start, ln):
    """rhai's calc_offset_len: (start, len) within n elements; a negative start counts from the end."""
    if start < 0:
        st = max(0, n + start)
    elif start >= n:
        return n, 0
    else:
        st = start
    return st, 0 if ln <= 0 else min(ln, n - st)


def _elem_index(n, i):
    """The element position of get / set / remove, or None out of range."""
    at = n + i if i < 0 else i
    return at if 0 <= at < n else None


def _sub_chars(s, start, ln):
    if not s or ln <= 0:
        return ""
    n = len(s)
    if start < 0:
        off = max(0, n + start)
    elif start >= n:
        return ""
    else:
        off = start
    return s[off:off + ln]


def _split_ws(s):
    out, cur = [], None
    for ch in s:
        if ch in _WS:
            if cur is not None:
                out.append(cur)
            cur = None
        else:
            cur = (cur or "") + ch
    if cur is not None:
        out.append(cur)
    return out


def _rsplit_pieces(s, d, rev, lim):
    """Rust's str::split / rsplit (and splitn / rsplitn with lim > 0). An empty pattern matches at
    every character boundary, both ends included."""
    if d:
        if rev:
            parts = s.rsplit(d, lim - 1) if lim else s.rsplit(d)
            return parts[::-1]
        return s.split(d, lim - 1) if lim else s.split(d)
    cuts = list(range(len(s) + 1))  # match positions (characters)
    out = []
    if not rev:
        prev = 0
        for c in cuts:
            if lim and len(out) + 1 == lim:
                break
            out.append(s[prev:c])
            prev = c
        out.append(s[prev:])
    else:
        prev = len(s)
        for c in reversed(cuts):
            if lim and len(out) + 1 == lim:
                break
            out.append(s[c:prev])
            prev = c
        out.append(s[:prev])
    return out


def _parse_int(text, radix):
    """i64::from_str_radix(text.trim(), radix) with its ParseIntError texts, as rhai words them."""
    t = text.strip(_WS)

    def err(e):
        raise ExprError(f"Error parsing integer number '{text}': {e}")
    if not t:
        err("cannot parse integer from empty string")
    neg = t[0] == "-"
    if t[0] in "+-":
        t = t[1:]
        if not t:
            err("invalid digit found in string")
    v = 0
    for ch in t:
        d = int(ch, 36) if ch.isascii() and ch.isalnum() else 99
        if d >= radix:
            err("invalid digit found in string")
        v = v * radix + d
        if (-v if neg else v) < I64_MIN or (-v if neg else v) > I64_MAX:
            err("number too small to fit in target type" if neg else "number too large to fit in target type")
    return -v if neg else v


def _utf8len(s):
    return len(s.encode("utf-8", "surrogatepass"))


class Run:
    """One evaluation of a program over member results (member_ok: list of bool)."""

    def __init__(self, prog, members, member_ok):
        self.prog, self.members, self.ok = prog, members, member_ok
        self.called = []
        self.ops = self.built = self.calls = 0
        self.steps = 0
        self.frames = [[]]  # per call: list of (name, value), innermost last

    # -- limits
    def charge(self, n):
        if n > MAX_ALLOC - self.built:
            raise ExprError(f"engine limit: more than {MAX_ALLOC} bytes of strings and arrays built")
        self.built += n

    def tick(self):
        self.ops += 1
        if self.ops > MAX_OPS:
            raise ExprError(f"engine limit: more than {MAX_OPS} loop iterations and script-function calls")

    # -- variables
    def get(self, name):
        for k in range(len(self.frames[-1]) - 1, -1, -1):
            if self.frames[-1][k][0] == name:
                return self.frames[-1][k][1]
        raise ExprError(f"Variable not found: {name}")

    def put(self, name, value):
        f = self.frames[-1]
        for k in range(len(f) - 1, -1, -1):
            if f[k][0] == name:
                f[k] = (name, value)
                return
        raise ExprError(f"Variable not found: {name}")

    # -- helpers
    @staticmethod
    def nf(name, *vals):
        raise ExprError(f"Function not found: {name} (" + ", ".join(type_name(v) for v in vals) + ")")

    def equal(self, a, b, depth=0):
        if _kind(a) != _kind(b):
            return False
        if isinstance(a, list):
            if len(a) != len(b):
                return False
            if not a:
                return True
            if depth == MAX_CMP:
                raise ExprError(f"engine limit: arrays nested more than {MAX_CMP} deep in a comparison")
            return all(self.equal(x, y, depth + 1) for x, y in zip(a, b))
        return a == b

    @staticmethod
    def text(v):
        if v is None:
            return ""
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, (int, str)):
            return str(v)
        raise ExprError(UNSUP + "converting an array to a string")

    @staticmethod
    def index_error(i, n):
        pre = f"Array index {i} out of bounds: "
        if n == 0:
            raise ExprError(pre + "array is empty")
        if n == 1:
            raise ExprError(pre + "only 1 element in array")
        raise ExprError(pre + f"only {n} elements in array")

    def position(self, arr, ix):
        if isinstance(arr, str):
            raise ExprError(UNSUP + "indexing a string (characters)")
        if not isinstance(arr, list):
            raise ExprError(f"Indexer unavailable: {type_name(arr)}")
        if not _is_int(ix):
            raise ExprError(f"Array index must be an i64, found {type_name(ix)}")
        at = ix + len(arr) if ix < 0 else ix
        if not 0 <= at < len(arr):
            self.index_error(ix, len(arr))
        return at

    def builtin(self, name, args):
        """A built-in over its arguments: its result; for a `&mut` function (_MUT) the pair
        (receiver as changed, result). Charges as expr.cpp's interpreter states: a new string its
        UTF-8 bytes, a new or copied array 16 B a cell; slices are free."""
        a = args
        mut = (name, len(a)) in _MUT
        kinds = [type_name(v) for v in a]

        def out(recv, res):
            return (recv, res) if mut else res

        def refuse(why):
            raise ExprError(UNSUP + f"{name} (" + ", ".join(kinds) + ")" + why)

        def isa(k, t):
            return len(a) > k and kinds[k] == t

        if name in ("len", "is_empty"):
            if isinstance(a[0], (list, str)):
                n = len(a[0])
            else:
                self.nf(name, *a)
            return n if name == "len" else n == 0
        if name == "type_of":
            return type_name(a[0])
        if name == "to_string":
            if isinstance(a[0], str):
                return a[0]
            t = self.text(a[0])
            self.charge(_utf8len(t))
            return t
        if name == "push":
            if not isinstance(a[0], list):
                self.nf(name, *a)
            self.charge(16 * (len(a[0]) + 1))
            return out(a[0] + [a[1]], None)
        if name in ("contains", "index_of"):
            if len(a) == 3 and not isa(2, "i64"):
                self.nf(name, *a)
            hay, x = a[0], a[1]
            idx = name == "index_of"
            if isinstance(hay, list):
                start = _offset_len(len(hay), a[2], 0)[0] if len(a) == 3 else 0
                for k in range(start, len(hay)):
                    if self.equal(hay[k], x):
                        return k if idx else True
                return -1 if idx else False
            if isinstance(hay, str) and isinstance(x, str):
                if not idx:
                    return x in hay
                if not hay:
                    return -1
                start = 0
                if len(a) == 3:
                    st, n = a[2], len(hay)
                    if st < 0:
                        start = max(0, n + st)
                    elif st >= n and st != 0:
                        return -1
                    else:
                        start = st
                return hay.find(x, start)
            self.nf(name, *a)
        if name in ("starts_with", "ends_with"):
            if not (isinstance(a[0], str) and isinstance(a[1], str)):
                self.nf(name, *a)
            return a[0].startswith(a[1]) if name == "starts_with" else a[0].endswith(a[1])
        # ---- integers
        if name in ("abs", "sign", "is_zero", "is_odd", "is_even", "to_hex", "to_octal", "to_binary"):
            if not isa(0, "i64"):
                self.nf(name, *a)
            x = a[0]
            if name == "abs":
                if x == I64_MIN:
                    raise ExprError(f"Negation overflow: -{x}")
                return abs(x)
            if name == "sign":
                return (x > 0) - (x < 0)
            if name in ("is_zero", "is_odd", "is_even"):
                return {"is_zero": x == 0, "is_odd": x % 2 == 1, "is_even": x % 2 == 0}[name]
            t = format(x & U64_MAX, {"to_hex": "x", "to_octal": "o", "to_binary": "b"}[name])
            self.charge(len(t))
            return t
        if name in ("max", "min"):
            if not (isa(0, "i64") and isa(1, "i64")):
                self.nf(name, *a)
            return max(a[0], a[1]) if name == "max" else min(a[0], a[1])
        if name == "parse_int":
            if not isa(0, "string") or (len(a) == 2 and not isa(1, "i64")):
                self.nf(name, *a)
            radix = a[1] if len(a) == 2 else 10
            if not 2 <= radix <= 36:
                raise ExprError(f"Invalid radix: '{radix}'")
            return _parse_int(a[0], radix)
        # ---- strings
        if name in ("to_upper", "to_lower", "make_upper", "make_lower"):
            if not isa(0, "string"):
                self.nf(name, *a)
            r = a[0].upper() if name.endswith("upper") else a[0].lower()
            self.charge(_utf8len(r))
            return r if name.startswith("to_") else (r, None)
        if name == "trim":
            if not isa(0, "string"):
                self.nf(name, *a)
            return a[0].strip(_WS), None
        if name in ("sub_string", "crop"):
            if not (isa(0, "string") and isa(1, "i64")) or (len(a) == 3 and not isa(2, "i64")):
                self.nf(name, *a)
            r = _sub_chars(a[0], a[1], a[2] if len(a) == 3 else _utf8len(a[0]))
            return r if name == "sub_string" else (r, None)
        if name == "replace":
            if not all(isinstance(v, str) for v in a):
                self.nf(name, *a)
            if not a[0]:
                return a[0], None
            r = a[2].join(_rsplit_pieces(a[0], a[1], False, 0))
            self.charge(_utf8len(r))
            return r, None
        if name in ("split", "split_rev"):
            if name == "split" and len(a) == 2 and isinstance(a[0], list) and isa(1, "i64"):
                st = _offset_len(len(a[0]), a[1], I64_MAX)[0]
                return a[0][:st], a[0][st:]
            if not isa(0, "string"):
                self.nf(name, *a)
            s = a[0]
            if len(a) == 1:
                parts = [p for p in _split_ws(s) if p]
            elif name == "split" and len(a) == 2 and isa(1, "i64"):
                i, n = a[1], len(s)
                at = (0 if -i > n else n + i) if i <= 0 else min(i, n)
                parts = [s[:at], s[at:]]
            else:
                if not isa(1, "string") or (len(a) == 3 and not isa(2, "i64")):
                    self.nf(name, *a)
                lim = (1 if a[2] < 1 else a[2]) if len(a) == 3 else 0
                parts = _rsplit_pieces(s, a[1], name == "split_rev", lim)
            self.charge(16 * len(parts))
            return out(s, parts)
        if name == "bytes":
            if not isa(0, "string"):
                self.nf(name, *a)
            return _utf8len(a[0])
        # ---- arrays, and the string forms of append / remove / clear / truncate
        if name == "append":
            if isinstance(a[0], list) and isinstance(a[1], list):
                self.charge(16 * (len(a[0]) + len(a[1])))
                return a[0] + a[1], None
            if isinstance(a[0], str):
                t = self.text(a[1])
                self.charge(_utf8len(a[0]) + _utf8len(t))
                return a[0] + t, None
            self.nf(name, *a)
        if name == "insert":
            if not (isinstance(a[0], list) and isa(1, "i64")):
                self.nf(name, *a)
            self.charge(16 * (len(a[0]) + 1))
            at = _offset_len(len(a[0]), a[1], 0)[0]
            return a[0][:at] + [a[2]] + a[0][at:], None
        if name in ("pop", "shift"):
            if isinstance(a[0], str):
                refuse(": it returns a character")
            if not isinstance(a[0], list):
                self.nf(name, *a)
            v = a[0]
            if not v:
                return v, None
            return (v[:-1], v[-1]) if name == "pop" else (v[1:], v[0])
        if name == "remove":
            if isinstance(a[0], str) and isinstance(a[1], str):
                if not a[0] or not a[1]:
                    return a[0], None
                r = "".join(_rsplit_pieces(a[0], a[1], False, 0))
                self.charge(_utf8len(r))
                return r, None
            if not (isinstance(a[0], list) and isa(1, "i64")):
                self.nf(name, *a)
            at = _elem_index(len(a[0]), a[1])
            if at is None:
                return a[0], None
            self.charge(16 * (len(a[0]) - 1))
            return a[0][:at] + a[0][at + 1:], a[0][at]
        if name == "reverse":
            if not isinstance(a[0], list):
                self.nf(name, *a)
            self.charge(16 * len(a[0]))
            return a[0][::-1], None
        if name == "sort":
            if not isinstance(a[0], list):
                self.nf(name, *a)
            v = a[0]
            if len(v) <= 1:
                return v, None
            ts = {type_name(e) for e in v}
            if len(ts) > 1:
                raise ExprError("Function not found: sort() cannot be called with elements of different types")
            if ts <= {"array", "()"}:
                return v, None
            self.charge(16 * len(v))
            return sorted(v), None  # (bool: False < True; str: code point order = Rust's byte order)
        if name == "clear":
            if isinstance(a[0], list):
                return [], None
            if isinstance(a[0], str):
                return "", None
            self.nf(name, *a)
        if name in ("truncate", "chop"):
            if not isa(1, "i64"):
                self.nf(name, *a)
            n = a[1]
            if isinstance(a[0], str) and name == "truncate":
                return ("" if n <= 0 else a[0][:n]), None
            if not isinstance(a[0], list):
                self.nf(name, *a)
            v = a[0]
            if n <= 0:
                return [], None
            if n >= len(v):
                return v, None
            return (v[:n] if name == "truncate" else v[len(v) - n:]), None
        if name in ("get", "set"):
            if isinstance(a[0], str) and isa(1, "i64"):
                refuse(": characters")
            if not (isinstance(a[0], list) and isa(1, "i64")):
                self.nf(name, *a)
            at = _elem_index(len(a[0]), a[1])
            if name == "get":
                return None if at is None else a[0][at]
            if at is None:
                return a[0], None
            self.charge(16 * len(a[0]))
            return a[0][:at] + [a[2]] + a[0][at + 1:], None
        if name in ("extract", "drain", "retain"):
            if not (isinstance(a[0], list) and isa(1, "i64")) or (len(a) == 3 and not isa(2, "i64")):
                self.nf(name, *a)
            v = a[0]
            ln = a[2] if len(a) == 3 else I64_MAX
            st, n = (0, 0) if not v or ln <= 0 else _offset_len(len(v), a[1], ln)
            mid, rest = v[st:st + n], v[:st] + v[st + n:]
            if name == "extract":
                return mid if n else []
            if n == 0:
                return v, []
            self.charge(16 * len(rest))
            return (rest, mid) if name == "drain" else (mid, rest)
        if name == "splice":
            if not (isinstance(a[0], list) and isa(1, "i64") and isa(2, "i64") and isinstance(a[3], list)):
                self.nf(name, *a)
            v = a[0]
            st, n = _offset_len(len(v), a[1], a[2]) if v else (0, 0)
            self.charge(16 * (len(v) - n + len(a[3])))
            return v[:st] + a[3] + v[st + n:], None
        if name == "dedup":
            if not isinstance(a[0], list):
                self.nf(name, *a)
            v = a[0]
            if len(v) <= 1:
                return v, None
            r = [v[0]]
            for e in v[1:]:
                if not self.equal(e, r[-1]):
                    r.append(e)
            self.charge(16 * len(r))
            return r, None
        if name == "pad":
            if isinstance(a[0], str) and isa(1, "i64"):
                refuse(": padding strings")
            if not (isinstance(a[0], list) and isa(1, "i64")):
                self.nf(name, *a)
            n = a[1]
            if n <= 0 or n <= len(a[0]):
                return a[0], None
            if n > MAX_ALLOC:
                raise ExprError(f"engine limit: more than {MAX_ALLOC} bytes of strings and arrays built")
            self.charge(16 * n)
            return a[0] + [a[2]] * (n - len(a[0])), None
        raise AssertionError(name)

    def arith(self, op, a, b, assign=False):
        if op in ("==", "!="):
            return self.equal(a, b) == (op == "==")
        if op in ("<", "<=", ">", ">="):
            if _kind(a) != _kind(b):
                return False
            if not (_is_int(a) or isinstance(a, str)):
                self.nf(op, a, b)
            return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]
        if op in ("|", "&", "^"):
            if isinstance(a, bool) and isinstance(b, bool):
                return {"|": a or b, "&": a and b, "^": a != b}[op]
            if _is_int(a) and _is_int(b):
                r = {"|": a | b, "&": a & b, "^": a ^ b}[op]
                return r
            self.nf(op, a, b)
        if op == "+" and isinstance(a, list) and (isinstance(b, list) or assign):
            extra = b if isinstance(b, list) else [b]
            self.charge(16 * (len(a) + len(extra)))
            return a + extra
        if op == "+" and (isinstance(a, str) or isinstance(b, str)):
            joined = self.text(a) + self.text(b)
            self.charge(_utf8len(joined))
            return joined
        if op == "-" and isinstance(a, str) and isinstance(b, str):  # every occurrence of b removed
            if not a or not b:
                return a
            r = a.replace(b, "")
            self.charge(_utf8len(r))
            return r
        if not (_is_int(a) and _is_int(b)):
            self.nf(op, a, b)
        text = f"{a} {op} {b}"
        if op in ("**", "<<", ">>"):
            return _int_pow_shift(op, a, b)
        if op in ("/", "%"):
            if b == 0:
                raise ExprError(f"Division by zero: {text}")
            if a == I64_MIN and b == -1:
                raise ExprError(("Division overflow: " if op == "/" else "Modulo overflow: ") + text)
            q = abs(a) // abs(b)
            q = q if (a >= 0) == (b >= 0) else -q
            return q if op == "/" else a - q * b
        r = a + b if op == "+" else a - b if op == "-" else a * b
        if not I64_MIN <= r <= I64_MAX:
            raise ExprError({"+": "Addition", "-": "Subtraction", "*": "Multiplication"}[op] + " overflow: " + text)
        return r

    def condition(self, node, what):
        v = self.ev(node)
        if not isinstance(v, bool):
            raise ExprError(f"Boolean value expected for the {what} condition, found {type_name(v)}")
        return v

    def bounds(self, r):
        lo, hi = self.ev(r[3]), self.ev(r[4])
        if not (_is_int(lo) and _is_int(hi)):
            self.nf(r[2], lo, hi)
        return lo, hi

    def iterate(self, node, values):
        """Run a for / while body per value; -> the loop's value."""
        _, var, counter, _, body = node
        frame = self.frames[-1]
        mark = len(frame)
        try:
            for k, x in values:
                del frame[mark:]
                frame.append((var, x))
                if counter:
                    frame.append((counter, k))
                self.tick()
                try:
                    self.ev(body)
                except _Continue:
                    pass
        except _Break as b:
            del frame[mark:]
            return b.value
        del frame[mark:]
        return None

    def call(self, node):
        _, name, argn, method = node
        args = [self.ev(a) for a in argn]
        fns = self.prog.fns
        if not method and (name, len(args)) in fns:
            params, body = fns[(name, len(args))]
            if len(self.frames) - 1 >= MAX_CALLS:
                raise ExprError("Stack overflow")
            self.tick()
            self.frames.append(list(zip(params, args)))
            try:
                return self.ev(body)
            except _Return as r:
                return r.value
            finally:
                self.frames.pop()
        if not method and not args and name in self.members:
            s = self.members.index(name)
            if s not in self.called:
                self.called.append(s)
            return bool(self.ok[s])
        if (name, len(args)) in _BUILTINS:
            v = self.builtin(name, args)
            if (name, len(args)) not in _MUT:
                return v
            recv, res = v
            if method and argn[0][0] == "var":  # rhai's `&mut` receiver: the variable changes
                self.put(argn[0][1], recv)
            return res
        self.nf(name, *args)

    def ev(self, n):
        self.steps += 1
        tag = n[0]
        if tag == "lit":
            return n[1]
        if tag == "var":
            return self.get(n[1])
        if tag == "call":
            return self.call(n)
        if tag == "un":
            a = self.ev(n[2])
            if n[1] == "!":
                if not isinstance(a, bool):
                    self.nf("!", a)
                return not a
            if not _is_int(a):
                self.nf(n[1], a)
            if n[1] == "-":
                if a == I64_MIN:
                    raise ExprError(f"Negation overflow: -{a}")
                return -a
            return a
        if tag == "bin":
            op = n[1]
            a = self.ev(n[2])
            if op in ("||", "&&"):
                if not isinstance(a, bool):
                    raise ExprError(f"Function not found: {op} ({type_name(a)}, ...)")
                if a == (op == "||"):
                    return a
                b = self.ev(n[3])
                if not isinstance(b, bool):
                    self.nf(op, a, b)
                return b
            return self.arith(op, a, self.ev(n[3]))
        if tag == "coalesce":
            a = self.ev(n[1])
            return a if a is not None else self.ev(n[2])
        if tag == "in":
            _, neg, needle, hay = n
            x = self.ev(needle)
            if hay[0] == "range":
                lo, hi = self.bounds(hay)
                if not _is_int(x):
                    raise ExprError(f"Function not found: contains ({'range=' if hay[1] else 'range'}, {type_name(x)})")
                r = lo <= x <= hi if hay[1] else lo <= x < hi
            else:
                r = self.builtin("contains", [self.ev(hay), x])
            return (not r) if neg else r
        if tag == "if":
            if self.condition(n[1], "if"):
                return self.ev(n[2])
            return self.ev(n[3]) if n[3] is not None else None
        if tag == "block":
            frame = self.frames[-1]
            mark = len(frame)
            v = None
            try:
                for st in n[1]:
                    v = self.ev(st)
            finally:
                del frame[mark:]
            return v if n[2] else None
        if tag == "let":
            v = self.ev(n[2]) if n[2] is not None else None
            self.frames[-1].append((n[1], v))
            return None
        if tag == "assign":
            _, name, op, rhs = n
            r = self.ev(rhs)
            cur = self.get(name)
            self.put(name, r if op == "" else self.arith(op, cur, r, assign=True))
            return None
        if tag == "setidx":
            _, name, op, ixn, rhs = n
            r = self.ev(rhs)
            ix = self.ev(ixn)
            arr = self.get(name)
            at = self.position(arr, ix)
            nv = r if op == "" else self.arith(op, arr[at], r, assign=True)
            self.charge(16 * len(arr))
            self.put(name, arr[:at] + [nv] + arr[at + 1:])
            return None
        if tag == "index":
            arr = self.ev(n[1])
            ix = self.ev(n[2])
            return arr[self.position(arr, ix)]
        if tag == "array":
            items = [self.ev(x) for x in n[1]]
            self.charge(16 * len(items))
            return items
        if tag == "switch":
            x = self.ev(n[1])
            cases = n[2]
            order = [c for c in cases if c["range"] is None and not c["wild"]] + \
                [c for c in cases if c["range"] is not None] + [c for c in cases if c["wild"]]
            for c in order:
                if c["wild"]:
                    hit = True
                elif c["range"] is not None:
                    lo, hi, incl = c["range"]
                    hit = _is_int(x) and (lo <= x <= hi if incl else lo <= x < hi)
                else:
                    hit = any(_kind(x) == _kind(v) and x == v for v in c["vals"])
                if hit and (c["guard"] is None or self.condition(c["guard"], "switch case")):
                    return self.ev(c["body"])
            return None
        if tag in ("while", "loop", "do"):
            try:
                first = True
                while True:
                    if tag == "while" and not self.condition(n[1], "while"):
                        break
                    if tag == "do" and not first:
                        c = self.condition(n[3], "do-until" if n[2] else "do-while")
                        if c == n[2]:
                            break
                    first = False
                    self.tick()
                    try:
                        self.ev(n[2] if tag == "while" else n[1])
                    except _Continue:
                        pass
            except _Break as b:
                return b.value
            return None
        if tag == "for":
            it = n[3]
            if it[0] == "range":
                lo, hi = self.bounds(it)
                top = hi if it[1] else hi - 1
                return self.iterate(n, ((k, lo + k) for k in range(max(0, top - lo + 1))))
            arr = self.ev(it)
            if isinstance(arr, str):
                raise ExprError(UNSUP + "iterating over a string (characters)")
            if not isinstance(arr, list):
                raise ExprError(f"For loop expects an iterable type, found {type_name(arr)}")
            return self.iterate(n, enumerate(arr))
        if tag == "break":
            raise _Break(self.ev(n[1]) if n[1] is not None else None)
        if tag == "continue":
            raise _Continue()
        if tag == "return":
            raise _Return(self.ev(n[1]) if n[1] is not None else None)
        raise AssertionError(tag)


def run(prog, members, member_ok):
    """-> (error message or None, bool value, called members in call order, nodes evaluated)."""
    r = Run(prog, members, member_ok)
    try:
        v = r.ev(prog.root)
    except _Return as ret:
        v = ret.value
    except (ExprError, RecursionError) as e:
        msg = str(e) if isinstance(e, ExprError) else "Stack overflow"
        return msg, False, r.called, r.steps
    if not isinstance(v, bool):
        return f"Output type incorrect: {type_name(v)} (expecting bool)", False, r.called, r.steps
    return None, v, r.called, r.steps


def calls_members(prog, members):
    def walk(n):
        if n[0] == "call" and not n[3] and not n[2] and n[1] in members and (n[1], 0) not in prog.fns:
            return True
        return any(walk(c) for c, _ in _children(n))
    return walk(prog.root) or any(walk(b) for _, b in prog.fns.values())


def bool_tree(prog, members):
    """The program as the bool-only tree (('const', 'bool', v) | ('call', slot) | ('not', a) |
    ('and'|'or'|'eq'|'ne', a, b)) when it is one — a single tail expression over member calls,
    bool literals, ! && || == != (call-free subtrees folded to their values) — else None."""
    if prog.fns:
        return None
    root = prog.root
    while root[0] == "block":
        if len(root[1]) != 1 or not root[2]:
            return None
        root = root[1][0]

    def has_var_or_call(n):
        if n[0] in ("call", "var", "let", "assign", "setidx", "array", "index", "for", "while", "loop", "do",
                    "switch", "break", "continue", "return", "in", "range"):
            return True
        if n[0] == "lit" and isinstance(n[1], str):
            return True
        return any(has_var_or_call(c) for c, _ in _children(n))

    def conv(n):
        if not has_var_or_call(n):
            r = Run(prog, members, [])
            try:
                v = r.ev(n)
            except ExprError:
                return None
            return ("const", "bool", v) if isinstance(v, bool) else None
        if n[0] == "call":
            if n[3] or n[2] or n[1] not in members:
                return None
            return ("call", members.index(n[1]))
        if n[0] == "un" and n[1] == "!":
            a = conv(n[2])
            return ("not", a) if a is not None else None
        if n[0] == "bin" and n[1] in ("&&", "||", "==", "!="):
            a, b = conv(n[2]), conv(n[3])
            if a is None or b is None:
                return None
            return ({"&&": "and", "||": "or", "==": "eq", "!=": "ne"}[n[1]], a, b)
        if n[0] == "block" and len(n[1]) == 1 and n[2]:
            return conv(n[1][0])
        return None

    return conv(root)
