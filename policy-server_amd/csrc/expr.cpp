// expr.cpp — see expr.hpp. Lexer, recursive-descent parser with rhai precedence, a host
// interpreter (validation, response messages, truth tables), constant folding of call-free
// subtrees, and the device forms: short-circuit jump code or a truth table.
#include "expr.hpp"

#include <cctype>
#include <climits>
#include <algorithm>
#include <map>

#include "kwdev.hpp"

namespace kw {

// ------------------------------------------------------------------------------------------
// Values and the tree
// ------------------------------------------------------------------------------------------
enum class VT : uint8_t { Unit, Bool, Int, Str };
struct Val {
  VT t = VT::Unit;
  bool b = false;
  int64_t i = 0;
  std::string s;
};
static const char* tname(VT t) { return t == VT::Bool ? "bool" : t == VT::Int ? "i64" : t == VT::Str ? "string" : "()"; }

struct Node {
  enum K { Lit, Var, Call, Unary, Bin, If, Block, Let } k = Lit;
  Val lit;            // Lit
  std::string name;   // Var / Let
  int slot = -1;      // Call
  std::string op;     // Unary / Bin
  std::vector<std::unique_ptr<Node>> kids;  // Unary: a; Bin: a b; If: cond then [else]; Block: statements; Let: init
  bool tail = false;  // Block: its last statement is a value (no `;` after it)
};
using P = std::unique_ptr<Node>;

struct ExprAst {
  P root;  // a Block (the script)
};

namespace {

// ------------------------------------------------------------------------------------------
// Lexer
// ------------------------------------------------------------------------------------------
enum class Tk { End, Ident, Int, Str, Punct };
struct Token {
  Tk t = Tk::End;
  std::string s;
  int64_t v = 0;
};

struct Lexer {
  std::vector<Token> toks;
  std::string err;
  bool run(const std::string& s) {
    size_t k = 0;
    while (k < s.size()) {
      const char c = s[k];
      if (isspace((unsigned char)c)) {
        ++k;
        continue;
      }
      if (c == '/' && k + 1 < s.size() && s[k + 1] == '/') {  // line comment
        while (k < s.size() && s[k] != '\n') ++k;
        continue;
      }
      Token t;
      if (isalpha((unsigned char)c) || c == '_') {
        const size_t b = k;
        while (k < s.size() && (isalnum((unsigned char)s[k]) || s[k] == '_')) ++k;
        t.t = Tk::Ident;
        t.s = s.substr(b, k - b);
      } else if (isdigit((unsigned char)c)) {
        const size_t b = k;
        while (k < s.size() && (isdigit((unsigned char)s[k]) || s[k] == '_')) ++k;
        std::string d;
        for (size_t j = b; j < k; ++j)
          if (s[j] != '_') d.push_back(s[j]);
        if (d.size() > 19 || (d.size() == 19 && d > "9223372036854775807")) {
          err = "Syntax error: integer literal too large";
          return false;
        }
        t.t = Tk::Int;
        t.v = std::stoll(d);
      } else if (c == '"') {
        ++k;
        t.t = Tk::Str;
        bool closed = false;
        while (k < s.size()) {
          const char q = s[k++];
          if (q == '"') {
            closed = true;
            break;
          }
          if (q != '\\') {
            t.s.push_back(q);
            continue;
          }
          if (k >= s.size()) break;
          const char e = s[k++];
          switch (e) {
            case 'n': t.s.push_back('\n'); break;
            case 't': t.s.push_back('\t'); break;
            case 'r': t.s.push_back('\r'); break;
            case '0': t.s.push_back('\0'); break;
            case '\\': t.s.push_back('\\'); break;
            case '"': t.s.push_back('"'); break;
            case '\'': t.s.push_back('\''); break;
            default: err = std::string("Syntax error: invalid escape sequence \\") + e; return false;
          }
        }
        if (!closed) {
          err = "Syntax error: unterminated string literal";
          return false;
        }
      } else {
        static const char* ops[] = {"||", "&&", "==", "!=", "<=", ">=", "<", ">", "+", "-", "*", "/", "%",
                                    "!",  "|",  "&",  "^",  "(",  ")",  "{", "}", ";", "="};
        bool ok = false;
        for (const char* o : ops) {
          const size_t n = std::char_traits<char>::length(o);
          if (s.compare(k, n, o) == 0) {
            t.t = Tk::Punct;
            t.s = o;
            k += n;
            ok = true;
            break;
          }
        }
        if (!ok) {
          err = std::string("Syntax error: unexpected character '") + c + "'";
          return false;
        }
      }
      toks.push_back(t);
    }
    toks.push_back(Token{});
    return true;
  }
};

bool is_kw(const std::string& s) { return s == "let" || s == "if" || s == "else" || s == "true" || s == "false"; }

// ------------------------------------------------------------------------------------------
// Parser (script mode: statements, blocks, if-else expressions)
// ------------------------------------------------------------------------------------------
struct Parser {
  const std::vector<Token>& toks;
  const std::vector<std::string>& members;
  size_t i = 0;
  std::string err;
  Parser(const std::vector<Token>& t, const std::vector<std::string>& m) : toks(t), members(m) {}

  const Token& peek() const { return toks[i]; }
  bool punct(const char* o) const { return peek().t == Tk::Punct && peek().s == o; }
  bool ident(const char* o) const { return peek().t == Tk::Ident && peek().s == o; }
  P fail(const std::string& m) {
    if (err.empty()) err = m;
    return nullptr;
  }
  std::string near() const {
    const Token& t = peek();
    if (t.t == Tk::End) return "end of script";
    if (t.t == Tk::Int) return std::to_string(t.v);
    if (t.t == Tk::Str) return "\"" + t.s + "\"";
    return "'" + t.s + "'";
  }

  // statements until `close` ("}" or end of script)
  P block_body(bool top) {
    auto b = std::make_unique<Node>();
    b->k = Node::Block;
    for (;;) {
      if (top ? peek().t == Tk::End : punct("}")) break;
      if (peek().t == Tk::End) return fail("Syntax error: expecting '}' to close the block");
      P st;
      bool block_like = false;
      if (ident("let")) {
        ++i;
        if (peek().t != Tk::Ident || is_kw(peek().s)) return fail("Syntax error: expecting a variable name after 'let'");
        auto l = std::make_unique<Node>();
        l->k = Node::Let;
        l->name = peek().s;
        ++i;
        if (!punct("=")) return fail("Syntax error: expecting '=' after the variable name");
        ++i;
        P init = expr();
        if (!init) return nullptr;
        l->kids.push_back(std::move(init));
        st = std::move(l);
      } else {
        block_like = ident("if") || punct("{");
        st = expr();
        if (!st) return nullptr;
      }
      const bool is_let = st->k == Node::Let;
      b->kids.push_back(std::move(st));
      if (punct(";")) {
        ++i;
        b->tail = false;
        continue;
      }
      if (top ? peek().t == Tk::End : punct("}")) {
        b->tail = !is_let;
        break;
      }
      if (!block_like) return fail("Syntax error: expecting ';' to terminate this statement, found " + near());
      b->tail = false;
    }
    return b;
  }

  // precedence climbing: || | ^ (30), && & (60), == != (90), < <= > >= (110), + - (150), * / % (180)
  static int prec(const Token& t) {
    if (t.t != Tk::Punct) return -1;
    const std::string& o = t.s;
    if (o == "||" || o == "|" || o == "^") return 30;
    if (o == "&&" || o == "&") return 60;
    if (o == "==" || o == "!=") return 90;
    if (o == "<" || o == "<=" || o == ">" || o == ">=") return 110;
    if (o == "+" || o == "-") return 150;
    if (o == "*" || o == "/" || o == "%") return 180;
    return -1;
  }
  P expr(int min_prec = 0) {
    P l = unary();
    while (l) {
      const int p = prec(peek());
      if (p < 0 || p < min_prec) break;
      auto n = std::make_unique<Node>();
      n->k = Node::Bin;
      n->op = peek().s;
      ++i;
      P r = expr(p + 1);
      if (!r) return nullptr;
      n->kids.push_back(std::move(l));
      n->kids.push_back(std::move(r));
      l = std::move(n);
    }
    return l;
  }
  P unary() {
    if (punct("!") || punct("-") || punct("+")) {
      auto n = std::make_unique<Node>();
      n->k = Node::Unary;
      n->op = peek().s;
      ++i;
      P a = unary();
      if (!a) return nullptr;
      n->kids.push_back(std::move(a));
      return n;
    }
    return primary();
  }
  P primary() {
    const Token t = peek();
    auto n = std::make_unique<Node>();
    if (t.t == Tk::Int) {
      ++i;
      n->lit.t = VT::Int;
      n->lit.i = t.v;
      return n;
    }
    if (t.t == Tk::Str) {
      ++i;
      n->lit.t = VT::Str;
      n->lit.s = t.s;
      return n;
    }
    if (punct("(")) {
      ++i;
      P e = expr();
      if (!e) return nullptr;
      if (!punct(")")) return fail("Syntax error: expecting ')', found " + near());
      ++i;
      return e;
    }
    if (punct("{")) {
      ++i;
      P b = block_body(false);
      if (!b) return nullptr;
      ++i;  // '}'
      return b;
    }
    if (t.t == Tk::Ident) {
      ++i;
      if (t.s == "true" || t.s == "false") {
        n->lit.t = VT::Bool;
        n->lit.b = t.s == "true";
        return n;
      }
      if (t.s == "if") {
        n->k = Node::If;
        P c = expr();
        if (!c) return nullptr;
        n->kids.push_back(std::move(c));
        if (!punct("{")) return fail("Syntax error: expecting '{' after the if condition, found " + near());
        ++i;
        P th = block_body(false);
        if (!th) return nullptr;
        ++i;
        n->kids.push_back(std::move(th));
        if (ident("else")) {
          ++i;
          if (ident("if")) {
            P e = primary();
            if (!e) return nullptr;
            n->kids.push_back(std::move(e));
          } else {
            if (!punct("{")) return fail("Syntax error: expecting '{' or 'if' after 'else', found " + near());
            ++i;
            P e = block_body(false);
            if (!e) return nullptr;
            ++i;
            n->kids.push_back(std::move(e));
          }
        }
        return n;
      }
      if (t.s == "let" || t.s == "else") return fail("Syntax error: unexpected '" + t.s + "'");
      if (!punct("(")) {
        n->k = Node::Var;
        n->name = t.s;
        return n;
      }
      ++i;
      if (!punct(")")) return fail("Syntax error: member policies take no arguments");
      ++i;
      int slot = -1;
      for (size_t m = 0; m < members.size(); ++m)
        if (members[m] == t.s) slot = (int)m;
      n->k = Node::Call;
      n->slot = slot;  // -1: "Function not found" when called (rhai resolves at run time)
      n->name = t.s;
      return n;
    }
    if (t.t == Tk::End) return fail("Syntax error: expecting an expression, found end of script");
    return fail("Syntax error: unexpected " + near());
  }
};

// ------------------------------------------------------------------------------------------
// Interpreter
// ------------------------------------------------------------------------------------------
struct Interp {
  std::function<bool(uint32_t)> ok;
  std::vector<std::pair<std::string, Val>> vars;
  std::vector<uint32_t> called;
  std::vector<uint8_t> seen;
  std::string err;
  explicit Interp(std::function<bool(uint32_t)> f) : ok(std::move(f)) {}

  bool fail(const std::string& m) {
    err = m;
    return false;
  }
  bool nf(const std::string& op, const Val& a, const Val& b) {
    return fail("Function not found: " + op + " (" + tname(a.t) + ", " + tname(b.t) + ")");
  }

  bool eval(const Node* n, Val* out) {
    switch (n->k) {
      case Node::Lit: *out = n->lit; return true;
      case Node::Var:
        for (size_t k = vars.size(); k-- > 0;)
          if (vars[k].first == n->name) {
            *out = vars[k].second;
            return true;
          }
        return fail("Variable not found: " + n->name);
      case Node::Call: {
        if (n->slot < 0) return fail("Function not found: " + n->name + " ()");
        const uint32_t s = (uint32_t)n->slot;
        if (s >= seen.size()) seen.resize(s + 1, 0);
        if (!seen[s]) {
          seen[s] = 1;
          called.push_back(s);
        }
        out->t = VT::Bool;
        out->b = ok(s);
        return true;
      }
      case Node::Unary: {
        Val a;
        if (!eval(n->kids[0].get(), &a)) return false;
        if (n->op == "!") {
          if (a.t != VT::Bool) return fail(std::string("Function not found: ! (") + tname(a.t) + ")");
          out->t = VT::Bool;
          out->b = !a.b;
          return true;
        }
        if (a.t != VT::Int) return fail("Function not found: " + n->op + " (" + tname(a.t) + ")");
        if (n->op == "-" && a.i == INT64_MIN) return fail("Negation overflow: -" + std::to_string(a.i));
        *out = a;
        if (n->op == "-") out->i = -a.i;
        return true;
      }
      case Node::Bin: return bin(n, out);
      case Node::If: {
        Val c;
        if (!eval(n->kids[0].get(), &c)) return false;
        if (c.t != VT::Bool) return fail("Boolean value expected for the if condition, found " + std::string(tname(c.t)));
        if (c.b) return eval(n->kids[1].get(), out);
        if (n->kids.size() > 2) return eval(n->kids[2].get(), out);
        *out = Val{};
        return true;
      }
      case Node::Block: {
        const size_t scope = vars.size();
        Val v;
        for (size_t k = 0; k < n->kids.size(); ++k) {
          const Node* st = n->kids[k].get();
          if (st->k == Node::Let) {
            Val x;
            if (!eval(st->kids[0].get(), &x)) return false;
            vars.push_back({st->name, x});
            v = Val{};
          } else if (!eval(st, &v)) {
            return false;
          }
        }
        vars.resize(scope);
        *out = n->tail ? v : Val{};
        return true;
      }
      case Node::Let: *out = Val{}; return true;  // (handled by Block)
    }
    return fail("internal: bad node");
  }

  bool bin(const Node* n, Val* out) {
    const std::string& op = n->op;
    Val a, b;
    if (!eval(n->kids[0].get(), &a)) return false;
    if (op == "||" || op == "&&") {
      if (a.t != VT::Bool) return fail("Function not found: " + op + " (" + tname(a.t) + ", ...)");
      if ((op == "||") == a.b) {  // short circuit
        out->t = VT::Bool;
        out->b = a.b;
        return true;
      }
      if (!eval(n->kids[1].get(), &b)) return false;
      if (b.t != VT::Bool) return nf(op, a, b);
      *out = b;
      return true;
    }
    if (!eval(n->kids[1].get(), &b)) return false;
    out->t = VT::Bool;
    if (op == "==" || op == "!=") {  // different types: false (!= true), rhai's built-in comparison
      bool eq = a.t == b.t && (a.t == VT::Unit || (a.t == VT::Bool && a.b == b.b) || (a.t == VT::Int && a.i == b.i) ||
                               (a.t == VT::Str && a.s == b.s));
      out->b = op == "==" ? eq : !eq;
      return true;
    }
    if (op == "<" || op == "<=" || op == ">" || op == ">=") {
      if (a.t != b.t) {
        out->b = false;
        return true;
      }
      int c;
      if (a.t == VT::Int) c = a.i < b.i ? -1 : a.i > b.i ? 1 : 0;
      else if (a.t == VT::Str) c = a.s.compare(b.s) < 0 ? -1 : a.s == b.s ? 0 : 1;
      else return nf(op, a, b);
      out->b = op == "<" ? c < 0 : op == "<=" ? c <= 0 : op == ">" ? c > 0 : c >= 0;
      return true;
    }
    if (op == "|" || op == "&" || op == "^") {
      if (a.t == VT::Bool && b.t == VT::Bool) {
        out->b = op == "|" ? (a.b || b.b) : op == "&" ? (a.b && b.b) : (a.b != b.b);
        return true;
      }
      if (a.t == VT::Int && b.t == VT::Int) {
        out->t = VT::Int;
        out->i = op == "|" ? (a.i | b.i) : op == "&" ? (a.i & b.i) : (a.i ^ b.i);
        return true;
      }
      return nf(op, a, b);
    }
    if (op == "+" && a.t == VT::Str && b.t == VT::Str) {
      out->t = VT::Str;
      out->s = a.s + b.s;
      return true;
    }
    if (a.t != VT::Int || b.t != VT::Int) return nf(op, a, b);
    out->t = VT::Int;
    const std::string expr = std::to_string(a.i) + " " + op + " " + std::to_string(b.i);
    long long r = 0;
    if (op == "+") {
      if (__builtin_add_overflow(a.i, b.i, &r)) return fail("Addition overflow: " + expr);
    } else if (op == "-") {
      if (__builtin_sub_overflow(a.i, b.i, &r)) return fail("Subtraction overflow: " + expr);
    } else if (op == "*") {
      if (__builtin_mul_overflow(a.i, b.i, &r)) return fail("Multiplication overflow: " + expr);
    } else {  // / %
      if (b.i == 0) return fail("Division by zero: " + expr);
      if (a.i == INT64_MIN && b.i == -1) return fail((op == "/" ? "Division overflow: " : "Modulo overflow: ") + expr);
      r = op == "/" ? a.i / b.i : a.i % b.i;
    }
    out->i = r;
    return true;
  }
};

ExprOutcome run_ast(const ExprAst& ast, const std::function<bool(uint32_t)>& ok) {
  Interp in(ok);
  Val v;
  ExprOutcome o;
  if (!in.eval(ast.root.get(), &v)) {
    o.error = true;
    o.message = in.err;
  } else if (v.t != VT::Bool) {
    o.error = true;
    o.message = std::string("Output type incorrect: ") + tname(v.t) + " (expecting bool)";
  } else {
    o.value = v.b;
  }
  o.called = std::move(in.called);
  return o;
}

// ------------------------------------------------------------------------------------------
// Folding and the bool-only subset
// ------------------------------------------------------------------------------------------
bool has_call(const Node* n) {
  if (n->k == Node::Call) return true;
  for (const P& k : n->kids)
    if (has_call(k.get())) return true;
  return false;
}

bool has_call_or_var(const Node* n) {
  if (n->k == Node::Call || n->k == Node::Var || n->k == Node::Let) return true;
  for (const P& k : n->kids)
    if (has_call_or_var(k.get())) return true;
  return false;
}

// Replace every call-free, variable-free subtree whose evaluation succeeds by its value (an erroring
// one stays: it may never run, e.g. behind a short circuit).
void fold(P* np) {
  Node* n = np->get();
  for (P& k : n->kids) fold(&k);
  if (n->k == Node::Lit || has_call_or_var(n)) return;
  const std::function<bool(uint32_t)> none = [](uint32_t) { return false; };
  Interp in(none);
  Val v;
  if (!in.eval(n, &v)) return;
  auto l = std::make_unique<Node>();
  l->lit = v;
  *np = std::move(l);
}

// bool-only: bool literals, member calls, ! && || == != (== / != over bools), a script that is a
// single tail expression
const Node* bool_root(const ExprAst& a) {
  const Node* r = a.root.get();
  while (r->k == Node::Block && r->tail && r->kids.size() == 1) r = r->kids[0].get();
  return r;
}
bool is_bool_subset(const Node* n) {
  switch (n->k) {
    case Node::Lit: return n->lit.t == VT::Bool;
    case Node::Call: return n->slot >= 0;
    case Node::Unary: return n->op == "!" && is_bool_subset(n->kids[0].get());
    case Node::Bin:
      if (n->op != "&&" && n->op != "||" && n->op != "==" && n->op != "!=") return false;
      return is_bool_subset(n->kids[0].get()) && is_bool_subset(n->kids[1].get());
    case Node::Block: return n->tail && n->kids.size() == 1 && is_bool_subset(n->kids[0].get());
    default: return false;
  }
}

// Short-circuit jump code (kwdev.hpp GOp): a || b = a, JT end, b; a && b = a, JF end, b; == / !=
// evaluate both sides and deepen the value stack by one.
void emit(const Node* n, bool wide, std::vector<uint8_t>* code, uint32_t depth, uint32_t* maxdepth) {
  if (depth > *maxdepth) *maxdepth = depth;
  switch (n->k) {
    case Node::Lit: code->push_back(n->lit.b ? G_CONST1 : G_CONST0); return;
    case Node::Call:
      if (wide) {
        code->push_back(G_CALL16);
        code->push_back((uint8_t)(n->slot & 0xff));
        code->push_back((uint8_t)(n->slot >> 8));
      } else {
        code->push_back(G_CALL);
        code->push_back((uint8_t)n->slot);
      }
      return;
    case Node::Unary:
      emit(n->kids[0].get(), wide, code, depth, maxdepth);
      code->push_back(G_NOT);
      return;
    case Node::Block: emit(n->kids[0].get(), wide, code, depth, maxdepth); return;
    case Node::Bin:
      emit(n->kids[0].get(), wide, code, depth, maxdepth);
      if (n->op == "&&" || n->op == "||") {
        code->push_back(n->op == "&&" ? G_JF : G_JT);
        const size_t at = code->size();
        code->push_back(0);
        code->push_back(0);
        if (wide) {
          code->push_back(0);
          code->push_back(0);
        }
        emit(n->kids[1].get(), wide, code, depth, maxdepth);
        const size_t to = code->size();
        (*code)[at] = (uint8_t)(to & 0xff);
        (*code)[at + 1] = (uint8_t)((to >> 8) & 0xff);
        if (wide) {
          (*code)[at + 2] = (uint8_t)((to >> 16) & 0xff);
          (*code)[at + 3] = (uint8_t)(to >> 24);
        }
        return;
      }
      emit(n->kids[1].get(), wide, code, depth + 1, maxdepth);
      code->push_back(n->op == "==" ? G_EQ : G_NE);
      return;
    default: return;
  }
}

// ---- script bytecode (kwdev.hpp SOp): the interpreter's semantics, compiled
struct ScriptEmitter {
  std::vector<uint8_t> code, pool;
  std::vector<std::vector<std::pair<std::string, uint32_t>>> scopes;  // name -> let slot, innermost last
  std::vector<uint64_t> slot_len;  // static bound of a let slot's string length
  uint32_t depth = 0, maxdepth = 0;
  uint64_t arena = 0;  // bytes of the concatenations a run may build (each runs at most once: no loops)
  void u8(uint8_t x) { code.push_back(x); }
  void u16(uint32_t x) {
    u8((uint8_t)x);
    u8((uint8_t)(x >> 8));
  }
  void u32(uint32_t x) {
    u16(x & 0xffff);
    u16(x >> 16);
  }
  void push(int n = 1) {
    depth += (uint32_t)n;
    maxdepth = std::max(maxdepth, depth);
  }
  size_t hole(uint8_t op) {
    u8(op);
    const size_t at = code.size();
    u32(0);
    return at;
  }
  void patch(size_t at) {
    const uint32_t to = (uint32_t)code.size();
    for (int k = 0; k < 4; ++k) code[at + (size_t)k] = (uint8_t)(to >> (8 * k));
  }
  bool lookup(const std::string& name, uint32_t* slot) const {
    for (size_t sc = scopes.size(); sc-- > 0;)
      for (size_t k = scopes[sc].size(); k-- > 0;)
        if (scopes[sc][k].first == name) {
          *slot = scopes[sc][k].second;
          return true;
        }
    return false;
  }
  // emits n (leaving one value on the stack); returns the static bound of its string length
  uint64_t emit(const Node* n) {
    switch (n->k) {
      case Node::Lit:
        push();
        if (n->lit.t == VT::Unit) {
          u8(S_UNIT);
        } else if (n->lit.t == VT::Bool) {
          u8(S_BOOL);
          u8(n->lit.b ? 1 : 0);
        } else if (n->lit.t == VT::Int) {
          u8(S_INT);
          for (int k = 0; k < 8; ++k) u8((uint8_t)((uint64_t)n->lit.i >> (8 * k)));
        } else {
          u8(S_STR);
          u32((uint32_t)pool.size());  // rebased to the program start at the end
          u32((uint32_t)n->lit.s.size());
          pool.insert(pool.end(), n->lit.s.begin(), n->lit.s.end());
          return n->lit.s.size();
        }
        return 0;
      case Node::Var: {
        uint32_t slot;
        push();
        if (!lookup(n->name, &slot)) {
          u8(S_FAIL);
          return 0;
        }
        u8(S_LOAD);
        u16(slot);
        return slot_len[slot];
      }
      case Node::Call:
        push();
        if (n->slot < 0) {
          u8(S_FAIL);
        } else {
          u8(S_CALL);
          u32((uint32_t)n->slot);
        }
        return 0;
      case Node::Unary:
        emit(n->kids[0].get());
        u8(n->op == "!" ? S_NOT : n->op == "-" ? S_NEG : S_POS);
        return 0;
      case Node::Bin: {
        const std::string& op = n->op;
        const uint64_t la = emit(n->kids[0].get());
        if (op == "||" || op == "&&") {
          const size_t at = hole(op == "||" ? S_OR : S_AND);
          --depth;  // (the continuing path pops the left side)
          emit(n->kids[1].get());
          u8(S_CHKB);
          patch(at);
          return 0;
        }
        const uint64_t lb = emit(n->kids[1].get());
        static const char* ops[] = {"|", "^", "&", "==", "!=", "<", "<=", ">", ">=", "+", "-", "*", "/", "%"};
        uint8_t code_op = 0;
        for (uint8_t k = 0; k < 14; ++k)
          if (op == ops[k]) code_op = k;
        u8(S_BIN);
        u8(code_op);
        --depth;
        if (code_op == SB_ADD) {
          arena += la + lb;
          return la + lb;
        }
        return 0;
      }
      case Node::If: {
        emit(n->kids[0].get());
        const size_t at_else = hole(S_IF);
        --depth;
        const uint32_t d0 = depth;
        const uint64_t lt = emit(n->kids[1].get());
        const size_t at_end = hole(S_JMP);
        patch(at_else);
        depth = d0;
        uint64_t le = 0;
        if (n->kids.size() > 2) {
          le = emit(n->kids[2].get());
        } else {
          push();
          u8(S_UNIT);
        }
        patch(at_end);
        return std::max(lt, le);
      }
      case Node::Block: {
        scopes.emplace_back();
        uint64_t last = 0;
        for (size_t k = 0; k < n->kids.size(); ++k) {
          const Node* st = n->kids[k].get();
          if (st->k == Node::Let) {
            const uint64_t l = emit(st->kids[0].get());
            const uint32_t slot = (uint32_t)slot_len.size();
            slot_len.push_back(l);
            u8(S_STORE);
            u16(slot);
            --depth;
            scopes.back().push_back({st->name, slot});
            last = 0;
          } else {
            last = emit(st);
            if (!(n->tail && k + 1 == n->kids.size())) {
              u8(S_POP);
              --depth;
            }
          }
        }
        scopes.pop_back();
        if (!n->tail) {
          push();
          u8(S_UNIT);
          return 0;
        }
        return last;
      }
      case Node::Let: push(); u8(S_UNIT); return 0;  // (handled by Block)
    }
    return 0;
  }
};

// The script form of a group (GroupProgram::script): header | code | string pool (kwdev.hpp SOp).
bool emit_script(const ExprAst& ast, std::vector<uint8_t>* out, uint32_t* depth, std::string* err) {
  ScriptEmitter e;
  e.emit(ast.root.get());
  e.u8(S_END);
  if (e.arena > kMaxScriptArena) {
    *err = "policy group expression can build strings longer than the engine's limit (65536 bytes)";
    return false;
  }
  if (e.slot_len.size() > 65535 || e.code.size() + e.pool.size() > 0x7fffffffu) {
    *err = "policy group expression exceeds the engine's limits";
    return false;
  }
  const uint32_t hdr = 16, code_len = (uint32_t)e.code.size();
  // rebase S_STR pool offsets to the program start: walk the code
  for (size_t pc = 0; pc < e.code.size();) {
    const uint8_t op = e.code[pc++];
    switch (op) {
      case S_BOOL: case S_BIN: pc += 1; break;
      case S_INT: pc += 8; break;
      case S_STR: {
        uint32_t off = 0;
        for (int k = 0; k < 4; ++k) off |= (uint32_t)e.code[pc + (size_t)k] << (8 * k);
        off += hdr + code_len;
        for (int k = 0; k < 4; ++k) e.code[pc + (size_t)k] = (uint8_t)(off >> (8 * k));
        pc += 8;
        break;
      }
      case S_LOAD: case S_STORE: pc += 2; break;
      case S_CALL: case S_AND: case S_OR: case S_IF: case S_JMP: pc += 4; break;
      default: break;
    }
  }
  out->clear();
  const uint32_t h[4] = {std::max(e.maxdepth, 1u), (uint32_t)e.slot_len.size(), (uint32_t)e.arena, code_len};
  out->insert(out->end(), (const uint8_t*)h, (const uint8_t*)h + 16);
  out->insert(out->end(), e.code.begin(), e.code.end());
  out->insert(out->end(), e.pool.begin(), e.pool.end());
  *depth = h[0];
  return true;
}

}  // namespace

std::string group_eval_message(const std::string& m) {
  if (m.rfind("Output type incorrect", 0) == 0) return "policy group expression did not evaluate to a boolean: " + m;
  return "policy group expression evaluation failed: " + m;
}

ExprOutcome GroupProgram::run(const std::function<bool(uint32_t)>& member_ok) const {
  if (!ast) {
    ExprOutcome o;
    o.error = true;
    o.message = error;
    return o;
  }
  return run_ast(*ast, member_ok);
}

GroupProgram compile_group_expression(const std::string& expr, const std::vector<std::string>& members) {
  GroupProgram g;
  g.nmem = (uint32_t)members.size();
  Lexer lx;
  if (!lx.run(expr)) {
    g.error = lx.err;
    return g;
  }
  Parser p(lx.toks, members);
  P root = p.block_body(true);
  if (!root) {
    g.error = p.err;
    return g;
  }
  auto ast = std::make_shared<ExprAst>();
  ast->root = std::move(root);
  // validation: the script runs with every member returning true (validate_settings)
  {
    Interp in([](uint32_t) { return true; });
    Val v;
    if (!in.eval(ast->root.get(), &v)) {
      g.error = in.err;
      return g;
    }
  }
  g.valid = true;
  fold(&ast->root);
  g.ast = ast;
  // a script without member calls has one outcome: a constant column or a constant program
  if (!has_call(ast->root.get())) {
    const ExprOutcome o = run_ast(*ast, [](uint32_t) { return true; });
    if (o.error) {
      g.eval_error = true;
      g.eval_message = group_eval_message(o.message);
      return g;
    }
    g.code.push_back(o.value ? G_CONST1 : G_CONST0);
    g.depth = 1;
    return g;
  }
  const Node* br = bool_root(*ast);
  if (is_bool_subset(br)) {
    uint32_t maxd = 1;
    emit(br, false, &g.code, 1, &maxd);
    g.depth = maxd;
    if (members.size() <= (size_t)kMaxGroupMembers && maxd <= (uint32_t)kMaxGroupStack && g.code.size() <= 65535) return g;
    // the wide path: u16 member operands, u32 jump targets, a value stack in global scratch
    g.code.clear();
    maxd = 1;
    emit(br, true, &g.code, 1, &maxd);
    g.depth = maxd;
    if (members.size() > 65535 || maxd > kMaxWideStack) {
      g.valid = false;
      g.error = "policy group expression exceeds the engine's limits (65535 members, value stack 65536)";
      g.code.clear();
      return g;
    }
    g.wide = true;
    return g;
  }
  if (members.size() > kMaxTableMembers) {
    // too many members for a truth table: typed bytecode, run by the wide path's combine kernel
    std::string err;
    if (!emit_script(*ast, &g.code, &g.depth, &err)) {
      g.valid = false;
      g.error = err;
      g.code.clear();
      return g;
    }
    g.wide = true;
    g.script = true;
    return g;
  }
  // truth table over the member results: value, error, and the members called that rejected
  const uint32_t n = (uint32_t)members.size();
  g.table.assign((size_t)1 << n, 0);
  for (uint32_t mask = 0; mask < (1u << n); ++mask) {
    const ExprOutcome o = run_ast(*ast, [mask](uint32_t s) { return ((mask >> s) & 1u) != 0; });
    uint32_t e = o.error ? kGtError : (o.value ? kGtValue : 0u);
    for (uint32_t s : o.called)
      if (!((mask >> s) & 1u)) e |= 1u << (16 + s);
    g.table[mask] = e;
  }
  return g;
}

}  // namespace kw
