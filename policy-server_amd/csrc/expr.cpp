// expr.cpp — see expr.hpp. Recursive-descent parser with rhai precedence
// (|| < && < comparison < + - < * / % < unary), static typing (member calls are bool, integer
// literals are i64), constant folding of every call-free subtree, postfix emission.
#include "expr.hpp"

#include <cctype>
#include <memory>

#include "kwdev.hpp"

namespace kw {
namespace {

enum class Tk { End, Ident, Int, LParen, RParen, Op, Bad };
struct Token {
  Tk t;
  std::string s;
  int64_t v = 0;
  size_t pos = 0;
};

struct Node {
  enum K { Const, Call, Not, Neg, Bin } k;
  bool is_bool = true;  // type
  bool bval = false;
  int64_t ival = 0;
  int slot = -1;
  std::string op;
  std::unique_ptr<Node> a, b;
};
using P = std::unique_ptr<Node>;

struct Parser {
  std::vector<Token> toks;
  size_t i = 0;
  const std::vector<std::string>& members;
  std::string err;
  explicit Parser(const std::vector<std::string>& m) : members(m) {}

  bool lex(const std::string& s) {
    size_t k = 0;
    while (k < s.size()) {
      char c = s[k];
      if (isspace((unsigned char)c)) {
        ++k;
        continue;
      }
      Token t;
      t.pos = k;
      if (isalpha((unsigned char)c) || c == '_') {
        size_t b = k;
        while (k < s.size() && (isalnum((unsigned char)s[k]) || s[k] == '_')) ++k;
        t.t = Tk::Ident;
        t.s = s.substr(b, k - b);
      } else if (isdigit((unsigned char)c)) {
        size_t b = k;
        while (k < s.size() && (isdigit((unsigned char)s[k]) || s[k] == '_')) ++k;
        std::string d;
        for (size_t j = b; j < k; ++j)
          if (s[j] != '_') d.push_back(s[j]);
        if (d.size() > 18) {
          err = "Syntax error: integer literal too large";
          return false;
        }
        t.t = Tk::Int;
        t.v = std::stoll(d);
      } else if (c == '(') {
        t.t = Tk::LParen;
        ++k;
      } else if (c == ')') {
        t.t = Tk::RParen;
        ++k;
      } else {
        static const char* ops[] = {"||", "&&", "==", "!=", "<=", ">=", "<", ">", "+", "-", "*", "/", "%", "!"};
        bool ok = false;
        for (const char* o : ops) {
          size_t n = std::char_traits<char>::length(o);
          if (s.compare(k, n, o) == 0) {
            t.t = Tk::Op;
            t.s = o;
            k += n;
            ok = true;
            break;
          }
        }
        if (!ok) {
          err = std::string("Syntax error: unexpected character '") + c + "' (line 1, position " +
                std::to_string(k + 1) + ")";
          return false;
        }
      }
      toks.push_back(t);
    }
    Token e;
    e.t = Tk::End;
    e.pos = s.size();
    toks.push_back(e);
    return true;
  }

  const Token& peek() const { return toks[i]; }
  bool isop(const char* o) const { return peek().t == Tk::Op && peek().s == o; }

  P bin(const std::string& op, P a, P b) {
    auto n = std::make_unique<Node>();
    n->k = Node::Bin;
    n->op = op;
    n->a = std::move(a);
    n->b = std::move(b);
    return n;
  }
  P expr() { return orx(); }
  P orx() {
    P l = andx();
    while (l && isop("||")) {
      ++i;
      P r = andx();
      if (!r) return nullptr;
      l = bin("||", std::move(l), std::move(r));
    }
    return l;
  }
  P andx() {
    P l = cmp();
    while (l && isop("&&")) {
      ++i;
      P r = cmp();
      if (!r) return nullptr;
      l = bin("&&", std::move(l), std::move(r));
    }
    return l;
  }
  P cmp() {
    P l = add();
    while (l && (isop("==") || isop("!=") || isop("<") || isop("<=") || isop(">") || isop(">="))) {
      std::string op = peek().s;
      ++i;
      P r = add();
      if (!r) return nullptr;
      l = bin(op, std::move(l), std::move(r));
    }
    return l;
  }
  P add() {
    P l = mul();
    while (l && (isop("+") || isop("-"))) {
      std::string op = peek().s;
      ++i;
      P r = mul();
      if (!r) return nullptr;
      l = bin(op, std::move(l), std::move(r));
    }
    return l;
  }
  P mul() {
    P l = unary();
    while (l && (isop("*") || isop("/") || isop("%"))) {
      std::string op = peek().s;
      ++i;
      P r = unary();
      if (!r) return nullptr;
      l = bin(op, std::move(l), std::move(r));
    }
    return l;
  }
  P unary() {
    if (isop("!") || isop("-")) {
      bool neg = peek().s == "-";
      ++i;
      P a = unary();
      if (!a) return nullptr;
      auto n = std::make_unique<Node>();
      n->k = neg ? Node::Neg : Node::Not;
      n->a = std::move(a);
      return n;
    }
    return primary();
  }
  P primary() {
    const Token& t = peek();
    auto n = std::make_unique<Node>();
    if (t.t == Tk::Int) {
      ++i;
      n->k = Node::Const;
      n->is_bool = false;
      n->ival = t.v;
      return n;
    }
    if (t.t == Tk::LParen) {
      ++i;
      P e = expr();
      if (!e) return nullptr;
      if (peek().t != Tk::RParen) {
        err = "Syntax error: expecting ')' (line 1, position " + std::to_string(peek().pos + 1) + ")";
        return nullptr;
      }
      ++i;
      return e;
    }
    if (t.t == Tk::Ident) {
      std::string name = t.s;
      ++i;
      if (name == "true" || name == "false") {
        n->k = Node::Const;
        n->bval = name == "true";
        return n;
      }
      if (peek().t != Tk::LParen) {
        err = "Variable not found: " + name + " (line 1, position " + std::to_string(t.pos + 1) + ")";
        return nullptr;
      }
      ++i;
      if (peek().t != Tk::RParen) {
        err = "Syntax error: member policies take no arguments (line 1, position " +
              std::to_string(peek().pos + 1) + ")";
        return nullptr;
      }
      ++i;
      int slot = -1;
      for (size_t m = 0; m < members.size(); ++m)
        if (members[m] == name) slot = (int)m;
      if (slot < 0) {
        err = "Function not found: " + name + " () (line 1, position " + std::to_string(t.pos + 1) + ")";
        return nullptr;
      }
      n->k = Node::Call;
      n->slot = slot;
      return n;
    }
    if (t.t == Tk::End) err = "Syntax error: expecting an expression (line 1, position " + std::to_string(t.pos + 1) + ")";
    else err = "Syntax error: unexpected '" + t.s + "' (line 1, position " + std::to_string(t.pos + 1) + ")";
    return nullptr;
  }
};

const char* tname(const Node& n) { return n.is_bool ? "bool" : "i64"; }

// type check + constant fold; returns false with err on a type error
bool check(Node* n, std::string* err) {
  switch (n->k) {
    case Node::Const:
    case Node::Call: return true;
    case Node::Not:
      if (!check(n->a.get(), err)) return false;
      if (!n->a->is_bool) {
        *err = "Function not found: ! (i64)";
        return false;
      }
      n->is_bool = true;
      if (n->a->k == Node::Const) {
        n->k = Node::Const;
        n->bval = !n->a->bval;
        n->a.reset();
      }
      return true;
    case Node::Neg:
      if (!check(n->a.get(), err)) return false;
      if (n->a->is_bool) {
        *err = "Function not found: - (bool)";
        return false;
      }
      n->is_bool = false;
      n->k = Node::Const;
      n->ival = -n->a->ival;
      n->a.reset();
      return true;
    case Node::Bin: {
      if (!check(n->a.get(), err) || !check(n->b.get(), err)) return false;
      Node& a = *n->a;
      Node& b = *n->b;
      const std::string& op = n->op;
      if (op == "&&" || op == "||") {
        if (!a.is_bool || !b.is_bool) {
          *err = "Function not found: " + op + " (" + tname(a) + ", " + tname(b) + ")";
          return false;
        }
        n->is_bool = true;
        if (a.k == Node::Const && b.k == Node::Const) {
          bool v = op == "&&" ? (a.bval && b.bval) : (a.bval || b.bval);
          n->k = Node::Const;
          n->bval = v;
          n->a.reset();
          n->b.reset();
        }
        return true;
      }
      if (op == "==" || op == "!=") {
        if (a.is_bool != b.is_bool) {
          *err = "Function not found: " + op + " (" + tname(a) + ", " + tname(b) + ")";
          return false;
        }
        n->is_bool = true;
        if (a.k == Node::Const && b.k == Node::Const) {
          bool eq = a.is_bool ? a.bval == b.bval : a.ival == b.ival;
          n->k = Node::Const;
          n->bval = op == "==" ? eq : !eq;
          n->a.reset();
          n->b.reset();
        }
        return true;
      }
      // int-only operators
      if (a.is_bool || b.is_bool) {
        *err = "Function not found: " + op + " (" + tname(a) + ", " + tname(b) + ")";
        return false;
      }
      // both int -> both constant (no member call returns an int)
      int64_t x = a.ival, y = b.ival;
      n->k = Node::Const;
      n->a.reset();
      n->b.reset();
      if (op == "<" || op == "<=" || op == ">" || op == ">=") {
        n->is_bool = true;
        n->bval = op == "<" ? x < y : op == "<=" ? x <= y : op == ">" ? x > y : x >= y;
        return true;
      }
      n->is_bool = false;
      if ((op == "/" || op == "%") && y == 0) {
        *err = "Division by zero: " + std::to_string(x) + " " + op + " 0";
        return false;
      }
      n->ival = op == "+" ? x + y : op == "-" ? x - y : op == "*" ? x * y : op == "/" ? x / y : x % y;
      return true;
    }
  }
  return true;
}

// Short-circuit jump code (kwdev.hpp GOp): a || b = a, JT end, b; a && b = a, JF end, b; the other
// operators evaluate both sides. Only == / != deepen the value stack.
void emit(const Node* n, std::vector<uint8_t>* code, int depth, int* maxdepth) {
  if (depth > *maxdepth) *maxdepth = depth;
  switch (n->k) {
    case Node::Const: code->push_back(n->bval ? G_CONST1 : G_CONST0); return;
    case Node::Call:
      code->push_back(G_CALL);
      code->push_back((uint8_t)n->slot);
      return;
    case Node::Not:
      emit(n->a.get(), code, depth, maxdepth);
      code->push_back(G_NOT);
      return;
    case Node::Neg: return;  // folded
    case Node::Bin:
      emit(n->a.get(), code, depth, maxdepth);
      if (n->op == "&&" || n->op == "||") {
        code->push_back(n->op == "&&" ? G_JF : G_JT);
        const size_t at = code->size();
        code->push_back(0);
        code->push_back(0);
        emit(n->b.get(), code, depth, maxdepth);
        (*code)[at] = (uint8_t)(code->size() & 0xff);
        (*code)[at + 1] = (uint8_t)(code->size() >> 8);
        return;
      }
      emit(n->b.get(), code, depth + 1, maxdepth);
      code->push_back(n->op == "==" ? G_EQ : G_NE);
      return;
  }
}

}  // namespace

GroupProgram compile_group_expression(const std::string& expr, const std::vector<std::string>& members) {
  GroupProgram g;
  Parser p(members);
  if (!p.lex(expr)) {
    g.error = p.err;
    return g;
  }
  P root = p.expr();
  if (root && p.peek().t != Tk::End) {
    p.err = "Syntax error: unexpected '" + p.peek().s + "' (line 1, position " + std::to_string(p.peek().pos + 1) + ")";
    root.reset();
  }
  if (!root) {
    g.error = p.err;
    return g;
  }
  std::string terr;
  if (!check(root.get(), &terr)) {
    g.error = terr;
    return g;
  }
  g.valid = true;
  if (!root->is_bool) {
    // rhai accepts the expression at validation time but evaluation yields an i64
    g.eval_error = true;
    g.eval_message = "policy group expression did not evaluate to a boolean: Output type incorrect: i64 (expecting bool)";
    return g;
  }
  int maxd = 1;
  emit(root.get(), &g.code, 1, &maxd);
  if (maxd > kMaxGroupStack || g.code.size() > 65535) {
    g.valid = false;
    g.error = "policy group expression nests too deeply for the engine (max stack 64)";
    g.code.clear();
  }
  return g;
}

}  // namespace kw
