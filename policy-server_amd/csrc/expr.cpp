// expr.cpp — see expr.hpp. Lexer, recursive-descent parser with rhai's precedence, a host
// interpreter (validation, response messages, truth tables), constant folding of call-free
// subtrees, and the device forms: short-circuit jump code, a truth table, or script bytecode
// (kwdev.hpp SOp) for the typed stack machine of slots.hpp.
#include "expr.hpp"

#include <cctype>
#include <climits>
#include <algorithm>
#include <cstdlib>
#include <map>
#include <set>

#include "kwdev.hpp"
#include "unicode_data.hpp"

namespace kw {

// ------------------------------------------------------------------------------------------
// Values and the tree
// ------------------------------------------------------------------------------------------
enum class VT : uint8_t { Unit, Bool, Int, Str, Arr };
struct Val {
  VT t = VT::Unit;
  bool b = false;
  int64_t i = 0;
  std::string s;
  std::vector<Val> a;  // arrays (values are copied: rhai's value semantics)
};
static const char* tname(VT t) {
  switch (t) {
    case VT::Bool: return "bool";
    case VT::Int: return "i64";
    case VT::Str: return "string";
    case VT::Arr: return "array";
    default: return "()";
  }
}
static Val vbool(bool b) {
  Val v;
  v.t = VT::Bool;
  v.b = b;
  return v;
}
static Val vint(int64_t i) {
  Val v;
  v.t = VT::Int;
  v.i = i;
  return v;
}
static Val vstr(std::string s) {
  Val v;
  v.t = VT::Str;
  v.s = std::move(s);
  return v;
}

const char* const kUnsupported = "unsupported by this engine: ";

struct Node;
using P = std::unique_ptr<Node>;
struct SwitchCase {
  std::vector<Val> vals;  // exact values (alternatives)
  bool range = false, incl = false, wildcard = false;
  int64_t lo = 0, hi = 0;
  P guard, body;
};
struct Node {
  enum K {
    Lit, Var, Call, Unary, Bin, Coalesce, In, Range, If, Block, Let, Assign, IndexAssign, Index, Array, Switch,
    While, DoWhile, Loop, For, Break, Continue, Return
  } k = Lit;
  Val lit;             // Lit
  std::string name;    // Var / Let / Assign / IndexAssign (the variable) / Call (the function) / For (loop variable)
  std::string name2;   // For: the index variable of `for (x, i) in ..` ("" none); Range: ".." "..=" or "range"
  std::string op;      // Unary / Bin; Assign / IndexAssign: "" for `=`, else the operator of `op=`
  bool flag = false;   // Block: tail value; Let: const; In: `!in`; Range: inclusive; DoWhile: until; Call: method style
  int slot = -1;       // Call: member slot (a member called with no arguments)
  int fn = -1;         // Call: script function (ExprAst::fns index)
  int builtin = -1;    // Call: SFn id
  std::vector<P> kids;
  std::vector<SwitchCase> cases;  // Switch (kids[0] is the scrutinee)
};

struct FnDef {
  std::string name;
  std::vector<std::string> params;
  P body;  // a Block
};

struct ExprAst {
  P root;  // a Block (the script)
  std::vector<FnDef> fns;
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

void put_utf8(uint32_t c, std::string* o) {
  if (c < 0x80) {
    o->push_back((char)c);
  } else if (c < 0x800) {
    o->push_back((char)(0xC0 | (c >> 6)));
    o->push_back((char)(0x80 | (c & 0x3F)));
  } else if (c < 0x10000) {
    o->push_back((char)(0xE0 | (c >> 12)));
    o->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
    o->push_back((char)(0x80 | (c & 0x3F)));
  } else {
    o->push_back((char)(0xF0 | (c >> 18)));
    o->push_back((char)(0x80 | ((c >> 12) & 0x3F)));
    o->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
    o->push_back((char)(0x80 | (c & 0x3F)));
  }
}

struct Lexer {
  std::vector<Token> toks;
  std::string err;
  bool unsupported(const std::string& what) {
    err = kUnsupported + what;
    return false;
  }
  bool run(const std::string& s) {
    size_t k = 0;
    auto is_id = [&](size_t j) { return j < s.size() && (isalnum((unsigned char)s[j]) || s[j] == '_'); };
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
      if (c == '/' && k + 1 < s.size() && s[k + 1] == '*') {  // block comment (rhai nests them)
        int lvl = 0;
        do {
          if (s.compare(k, 2, "/*") == 0) {
            ++lvl;
            k += 2;
          } else if (s.compare(k, 2, "*/") == 0) {
            --lvl;
            k += 2;
          } else {
            ++k;
          }
        } while (lvl > 0 && k < s.size());
        if (lvl > 0) {
          err = "Syntax error: unterminated block comment";
          return false;
        }
        continue;
      }
      Token t;
      if (isalpha((unsigned char)c) || c == '_') {
        const size_t b = k;
        while (is_id(k)) ++k;
        t.t = Tk::Ident;
        t.s = s.substr(b, k - b);
      } else if (isdigit((unsigned char)c)) {
        const size_t b = k;
        int base = 10;
        if (c == '0' && k + 1 < s.size() && (s[k + 1] == 'x' || s[k + 1] == 'o' || s[k + 1] == 'b')) {
          base = s[k + 1] == 'x' ? 16 : s[k + 1] == 'o' ? 8 : 2;
          k += 2;
        }
        std::string d;
        while (k < s.size() && (isalnum((unsigned char)s[k]) || s[k] == '_')) {
          if (s[k] != '_') d.push_back(s[k]);
          ++k;
        }
        if (base == 10 && k + 1 < s.size() && s[k] == '.' && isdigit((unsigned char)s[k + 1]))
          return unsupported("floating-point numbers");
        if (base == 10 && (d.find('e') != std::string::npos || d.find('E') != std::string::npos))
          return unsupported("floating-point numbers");
        if (d.empty()) {
          err = "Syntax error: invalid number: " + s.substr(b, k - b);
          return false;
        }
        unsigned __int128 v = 0;
        for (char ch : d) {
          int dv = isdigit((unsigned char)ch) ? ch - '0' : isxdigit((unsigned char)ch) ? (tolower(ch) - 'a' + 10) : 99;
          if (dv >= base) {
            err = "Syntax error: invalid number: " + s.substr(b, k - b);
            return false;
          }
          v = std::min<unsigned __int128>(v * (unsigned)base + (unsigned)dv, (unsigned __int128)UINT64_MAX + 1);
        }
        // decimal literals are i64 (a leading '-' is the negation operator); rhai reads a
        // hexadecimal / octal / binary literal as the bits of an i64
        if ((base == 10 && v > (unsigned __int128)INT64_MAX) || v > (unsigned __int128)UINT64_MAX) {
          err = "Syntax error: integer literal too large";
          return false;
        }
        t.t = Tk::Int;
        t.v = (int64_t)(uint64_t)v;
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
            case '\n':  // line continuation: the newline and the next line's leading spaces go
              while (k < s.size() && (s[k] == ' ' || s[k] == '\t')) ++k;
              break;
            case 'x':
            case 'u':
            case 'U': {
              const int n = e == 'x' ? 2 : e == 'u' ? 4 : 8;
              uint32_t cp = 0;
              for (int j = 0; j < n; ++j) {
                if (k >= s.size() || !isxdigit((unsigned char)s[k])) {
                  err = std::string("Syntax error: invalid escape sequence \\") + e;
                  return false;
                }
                const char h = s[k++];
                cp = cp * 16u + (uint32_t)(isdigit((unsigned char)h) ? h - '0' : tolower(h) - 'a' + 10);
              }
              if (cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) {
                err = std::string("Syntax error: invalid escape sequence \\") + e;
                return false;
              }
              put_utf8(cp, &t.s);
              break;
            }
            default: err = std::string("Syntax error: invalid escape sequence \\") + e; return false;
          }
        }
        if (!closed) {
          err = "Syntax error: unterminated string literal";
          return false;
        }
      } else if (c == '\'') {
        return unsupported("character literals");
      } else if (c == '`') {
        return unsupported("back-tick strings and string interpolation");
      } else {
        if (c == '!' && s.compare(k, 3, "!in") == 0 && !is_id(k + 3)) {
          t.t = Tk::Punct;
          t.s = "!in";
          k += 3;
          toks.push_back(t);
          continue;
        }
        static const char* bad[][2] = {{"#{", "object maps"}, {"::", "modules and namespaces"},
                                       {"?.", "the ?. operator"}, {"?[", "the ?[ operator"}};
        for (auto& b : bad)
          if (s.compare(k, std::char_traits<char>::length(b[0]), b[0]) == 0) return unsupported(b[1]);
        static const char* ops[] = {"..=", "**=", "<<=", ">>=", "=>", "??", "..", "**", "<<", ">>", "||", "&&", "==", "!=", "<=", ">=", "+=", "-=", "*=", "/=",
                                    "%=",  "|=", "&=", "^=", "<",  ">",  "+",  "-",  "*",  "/",  "%",  "!",  "|",  "&",
                                    "^",   "(",  ")",  "{",  "}",  "[",  "]",  ";",  "=",  ",",  "."};
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
        if (!ok) {  // (the whole UTF-8 sequence of a non-ASCII character)
          const unsigned char u = (unsigned char)c;
          const size_t n = u < 0xC0 ? 1 : u < 0xE0 ? 2 : u < 0xF0 ? 3 : 4;
          err = "Syntax error: unexpected character '" + s.substr(k, n) + "'";
          return false;
        }
      }
      toks.push_back(t);
    }
    toks.push_back(Token{});
    return true;
  }
};

// Built-in functions: rhai 1.21's standard packages (Engine::new()) over the
// engine's values, one SFn id per (name, arity). `mut`: rhai gives the function a `&mut` first
// parameter, so a method-style call on a variable changes the variable (a function-style call works
// on a copy). Argument types are dispatched when the call runs, as rhai dispatches its overloads.
struct BuiltinDef {
  const char* name;
  uint8_t nargs, fid;
  bool mut;
};
const BuiltinDef kBuiltins[] = {
    {"len", 1, F_LEN, false}, {"is_empty", 1, F_IS_EMPTY, false}, {"contains", 2, F_CONTAINS, false},
    {"to_string", 1, F_TO_STRING, false}, {"type_of", 1, F_TYPE_OF, false}, {"starts_with", 2, F_STARTS_WITH, false},
    {"ends_with", 2, F_ENDS_WITH, false}, {"push", 2, F_PUSH, true},
    {"abs", 1, F_ABS, false}, {"sign", 1, F_SIGN, false}, {"is_zero", 1, F_IS_ZERO, false},
    {"is_odd", 1, F_IS_ODD, false}, {"is_even", 1, F_IS_EVEN, false}, {"max", 2, F_MAX, false},
    {"min", 2, F_MIN, false}, {"to_hex", 1, F_TO_HEX, false}, {"to_octal", 1, F_TO_OCTAL, false},
    {"to_binary", 1, F_TO_BINARY, false}, {"parse_int", 1, F_PARSE_INT, false}, {"parse_int", 2, F_PARSE_INT_R, false},
    {"to_upper", 1, F_TO_UPPER, false}, {"to_lower", 1, F_TO_LOWER, false}, {"make_upper", 1, F_MAKE_UPPER, true},
    {"make_lower", 1, F_MAKE_LOWER, true}, {"trim", 1, F_TRIM, true}, {"sub_string", 2, F_SUB_STRING, false},
    {"sub_string", 3, F_SUB_STRING_N, false}, {"crop", 2, F_CROP, true}, {"crop", 3, F_CROP_N, true},
    {"index_of", 2, F_INDEX_OF, false}, {"index_of", 3, F_INDEX_OF_FROM, false}, {"replace", 3, F_REPLACE, true},
    {"split", 1, F_SPLIT_WS, false}, {"split", 2, F_SPLIT, true}, {"split", 3, F_SPLIT_N, false},
    {"split_rev", 2, F_SPLIT_REV, false}, {"split_rev", 3, F_SPLIT_REV_N, false}, {"bytes", 1, F_BYTES, false},
    {"append", 2, F_APPEND, true}, {"insert", 3, F_INSERT, true}, {"pop", 1, F_POP, true}, {"shift", 1, F_SHIFT, true},
    {"remove", 2, F_REMOVE, true}, {"reverse", 1, F_REVERSE, true}, {"sort", 1, F_SORT, true},
    {"clear", 1, F_CLEAR, true}, {"truncate", 2, F_TRUNCATE, true}, {"chop", 2, F_CHOP, true},
    {"get", 2, F_GET, false}, {"set", 3, F_SET, true}, {"extract", 2, F_EXTRACT, false},
    {"extract", 3, F_EXTRACT_N, false}, {"drain", 3, F_DRAIN, true}, {"retain", 3, F_RETAIN, true},
    {"splice", 4, F_SPLICE, true}, {"dedup", 1, F_DEDUP, true}, {"pad", 3, F_PAD, true},
};

int builtin_id(const std::string& name, size_t nargs) {
  for (const BuiltinDef& b : kBuiltins)
    if (name == b.name && nargs == b.nargs) return b.fid;
  return -1;
}
bool builtin_mut(int fid) {
  for (const BuiltinDef& b : kBuiltins)
    if (b.fid == fid) return b.mut;
  return false;
}
// a method that always changes its receiver (split changes arrays only): never on a constant or on
// an element in place
bool always_mutates(const std::string& m) {
  for (const BuiltinDef& b : kBuiltins)
    if (m == b.name && b.mut && b.fid != F_SPLIT) return true;
  return false;
}

// The rest of rhai 1.21's standard packages (Engine::new(): CorePackage, BitFieldPackage,
// BasicMathPackage, BasicArrayPackage, BasicBlobPackage, BasicMapPackage, BasicTimePackage,
// MoreStringPackage; the language keywords are refused by the parser). A call of one of these names
// that no script function or member takes is refused by name at load, as the engine's other
// omissions are, never answered with rhai's own "Function not found".
const char* const kStdRefused[] = {
    // core and function pointers (LanguageCorePackage, BasicFnPackage)
    "tag", "set_tag", "take", "sleep", "name", "is_anonymous", "to_debug",
    // keyword functions in method style (as functions the parser refuses them by their own words)
    "print", "debug", "eval", "Fn", "call", "curry", "is_def_var", "is_def_fn", "is_shared",
    // bit fields
    "get_bit", "set_bit", "get_bits", "set_bits", "bits",
    // floating point and conversions
    "to_int", "to_float", "parse_float", "sqrt", "exp", "ln", "log", "floor", "ceiling", "round", "int", "fraction",
    "is_nan", "is_finite", "is_infinite", "sin", "cos", "tan", "sinh", "cosh", "tanh", "asin", "acos", "atan",
    "asinh", "acosh", "atanh", "hypot", "to_degrees", "to_radians", "PI", "E",
    // characters
    "chars", "to_chars",
    // arrays through function pointers
    "map", "filter", "reduce", "reduce_rev", "some", "all", "find", "find_map", "for_each", "zip", "sort_desc",
    // blobs
    "blob", "to_blob", "as_string", "write_ascii", "write_utf8", "write_le", "write_be", "parse_le_int",
    "parse_be_int", "parse_le_float", "parse_be_float",
    // object maps
    "keys", "values", "mixin", "fill_with", "to_json",
    // time
    "timestamp", "elapsed",
};
bool std_refused(const std::string& name) {
  for (const char* r : kStdRefused)
    if (name == r) return true;
  return false;
}

bool is_kw(const std::string& s) {
  static const std::set<std::string> kw = {"let",   "const", "if",     "else",  "true", "false", "switch", "while",
                                           "loop",  "do",    "until",  "for",   "in",   "break", "continue",
                                           "return", "fn"};
  return kw.count(s) > 0;
}
// rhai keywords and functions this engine does not implement: refused by name
const char* unsupported_word(const std::string& s) {
  static const std::map<std::string, const char*> m = {
      {"import", "modules (import)"}, {"export", "modules (export)"}, {"as", "modules (as)"},
      {"private", "private functions"}, {"try", "try / catch"}, {"catch", "try / catch"}, {"throw", "throw"},
      {"this", "this"}, {"global", "the global namespace"}, {"Fn", "function pointers"}, {"call", "function pointers"},
      {"curry", "function pointers"}, {"eval", "eval"}, {"print", "print"}, {"debug", "debug"},
      {"is_def_var", "is_def_var"}, {"is_def_fn", "is_def_fn"}, {"is_shared", "shared values"},
      {"static", "static"}, {"exit", "exit"}};
  auto it = m.find(s);
  return it == m.end() ? nullptr : it->second;
}

// ------------------------------------------------------------------------------------------
// Parser
// ------------------------------------------------------------------------------------------
struct Parser {
  const std::vector<Token>& toks;
  size_t i = 0;
  std::string err;
  ExprAst* ast = nullptr;
  int loops = 0;      // enclosing loops (break / continue)
  bool in_fn = false;
  std::vector<std::vector<std::pair<std::string, bool>>> scopes;  // (name, const) per block
  explicit Parser(const std::vector<Token>& t) : toks(t) {}

  const Token& peek(size_t d = 0) const { return toks[std::min(i + d, toks.size() - 1)]; }
  bool punct(const char* o, size_t d = 0) const { return peek(d).t == Tk::Punct && peek(d).s == o; }
  bool ident(const char* o) const { return peek().t == Tk::Ident && peek().s == o; }
  P fail(const std::string& m) {
    if (err.empty()) err = m;
    return nullptr;
  }
  P unsupported(const std::string& what) { return fail(kUnsupported + what); }
  std::string near() const {
    const Token& t = peek();
    if (t.t == Tk::End) return "end of script";
    if (t.t == Tk::Int) return std::to_string(t.v);
    if (t.t == Tk::Str) return "\"" + t.s + "\"";
    return "'" + t.s + "'";
  }
  bool expect(const char* o, const char* what) {
    if (punct(o)) {
      ++i;
      return true;
    }
    fail(std::string("Syntax error: expecting '") + o + "' " + what + ", found " + near());
    return false;
  }
  void declare(const std::string& n, bool is_const) { scopes.back().push_back({n, is_const}); }
  bool is_const_var(const std::string& n) const {
    for (size_t s = scopes.size(); s-- > 0;)
      for (size_t k = scopes[s].size(); k-- > 0;)
        if (scopes[s][k].first == n) return scopes[s][k].second;
    return false;
  }
  static bool block_like(const Node* n) {
    return n->k == Node::If || n->k == Node::Switch || n->k == Node::While || n->k == Node::Loop || n->k == Node::For ||
           n->k == Node::Block;
  }

  // statements until "}" (or the end of the script at the top level)
  P block_body(bool top) {
    auto b = std::make_unique<Node>();
    b->k = Node::Block;
    scopes.emplace_back();
    for (;;) {
      if (top ? peek().t == Tk::End : punct("}")) break;
      if (peek().t == Tk::End) return fail("Syntax error: expecting '}' to close the block");
      if (punct(";")) {  // an empty statement
        ++i;
        continue;
      }
      if (ident("fn")) {
        if (!top || in_fn) return fail("Syntax error: functions can only be defined at global level");
        if (!fn_def()) return nullptr;
        continue;
      }
      P st = statement();
      if (!st) return nullptr;
      const bool is_decl = st->k == Node::Let || st->k == Node::Assign || st->k == Node::IndexAssign;
      const bool blk = block_like(st.get());
      b->kids.push_back(std::move(st));
      if (punct(";")) {
        ++i;
        b->flag = false;
        continue;
      }
      if (top ? peek().t == Tk::End : punct("}")) {
        b->flag = !is_decl;
        break;
      }
      if (!blk) return fail("Syntax error: expecting ';' to terminate this statement, found " + near());
      b->flag = false;
    }
    scopes.pop_back();
    return b;
  }

  bool fn_def() {
    ++i;  // fn
    if (peek().t != Tk::Ident || is_kw(peek().s)) {
      fail("Syntax error: expecting a function name after 'fn'");
      return false;
    }
    FnDef f;
    f.name = peek().s;
    ++i;
    if (!expect("(", "after the function name")) return false;
    while (!punct(")")) {
      if (peek().t != Tk::Ident || is_kw(peek().s)) {
        fail("Syntax error: expecting a parameter name, found " + near());
        return false;
      }
      if (std::find(f.params.begin(), f.params.end(), peek().s) != f.params.end()) {
        fail("Syntax error: duplicated parameter '" + peek().s + "' in function '" + f.name + "'");
        return false;
      }
      f.params.push_back(peek().s);
      ++i;
      if (punct(",")) ++i;
      else if (!punct(")")) {
        fail("Syntax error: expecting ',' or ')' in the parameter list, found " + near());
        return false;
      }
    }
    ++i;
    for (const FnDef& g : ast->fns)
      if (g.name == f.name && g.params.size() == f.params.size()) {
        fail("Syntax error: function '" + f.name + "' with " + std::to_string(f.params.size()) +
             " parameters is defined more than once");
        return false;
      }
    if (!expect("{", "to start the function body")) return false;
    const int saved_loops = loops;
    auto saved_scopes = std::move(scopes);
    scopes.clear();
    scopes.emplace_back();
    for (const std::string& p : f.params) declare(p, false);
    loops = 0;
    in_fn = true;
    f.body = block_body(false);
    in_fn = false;
    loops = saved_loops;
    scopes = std::move(saved_scopes);
    if (!f.body) return false;
    ++i;  // '}'
    ast->fns.push_back(std::move(f));
    return true;
  }

  P statement() {
    if (ident("let") || ident("const")) {
      const bool c = ident("const");
      ++i;
      if (peek().t != Tk::Ident || is_kw(peek().s)) return fail("Syntax error: expecting a variable name after 'let'");
      auto l = std::make_unique<Node>();
      l->k = Node::Let;
      l->flag = c;
      l->name = peek().s;
      ++i;
      if (punct("=")) {
        ++i;
        P init = expr();
        if (!init) return nullptr;
        l->kids.push_back(std::move(init));
      } else if (c) {
        return fail("Syntax error: expecting '=' after the constant name");
      }
      declare(l->name, c);
      return l;
    }
    if (ident("break") || ident("continue") || ident("return")) {
      auto n = std::make_unique<Node>();
      n->k = ident("break") ? Node::Break : ident("continue") ? Node::Continue : Node::Return;
      ++i;
      if (n->k != Node::Return && loops == 0)
        return fail(std::string("Syntax error: ") + (n->k == Node::Break ? "break" : "continue") +
                    " should only be used inside a loop");
      if (n->k != Node::Continue && !punct(";") && !punct("}") && peek().t != Tk::End && !punct(",")) {
        P v = expr();
        if (!v) return nullptr;
        n->kids.push_back(std::move(v));
      }
      return n;
    }
    // an if / switch / loop / block at the start of a statement is a statement of its own: no
    // operator, index or method call continues it (rhai's parse_stmt; `for .. { } [1]` is two)
    if (ident("if") || ident("switch") || ident("while") || ident("loop") || ident("do") || ident("for") || punct("{"))
      return primary();
    P e = expr();
    if (!e) return nullptr;
    static const char* aops[] = {"=", "+=", "-=", "*=", "/=", "%=", "|=", "&=", "^=", "**=", "<<=", ">>="};
    for (const char* ao : aops) {
      if (!punct(ao)) continue;
      ++i;
      P rhs = expr();
      if (!rhs) return nullptr;
      auto a = std::make_unique<Node>();
      a->op = std::string(ao) == "=" ? "" : std::string(ao).substr(0, std::char_traits<char>::length(ao) - 1);
      if (e->k == Node::Var) {
        a->k = Node::Assign;
        a->name = e->name;
        a->kids.push_back(std::move(rhs));
      } else if (e->k == Node::Index && e->kids[0]->k == Node::Var) {
        a->k = Node::IndexAssign;
        a->name = e->kids[0]->name;
        a->kids.push_back(std::move(e->kids[1]));
        a->kids.push_back(std::move(rhs));
      } else if (e->k == Node::Index) {
        return unsupported("assigning to a nested index or to an element of a temporary value");
      } else {
        return fail("Syntax error: cannot assign to this expression");
      }
      if (is_const_var(a->name)) return fail("Syntax error: cannot assign to the constant '" + a->name + "'");
      return a;
    }
    return e;
  }

  // precedence climbing (rhai 1.x): || | ^ (30), && & (60), == != (90), in !in (110),
  // < <= > >= (130), ?? (135), .. ..= (140), + - (150), * / % (180), ** (190, right-associative),
  // << >> (210)
  static int prec(const Token& t) {
    if (t.t == Tk::Ident) return t.s == "in" ? 110 : -1;
    if (t.t != Tk::Punct) return -1;
    const std::string& o = t.s;
    if (o == "||" || o == "|" || o == "^") return 30;
    if (o == "&&" || o == "&") return 60;
    if (o == "==" || o == "!=") return 90;
    if (o == "!in") return 110;
    if (o == "<" || o == "<=" || o == ">" || o == ">=") return 130;
    if (o == "??") return 135;
    if (o == ".." || o == "..=") return 140;
    if (o == "+" || o == "-") return 150;
    if (o == "*" || o == "/" || o == "%") return 180;
    if (o == "**") return 190;
    if (o == "<<" || o == ">>") return 210;
    return -1;
  }
  P expr(int min_prec = 0) {
    P l = unary();
    while (l) {
      const int p = prec(peek());
      if (p < 0 || p < min_prec) break;
      const std::string o = peek().s;
      ++i;
      P r = expr(o == "**" ? p : p + 1);
      if (!r) return nullptr;
      auto n = std::make_unique<Node>();
      if (o == "in" || o == "!in") {
        n->k = Node::In;
        n->flag = o == "!in";
      } else if (o == "??") {
        n->k = Node::Coalesce;
      } else if (o == ".." || o == "..=") {
        n->k = Node::Range;
        n->flag = o == "..=";
        n->name2 = o;
      } else {
        n->k = Node::Bin;
        n->op = o;
      }
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
    return postfix();
  }
  bool args(std::vector<P>* out) {  // after '('
    while (!punct(")")) {
      P a = expr();
      if (!a) return false;
      out->push_back(std::move(a));
      if (punct(",")) ++i;
      else if (!punct(")")) {
        fail("Syntax error: expecting ',' or ')' in the argument list, found " + near());
        return false;
      }
    }
    ++i;
    return true;
  }
  P postfix() {
    P e = primary();
    while (e) {
      if (punct(".")) {
        ++i;
        if (peek().t != Tk::Ident) return fail("Syntax error: expecting a method name after '.', found " + near());
        const std::string m = peek().s;
        ++i;
        auto c = std::make_unique<Node>();
        c->k = Node::Call;
        c->name = m;
        c->flag = true;
        c->kids.push_back(std::move(e));
        if (!punct("(")) {
          // the packages' property getters (len, is_empty: strings and arrays; bytes: strings) read
          // as the method call; any other property needs object maps or custom types
          if (m != "len" && m != "is_empty" && m != "bytes") return unsupported("property access (." + m + ")");
          e = std::move(c);
          continue;
        }
        ++i;
        if (!args(&c->kids)) return nullptr;
        if (always_mutates(m) && c->kids[0]->k == Node::Index)
          return unsupported("mutating an element in place (x[i]." + m + "(..))");
        if (always_mutates(m) && c->kids[0]->k == Node::Var && is_const_var(c->kids[0]->name))
          return fail("Syntax error: cannot assign to the constant '" + c->kids[0]->name + "'");
        e = std::move(c);
      } else if (punct("[")) {
        ++i;
        P ix = expr();
        if (!ix) return nullptr;
        if (!expect("]", "to close the index")) return nullptr;
        auto n = std::make_unique<Node>();
        n->k = Node::Index;
        n->kids.push_back(std::move(e));
        n->kids.push_back(std::move(ix));
        e = std::move(n);
      } else {
        break;
      }
    }
    return e;
  }
  P loop_body() {
    if (!punct("{")) return fail("Syntax error: expecting '{' to start the loop body, found " + near());
    ++i;
    ++loops;
    P b = block_body(false);
    --loops;
    if (!b) return nullptr;
    ++i;
    return b;
  }
  P inner_block(const char* what) {
    if (!punct("{")) return fail(std::string("Syntax error: expecting '{' ") + what + ", found " + near());
    ++i;
    P b = block_body(false);
    if (!b) return nullptr;
    ++i;
    return b;
  }
  bool case_literal(Val* v) {
    bool neg = false;
    if (punct("-")) {
      neg = true;
      ++i;
    }
    const Token t = peek();
    if (t.t == Tk::Int) {
      ++i;
      *v = vint(neg ? -t.v : t.v);
      return true;
    }
    if (neg) return false;
    if (t.t == Tk::Str) {
      ++i;
      *v = vstr(t.s);
      return true;
    }
    if (t.t == Tk::Ident && (t.s == "true" || t.s == "false")) {
      ++i;
      *v = vbool(t.s == "true");
      return true;
    }
    if (punct("(") && punct(")", 1)) {
      i += 2;
      *v = Val{};
      return true;
    }
    return false;
  }
  P switch_expr() {
    auto n = std::make_unique<Node>();
    n->k = Node::Switch;
    P scr = expr();
    if (!scr) return nullptr;
    n->kids.push_back(std::move(scr));
    if (!expect("{", "after the switch value")) return nullptr;
    bool seen_default = false;
    std::vector<std::pair<Val, bool>> unguarded;
    while (!punct("}")) {
      if (seen_default) return fail("Syntax error: the wildcard case '_' must be the last case");
      SwitchCase c;
      if (ident("_")) {
        ++i;
        c.wildcard = true;
        seen_default = true;
      } else {
        for (;;) {
          Val v;
          if (!case_literal(&v)) return fail("Syntax error: a switch case must be a constant value, found " + near());
          if (punct("..") || punct("..=")) {
            c.incl = punct("..=");
            ++i;
            Val h;
            if (v.t != VT::Int || !case_literal(&h) || h.t != VT::Int)
              return fail("Syntax error: a switch range case needs integer bounds");
            c.range = true;
            c.lo = v.i;
            c.hi = h.i;
            break;
          }
          c.vals.push_back(v);
          if (!punct("|")) break;
          ++i;
        }
      }
      if (ident("if")) {
        if (c.wildcard) return fail("Syntax error: the wildcard case '_' cannot have a condition");
        ++i;
        c.guard = expr();
        if (!c.guard) return nullptr;
      }
      if (!expect("=>", "after the switch case")) return nullptr;
      if (!c.range && !c.wildcard && !c.guard) {
        for (const Val& v : c.vals) {
          for (auto& u : unguarded)
            if (u.first.t == v.t && u.first.b == v.b && u.first.i == v.i && u.first.s == v.s)
              return fail("Syntax error: duplicated switch case");
          unguarded.push_back({v, true});
        }
      }
      bool blk = false;
      if (punct("{")) {
        c.body = inner_block("");
        blk = true;
      } else {
        c.body = statement();
        if (c.body && (c.body->k == Node::Let || c.body->k == Node::Assign || c.body->k == Node::IndexAssign))
          return fail("Syntax error: a switch case body must be an expression or a block");
      }
      if (!c.body) return nullptr;
      n->cases.push_back(std::move(c));
      if (punct(",")) ++i;
      else if (!punct("}") && !blk) return fail("Syntax error: expecting ',' between switch cases, found " + near());
    }
    ++i;
    return n;
  }
  P primary() {
    const Token t = peek();
    auto n = std::make_unique<Node>();
    if (t.t == Tk::Int) {
      ++i;
      n->lit = vint(t.v);
      return n;
    }
    if (t.t == Tk::Str) {
      ++i;
      n->lit = vstr(t.s);
      return n;
    }
    if (punct("(")) {
      ++i;
      if (punct(")")) {  // ()
        ++i;
        return n;
      }
      P e = expr();
      if (!e) return nullptr;
      if (!punct(")")) return fail("Syntax error: expecting ')', found " + near());
      ++i;
      return e;
    }
    if (punct("[")) {
      ++i;
      n->k = Node::Array;
      while (!punct("]")) {
        P e = expr();
        if (!e) return nullptr;
        n->kids.push_back(std::move(e));
        if (punct(",")) ++i;
        else if (!punct("]")) return fail("Syntax error: expecting ',' or ']' in the array literal, found " + near());
      }
      ++i;
      return n;
    }
    if (punct("{")) {
      ++i;
      P b = block_body(false);
      if (!b) return nullptr;
      ++i;  // '}'
      return b;
    }
    if (punct("|") || punct("||")) return unsupported("closures");
    if (t.t == Tk::Ident) {
      if (const char* u = unsupported_word(t.s)) return unsupported(u);
      ++i;
      if (t.s == "true" || t.s == "false") {
        n->lit = vbool(t.s == "true");
        return n;
      }
      if (t.s == "if") {
        n->k = Node::If;
        P c = expr();
        if (!c) return nullptr;
        n->kids.push_back(std::move(c));
        P th = inner_block("after the if condition");
        if (!th) return nullptr;
        n->kids.push_back(std::move(th));
        if (ident("else")) {
          ++i;
          if (ident("if")) {
            P e = primary();
            if (!e) return nullptr;
            n->kids.push_back(std::move(e));
          } else {
            P e = inner_block("or 'if' after 'else'");
            if (!e) return nullptr;
            n->kids.push_back(std::move(e));
          }
        }
        return n;
      }
      if (t.s == "switch") return switch_expr();
      if (t.s == "while") {
        n->k = Node::While;
        P c = expr();
        if (!c) return nullptr;
        P b = loop_body();
        if (!b) return nullptr;
        n->kids.push_back(std::move(c));
        n->kids.push_back(std::move(b));
        return n;
      }
      if (t.s == "loop") {
        n->k = Node::Loop;
        P b = loop_body();
        if (!b) return nullptr;
        n->kids.push_back(std::move(b));
        return n;
      }
      if (t.s == "do") {
        n->k = Node::DoWhile;
        P b = loop_body();
        if (!b) return nullptr;
        if (!ident("while") && !ident("until")) return fail("Syntax error: expecting 'while' or 'until' after the do block");
        n->flag = ident("until");
        ++i;
        P c = expr();
        if (!c) return nullptr;
        n->kids.push_back(std::move(b));
        n->kids.push_back(std::move(c));
        return n;
      }
      if (t.s == "for") {
        n->k = Node::For;
        const bool paren = punct("(");
        if (paren) ++i;
        if (peek().t != Tk::Ident || is_kw(peek().s)) return fail("Syntax error: expecting a loop variable after 'for'");
        n->name = peek().s;
        ++i;
        if (paren) {
          if (!expect(",", "after the loop variable")) return nullptr;
          if (peek().t != Tk::Ident || is_kw(peek().s)) return fail("Syntax error: expecting the counter variable");
          n->name2 = peek().s;
          ++i;
          if (!expect(")", "after the counter variable")) return nullptr;
        }
        if (!ident("in")) return fail("Syntax error: expecting 'in' after the loop variable, found " + near());
        ++i;
        P it = expr();
        if (!it) return nullptr;
        if (it->k == Node::Call && !it->flag && it->name == "range") {  // range(a, b): a..b
          if (it->kids.size() != 2) return unsupported("range() with a step");
          it->k = Node::Range;
          it->flag = false;
          it->name2 = "range";
        }
        n->kids.push_back(std::move(it));
        scopes.emplace_back();
        declare(n->name, false);
        if (!n->name2.empty()) declare(n->name2, false);
        P b = loop_body();
        scopes.pop_back();
        if (!b) return nullptr;
        n->kids.push_back(std::move(b));
        return n;
      }
      if (t.s == "let" || t.s == "const" || t.s == "else" || t.s == "fn" || t.s == "in" || t.s == "until" ||
          t.s == "break" || t.s == "continue" || t.s == "return")
        return fail("Syntax error: unexpected '" + t.s + "'");
      if (!punct("(")) {
        n->k = Node::Var;
        n->name = t.s;
        return n;
      }
      ++i;
      n->k = Node::Call;
      n->name = t.s;
      if (!args(&n->kids)) return nullptr;
      return n;
    }
    if (t.t == Tk::End) return fail("Syntax error: expecting an expression, found end of script");
    return fail("Syntax error: unexpected " + near());
  }
};

// ranges are values only as the right side of `in` / `!in` and as a `for` iterable
bool check_ranges(const Node* n, bool allowed, std::string* err) {
  if (n->k == Node::Range && !allowed) {
    *err = std::string(kUnsupported) + "range values outside `for` and `in`";
    return false;
  }
  for (size_t k = 0; k < n->kids.size(); ++k) {
    const bool ok = (n->k == Node::In && k == 1) || (n->k == Node::For && k == 0);
    if (!check_ranges(n->kids[k].get(), ok, err)) return false;
  }
  for (const SwitchCase& c : n->cases) {
    if (c.guard && !check_ranges(c.guard.get(), false, err)) return false;
    if (!check_ranges(c.body.get(), false, err)) return false;
  }
  return true;
}

// call resolution, as rhai's: a script function of that name and arity, else a member policy
// (a native function of no arguments), else a built-in; anything else is "Function not found"
// when called (after its arguments ran)
void resolve(Node* n, const ExprAst& ast, const std::vector<std::string>& members) {
  if (n->k == Node::Call) {
    n->fn = -1;
    n->slot = -1;
    n->builtin = -1;
    for (size_t f = 0; f < ast.fns.size(); ++f)
      if (!n->flag && ast.fns[f].name == n->name && ast.fns[f].params.size() == n->kids.size()) n->fn = (int)f;
    if (n->fn < 0 && !n->flag && n->kids.empty())
      for (size_t m = 0; m < members.size(); ++m)
        if (members[m] == n->name) n->slot = (int)m;
    if (n->fn < 0 && n->slot < 0) n->builtin = builtin_id(n->name, n->kids.size());
  }
  for (P& k : n->kids) resolve(k.get(), ast, members);
  for (SwitchCase& c : n->cases) {
    if (c.guard) resolve(c.guard.get(), ast, members);
    resolve(c.body.get(), ast, members);
  }
}

// a call of a standard-package function the engine does not implement (kStdRefused): its name
const Node* refused_call(const Node* n) {
  if (n->k == Node::Call && n->fn < 0 && n->slot < 0 && n->builtin < 0 && std_refused(n->name)) return n;
  for (const P& k : n->kids)
    if (const Node* r = refused_call(k.get())) return r;
  for (const SwitchCase& c : n->cases) {
    if (c.guard)
      if (const Node* r = refused_call(c.guard.get())) return r;
    if (const Node* r = refused_call(c.body.get())) return r;
  }
  return nullptr;
}

// range(a, b) outside a `for` would be a range value: not supported (check_ranges)
bool stray_range_call(const Node* n) {
  if (n->k == Node::Call && n->name == "range" && n->fn < 0 && n->slot < 0 && n->builtin < 0) return true;
  for (const P& k : n->kids)
    if (stray_range_call(k.get())) return true;
  for (const SwitchCase& c : n->cases)
    if ((c.guard && stray_range_call(c.guard.get())) || stray_range_call(c.body.get())) return true;
  return false;
}

// ------------------------------------------------------------------------------------------
// Strings as Rust's str methods see them (rhai's string functions are Rust's): code points of
// valid UTF-8 (every string here is), White_Space, and the full case mappings with Σ's
// Final_Sigma context (unicode_data.hpp, Unicode 13.0)
// ------------------------------------------------------------------------------------------
std::vector<uint32_t> cps_of(const std::string& s) {
  std::vector<uint32_t> out;
  for (size_t k = 0; k < s.size();) {
    const unsigned char c = (unsigned char)s[k];
    const size_t n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
    uint32_t v = n == 1 ? c : n == 2 ? (c & 0x1Fu) : n == 3 ? (c & 0x0Fu) : (c & 0x07u);
    for (size_t j = 1; j < n && k + j < s.size(); ++j) v = (v << 6) | ((unsigned char)s[k + j] & 0x3Fu);
    out.push_back(v);
    k += n;
  }
  return out;
}
std::string utf8_of(const std::vector<uint32_t>& v, size_t lo = 0, size_t hi = SIZE_MAX) {
  std::string o;
  for (size_t k = lo; k < v.size() && k < hi; ++k) put_utf8(v[k], &o);
  return o;
}
bool uni_ws(uint32_t c) {
  return (c >= 9 && c <= 13) || c == ' ' || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
bool uni_in(const UniRange* r, uint32_t n, uint32_t c) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t m = (lo + hi) / 2;
    if (r[m].hi < c) lo = m + 1;
    else hi = m;
  }
  return lo < n && r[lo].lo <= c;
}
const UniCaseMap* uni_map(const UniCaseMap* t, uint32_t n, uint32_t c) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t m = (lo + hi) / 2;
    if (t[m].cp < c) lo = m + 1;
    else hi = m;
  }
  return lo < n && t[lo].cp == c ? &t[lo] : nullptr;
}
bool uni_ignorable(uint32_t c) { return uni_in(kUniCaseIgnorable, kUniCaseIgnorableN, c); }
bool uni_cased(uint32_t c) { return uni_in(kUniCased, kUniCasedN, c); }  // (and not Case_Ignorable)
// str::to_lowercase / str::to_uppercase
std::string str_case(const std::string& s, bool upper) {
  const std::vector<uint32_t> v = cps_of(s);
  std::vector<uint32_t> o;
  for (size_t k = 0; k < v.size(); ++k) {
    const uint32_t c = v[k];
    if (!upper && c == 0x3A3) {  // Σ: ς at the end of a word (Unicode 3.13 Final_Sigma)
      size_t j = k;
      while (j > 0 && uni_ignorable(v[j - 1])) --j;
      bool fin = j > 0 && uni_cased(v[j - 1]);
      if (fin) {
        j = k + 1;
        while (j < v.size() && uni_ignorable(v[j])) ++j;
        fin = !(j < v.size() && uni_cased(v[j]));
      }
      o.push_back(fin ? 0x3C2 : 0x3C3);
      continue;
    }
    const UniCaseMap* m = upper ? uni_map(kUniUpper, kUniUpperN, c) : uni_map(kUniLower, kUniLowerN, c);
    if (!m) o.push_back(c);
    else
      for (uint32_t j = 0; j < m->n; ++j) o.push_back(m->m[j]);
  }
  return utf8_of(o);
}
// rhai's checked ** << >> on i64: a negative shift shifts the other way; 64 or more bits, an exponent
// outside [0, u32::MAX] or a power past i64 is an error; >> is arithmetic (slots.hpp int_pow_shift
// is the device form)
bool int_pow_shift(const std::string& op, int64_t x, int64_t y, int64_t* r, std::string* err) {
  const std::string ex = std::to_string(x) + " " + op + " " + std::to_string(y);
  if (op == "**") {
    if (y > (int64_t)0xFFFFFFFFll) return *err = "Integer raised to too large an index: " + ex, false;
    if (y < 0) return *err = "Integer raised to a negative index: " + ex, false;
    long long v = 1;
    for (int64_t k = 0; k < y; ++k) {
      if (__builtin_mul_overflow(v, (long long)x, &v)) return *err = "Exponential overflow: " + ex, false;
      if (v == 0 || ((v == 1 || v == -1) && (x == 1 || x == -1))) {  // 0, 1, -1: the rest is a parity
        if (v != 0 && x == -1) v = (y % 2 == 0) ? 1 : -1;
        break;
      }
    }
    *r = v;
    return true;
  }
  const bool left = op == "<<";
  const std::string name = left ? "Left-shift" : "Right-shift";
  if (y > (int64_t)0xFFFFFFFFll || y == INT64_MIN) return *err = name + " by too many bits: " + ex, false;
  if (y < 0) return int_pow_shift(left ? ">>" : "<<", x, -y, r, err);
  if (y >= 64) return *err = name + " by too many bits: " + ex, false;
  *r = left ? (int64_t)((uint64_t)x << y) : (x >> y);
  return true;
}

// rhai's calc_offset_len (start counts from the end when negative, clamped; len clamped)
void offset_len(size_t n, int64_t start, int64_t len, size_t* st, size_t* ln) {
  size_t s0;
  if (start < 0) {
    const uint64_t a = (uint64_t)0 - (uint64_t)start;
    s0 = a >= n ? 0 : n - (size_t)a;
  } else if ((uint64_t)start >= n) {
    *st = n;
    *ln = 0;
    return;
  } else {
    s0 = (size_t)start;
  }
  *st = s0;
  *ln = len <= 0 ? 0 : (uint64_t)len > n - s0 ? n - s0 : (size_t)len;
}
// an element position for get / set / remove: negative from the end; out of range: none
bool elem_index(size_t n, int64_t i, size_t* at) {
  if (i < 0) {
    const uint64_t a = (uint64_t)0 - (uint64_t)i;
    if (a > n) return false;
    *at = n - (size_t)a;
    return true;
  }
  if ((uint64_t)i >= n) return false;
  *at = (size_t)i;
  return true;
}
// the characters [from, from + len) of a string by rhai's sub_string rules
std::string sub_chars(const std::string& s, int64_t start, int64_t len) {
  const std::vector<uint32_t> v = cps_of(s);
  if (v.empty() || len <= 0) return "";
  size_t off;
  if (start < 0) {
    const uint64_t a = (uint64_t)0 - (uint64_t)start;
    off = a > v.size() ? 0 : v.size() - (size_t)a;
  } else if ((uint64_t)start >= v.size()) {
    return "";
  } else {
    off = (size_t)start;
  }
  const size_t take = (uint64_t)len > v.size() - off ? v.size() - off : (size_t)len;
  return utf8_of(v, off, off + take);
}
// Rust's str::split / rsplit / splitn / rsplitn over a string pattern (an empty pattern matches at
// every character boundary, both ends included); n = 0: no limit
std::vector<std::string> str_split(const std::string& s, const std::string& d, bool rev, size_t n) {
  std::vector<size_t> at;  // match starts (byte offsets), left to right
  if (d.empty()) {
    for (size_t k = 0; k <= s.size(); ++k)
      if (k == s.size() || ((unsigned char)s[k] & 0xC0u) != 0x80u) at.push_back(k);
  } else if (!rev) {
    for (size_t k = s.find(d); k != std::string::npos; k = s.find(d, k + d.size())) at.push_back(k);
  } else {  // right to left, non-overlapping
    std::vector<size_t> r;
    for (size_t e = s.size(); e >= d.size();) {
      const size_t k = s.rfind(d, e - d.size());
      if (k == std::string::npos) break;
      r.push_back(k);
      if (k < d.size()) break;
      e = k;
    }
    at.assign(r.rbegin(), r.rend());
  }
  std::vector<std::string> out;
  if (!rev) {
    size_t from = 0;
    for (size_t k : at) {
      if (n && out.size() + 1 == n) break;
      out.push_back(s.substr(from, k - from));
      from = k + d.size();
    }
    out.push_back(s.substr(from));
  } else {
    size_t to = s.size();
    for (size_t j = at.size(); j-- > 0;) {
      if (n && out.size() + 1 == n) break;
      const size_t k = at[j];
      out.push_back(s.substr(k + d.size(), to - k - d.size()));
      to = k;
    }
    out.push_back(s.substr(0, to));
  }
  return out;
}
// i64::from_str_radix(s.trim(), radix) and its ParseIntError texts
bool parse_i64(const std::string& text, int64_t radix, int64_t* out, std::string* err) {
  std::vector<uint32_t> v = cps_of(text);
  size_t a = 0, b = v.size();
  while (a < b && uni_ws(v[a])) ++a;
  while (b > a && uni_ws(v[b - 1])) --b;
  if (a == b) {
    *err = "cannot parse integer from empty string";
    return false;
  }
  bool neg = false;
  if (v[a] == '+' || v[a] == '-') {
    neg = v[a] == '-';
    ++a;
    if (a == b) {
      *err = "invalid digit found in string";
      return false;
    }
  }
  long long r = 0;
  for (size_t k = a; k < b; ++k) {
    const uint32_t c = v[k];
    int64_t d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'z' ? c - 'a' + 10 : c >= 'A' && c <= 'Z' ? c - 'A' + 10 : 99;
    if (d >= radix) {
      *err = "invalid digit found in string";
      return false;
    }
    if (__builtin_mul_overflow(r, (long long)radix, &r) ||
        (neg ? __builtin_sub_overflow(r, (long long)d, &r) : __builtin_add_overflow(r, (long long)d, &r))) {
      *err = neg ? "number too small to fit in target type" : "number too large to fit in target type";
      return false;
    }
  }
  *out = r;
  return true;
}
std::string radix_text(int64_t v, unsigned bits) {  // Rust's {:x} / {:o} / {:b} of an i64 (two's complement)
  uint64_t u = (uint64_t)v;
  const char* dig = "0123456789abcdef";
  std::string o;
  const unsigned mask = (1u << bits) - 1u;
  do {
    o.push_back(dig[u & mask]);
    u >>= bits;
  } while (u);
  std::reverse(o.begin(), o.end());
  return o;
}

// ------------------------------------------------------------------------------------------
// Interpreter
// ------------------------------------------------------------------------------------------
enum Flow { OK, ERR, BRK, CNT, RET };

std::string limit_ops() {
  return "engine limit: more than " + std::to_string(kMaxScriptOps) + " loop iterations and script-function calls";
}
std::string limit_alloc() {
  return "engine limit: more than " + std::to_string(kMaxScriptAlloc) + " bytes of strings and arrays built";
}
std::string limit_depth() {
  return "engine limit: arrays nested more than " + std::to_string(kMaxCompareDepth) + " deep in a comparison";
}

struct Interp {
  const ExprAst* ast = nullptr;
  std::function<bool(uint32_t)> ok;
  std::vector<std::pair<std::string, Val>> vars;
  size_t base = 0;  // the current function frame's first variable
  std::vector<uint32_t> called;
  std::vector<uint8_t> seen;
  std::string err;
  uint32_t ops = 0, alloc = 0, depth = 0;
  uint64_t steps = 0;  // nodes evaluated (the cost of one run, for the truth-table decision)
  Val fv;              // the value a `break` / `return` carries to its loop / call              // the value a `break` / `return` carries to its loop / call  // nodes evaluated (the cost of one run, for the truth-table decision)
  explicit Interp(std::function<bool(uint32_t)> f) : ok(std::move(f)) {}

  Flow fail(const std::string& m) {
    err = m;
    return ERR;
  }
  Flow nf(const std::string& fn, const std::vector<const Val*>& a) {
    std::string s = "Function not found: " + fn + " (";
    for (size_t k = 0; k < a.size(); ++k) s += (k ? ", " : "") + std::string(tname(a[k]->t));
    return fail(s + ")");
  }
  bool charge(uint64_t n) {
    if (n > (uint64_t)(kMaxScriptAlloc - alloc)) return false;
    alloc += (uint32_t)n;
    return true;
  }
  Val* lookup(const std::string& name) {
    for (size_t k = vars.size(); k-- > base;)
      if (vars[k].first == name) return &vars[k].second;
    return nullptr;
  }
  // deep equality: 1 / 0, -1 past kMaxCompareDepth (slots.hpp veq walks in the same order)
  int eq(const Val& a, const Val& b, uint32_t d) const {
    if (a.t != b.t) return 0;
    switch (a.t) {
      case VT::Unit: return 1;
      case VT::Bool: return a.b == b.b;
      case VT::Int: return a.i == b.i;
      case VT::Str: return a.s == b.s;
      case VT::Arr: {
        if (a.a.size() != b.a.size()) return 0;
        if (a.a.empty()) return 1;
        if (d == kMaxCompareDepth) return -1;
        for (size_t k = 0; k < a.a.size(); ++k) {
          const int e = eq(a.a[k], b.a[k], d + 1);
          if (e != 1) return e;
        }
        return 1;
      }
    }
    return 0;
  }
  // to_string of a non-array value
  static bool text(const Val& v, std::string* out) {
    switch (v.t) {
      case VT::Unit: out->clear(); return true;
      case VT::Bool: *out = v.b ? "true" : "false"; return true;
      case VT::Int: *out = std::to_string(v.i); return true;
      case VT::Str: *out = v.s; return true;
      default: return false;
    }
  }
  static size_t chars(const std::string& s) {
    size_t n = 0;
    for (unsigned char c : s) n += (c & 0xC0u) != 0x80u;
    return n;
  }
  static bool index_of(int64_t i, size_t n, size_t* at) {
    if (i < 0) i += (int64_t)n;
    if (i < 0 || i >= (int64_t)n) return false;
    *at = (size_t)i;
    return true;
  }
  Flow bounds(int64_t i, size_t n) {
    const std::string s = "Array index " + std::to_string(i) + " out of bounds: ";
    if (n == 0) return fail(s + "array is empty");
    if (n == 1) return fail(s + "only 1 element in array");
    return fail(s + "only " + std::to_string(n) + " elements in array");
  }
  Flow not_indexable(const Val& v) {
    if (v.t == VT::Str) return fail(std::string(kUnsupported) + "indexing a string (characters)");
    return fail(std::string("Indexer unavailable: ") + tname(v.t));
  }

  // A built-in over its arguments a (a[0] by value: the function changes it in place when rhai's
  // takes `&mut`, and the caller stores it back for a method-style call on a variable). Charges
  // against kMaxScriptAlloc (slots.hpp charges the same): a new string its bytes, a new or copied
  // array 16 B a cell; slices (sub_string, trim, split pieces, extract, pop, ...) are free.
  Flow builtin(int fid, const std::string& name, std::vector<Val>& a, Val* out) {
    std::vector<const Val*> ap;
    for (const Val& v : a) ap.push_back(&v);
    auto refuse = [&](const char* why) {
      std::string s = std::string(kUnsupported) + name + " (";
      for (size_t k = 0; k < a.size(); ++k) s += (k ? ", " : "") + std::string(tname(a[k].t));
      return fail(s + ")" + why);
    };
    auto is = [&](size_t k, VT t) { return a.size() > k && a[k].t == t; };
    auto new_str = [&](std::string s) -> Flow {
      if (!charge(s.size())) return fail(limit_alloc());
      *out = vstr(std::move(s));
      return OK;
    };
    *out = Val{};
    switch (fid) {
      case F_LEN:
      case F_IS_EMPTY: {
        size_t n;
        if (a[0].t == VT::Arr) n = a[0].a.size();
        else if (a[0].t == VT::Str) n = chars(a[0].s);
        else return nf(name, ap);
        *out = fid == F_LEN ? vint((int64_t)n) : vbool(n == 0);
        return OK;
      }
      case F_TYPE_OF: *out = vstr(tname(a[0].t)); return OK;
      case F_TO_STRING: {
        if (a[0].t == VT::Str) {
          *out = a[0];
          return OK;
        }
        std::string s;
        if (!text(a[0], &s)) return fail(std::string(kUnsupported) + "converting an array to a string");
        return new_str(s);
      }
      case F_PUSH: {
        if (a[0].t != VT::Arr) return nf(name, ap);
        if (!charge(16ull * (a[0].a.size() + 1))) return fail(limit_alloc());
        a[0].a.push_back(a[1]);
        return OK;
      }
      case F_CONTAINS:
      case F_INDEX_OF:
      case F_INDEX_OF_FROM: {
        const Val &c = a[0], &x = a[1];
        if (fid == F_INDEX_OF_FROM && !is(2, VT::Int)) return nf(name, ap);
        if (c.t == VT::Arr) {
          size_t from = 0, ln;
          if (fid == F_INDEX_OF_FROM) offset_len(c.a.size(), a[2].i, 0, &from, &ln);
          for (size_t k = from; k < c.a.size(); ++k) {
            const int r = eq(c.a[k], x, 0);
            if (r < 0) return fail(limit_depth());
            if (r) {
              *out = fid == F_CONTAINS ? vbool(true) : vint((int64_t)k);
              return OK;
            }
          }
          *out = fid == F_CONTAINS ? vbool(false) : vint(-1);
          return OK;
        }
        if (c.t == VT::Str && x.t == VT::Str) {
          if (fid == F_CONTAINS) {
            *out = vbool(c.s.find(x.s) != std::string::npos);
            return OK;
          }
          // index_of: the character position of the first match at or after `start` characters
          int64_t r = -1;
          if (!c.s.empty()) {
            const std::vector<uint32_t> v = cps_of(c.s);
            size_t from = 0;
            bool none = false;
            if (fid == F_INDEX_OF_FROM) {
              const int64_t st = a[2].i;
              if (st < 0) {
                const uint64_t m = (uint64_t)0 - (uint64_t)st;
                from = m > v.size() ? 0 : utf8_of(v, 0, v.size() - (size_t)m).size();
              } else if ((uint64_t)st >= v.size()) {
                none = st != 0;
              } else {
                from = utf8_of(v, 0, (size_t)st).size();
              }
            }
            const size_t k = none ? std::string::npos : c.s.find(x.s, from);
            if (k != std::string::npos) r = (int64_t)chars(c.s.substr(0, k));
          }
          *out = vint(r);
          return OK;
        }
        return nf(name, ap);
      }
      case F_STARTS_WITH:
      case F_ENDS_WITH: {
        if (a[0].t != VT::Str || a[1].t != VT::Str) return nf(name, ap);
        const std::string &h = a[0].s, &n = a[1].s;
        const bool r = n.size() <= h.size() && (fid == F_STARTS_WITH ? h.compare(0, n.size(), n) == 0
                                                                      : h.compare(h.size() - n.size(), n.size(), n) == 0);
        *out = vbool(r);
        return OK;
      }
      // ---- integers (ArithmeticPackage, LogicPackage, BasicMathPackage)
      case F_ABS:
      case F_SIGN:
      case F_IS_ZERO:
      case F_IS_ODD:
      case F_IS_EVEN:
      case F_TO_HEX:
      case F_TO_OCTAL:
      case F_TO_BINARY: {
        if (a[0].t != VT::Int) return nf(name, ap);
        const int64_t x = a[0].i;
        switch (fid) {
          case F_ABS:
            if (x == INT64_MIN) return fail("Negation overflow: -" + std::to_string(x));
            *out = vint(x < 0 ? -x : x);
            return OK;
          case F_SIGN: *out = vint(x < 0 ? -1 : x > 0 ? 1 : 0); return OK;
          case F_IS_ZERO: *out = vbool(x == 0); return OK;
          case F_IS_ODD: *out = vbool((x & 1) != 0); return OK;
          case F_IS_EVEN: *out = vbool((x & 1) == 0); return OK;
          default: return new_str(radix_text(x, fid == F_TO_HEX ? 4 : fid == F_TO_OCTAL ? 3 : 1));
        }
      }
      case F_MAX:
      case F_MIN:
        if (a[0].t != VT::Int || a[1].t != VT::Int) return nf(name, ap);
        *out = vint(fid == F_MAX ? std::max(a[0].i, a[1].i) : std::min(a[0].i, a[1].i));
        return OK;
      case F_PARSE_INT:
      case F_PARSE_INT_R: {
        if (a[0].t != VT::Str || (fid == F_PARSE_INT_R && a[1].t != VT::Int)) return nf(name, ap);
        const int64_t radix = fid == F_PARSE_INT_R ? a[1].i : 10;
        if (radix < 2 || radix > 36) return fail("Invalid radix: '" + std::to_string(radix) + "'");
        int64_t v;
        std::string e;
        if (!parse_i64(a[0].s, radix, &v, &e)) return fail("Error parsing integer number '" + a[0].s + "': " + e);
        *out = vint(v);
        return OK;
      }
      // ---- strings (BasicStringPackage, MoreStringPackage)
      case F_TO_UPPER:
      case F_TO_LOWER:
      case F_MAKE_UPPER:
      case F_MAKE_LOWER: {
        if (a[0].t != VT::Str) return nf(name, ap);
        const std::string r = str_case(a[0].s, fid == F_TO_UPPER || fid == F_MAKE_UPPER);
        if (!charge(r.size())) return fail(limit_alloc());
        if (fid == F_TO_UPPER || fid == F_TO_LOWER) *out = vstr(r);
        else a[0].s = r;
        return OK;
      }
      case F_TRIM: {
        if (a[0].t != VT::Str) return nf(name, ap);
        const std::vector<uint32_t> v = cps_of(a[0].s);
        size_t lo = 0, hi = v.size();
        while (lo < hi && uni_ws(v[lo])) ++lo;
        while (hi > lo && uni_ws(v[hi - 1])) --hi;
        a[0].s = utf8_of(v, lo, hi);
        return OK;
      }
      case F_SUB_STRING:
      case F_SUB_STRING_N:
      case F_CROP:
      case F_CROP_N: {
        const bool n3 = fid == F_SUB_STRING_N || fid == F_CROP_N;
        if (a[0].t != VT::Str || a[1].t != VT::Int || (n3 && a[2].t != VT::Int)) return nf(name, ap);
        const int64_t len = n3 ? a[2].i : (int64_t)a[0].s.size();
        std::string r = sub_chars(a[0].s, a[1].i, len);
        if (fid == F_SUB_STRING || fid == F_SUB_STRING_N) *out = vstr(std::move(r));
        else a[0].s = std::move(r);
        return OK;
      }
      case F_REPLACE: {
        if (a[0].t != VT::Str || a[1].t != VT::Str || a[2].t != VT::Str) return nf(name, ap);
        if (a[0].s.empty()) return OK;
        const std::vector<std::string> parts = str_split(a[0].s, a[1].s, false, 0);
        std::string r;
        for (size_t k = 0; k < parts.size(); ++k) r += (k ? a[2].s : "") + parts[k];
        if (!charge(r.size())) return fail(limit_alloc());
        a[0].s = std::move(r);
        return OK;
      }
      case F_SPLIT_WS:
      case F_SPLIT:
      case F_SPLIT_N:
      case F_SPLIT_REV:
      case F_SPLIT_REV_N: {
        if (fid == F_SPLIT && a[0].t == VT::Arr && a[1].t == VT::Int) {  // array: cut off the tail from index
          size_t st, ln;
          offset_len(a[0].a.size(), a[1].i, INT64_MAX, &st, &ln);
          out->t = VT::Arr;
          out->a.assign(a[0].a.begin() + (std::ptrdiff_t)st, a[0].a.end());
          a[0].a.resize(st);
          return OK;
        }
        if (a[0].t != VT::Str) return nf(name, ap);
        std::vector<std::string> parts;
        if (fid == F_SPLIT_WS) {
          const std::vector<uint32_t> v = cps_of(a[0].s);
          for (size_t k = 0; k < v.size();) {
            while (k < v.size() && uni_ws(v[k])) ++k;
            const size_t b = k;
            while (k < v.size() && !uni_ws(v[k])) ++k;
            if (k > b) parts.push_back(utf8_of(v, b, k));
          }
        } else if (fid == F_SPLIT && a[1].t == VT::Int) {  // at a character position
          const std::vector<uint32_t> v = cps_of(a[0].s);
          const int64_t i = a[1].i;
          size_t at;
          if (i <= 0) {
            const uint64_t m = (uint64_t)0 - (uint64_t)i;
            at = m > v.size() ? 0 : v.size() - (size_t)m;
          } else {
            at = (uint64_t)i > v.size() ? v.size() : (size_t)i;
          }
          parts = {utf8_of(v, 0, at), utf8_of(v, at)};
        } else {
          if (a[1].t != VT::Str) return nf(name, ap);
          const bool lim = fid == F_SPLIT_N || fid == F_SPLIT_REV_N;
          if (lim && a[2].t != VT::Int) return nf(name, ap);
          size_t n = 0;
          if (lim) n = a[2].i < 1 ? 1 : (size_t)std::min<int64_t>(a[2].i, INT64_MAX);
          parts = str_split(a[0].s, a[1].s, fid == F_SPLIT_REV || fid == F_SPLIT_REV_N, n);
        }
        if (!charge(16ull * parts.size())) return fail(limit_alloc());
        out->t = VT::Arr;
        for (std::string& p : parts) out->a.push_back(vstr(std::move(p)));
        return OK;
      }
      case F_BYTES:
        if (a[0].t != VT::Str) return nf(name, ap);
        *out = vint((int64_t)a[0].s.size());
        return OK;
      // ---- arrays (BasicArrayPackage), and the string forms of append / remove / clear / truncate
      case F_APPEND:
        if (a[0].t == VT::Arr && a[1].t == VT::Arr) {
          if (!charge(16ull * (a[0].a.size() + a[1].a.size()))) return fail(limit_alloc());
          a[0].a.insert(a[0].a.end(), a[1].a.begin(), a[1].a.end());
          return OK;
        }
        if (a[0].t == VT::Str) {
          std::string t;
          if (!text(a[1], &t)) return fail(std::string(kUnsupported) + "converting an array to a string");
          if (!charge(a[0].s.size() + t.size())) return fail(limit_alloc());
          a[0].s += t;
          return OK;
        }
        return nf(name, ap);
      case F_INSERT: {
        if (a[0].t != VT::Arr || a[1].t != VT::Int) return nf(name, ap);
        if (!charge(16ull * (a[0].a.size() + 1))) return fail(limit_alloc());
        size_t st, ln;
        offset_len(a[0].a.size(), a[1].i, 0, &st, &ln);
        a[0].a.insert(a[0].a.begin() + (std::ptrdiff_t)st, a[2]);
        return OK;
      }
      case F_POP:
      case F_SHIFT:
        if (a[0].t == VT::Str) return refuse(": it returns a character");
        if (a[0].t != VT::Arr) return nf(name, ap);
        if (!a[0].a.empty()) {
          if (fid == F_POP) {
            *out = std::move(a[0].a.back());
            a[0].a.pop_back();
          } else {
            *out = std::move(a[0].a.front());
            a[0].a.erase(a[0].a.begin());
          }
        }
        return OK;
      case F_REMOVE: {
        if (a[0].t == VT::Str && a[1].t == VT::Str) {  // every occurrence of the substring
          if (a[1].s.empty() || a[0].s.empty()) return OK;
          std::string r;
          for (const std::string& p : str_split(a[0].s, a[1].s, false, 0)) r += p;
          if (!charge(r.size())) return fail(limit_alloc());
          a[0].s = std::move(r);
          return OK;
        }
        if (a[0].t != VT::Arr || a[1].t != VT::Int) return nf(name, ap);
        size_t at;
        if (!elem_index(a[0].a.size(), a[1].i, &at)) return OK;
        if (!charge(16ull * (a[0].a.size() - 1))) return fail(limit_alloc());
        *out = std::move(a[0].a[at]);
        a[0].a.erase(a[0].a.begin() + (std::ptrdiff_t)at);
        return OK;
      }
      case F_REVERSE:
        if (a[0].t != VT::Arr) return nf(name, ap);
        if (!charge(16ull * a[0].a.size())) return fail(limit_alloc());
        std::reverse(a[0].a.begin(), a[0].a.end());
        return OK;
      case F_SORT: {
        if (a[0].t != VT::Arr) return nf(name, ap);
        std::vector<Val>& v = a[0].a;
        if (v.size() <= 1) return OK;
        for (const Val& e : v)
          if (e.t != v[0].t) return fail("Function not found: sort() cannot be called with elements of different types");
        if (v[0].t == VT::Arr || v[0].t == VT::Unit) return OK;
        if (!charge(16ull * v.size())) return fail(limit_alloc());
        std::stable_sort(v.begin(), v.end(), [](const Val& x, const Val& y) {
          if (x.t == VT::Int) return x.i < y.i;
          if (x.t == VT::Bool) return !x.b && y.b;
          return x.s < y.s;  // (byte order: Rust's str ordering)
        });
        return OK;
      }
      case F_CLEAR:
        if (a[0].t == VT::Arr) a[0].a.clear();
        else if (a[0].t == VT::Str) a[0].s.clear();
        else return nf(name, ap);
        return OK;
      case F_TRUNCATE:
      case F_CHOP: {
        if (a[1].t != VT::Int) return nf(name, ap);
        const int64_t n = a[1].i;
        if (a[0].t == VT::Str && fid == F_TRUNCATE) {
          const std::vector<uint32_t> v = cps_of(a[0].s);
          if (n <= 0) a[0].s.clear();
          else if ((uint64_t)n < v.size()) a[0].s = utf8_of(v, 0, (size_t)n);
          return OK;
        }
        if (a[0].t != VT::Arr) return nf(name, ap);
        std::vector<Val>& v = a[0].a;
        if (n <= 0) v.clear();
        else if ((uint64_t)n < v.size()) {
          if (fid == F_TRUNCATE) v.resize((size_t)n);
          else v.erase(v.begin(), v.end() - (std::ptrdiff_t)n);
        }
        return OK;
      }
      case F_GET:
      case F_SET: {
        if (a[0].t == VT::Str && a[1].t == VT::Int) return refuse(": characters");
        if (a[0].t != VT::Arr || a[1].t != VT::Int) return nf(name, ap);
        size_t at;
        if (!elem_index(a[0].a.size(), a[1].i, &at)) return OK;
        if (fid == F_GET) {
          *out = a[0].a[at];
          return OK;
        }
        if (!charge(16ull * a[0].a.size())) return fail(limit_alloc());
        a[0].a[at] = a[2];
        return OK;
      }
      case F_EXTRACT:
      case F_EXTRACT_N:
      case F_DRAIN:
      case F_RETAIN: {
        const bool n3 = fid != F_EXTRACT;
        if (a[0].t != VT::Arr || a[1].t != VT::Int || (n3 && a[2].t != VT::Int)) return nf(name, ap);
        std::vector<Val>& v = a[0].a;
        out->t = VT::Arr;
        const int64_t len = n3 ? a[2].i : INT64_MAX;
        if (v.empty() || len <= 0) return OK;
        size_t st, ln;
        offset_len(v.size(), a[1].i, len, &st, &ln);
        if (ln == 0) return OK;
        const auto b = v.begin() + (std::ptrdiff_t)st, e = b + (std::ptrdiff_t)ln;
        if (fid == F_EXTRACT || fid == F_EXTRACT_N) {
          out->a.assign(b, e);
        } else if (fid == F_DRAIN) {  // the range out; the rest is a copy
          if (!charge(16ull * (v.size() - ln))) return fail(limit_alloc());
          out->a.assign(b, e);
          v.erase(b, e);
        } else {  // retain the range; what is cut off is a copy
          if (!charge(16ull * (v.size() - ln))) return fail(limit_alloc());
          out->a.assign(v.begin(), b);
          out->a.insert(out->a.end(), e, v.end());
          std::vector<Val> keep(b, e);
          v = std::move(keep);
        }
        return OK;
      }
      case F_SPLICE: {
        if (a[0].t != VT::Arr || a[1].t != VT::Int || a[2].t != VT::Int || a[3].t != VT::Arr) return nf(name, ap);
        std::vector<Val>& v = a[0].a;
        size_t st = 0, ln = 0;
        if (!v.empty()) offset_len(v.size(), a[1].i, a[2].i, &st, &ln);
        if (!charge(16ull * (v.size() - ln + a[3].a.size()))) return fail(limit_alloc());
        if (v.empty()) {
          v = a[3].a;
        } else {
          v.erase(v.begin() + (std::ptrdiff_t)st, v.begin() + (std::ptrdiff_t)(st + ln));
          v.insert(v.begin() + (std::ptrdiff_t)st, a[3].a.begin(), a[3].a.end());
        }
        return OK;
      }
      case F_DEDUP: {
        if (a[0].t != VT::Arr) return nf(name, ap);
        std::vector<Val>& v = a[0].a;
        if (v.size() <= 1) return OK;
        std::vector<Val> r;
        r.push_back(v[0]);
        for (size_t k = 1; k < v.size(); ++k) {
          const int e = eq(v[k], r.back(), 0);
          if (e < 0) return fail(limit_depth());
          if (!e) r.push_back(v[k]);
        }
        if (!charge(16ull * r.size())) return fail(limit_alloc());
        v = std::move(r);
        return OK;
      }
      case F_PAD: {
        if (a[0].t == VT::Str && a[1].t == VT::Int) return refuse(": padding strings");
        if (a[0].t != VT::Arr || a[1].t != VT::Int) return nf(name, ap);
        const int64_t n = a[1].i;
        if (n <= 0 || (uint64_t)n <= a[0].a.size()) return OK;
        if ((uint64_t)n > kMaxScriptAlloc || !charge(16ull * (uint64_t)n)) return fail(limit_alloc());
        a[0].a.resize((size_t)n, a[2]);
        return OK;
      }
    }
    return fail("internal: bad built-in");
  }

  Flow call(const Node* n, Val* out) {
    std::vector<Val> a(n->kids.size());
    for (size_t k = 0; k < n->kids.size(); ++k)
      if (Flow f = eval(n->kids[k].get(), &a[k])) return f;
    if (n->fn >= 0) {
      const FnDef& F = ast->fns[(size_t)n->fn];
      if (depth >= kMaxCallDepth) return fail("Stack overflow");
      if (++ops > kMaxScriptOps) return fail(limit_ops());
      const size_t saved = base;
      base = vars.size();
      for (size_t k = 0; k < a.size(); ++k) vars.push_back({F.params[k], std::move(a[k])});
      ++depth;
      Flow f = eval(F.body.get(), out);
      --depth;
      vars.resize(base);
      base = saved;
      if (f == RET) {
        *out = std::move(fv);
        f = OK;
      }
      return f;
    }
    if (n->slot >= 0) {
      const uint32_t s = (uint32_t)n->slot;
      if (s >= seen.size()) seen.resize(s + 1, 0);
      if (!seen[s]) {
        seen[s] = 1;
        called.push_back(s);
      }
      *out = vbool(ok(s));
      return OK;
    }
    if (n->builtin >= 0) {
      if (Flow f = builtin(n->builtin, n->name, a, out)) return f;
      // a method-style call on a variable changes it (rhai's `&mut` first parameter; a constant
      // never reaches here for a function that always changes it, the parser refuses that)
      if (n->flag && builtin_mut(n->builtin) && n->kids[0]->k == Node::Var) {
        Val* v = lookup(n->kids[0]->name);
        if (!v) return fail("Variable not found: " + n->kids[0]->name);
        *v = std::move(a[0]);
      }
      return OK;
    }
    std::vector<const Val*> ap;
    for (const Val& v : a) ap.push_back(&v);
    return nf(n->name, ap);
  }

  // a op b for the binary operators and compound assignments (`+=` pushes onto arrays)
  Flow binop(const std::string& op, bool assign, Val& a, Val& b, Val* out) {
    const std::string shown = op;
    if (op == "==" || op == "!=") {
      const int e = eq(a, b, 0);
      if (e < 0) return fail(limit_depth());
      *out = vbool((op == "==") == (e == 1));
      return OK;
    }
    if (op == "<" || op == "<=" || op == ">" || op == ">=") {
      if (a.t != b.t) {
        *out = vbool(false);
        return OK;
      }
      int c;
      if (a.t == VT::Int) c = a.i < b.i ? -1 : a.i > b.i ? 1 : 0;
      else if (a.t == VT::Str) c = a.s.compare(b.s) < 0 ? -1 : a.s == b.s ? 0 : 1;
      else return nf(shown, {&a, &b});
      *out = vbool(op == "<" ? c < 0 : op == "<=" ? c <= 0 : op == ">" ? c > 0 : c >= 0);
      return OK;
    }
    if (op == "|" || op == "&" || op == "^") {
      if (a.t == VT::Bool && b.t == VT::Bool) {
        *out = vbool(op == "|" ? (a.b || b.b) : op == "&" ? (a.b && b.b) : (a.b != b.b));
        return OK;
      }
      if (a.t == VT::Int && b.t == VT::Int) {
        *out = vint(op == "|" ? (a.i | b.i) : op == "&" ? (a.i & b.i) : (a.i ^ b.i));
        return OK;
      }
      return nf(shown, {&a, &b});
    }
    if (op == "+" && a.t == VT::Arr && (b.t == VT::Arr || assign)) {
      const size_t nb = b.t == VT::Arr ? b.a.size() : 1;
      if (!charge(16ull * (a.a.size() + nb))) return fail(limit_alloc());
      *out = a;
      if (b.t == VT::Arr) out->a.insert(out->a.end(), b.a.begin(), b.a.end());
      else out->a.push_back(b);
      return OK;
    }
    if (op == "+" && (a.t == VT::Str || b.t == VT::Str) && a.t != VT::Arr && b.t != VT::Arr) {
      std::string sa, sb;
      text(a, &sa);
      text(b, &sb);
      if (!charge(sa.size() + sb.size())) return fail(limit_alloc());
      *out = vstr(sa + sb);
      return OK;
    }
    if (op == "+" && (a.t == VT::Str || b.t == VT::Str))
      return fail(std::string(kUnsupported) + "converting an array to a string");
    if (op == "-" && a.t == VT::Str && b.t == VT::Str) {  // every occurrence of b removed
      if (a.s.empty() || b.s.empty()) {
        *out = a;
        return OK;
      }
      std::string r;
      for (const std::string& p : str_split(a.s, b.s, false, 0)) r += p;
      if (!charge(r.size())) return fail(limit_alloc());
      *out = vstr(std::move(r));
      return OK;
    }
    if (a.t != VT::Int || b.t != VT::Int) return nf(shown, {&a, &b});
    const std::string ex = std::to_string(a.i) + " " + op + " " + std::to_string(b.i);
    if (op == "**" || op == "<<" || op == ">>") {  // rhai's checked power / shifts (ArithmeticPackage)
      int64_t r;
      std::string e;
      if (!int_pow_shift(op, a.i, b.i, &r, &e)) return fail(e);
      *out = vint(r);
      return OK;
    }
    long long r = 0;
    if (op == "+") {
      if (__builtin_add_overflow(a.i, b.i, &r)) return fail("Addition overflow: " + ex);
    } else if (op == "-") {
      if (__builtin_sub_overflow(a.i, b.i, &r)) return fail("Subtraction overflow: " + ex);
    } else if (op == "*") {
      if (__builtin_mul_overflow(a.i, b.i, &r)) return fail("Multiplication overflow: " + ex);
    } else {  // / %
      if (b.i == 0) return fail("Division by zero: " + ex);
      if (a.i == INT64_MIN && b.i == -1) return fail((op == "/" ? "Division overflow: " : "Modulo overflow: ") + ex);
      r = op == "/" ? a.i / b.i : a.i % b.i;
    }
    *out = vint(r);
    return OK;
  }

  Flow cond(const Node* n, const char* what, bool* c) {
    Val v;
    if (Flow f = eval(n, &v)) return f;
    if (v.t != VT::Bool) return fail(std::string("Boolean value expected for the ") + what + " condition, found " + tname(v.t));
    *c = v.b;
    return OK;
  }
  bool tick() { return ++ops <= kMaxScriptOps; }

  // a loop body's outcome: OK go on, BRK leave with *out, anything else propagates
  Flow body(const Node* b, Val* out, bool* leave) {
    Val v;
    *leave = false;
    Flow f = eval(b, &v);
    if (f == CNT) return OK;
    if (f == BRK) {
      *leave = true;
      *out = std::move(fv);
      return OK;
    }
    return f;
  }

  Flow range_bounds(const Node* r, int64_t* lo, int64_t* hi) {
    Val a, b;
    if (Flow f = eval(r->kids[0].get(), &a)) return f;
    if (Flow f = eval(r->kids[1].get(), &b)) return f;
    if (a.t != VT::Int || b.t != VT::Int) return nf(r->name2, {&a, &b});
    *lo = a.i;
    *hi = b.i;
    return OK;
  }

  Flow eval(const Node* n, Val* out) {
    ++steps;
    switch (n->k) {
      case Node::Lit: *out = n->lit; return OK;
      case Node::Var: {
        Val* v = lookup(n->name);
        if (!v) return fail("Variable not found: " + n->name);
        *out = *v;
        return OK;
      }
      case Node::Call: return call(n, out);
      case Node::Unary: {
        Val a;
        if (Flow f = eval(n->kids[0].get(), &a)) return f;
        if (n->op == "!") {
          if (a.t != VT::Bool) return nf("!", {&a});
          *out = vbool(!a.b);
          return OK;
        }
        if (a.t != VT::Int) return nf(n->op, {&a});
        if (n->op == "-" && a.i == INT64_MIN) return fail("Negation overflow: -" + std::to_string(a.i));
        *out = vint(n->op == "-" ? -a.i : a.i);
        return OK;
      }
      case Node::Bin: {
        const std::string& op = n->op;
        Val a, b;
        if (Flow f = eval(n->kids[0].get(), &a)) return f;
        if (op == "||" || op == "&&") {
          if (a.t != VT::Bool) return fail("Function not found: " + op + " (" + tname(a.t) + ", ...)");
          if ((op == "||") == a.b) {  // short circuit
            *out = a;
            return OK;
          }
          if (Flow f = eval(n->kids[1].get(), &b)) return f;
          if (b.t != VT::Bool) return nf(op, {&a, &b});
          *out = b;
          return OK;
        }
        if (Flow f = eval(n->kids[1].get(), &b)) return f;
        return binop(op, false, a, b, out);
      }
      case Node::Coalesce: {
        if (Flow f = eval(n->kids[0].get(), out)) return f;
        if (out->t != VT::Unit) return OK;
        return eval(n->kids[1].get(), out);
      }
      case Node::In: {
        Val x;
        if (Flow f = eval(n->kids[0].get(), &x)) return f;
        const Node* h = n->kids[1].get();
        bool r;
        if (h->k == Node::Range) {
          int64_t lo, hi;
          if (Flow f = range_bounds(h, &lo, &hi)) return f;
          if (x.t != VT::Int) {
            const std::string sig = std::string("Function not found: contains (") + (h->flag ? "range=" : "range") + ", " +
                                    tname(x.t) + ")";
            return fail(sig);
          }
          r = x.i >= lo && (h->flag ? x.i <= hi : x.i < hi);
        } else {
          std::vector<Val> a(2);
          if (Flow f = eval(h, &a[0])) return f;
          a[1] = std::move(x);
          Val v;
          if (Flow f = builtin(F_CONTAINS, "contains", a, &v)) return f;
          r = v.b;
        }
        *out = vbool(n->flag ? !r : r);
        return OK;
      }
      case Node::Range: return fail("internal: range value");
      case Node::If: {
        bool c;
        if (Flow f = cond(n->kids[0].get(), "if", &c)) return f;
        if (c) return eval(n->kids[1].get(), out);
        if (n->kids.size() > 2) return eval(n->kids[2].get(), out);
        *out = Val{};
        return OK;
      }
      case Node::Block: {
        const size_t scope = vars.size();
        Val v;
        for (size_t k = 0; k < n->kids.size(); ++k) {
          if (Flow f = eval(n->kids[k].get(), &v)) {
            vars.resize(scope);
            return f;
          }
        }
        vars.resize(scope);
        *out = n->flag ? std::move(v) : Val{};
        return OK;
      }
      case Node::Let: {
        Val x;
        if (!n->kids.empty())
          if (Flow f = eval(n->kids[0].get(), &x)) return f;
        vars.push_back({n->name, std::move(x)});
        *out = Val{};
        return OK;
      }
      case Node::Assign: {
        Val r;
        if (Flow f = eval(n->kids[0].get(), &r)) return f;  // (rhai evaluates the right side first)
        Val* v = lookup(n->name);
        if (!v) return fail("Variable not found: " + n->name);
        if (n->op.empty()) {
          *v = std::move(r);
        } else {
          Val nv;
          if (Flow f = binop(n->op, true, *v, r, &nv)) return f;
          *v = std::move(nv);
        }
        *out = Val{};
        return OK;
      }
      case Node::IndexAssign: {
        Val r, ix;
        if (Flow f = eval(n->kids[1].get(), &r)) return f;
        if (Flow f = eval(n->kids[0].get(), &ix)) return f;
        Val* v = lookup(n->name);
        if (!v) return fail("Variable not found: " + n->name);
        if (v->t != VT::Arr) return not_indexable(*v);
        if (ix.t != VT::Int) return fail(std::string("Array index must be an i64, found ") + tname(ix.t));
        size_t at;
        if (!index_of(ix.i, v->a.size(), &at)) return bounds(ix.i, v->a.size());
        Val nv;
        if (n->op.empty()) {
          nv = std::move(r);
        } else if (Flow f = binop(n->op, true, v->a[at], r, &nv)) {
          return f;
        }
        if (!charge(16ull * v->a.size())) return fail(limit_alloc());
        v->a[at] = std::move(nv);
        *out = Val{};
        return OK;
      }
      case Node::Index: {
        Val a, ix;
        if (Flow f = eval(n->kids[0].get(), &a)) return f;
        if (Flow f = eval(n->kids[1].get(), &ix)) return f;
        if (a.t != VT::Arr) return not_indexable(a);
        if (ix.t != VT::Int) return fail(std::string("Array index must be an i64, found ") + tname(ix.t));
        size_t at;
        if (!index_of(ix.i, a.a.size(), &at)) return bounds(ix.i, a.a.size());
        *out = std::move(a.a[at]);
        return OK;
      }
      case Node::Array: {
        Val v;
        v.t = VT::Arr;
        v.a.resize(n->kids.size());
        for (size_t k = 0; k < n->kids.size(); ++k)
          if (Flow f = eval(n->kids[k].get(), &v.a[k])) return f;
        if (!charge(16ull * n->kids.size())) return fail(limit_alloc());
        *out = std::move(v);
        return OK;
      }
      case Node::Switch: {
        Val x;
        if (Flow f = eval(n->kids[0].get(), &x)) return f;
        // exact cases first (in order), then range cases, then the wildcard
        for (int pass = 0; pass < 3; ++pass)
          for (const SwitchCase& c : n->cases) {
            if ((pass == 0) != (!c.range && !c.wildcard) || (pass == 1) != c.range || (pass == 2) != c.wildcard) continue;
            bool m = c.wildcard;
            if (c.range) m = x.t == VT::Int && x.i >= c.lo && (c.incl ? x.i <= c.hi : x.i < c.hi);
            for (const Val& v : c.vals) m = m || eq(x, v, 0) == 1;
            if (!m) continue;
            if (c.guard) {
              bool g;
              if (Flow f = cond(c.guard.get(), "switch case", &g)) return f;
              if (!g) continue;
            }
            return eval(c.body.get(), out);
          }
        *out = Val{};
        return OK;
      }
      case Node::While:
      case Node::Loop:
      case Node::DoWhile: {
        const bool is_do = n->k == Node::DoWhile;
        const Node* b = n->kids[is_do ? 0 : n->k == Node::Loop ? 0 : 1].get();
        for (bool first = true;; first = false) {
          if (n->k == Node::While) {
            bool c;
            if (Flow f = cond(n->kids[0].get(), "while", &c)) return f;
            if (!c) break;
          } else if (is_do && !first) {
            bool c;
            if (Flow f = cond(n->kids[1].get(), n->flag ? "do-until" : "do-while", &c)) return f;
            if (c == n->flag) break;
          }
          if (!tick()) return fail(limit_ops());
          bool leave;
          if (Flow f = body(b, out, &leave)) return f;
          if (leave) return OK;
        }
        *out = Val{};
        return OK;
      }
      case Node::For: {
        const Node* it = n->kids[0].get();
        const Node* b = n->kids[1].get();
        const size_t scope = vars.size();
        auto run = [&](Val x, int64_t idx, bool* leave) -> Flow {
          vars.resize(scope);
          vars.push_back({n->name, std::move(x)});
          if (!n->name2.empty()) vars.push_back({n->name2, vint(idx)});
          if (!tick()) return fail(limit_ops());
          Flow f = body(b, out, leave);
          vars.resize(scope);
          return f;
        };
        bool leave = false;
        if (it->k == Node::Range) {
          int64_t lo, hi;
          if (Flow f = range_bounds(it, &lo, &hi)) return f;
          int64_t k = 0;
          for (int64_t x = lo; it->flag ? x <= hi : x < hi; ++x, ++k) {
            if (Flow f = run(vint(x), k, &leave)) return f;
            if (leave) return OK;
            if (x == INT64_MAX) break;
          }
        } else {
          Val a;
          if (Flow f = eval(it, &a)) return f;
          if (a.t == VT::Str) return fail(std::string(kUnsupported) + "iterating over a string (characters)");
          if (a.t != VT::Arr) return fail(std::string("For loop expects an iterable type, found ") + tname(a.t));
          for (size_t k = 0; k < a.a.size(); ++k) {
            if (Flow f = run(a.a[k], (int64_t)k, &leave)) return f;
            if (leave) return OK;
          }
        }
        *out = Val{};
        return OK;
      }
      case Node::Break:
      case Node::Return: {
        Val v;
        if (!n->kids.empty())
          if (Flow f = eval(n->kids[0].get(), &v)) return f;
        fv = std::move(v);
        return n->k == Node::Break ? BRK : RET;
      }
      case Node::Continue: return CNT;
    }
    return fail("internal: bad node");
  }
};

ExprOutcome run_ast(const ExprAst& ast, const std::function<bool(uint32_t)>& ok, uint64_t* steps = nullptr) {
  Interp in(ok);
  in.ast = &ast;
  Val v;
  ExprOutcome o;
  Flow f = in.eval(ast.root.get(), &v);
  if (f == RET) v = std::move(in.fv);
  if (f == ERR) {
    o.error = true;
    o.message = in.err;
  } else if (v.t != VT::Bool) {
    o.error = true;
    o.message = std::string("Output type incorrect: ") + tname(v.t) + " (expecting bool)";
  } else {
    o.value = v.b;
  }
  o.called = std::move(in.called);
  if (steps) *steps = in.steps;
  return o;
}

// ------------------------------------------------------------------------------------------
// Folding and the bool-only subset
// ------------------------------------------------------------------------------------------
bool has_member_call(const Node* n) {
  if (n->k == Node::Call && n->slot >= 0) return true;
  for (const P& k : n->kids)
    if (has_member_call(k.get())) return true;
  for (const SwitchCase& c : n->cases)
    if ((c.guard && has_member_call(c.guard.get())) || has_member_call(c.body.get())) return true;
  return false;
}
bool program_calls_members(const ExprAst& a) {
  if (has_member_call(a.root.get())) return true;
  for (const FnDef& f : a.fns)
    if (has_member_call(f.body.get())) return true;
  return false;
}

// a subtree that folds: literals and operators over them only (no variables, calls, loops,
// arrays or strings: a folded string would change what a run charges against its budget)
bool foldable(const Node* n) {
  switch (n->k) {
    case Node::Lit: return n->lit.t != VT::Str;
    case Node::Unary:
    case Node::Bin:
    case Node::Coalesce:
    case Node::If:
      for (const P& k : n->kids)
        if (!foldable(k.get())) return false;
      return true;
    case Node::Block:
      for (const P& k : n->kids)
        if (!foldable(k.get())) return false;
      return true;
    default: return false;
  }
}

// Replace every foldable subtree whose evaluation succeeds by its value (an erroring one stays:
// it may never run, e.g. behind a short circuit).
void fold(P* np, const ExprAst& ast) {
  Node* n = np->get();
  for (P& k : n->kids) fold(&k, ast);
  for (SwitchCase& c : n->cases) {
    if (c.guard) fold(&c.guard, ast);
    fold(&c.body, ast);
  }
  if (n->k == Node::Lit || !foldable(n)) return;
  Interp in([](uint32_t) { return false; });
  in.ast = &ast;
  Val v;
  if (in.eval(n, &v) != OK || (v.t != VT::Bool && v.t != VT::Int && v.t != VT::Unit)) return;
  auto l = std::make_unique<Node>();
  l->lit = v;
  *np = std::move(l);
}

// bool-only: bool literals, member calls, ! && || == != (== / != over bools), a script that is a
// single tail expression
const Node* bool_root(const ExprAst& a) {
  const Node* r = a.root.get();
  while (r->k == Node::Block && r->flag && r->kids.size() == 1) r = r->kids[0].get();
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
    case Node::Block: return n->flag && n->kids.size() == 1 && is_bool_subset(n->kids[0].get());
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
  const ExprAst& ast;
  std::vector<uint8_t> code, pool;
  bool allocates = false, uses_type_of = false;
  struct Loop {
    uint32_t depth;                  // value-stack depth before the loop expression
    std::vector<size_t> breaks, conts;  // jump operands to patch
  };
  struct Fn {  // the function being emitted
    std::vector<std::vector<std::pair<std::string, uint32_t>>> scopes;
    uint32_t nslots = 0, depth = 0, maxdepth = 0;
    std::vector<Loop> loops;
    std::vector<size_t> slot_patches;  // S_CALLF caller-slot operands of this function's calls
  };
  Fn* cur = nullptr;
  std::vector<size_t> fn_at;                          // code offset of each script function
  std::vector<std::pair<size_t, int>> call_patches;  // (operand, fn)
  explicit ScriptEmitter(const ExprAst& a) : ast(a) {}

  void u8(uint8_t x) { code.push_back(x); }
  void u16(uint32_t x) {
    u8((uint8_t)x);
    u8((uint8_t)(x >> 8));
  }
  void u32(uint32_t x) {
    u16(x & 0xffff);
    u16(x >> 16);
  }
  void u64(uint64_t x) {
    u32((uint32_t)x);
    u32((uint32_t)(x >> 32));
  }
  void push(int n = 1) {
    cur->depth = (uint32_t)((int)cur->depth + n);
    cur->maxdepth = std::max(cur->maxdepth, cur->depth);
  }
  void pop(int n = 1) { cur->depth = (uint32_t)((int)cur->depth - n); }
  size_t hole(uint8_t op) {
    u8(op);
    const size_t at = code.size();
    u32(0);
    return at;
  }
  void patch_to(size_t at, uint32_t to) {
    for (int k = 0; k < 4; ++k) code[at + (size_t)k] = (uint8_t)(to >> (8 * k));
  }
  void patch(size_t at) { patch_to(at, (uint32_t)code.size()); }
  uint32_t new_slot() { return cur->nslots++; }
  uint32_t declare(const std::string& name) {
    const uint32_t s = new_slot();
    cur->scopes.back().push_back({name, s});
    return s;
  }
  bool lookup(const std::string& name, uint32_t* slot) const {
    for (size_t sc = cur->scopes.size(); sc-- > 0;)
      for (size_t k = cur->scopes[sc].size(); k-- > 0;)
        if (cur->scopes[sc][k].first == name) {
          *slot = cur->scopes[sc][k].second;
          return true;
        }
    return false;
  }
  void load(uint32_t s) {
    u8(S_LOAD);
    u16(s);
    push();
  }
  void store(uint32_t s) {
    u8(S_STORE);
    u16(s);
    pop();
  }
  void lit(const Val& v) {
    push();
    if (v.t == VT::Unit) {
      u8(S_UNIT);
    } else if (v.t == VT::Bool) {
      u8(S_BOOL);
      u8(v.b ? 1 : 0);
    } else if (v.t == VT::Int) {
      u8(S_INT);
      u64((uint64_t)v.i);
    } else {
      u8(S_STR);
      u32((uint32_t)pool.size());  // rebased to the program start at the end
      u32((uint32_t)v.s.size());
      pool.insert(pool.end(), v.s.begin(), v.s.end());
    }
  }
  void bin(uint8_t b) {
    u8(S_BIN);
    u8(b);
    pop();
    if (b == SB_ADD || b == SB_ADDA || b == SB_SUB) allocates = true;
  }
  static uint8_t bin_code(const std::string& op, bool assign) {
    static const char* ops[] = {"|", "^", "&", "==", "!=", "<", "<=", ">", ">=", "+", "-", "*", "/", "%"};
    if (assign && op == "+") return SB_ADDA;
    for (uint8_t k = 0; k < 14; ++k)
      if (op == ops[k]) return k;
    if (op == "**") return SB_POW;
    if (op == "<<") return SB_SHL;
    if (op == ">>") return SB_SHR;
    return 0;
  }
  bool uses_chars = false;  // a function that reads character properties (the char table)
  void note_fn(int fid) {
    if (fid == F_TYPE_OF) uses_type_of = true;
    if (fid == F_TO_UPPER || fid == F_TO_LOWER || fid == F_MAKE_UPPER || fid == F_MAKE_LOWER || fid == F_TRIM ||
        fid == F_SPLIT_WS || fid == F_PARSE_INT || fid == F_PARSE_INT_R)
      uses_chars = true;
    static const int pure[] = {F_LEN, F_IS_EMPTY, F_CONTAINS, F_TYPE_OF, F_STARTS_WITH, F_ENDS_WITH, F_ABS, F_SIGN,
                               F_IS_ZERO, F_IS_ODD, F_IS_EVEN, F_MAX, F_MIN, F_PARSE_INT, F_PARSE_INT_R, F_BYTES};
    if (std::find(std::begin(pure), std::end(pure), fid) == std::end(pure)) allocates = true;
  }
  void fail_op() {  // a value the run never gets past
    u8(S_FAIL);
    push();
  }
  // drop the values above depth d (keeping the top when `keep`)
  void unwind(uint32_t d, bool keep) {
    const uint32_t n = cur->depth - d - (keep ? 1u : 0u);
    if (n == 0) return;
    u8(keep ? S_DROPKEEP : S_DROP);
    u16(n);
  }

  // emits n, leaving one value on the stack
  void emit(const Node* n) {
    switch (n->k) {
      case Node::Lit: lit(n->lit); return;
      case Node::Var: {
        uint32_t s;
        if (lookup(n->name, &s)) load(s);
        else fail_op();
        return;
      }
      case Node::Call: {
        for (const P& k : n->kids) emit(k.get());
        const int na = (int)n->kids.size();
        if (n->fn >= 0) {
          u8(S_CALLF);
          call_patches.push_back({code.size(), n->fn});
          u32(0);
          u8((uint8_t)na);
          cur->slot_patches.push_back(code.size());
          u16(0);
          pop(na);
          push();
          return;
        }
        if (n->slot >= 0) {
          u8(S_CALL);
          u32((uint32_t)n->slot);
          push();
          return;
        }
        if (n->builtin >= 0) {
          const int fid = n->builtin;
          const bool mut = builtin_mut(fid);
          u8(S_FN);
          u8((uint8_t)fid);
          u8((uint8_t)(na | (mut ? 0x80 : 0)));
          pop(na);
          push(mut ? 2 : 1);
          note_fn(fid);
          if (mut) {  // [receiver as changed, result]: into the variable for a method call on one
            uint32_t s;
            if (n->flag && n->kids[0]->k == Node::Var && lookup(n->kids[0]->name, &s)) {
              u8(S_XSTORE);
              u16(s);
            } else {
              u8(S_DROPKEEP);
              u16(1);
            }
            pop();
          }
          return;
        }
        u8(S_FAIL);
        pop(na);
        push();
        return;
      }
      case Node::Unary:
        emit(n->kids[0].get());
        u8(n->op == "!" ? S_NOT : n->op == "-" ? S_NEG : S_POS);
        return;
      case Node::Bin: {
        const std::string& op = n->op;
        emit(n->kids[0].get());
        if (op == "||" || op == "&&") {
          const size_t at = hole(op == "||" ? S_OR : S_AND);
          pop();  // (the continuing path pops the left side)
          emit(n->kids[1].get());
          u8(S_CHKB);
          patch(at);
          return;
        }
        emit(n->kids[1].get());
        bin(bin_code(op, false));
        return;
      }
      case Node::Coalesce: {
        emit(n->kids[0].get());
        const size_t at = hole(S_COAL);
        pop();
        emit(n->kids[1].get());
        patch(at);
        return;
      }
      case Node::In: {
        emit(n->kids[0].get());
        const Node* h = n->kids[1].get();
        if (h->k == Node::Range) {
          emit(h->kids[0].get());
          emit(h->kids[1].get());
          u8(S_INRANGE);
          u8(h->flag ? 1 : 0);
          pop(2);
        } else {
          emit(h);
          u8(S_FN);
          u8(F_IN);
          u8(2);
          pop();
        }
        if (n->flag) u8(S_NOT);
        return;
      }
      case Node::Range: fail_op(); return;
      case Node::If: {
        emit(n->kids[0].get());
        const size_t at_else = hole(S_IF);
        pop();
        const uint32_t d0 = cur->depth;
        emit(n->kids[1].get());
        const size_t at_end = hole(S_JMP);
        patch(at_else);
        cur->depth = d0;
        if (n->kids.size() > 2) emit(n->kids[2].get());
        else lit(Val{});
        patch(at_end);
        return;
      }
      case Node::Block: {
        cur->scopes.emplace_back();
        for (size_t k = 0; k < n->kids.size(); ++k) {
          const Node* st = n->kids[k].get();
          emit(st);
          if (!(n->flag && k + 1 == n->kids.size())) {
            u8(S_POP);
            pop();
          }
        }
        cur->scopes.pop_back();
        if (!n->flag) lit(Val{});
        return;
      }
      case Node::Let: {
        if (n->kids.empty()) lit(Val{});
        else emit(n->kids[0].get());
        const uint32_t s = declare(n->name);  // (after the initializer: `let x = x + 1` reads the old x)
        store(s);
        lit(Val{});
        return;
      }
      case Node::Assign: {
        uint32_t s;
        const bool found = lookup(n->name, &s);
        emit(n->kids[0].get());
        if (!found) {
          u8(S_FAIL);
          return;  // (the right side's value stands for the statement)
        }
        if (n->op.empty()) {
          store(s);
        } else {
          const uint32_t t = new_slot();
          store(t);
          load(s);
          load(t);
          bin(bin_code(n->op, true));
          store(s);
        }
        lit(Val{});
        return;
      }
      case Node::IndexAssign: {
        uint32_t s;
        const bool found = lookup(n->name, &s);
        const uint32_t tv = new_slot(), ti = new_slot();
        emit(n->kids[1].get());  // value first (rhai evaluates the right side first)
        store(tv);
        emit(n->kids[0].get());
        store(ti);
        if (!found) {
          fail_op();
          return;
        }
        load(ti);
        if (n->op.empty()) {
          load(tv);
        } else {
          load(s);
          load(ti);
          u8(S_INDEX);
          pop();
          load(tv);
          bin(bin_code(n->op, true));
        }
        u8(S_SETIDX);
        u16(s);
        pop(2);
        allocates = true;
        lit(Val{});
        return;
      }
      case Node::Index:
        emit(n->kids[0].get());
        emit(n->kids[1].get());
        u8(S_INDEX);
        pop();
        return;
      case Node::Array:
        for (const P& k : n->kids) emit(k.get());
        u8(S_ARR);
        u16((uint32_t)n->kids.size());
        pop((int)n->kids.size());
        push();
        allocates = true;
        return;
      case Node::Switch: {
        emit(n->kids[0].get());
        const uint32_t s = new_slot();
        store(s);
        std::vector<size_t> ends;
        const uint32_t d0 = cur->depth;
        for (int pass = 0; pass < 3; ++pass)
          for (const SwitchCase& c : n->cases) {
            if ((pass == 0) != (!c.range && !c.wildcard) || (pass == 1) != c.range || (pass == 2) != c.wildcard) continue;
            std::vector<size_t> nexts;
            if (!c.wildcard) {
              if (c.range) {
                load(s);
                u8(S_RCASE);
                u64((uint64_t)c.lo);
                u64((uint64_t)c.hi);
                u8(c.incl ? 1 : 0);
              } else {
                std::vector<size_t> ors;
                for (size_t v = 0; v < c.vals.size(); ++v) {
                  load(s);
                  lit(c.vals[v]);
                  bin(SB_EQ);
                  if (v + 1 < c.vals.size()) {
                    ors.push_back(hole(S_OR));
                    pop();
                  }
                }
                for (size_t at : ors) patch(at);
              }
              nexts.push_back(hole(S_IF));
              pop();
            }
            if (c.guard) {
              emit(c.guard.get());
              nexts.push_back(hole(S_IF));
              pop();
            }
            emit(c.body.get());
            ends.push_back(hole(S_JMP));
            cur->depth = d0;
            for (size_t at : nexts) patch(at);
          }
        lit(Val{});
        for (size_t at : ends) patch(at);
        return;
      }
      case Node::While:
      case Node::Loop:
      case Node::DoWhile: {
        const uint32_t d0 = cur->depth;
        cur->loops.push_back({d0, {}, {}});
        size_t exit_at = 0;
        bool has_exit = false;
        uint32_t top = (uint32_t)code.size(), cont;
        if (n->k == Node::DoWhile) {
          u8(S_TICK);
          emit(n->kids[0].get());
          u8(S_POP);
          pop();
          cont = (uint32_t)code.size();
          emit(n->kids[1].get());
          if (n->flag) u8(S_NOT);
          exit_at = hole(S_IF);  // while: false leaves; until: true leaves
          pop();
          has_exit = true;
          const size_t j = hole(S_JMP);
          patch_to(j, top);
        } else {
          cont = top;
          if (n->k == Node::While) {
            emit(n->kids[0].get());
            exit_at = hole(S_IF);
            pop();
            has_exit = true;
          }
          u8(S_TICK);
          emit(n->kids[n->k == Node::Loop ? 0 : 1].get());
          u8(S_POP);
          pop();
          const size_t j = hole(S_JMP);
          patch_to(j, top);
        }
        if (has_exit) patch(exit_at);
        lit(Val{});  // the normal exit's value
        Loop L = std::move(cur->loops.back());
        cur->loops.pop_back();
        for (size_t at : L.breaks) patch(at);
        for (size_t at : L.conts) patch_to(at, cont);
        cur->depth = d0 + 1;
        return;
      }
      case Node::For: {
        const uint32_t d0 = cur->depth;
        const Node* it = n->kids[0].get();
        const uint32_t sa = new_slot(), si = new_slot();
        const bool range = it->k == Node::Range;
        if (range) {
          emit(it->kids[0].get());
          emit(it->kids[1].get());
          u8(S_RANGECHK);
          store(si);  // hi (the end slot is `si` here; `sa` holds the cursor)
          store(sa);
        } else {
          emit(it);
          store(sa);
          lit(vint(0));
          store(si);
        }
        uint32_t sc = 0;
        if (range && !n->name2.empty()) {
          sc = new_slot();
          lit(vint(0));
          store(sc);
        }
        cur->loops.push_back({d0, {}, {}});
        const uint32_t top = (uint32_t)code.size();
        size_t exit_at;
        if (range) {
          u8(S_FORR);
          u16(sa);
          u16(si);
          u8(it->flag ? 1 : 0);
          exit_at = code.size();
          u32(0);
          push();
        } else {
          u8(S_FORA);
          u16(sa);
          u16(si);
          u8(n->name2.empty() ? 0 : 1);
          exit_at = code.size();
          u32(0);
          push(n->name2.empty() ? 1 : 2);
        }
        cur->scopes.emplace_back();
        const uint32_t sx = declare(n->name);
        if (!n->name2.empty()) {
          const uint32_t sk = declare(n->name2);
          if (range) {  // the counter of a range loop lives in slot sc (zeroed before `top`)
            store(sx);
            load(sc);
            store(sk);
            load(sc);
            lit(vint(1));
            bin(SB_ADD);
            store(sc);
          } else {
            store(sk);
            store(sx);
          }
        } else {
          store(sx);
        }
        u8(S_TICK);
        emit(n->kids[1].get());
        u8(S_POP);
        pop();
        cur->scopes.pop_back();
        const size_t j = hole(S_JMP);
        patch_to(j, top);
        patch(exit_at);
        lit(Val{});
        Loop L = std::move(cur->loops.back());
        cur->loops.pop_back();
        for (size_t at : L.breaks) patch(at);
        for (size_t at : L.conts) patch_to(at, top);
        cur->depth = d0 + 1;
        return;
      }
      case Node::Break:
      case Node::Continue: {
        Loop& L = cur->loops.back();
        if (n->k == Node::Break) {
          if (n->kids.empty()) lit(Val{});
          else emit(n->kids[0].get());
          unwind(L.depth, true);
          L.breaks.push_back(hole(S_JMP));
        } else {
          unwind(L.depth, false);
          L.conts.push_back(hole(S_JMP));
          push();
        }
        cur->depth = L.depth + 1;  // (unreachable after the jump; keeps the bookkeeping whole)
        return;
      }
      case Node::Return: {
        if (n->kids.empty()) lit(Val{});
        else emit(n->kids[0].get());
        u8(cur == &main_fn ? S_END : S_RET);
        return;
      }
    }
  }

  Fn main_fn;
  std::vector<Fn> fns;
};

// The script form of a group (GroupProgram::script): header | code | string pool (kwdev.hpp SOp).
bool emit_script(const ExprAst& ast, std::vector<uint8_t>* out, uint32_t* depth, std::string* err) {
  ScriptEmitter e(ast);
  e.cur = &e.main_fn;
  e.main_fn.scopes.emplace_back();
  e.emit(ast.root.get());
  e.u8(S_END);
  e.fns.resize(ast.fns.size());
  e.fn_at.assign(ast.fns.size(), 0);
  for (size_t f = 0; f < ast.fns.size(); ++f) {
    e.cur = &e.fns[f];
    e.cur->scopes.emplace_back();
    for (const std::string& p : ast.fns[f].params) e.declare(p);
    e.fn_at[f] = e.code.size();
    e.emit(ast.fns[f].body.get());
    e.u8(S_RET);
  }
  for (auto& c : e.call_patches) e.patch_to(c.first, (uint32_t)e.fn_at[(size_t)c.second]);
  auto patch_slots = [&](ScriptEmitter::Fn& f) {
    for (size_t at : f.slot_patches) {
      e.code[at] = (uint8_t)f.nslots;
      e.code[at + 1] = (uint8_t)(f.nslots >> 8);
    }
  };
  patch_slots(e.main_fn);
  uint32_t fn_depth = 0, fn_slots = 0;
  for (ScriptEmitter::Fn& f : e.fns) {
    patch_slots(f);
    fn_depth = std::max(fn_depth, f.maxdepth);
    fn_slots = std::max(fn_slots, f.nslots);
  }
  const bool has_fns = !ast.fns.empty();
  const uint64_t total_depth = (uint64_t)e.main_fn.maxdepth + (has_fns ? (uint64_t)kMaxCallDepth * fn_depth : 0) + 1;
  const uint64_t total_slots = (uint64_t)e.main_fn.nslots + (has_fns ? (uint64_t)kMaxCallDepth * fn_slots : 0);
  if (e.main_fn.nslots > 65535 || fn_slots > 65535 || total_depth > (1u << 24) || total_slots > (1u << 24) ||
      e.code.size() + e.pool.size() > 0x7fffffffu) {
    *err = "policy group expression exceeds the engine's limits";
    return false;
  }
  // the char table: every non-ASCII code point a run can hold (the literals', closed under the case
  // mappings; ς for Σ's final form), with its White_Space / Cased / Case_Ignorable bits and mappings
  uint32_t ctab = 0, nchar = 0;
  if (e.uses_chars) {
    std::set<uint32_t> cs;
    std::function<void(const Node*)> walk = [&](const Node* n) {
      auto add = [&](const Val& v) {
        if (v.t == VT::Str)
          for (uint32_t c : cps_of(v.s))
            if (c >= 0x80) cs.insert(c);
      };
      add(n->lit);
      for (const P& k : n->kids) walk(k.get());
      for (const SwitchCase& c : n->cases) {
        for (const Val& v : c.vals) add(v);
        if (c.guard) walk(c.guard.get());
        walk(c.body.get());
      }
    };
    walk(ast.root.get());
    for (const FnDef& f : ast.fns) walk(f.body.get());
    std::vector<uint32_t> work(cs.begin(), cs.end());
    if (cs.count(0x3A3)) work.push_back(0x3C2);
    while (!work.empty()) {
      const uint32_t c = work.back();
      work.pop_back();
      cs.insert(c);
      for (const UniCaseMap* m : {uni_map(kUniLower, kUniLowerN, c), uni_map(kUniUpper, kUniUpperN, c)})
        if (m)
          for (uint32_t j = 0; j < m->n; ++j)
            if (m->m[j] >= 0x80 && !cs.count(m->m[j])) work.push_back(m->m[j]);
    }
    while (e.pool.size() % 4) e.pool.push_back(0);
    ctab = (uint32_t)e.pool.size();
    for (uint32_t c : cs) {
      const UniCaseMap* lo = uni_map(kUniLower, kUniLowerN, c);
      const UniCaseMap* up = uni_map(kUniUpper, kUniUpperN, c);
      const uint32_t nlo = lo ? lo->n : 1u, nup = up ? up->n : 1u;
      uint32_t w[8] = {c,
                       (uni_ws(c) ? kChWs : 0u) | (uni_cased(c) ? kChCased : 0u) | (uni_ignorable(c) ? kChIgnorable : 0u) |
                           (nlo << 8) | (nup << 10),
                       lo ? lo->m[0] : c, lo ? lo->m[1] : 0u, lo ? lo->m[2] : 0u,
                       up ? up->m[0] : c, up ? up->m[1] : 0u, up ? up->m[2] : 0u};
      e.pool.insert(e.pool.end(), (const uint8_t*)w, (const uint8_t*)w + kChEntry);
      ++nchar;
    }
  }
  uint32_t tnames = 0;
  if (e.uses_type_of) {
    tnames = (uint32_t)e.pool.size();
    const char* names = "()booli64stringarray";
    e.pool.insert(e.pool.end(), names, names + 20);
  }
  const uint32_t code_len = (uint32_t)e.code.size();
  // rebase S_STR pool offsets to the program start: walk the code
  for (size_t pc = 0; pc < e.code.size();) {
    const uint8_t op = e.code[pc++];
    switch (op) {
      case S_BOOL: case S_BIN: case S_INRANGE: pc += 1; break;
      case S_FN: case S_XSTORE: pc += 2; break;
      case S_INT: pc += 8; break;
      case S_STR: {
        uint32_t off = 0;
        for (int k = 0; k < 4; ++k) off |= (uint32_t)e.code[pc + (size_t)k] << (8 * k);
        off += kScriptHeader + code_len;
        for (int k = 0; k < 4; ++k) e.code[pc + (size_t)k] = (uint8_t)(off >> (8 * k));
        pc += 8;
        break;
      }
      case S_LOAD: case S_STORE: case S_ARR: case S_SETIDX: case S_DROP: case S_DROPKEEP: pc += 2; break;
      case S_CALL: case S_AND: case S_OR: case S_IF: case S_JMP: case S_COAL: pc += 4; break;
      case S_RCASE: pc += 17; break;
      case S_FORR: case S_FORA: pc += 9; break;
      case S_CALLF: pc += 7; break;
      default: break;
    }
  }
  out->clear();
  const uint32_t h[8] = {(uint32_t)total_depth,
                         (uint32_t)std::max<uint64_t>(total_slots, 1),
                         e.allocates ? kMaxScriptAlloc : 0u,
                         code_len,
                         has_fns ? kMaxCallDepth : 0u,
                         tnames + kScriptHeader + code_len,
                         nchar ? ctab + kScriptHeader + code_len : 0u,
                         nchar};
  out->insert(out->end(), (const uint8_t*)h, (const uint8_t*)h + kScriptHeader);
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

GroupProgram compile_group_expression(const std::string& expr, const std::vector<std::string>& members,
                                      bool force_wide) {
  GroupProgram g;
  g.nmem = (uint32_t)members.size();
  Lexer lx;
  if (!lx.run(expr)) {
    g.error = lx.err;
    return g;
  }
  auto ast = std::make_shared<ExprAst>();
  Parser p(lx.toks);
  p.ast = ast.get();
  P root = p.block_body(true);
  if (!root) {
    g.error = p.err;
    return g;
  }
  ast->root = std::move(root);
  {
    std::string rerr;
    bool ok = check_ranges(ast->root.get(), false, &rerr);
    for (const FnDef& f : ast->fns) ok = ok && check_ranges(f.body.get(), false, &rerr);
    if (!ok) {
      g.error = rerr;
      return g;
    }
  }
  resolve(ast->root.get(), *ast, members);
  for (FnDef& f : ast->fns) resolve(f.body.get(), *ast, members);
  {
    bool stray = stray_range_call(ast->root.get());
    for (const FnDef& f : ast->fns) stray = stray || stray_range_call(f.body.get());
    if (stray) {
      g.error = std::string(kUnsupported) + "range values outside `for` and `in`";
      return g;
    }
    const Node* r = refused_call(ast->root.get());
    for (const FnDef& f : ast->fns) r = r ? r : refused_call(f.body.get());
    if (r) {
      g.error = std::string(kUnsupported) + r->name;
      return g;
    }
  }
  // validation: the script runs with every member returning true (validate_settings)
  uint64_t steps = 0;
  {
    const ExprOutcome o = run_ast(*ast, [](uint32_t) { return true; }, &steps);
    if (o.error && o.message.rfind("Output type incorrect", 0) != 0) {
      g.error = o.message;
      return g;
    }
  }
  g.valid = true;
  fold(&ast->root, *ast);
  for (FnDef& f : ast->fns) fold(&f.body, *ast);
  g.ast = ast;
  // a script without member calls has one outcome: a constant column or a constant program
  if (!program_calls_members(*ast) && !force_wide) {
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
  // KW_GROUP_FORM=script: every group with member calls takes the bytecode form (a test knob: the
  // CPU suite runs the stack machine through the host walk, the GPU suite through the combine kernel)
  const bool force_script = getenv("KW_GROUP_FORM") && std::string(getenv("KW_GROUP_FORM")) == "script";
  const Node* br = bool_root(*ast);
  if (!force_script && ast->fns.empty() && is_bool_subset(br)) {
    uint32_t maxd = 1;
    emit(br, false, &g.code, 1, &maxd);
    g.depth = maxd;
    if (!force_wide && members.size() <= (size_t)kMaxGroupMembers && maxd <= (uint32_t)kMaxGroupStack &&
        g.code.size() <= 65535)
      return g;
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
  // a truth table when it is small and cheap to fill (2^n runs of the interpreter); otherwise
  // typed bytecode, run per request by the wide path's combine kernel
  const bool table = !force_script && !force_wide && members.size() <= kMaxTableMembers &&
                     (std::max<uint64_t>(steps, 1) << members.size()) <= (1ull << 24);
  if (!table) {
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
