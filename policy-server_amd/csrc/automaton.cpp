// automaton.cpp — glob / literal / regex pattern sets -> minimised multi-pattern DFA.
// See automaton.hpp for semantics. Construction: each pattern becomes an NFA fragment (glob
// chain or Thompson construction), all fragments share one start; subset construction with
// beginning-of-string assertions followed only from the initial closure and end-of-string
// assertions followed only when computing a state's accept mask; byte classes from the partition
// of all edge sets; Moore minimisation.
#include "automaton.hpp"

#include <algorithm>
#include <map>
#include <unordered_map>

namespace kw {
namespace {

struct BSet {
  uint64_t w[4] = {0, 0, 0, 0};
  void set(unsigned b) { w[b >> 6] |= 1ull << (b & 63); }
  bool has(unsigned b) const { return (w[b >> 6] >> (b & 63)) & 1; }
  void fill() { w[0] = w[1] = w[2] = w[3] = ~0ull; }
  void invert() {
    for (auto& x : w) x = ~x;
  }
  void range(unsigned a, unsigned b) {
    for (unsigned c = a; c <= b && c < 256; ++c) set(c);
  }
  bool operator<(const BSet& o) const {
    for (int i = 0; i < 4; ++i)
      if (w[i] != o.w[i]) return w[i] < o.w[i];
    return false;
  }
};

struct NState {
  std::vector<std::pair<uint32_t, uint32_t>> tr;  // (set id, target)
  std::vector<uint32_t> eps, bol, eol;
  int acc = -1;
};

struct Nfa {
  std::vector<NState> st;
  std::vector<BSet> sets;
  std::map<BSet, uint32_t> set_ids;
  uint32_t add() {
    st.emplace_back();
    return (uint32_t)st.size() - 1;
  }
  uint32_t sid(const BSet& s) {
    auto it = set_ids.find(s);
    if (it != set_ids.end()) return it->second;
    uint32_t id = (uint32_t)sets.size();
    sets.push_back(s);
    set_ids[s] = id;
    return id;
  }
  void edge(uint32_t a, const BSet& s, uint32_t b) { st[a].tr.push_back({sid(s), b}); }
  void eps(uint32_t a, uint32_t b) { st[a].eps.push_back(b); }
};

constexpr size_t kMaxNfaStates = 200000;

bool class_set(const std::string& name, BSet* s) {
  for (unsigned c = 0; c < 128; ++c) {
    bool in = false;
    if (name == "alpha") in = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
    else if (name == "digit") in = c >= '0' && c <= '9';
    else if (name == "alnum") in = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9');
    else if (name == "upper") in = c >= 'A' && c <= 'Z';
    else if (name == "lower") in = c >= 'a' && c <= 'z';
    else if (name == "space") in = c == ' ' || (c >= 9 && c <= 13);
    else if (name == "blank") in = c == ' ' || c == '\t';
    else if (name == "punct") in = (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
    else if (name == "xdigit") in = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
    else if (name == "cntrl") in = c < 32 || c == 127;
    else if (name == "print") in = c >= 32 && c <= 126;
    else if (name == "graph") in = c >= 33 && c <= 126;
    else return false;
    if (in) s->set(c);
  }
  return true;
}

// ---------------------------------------------------------------- glob (fnmatch, flags 0)
enum class GTok : uint8_t { Set, Star };
struct GItem {
  GTok t;
  BSet s;
};

// Returns false on unsupported syntax; *never = true if glibc would never match (trailing '\').
bool parse_glob(const std::string& p, std::vector<GItem>* out, bool* never, std::string* err) {
  *never = false;
  size_t i = 0, n = p.size();
  while (i < n) {
    unsigned char c = (unsigned char)p[i];
    if (c == '*') {
      out->push_back({GTok::Star, {}});
      ++i;
      continue;
    }
    if (c == '?') {
      GItem g{GTok::Set, {}};
      g.s.fill();
      out->push_back(g);
      ++i;
      continue;
    }
    if (c == '\\') {
      if (i + 1 >= n) {
        *never = true;  // glibc: "Trailing \ loses."
        return true;
      }
      GItem g{GTok::Set, {}};
      g.s.set((unsigned char)p[i + 1]);
      out->push_back(g);
      i += 2;
      continue;
    }
    if (c == '[') {
      size_t j = i + 1;
      bool neg = false;
      if (j < n && (p[j] == '!' || p[j] == '^')) {
        neg = true;
        ++j;
      }
      BSet s;
      bool first = true, closed = false;
      while (j < n) {
        unsigned char x = (unsigned char)p[j];
        if (x == ']' && !first) {
          closed = true;
          ++j;
          break;
        }
        first = false;
        if (x == '[' && j + 1 < n && p[j + 1] == ':') {
          size_t e = p.find(":]", j + 2);
          if (e == std::string::npos) {
            s.set('[');
            ++j;
            continue;
          }
          if (!class_set(p.substr(j + 2, e - j - 2), &s)) {
            *err = "unsupported character class in glob '" + p + "'";
            return false;
          }
          j = e + 2;
          continue;
        }
        if (x == '[' && j + 1 < n && (p[j + 1] == '.' || p[j + 1] == '=')) {
          *err = "collating elements are not supported in glob '" + p + "'";
          return false;
        }
        unsigned lo = x;
        if (x == '\\') {
          if (j + 1 >= n) break;  // unterminated
          lo = (unsigned char)p[j + 1];
          ++j;
        }
        ++j;
        if (j + 1 < n && p[j] == '-' && p[j + 1] != ']') {
          unsigned hi = (unsigned char)p[j + 1];
          j += 2;
          if (hi == '\\' && j < n) {
            hi = (unsigned char)p[j];
            ++j;
          }
          if (lo <= hi) s.range(lo, hi);
        } else {
          s.set(lo);
        }
      }
      if (!closed) {  // glibc: unterminated '[' is an ordinary character
        GItem g{GTok::Set, {}};
        g.s.set('[');
        out->push_back(g);
        ++i;
        continue;
      }
      if (neg) s.invert();
      out->push_back({GTok::Set, s});
      i = j;
      continue;
    }
    GItem g{GTok::Set, {}};
    g.s.set(c);
    out->push_back(g);
    ++i;
  }
  return true;
}

// ---------------------------------------------------------------- regex (ERE subset)
struct RNode {
  enum K : uint8_t { Empty, Set, Cat, Alt, Star, Plus, Opt, Rep, Bol, Eol } k = Empty;
  BSet s;
  int a = -1, b = -1;
  int lo = 0, hi = 0;  // Rep; hi < 0 = unbounded
};

struct RParser {
  const std::string& p;
  size_t i = 0;
  std::vector<RNode> nodes;
  std::string err;
  explicit RParser(const std::string& s) : p(s) {}
  int mk(RNode n) {
    nodes.push_back(n);
    return (int)nodes.size() - 1;
  }
  bool eof() const { return i >= p.size(); }
  int alt() {
    int l = cat();
    if (l < 0) return -1;
    while (!eof() && p[i] == '|') {
      ++i;
      int r = cat();
      if (r < 0) return -1;
      RNode n;
      n.k = RNode::Alt;
      n.a = l;
      n.b = r;
      l = mk(n);
    }
    return l;
  }
  int cat() {
    int l = mk(RNode{});
    while (!eof() && p[i] != '|' && p[i] != ')') {
      int r = rep();
      if (r < 0) return -1;
      RNode n;
      n.k = RNode::Cat;
      n.a = l;
      n.b = r;
      l = mk(n);
    }
    return l;
  }
  bool number(int* v) {
    size_t s = i;
    int x = 0;
    while (!eof() && p[i] >= '0' && p[i] <= '9') {
      x = x * 10 + (p[i] - '0');
      if (x > 1000) return false;
      ++i;
    }
    *v = x;
    return i > s;
  }
  int rep() {
    int a = atom();
    if (a < 0) return -1;
    while (!eof()) {
      char c = p[i];
      RNode n;
      n.a = a;
      if (c == '*') n.k = RNode::Star;
      else if (c == '+') n.k = RNode::Plus;
      else if (c == '?') n.k = RNode::Opt;
      else if (c == '{') {
        ++i;
        int lo, hi;
        if (!number(&lo)) {
          err = "invalid repetition";
          return -1;
        }
        hi = lo;
        if (!eof() && p[i] == ',') {
          ++i;
          if (!eof() && p[i] == '}') hi = -1;
          else if (!number(&hi) || hi < lo) {
            err = "invalid repetition";
            return -1;
          }
        }
        if (eof() || p[i] != '}') {
          err = "unterminated repetition";
          return -1;
        }
        n.k = RNode::Rep;
        n.lo = lo;
        n.hi = hi;
      } else {
        break;
      }
      ++i;
      a = mk(n);
    }
    return a;
  }
  int atom() {
    char c = p[i];
    RNode n;
    if (c == '(') {
      ++i;
      int a = alt();
      if (a < 0) return -1;
      if (eof() || p[i] != ')') {
        err = "unmatched (";
        return -1;
      }
      ++i;
      return a;
    }
    if (c == '*' || c == '+' || c == '?' || c == '{') {
      err = "repetition operator without operand";
      return -1;
    }
    if (c == '^') {
      ++i;
      n.k = RNode::Bol;
      return mk(n);
    }
    if (c == '$') {
      ++i;
      n.k = RNode::Eol;
      return mk(n);
    }
    n.k = RNode::Set;
    if (c == '.') {
      ++i;
      n.s.fill();
      return mk(n);
    }
    if (c == '[') return bracket();
    if (c == '\\') {
      if (i + 1 >= p.size()) {
        err = "trailing backslash";
        return -1;
      }
      char x = p[i + 1];
      i += 2;
      switch (x) {
        case 'd': n.s.range('0', '9'); break;
        case 'D': n.s.range('0', '9'); n.s.invert(); break;
        case 'w': class_set("alnum", &n.s); n.s.set('_'); break;
        case 'W': class_set("alnum", &n.s); n.s.set('_'); n.s.invert(); break;
        case 's': class_set("space", &n.s); break;
        case 'S': class_set("space", &n.s); n.s.invert(); break;
        case 'b': case 'B': case '<': case '>': case '`': case '\'':
          err = "word-boundary assertions are not supported";
          return -1;
        default:
          if (x >= '1' && x <= '9') {
            err = "back-references are not supported";
            return -1;
          }
          n.s.set((unsigned char)x);
      }
      return mk(n);
    }
    ++i;
    n.s.set((unsigned char)c);
    return mk(n);
  }
  int bracket() {
    // POSIX bracket: backslash is literal; ']' first is literal.
    ++i;
    RNode n;
    n.k = RNode::Set;
    bool neg = false;
    if (!eof() && p[i] == '^') {
      neg = true;
      ++i;
    }
    bool first = true;
    while (true) {
      if (eof()) {
        err = "unmatched [";
        return -1;
      }
      unsigned char x = (unsigned char)p[i];
      if (x == ']' && !first) {
        ++i;
        break;
      }
      first = false;
      if (x == '[' && i + 1 < p.size() && p[i + 1] == ':') {
        size_t e = p.find(":]", i + 2);
        if (e == std::string::npos || !class_set(p.substr(i + 2, e - i - 2), &n.s)) {
          err = "invalid character class";
          return -1;
        }
        i = e + 2;
        continue;
      }
      if (x == '[' && i + 1 < p.size() && (p[i + 1] == '.' || p[i + 1] == '=')) {
        err = "collating elements are not supported";
        return -1;
      }
      ++i;
      if (i + 1 < p.size() && p[i] == '-' && p[i + 1] != ']') {
        unsigned hi = (unsigned char)p[i + 1];
        i += 2;
        if (hi < x) {
          err = "invalid range end";
          return -1;
        }
        n.s.range(x, hi);
      } else {
        n.s.set(x);
      }
    }
    if (neg) n.s.invert();
    return mk(n);
  }
};

struct Frag {
  uint32_t s, e;
};

struct Thompson {
  Nfa& nfa;
  const std::vector<RNode>& t;
  bool overflow = false;
  Frag build(int x) {
    if (nfa.st.size() > kMaxNfaStates) {
      overflow = true;
      uint32_t a = nfa.add();
      return {a, a};
    }
    const RNode& n = t[(size_t)x];
    switch (n.k) {
      case RNode::Empty: {
        uint32_t a = nfa.add();
        return {a, a};
      }
      case RNode::Set: {
        uint32_t a = nfa.add(), b = nfa.add();
        nfa.edge(a, n.s, b);
        return {a, b};
      }
      case RNode::Bol: {
        uint32_t a = nfa.add(), b = nfa.add();
        nfa.st[a].bol.push_back(b);
        return {a, b};
      }
      case RNode::Eol: {
        uint32_t a = nfa.add(), b = nfa.add();
        nfa.st[a].eol.push_back(b);
        return {a, b};
      }
      case RNode::Cat: {
        Frag l = build(n.a), r = build(n.b);
        nfa.eps(l.e, r.s);
        return {l.s, r.e};
      }
      case RNode::Alt: {
        Frag l = build(n.a), r = build(n.b);
        uint32_t a = nfa.add(), b = nfa.add();
        nfa.eps(a, l.s);
        nfa.eps(a, r.s);
        nfa.eps(l.e, b);
        nfa.eps(r.e, b);
        return {a, b};
      }
      case RNode::Star:
      case RNode::Plus:
      case RNode::Opt: {
        Frag f = build(n.a);
        uint32_t a = nfa.add(), b = nfa.add();
        nfa.eps(a, f.s);
        nfa.eps(f.e, b);
        if (n.k != RNode::Plus) nfa.eps(a, b);
        if (n.k != RNode::Opt) nfa.eps(f.e, f.s);
        return {a, b};
      }
      case RNode::Rep: {
        uint32_t a = nfa.add();
        uint32_t cur = a;
        for (int k = 0; k < n.lo; ++k) {
          Frag f = build(n.a);
          nfa.eps(cur, f.s);
          cur = f.e;
        }
        if (n.hi < 0) {
          Frag f = build(n.a);
          uint32_t b = nfa.add();
          nfa.eps(cur, f.s);
          nfa.eps(cur, b);
          nfa.eps(f.e, f.s);
          nfa.eps(f.e, b);
          return {a, b};
        }
        uint32_t b = nfa.add();
        nfa.eps(cur, b);
        for (int k = n.lo; k < n.hi; ++k) {
          Frag f = build(n.a);
          nfa.eps(cur, f.s);
          nfa.eps(f.e, b);
          cur = f.e;
        }
        return {a, b};
      }
    }
    uint32_t a = nfa.add();
    return {a, a};
  }
};

// ---------------------------------------------------------------- subset construction
struct SetHash {
  size_t operator()(const std::vector<uint32_t>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t x : v) {
      h ^= x;
      h *= 1099511628211ull;
    }
    return (size_t)h;
  }
};

void closure(const Nfa& nfa, std::vector<uint32_t>* set, bool bol, bool eol,
             std::vector<uint32_t>* mark, uint32_t stamp) {
  std::vector<uint32_t> stack(set->begin(), set->end());
  for (uint32_t x : *set) (*mark)[x] = stamp;
  while (!stack.empty()) {
    uint32_t x = stack.back();
    stack.pop_back();
    auto push = [&](uint32_t y) {
      if ((*mark)[y] != stamp) {
        (*mark)[y] = stamp;
        set->push_back(y);
        stack.push_back(y);
      }
    };
    for (uint32_t y : nfa.st[x].eps) push(y);
    if (bol)
      for (uint32_t y : nfa.st[x].bol) push(y);
    if (eol)
      for (uint32_t y : nfa.st[x].eol) push(y);
  }
  std::sort(set->begin(), set->end());
}

}  // namespace

bool regex_ok(const std::string& re, std::string* err) {
  RParser rp(re);
  int root = rp.alt();
  if (root >= 0 && !rp.eof()) {
    rp.err = "unmatched )";
    root = -1;
  }
  if (root < 0) {
    if (err) *err = rp.err;
    return false;
  }
  return true;
}

uint32_t Dfa::run(const uint8_t* s, size_t n) const {
  uint32_t st = start;
  for (size_t i = 0; i < n && st != 0; ++i) st = trans[(size_t)st * ncls + cls[s[i]]];
  return acc[st];
}

bool compile_dfa(const std::vector<Pattern>& pats, Dfa* out, std::string* err, uint32_t max_states) {
  Nfa nfa;
  uint32_t root = nfa.add();
  BSet any;
  any.fill();
  for (size_t k = 0; k < pats.size(); ++k) {
    const Pattern& P = pats[k];
    if (P.kind == Pattern::Literal) {
      uint32_t cur = nfa.add();
      nfa.eps(root, cur);
      for (unsigned char c : P.text) {
        BSet s;
        s.set(c);
        uint32_t nx = nfa.add();
        nfa.edge(cur, s, nx);
        cur = nx;
      }
      nfa.st[cur].acc = (int)k;
    } else if (P.kind == Pattern::Glob) {
      std::vector<GItem> items;
      bool never = false;
      if (!parse_glob(P.text, &items, &never, err)) return false;
      if (never) continue;
      uint32_t cur = nfa.add();
      nfa.eps(root, cur);
      for (const GItem& g : items) {
        if (g.t == GTok::Star) {
          uint32_t nx = nfa.add();
          nfa.eps(cur, nx);
          nfa.edge(nx, any, nx);
          cur = nx;
        } else {
          uint32_t nx = nfa.add();
          nfa.edge(cur, g.s, nx);
          cur = nx;
        }
      }
      nfa.st[cur].acc = (int)k;
    } else {
      RParser rp(P.text);
      int r = rp.alt();
      if (r >= 0 && !rp.eof()) {
        rp.err = "unmatched )";
        r = -1;
      }
      if (r < 0) {
        *err = "invalid regular expression '" + P.text + "': " + rp.err;
        return false;
      }
      // search semantics: unanchored prefix loop -> pattern -> sticky accept
      uint32_t pre = nfa.add();
      nfa.eps(root, pre);
      nfa.edge(pre, any, pre);
      Thompson th{nfa, rp.nodes};
      Frag f = th.build(r);
      if (th.overflow) {
        *err = "regular expression too large";
        return false;
      }
      nfa.eps(pre, f.s);
      uint32_t acc = nfa.add();
      nfa.eps(f.e, acc);
      nfa.edge(acc, any, acc);
      nfa.st[acc].acc = (int)k;
    }
  }
  if (nfa.st.size() > kMaxNfaStates) {
    *err = "pattern set too large";
    return false;
  }

  // byte classes: refine the single class by every edge set
  std::array<uint16_t, 256> cl{};
  uint32_t ncl = 1;
  for (const BSet& s : nfa.sets) {
    std::map<std::pair<uint16_t, bool>, uint16_t> remap;
    uint32_t next = 0;
    std::array<uint16_t, 256> nc{};
    for (unsigned b = 0; b < 256; ++b) {
      auto key = std::make_pair(cl[b], s.has(b));
      auto it = remap.find(key);
      if (it == remap.end()) it = remap.emplace(key, (uint16_t)next++).first;
      nc[b] = it->second;
    }
    cl = nc;
    ncl = next;
  }
  std::vector<unsigned> rep(ncl);
  for (int b = 255; b >= 0; --b) rep[cl[(unsigned)b]] = (unsigned)b;
  // per NFA set: membership per class
  std::vector<std::vector<uint8_t>> set_has(nfa.sets.size(), std::vector<uint8_t>(ncl));
  for (size_t s = 0; s < nfa.sets.size(); ++s)
    for (uint32_t c = 0; c < ncl; ++c) set_has[s][c] = nfa.sets[s].has(rep[c]);

  std::vector<uint32_t> mark(nfa.st.size(), 0);
  uint32_t stamp = 0;
  std::unordered_map<std::vector<uint32_t>, uint32_t, SetHash> ids;
  std::vector<std::vector<uint32_t>> dstates;
  std::vector<uint32_t> trans;
  std::vector<uint32_t> acc;  // accept class per DFA state
  std::map<std::vector<uint32_t>, uint32_t> class_ids;
  std::vector<std::vector<uint32_t>> classes;
  class_ids[{}] = 0;
  classes.push_back({});
  auto accept_of = [&](const std::vector<uint32_t>& set) {
    std::vector<uint32_t> e = set;
    closure(nfa, &e, false, true, &mark, ++stamp);
    std::vector<uint32_t> m;
    for (uint32_t x : e)
      if (nfa.st[x].acc >= 0) m.push_back((uint32_t)nfa.st[x].acc);
    std::sort(m.begin(), m.end());
    m.erase(std::unique(m.begin(), m.end()), m.end());
    auto it = class_ids.find(m);
    if (it == class_ids.end()) {
      it = class_ids.emplace(m, (uint32_t)classes.size()).first;
      classes.push_back(m);
    }
    return it->second;
  };
  // dead state 0
  dstates.push_back({});
  ids[{}] = 0;
  acc.push_back(0);
  std::vector<uint32_t> s0 = {root};
  closure(nfa, &s0, true, false, &mark, ++stamp);
  ids[s0] = 1;
  dstates.push_back(s0);
  acc.push_back(accept_of(s0));
  std::vector<uint32_t> work = {1};
  trans.assign((size_t)2 * ncl, 0);
  while (!work.empty()) {
    uint32_t d = work.back();
    work.pop_back();
    for (uint32_t c = 0; c < ncl; ++c) {
      std::vector<uint32_t> nx;
      ++stamp;
      for (uint32_t x : dstates[d])
        for (auto& e : nfa.st[x].tr)
          if (set_has[e.first][c] && mark[e.second] != stamp) {
            mark[e.second] = stamp;
            nx.push_back(e.second);
          }
      closure(nfa, &nx, false, false, &mark, ++stamp);
      uint32_t id;
      auto it = ids.find(nx);
      if (it != ids.end()) {
        id = it->second;
      } else {
        id = (uint32_t)dstates.size();
        if (id >= max_states) {
          *err = "automaton exceeds the state limit";
          return false;
        }
        ids.emplace(nx, id);
        dstates.push_back(nx);
        acc.push_back(accept_of(nx));
        trans.resize((size_t)(id + 1) * ncl, 0);
        work.push_back(id);
      }
      trans[(size_t)d * ncl + c] = (uint16_t)id;
    }
  }
  uint32_t ns = (uint32_t)dstates.size();

  // Moore minimisation: initial partition by accept class (dead state keeps its own block when
  // its class is 0 and its transitions are all dead — it merges with equivalent states, fine).
  std::vector<uint32_t> blk(ns);
  {
    std::map<uint32_t, uint32_t> m;
    for (uint32_t s = 0; s < ns; ++s) {
      auto it = m.find(acc[s]);
      if (it == m.end()) it = m.emplace(acc[s], (uint32_t)m.size()).first;
      blk[s] = it->second;
    }
  }
  uint32_t nblk = 0;
  for (uint32_t b : blk) nblk = std::max(nblk, b + 1);
  while (true) {
    std::map<std::vector<uint32_t>, uint32_t> sig;
    std::vector<uint32_t> nb(ns);
    for (uint32_t s = 0; s < ns; ++s) {
      std::vector<uint32_t> k;
      k.reserve(ncl + 1);
      k.push_back(blk[s]);
      for (uint32_t c = 0; c < ncl; ++c) k.push_back(blk[trans[(size_t)s * ncl + c]]);
      auto it = sig.find(k);
      if (it == sig.end()) it = sig.emplace(std::move(k), (uint32_t)sig.size()).first;
      nb[s] = it->second;
    }
    uint32_t n2 = (uint32_t)sig.size();
    blk = nb;
    if (n2 == nblk) break;
    nblk = n2;
  }
  // renumber: block of the dead state -> 0, start block -> as found
  std::vector<int64_t> newid(nblk, -1);
  uint32_t next = 0;
  newid[blk[0]] = next++;
  for (uint32_t s = 1; s < ns; ++s)
    if (newid[blk[s]] < 0) newid[blk[s]] = next++;
  out->nstates = next;
  out->ncls = ncl;
  out->start = (uint32_t)newid[blk[1]];
  for (unsigned b = 0; b < 256; ++b) out->cls[b] = (uint8_t)cl[b];
  if (next > max_states) {
    *err = "automaton exceeds the state limit";
    return false;
  }
  out->trans.assign((size_t)next * ncl, 0);
  out->acc.assign(next, 0);
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t t = (uint32_t)newid[blk[s]];
    out->acc[t] = acc[s];
    for (uint32_t c = 0; c < ncl; ++c)
      out->trans[(size_t)t * ncl + c] = (uint16_t)newid[blk[trans[(size_t)s * ncl + c]]];
  }
  if (ncl > 256) {
    *err = "too many byte classes";
    return false;
  }
  // absorbing states (all transitions to themselves; e.g. a glob's trailing `*` reached, an
  // unanchored regex matched) move to the end, [abs_lo, nstates): the kernels' walks stop there
  {
    const uint32_t n = out->nstates;
    std::vector<uint32_t> perm(n, 0);
    uint32_t at = 1;
    auto absorbing = [&](uint32_t t) {
      for (uint32_t c = 0; c < ncl; ++c)
        if (out->trans[(size_t)t * ncl + c] != t) return false;
      return true;
    };
    for (uint32_t t = 1; t < n; ++t)
      if (!absorbing(t)) perm[t] = at++;
    out->abs_lo = at;
    for (uint32_t t = 1; t < n; ++t)
      if (absorbing(t)) perm[t] = at++;
    std::vector<uint16_t> tr(out->trans.size());
    std::vector<uint32_t> ac(n);
    for (uint32_t t = 0; t < n; ++t) {
      ac[perm[t]] = out->acc[t];
      for (uint32_t c = 0; c < ncl; ++c) tr[(size_t)perm[t] * ncl + c] = (uint16_t)perm[out->trans[(size_t)t * ncl + c]];
    }
    out->trans.swap(tr);
    out->acc.swap(ac);
    out->start = perm[out->start];
  }
  // class ids in order of first use by a state (the dead state's empty set stays 0), unused sets
  // of the unminimised automaton dropped
  std::vector<int64_t> cmap(classes.size(), -1);
  cmap[0] = 0;
  out->classes.assign(1, {});
  for (uint32_t& a : out->acc) {
    if (cmap[a] < 0) {
      cmap[a] = (int64_t)out->classes.size();
      out->classes.push_back(classes[a]);
    }
    a = (uint32_t)cmap[a];
  }
  return true;
}

bool compile_column(const std::vector<Pattern>& pats, size_t max_bytes, uint32_t max_states, std::vector<Dfa>* out,
                    std::string* err, std::vector<uint32_t>* firsts) {
  out->clear();
  if (firsts) firsts->clear();
  size_t i = 0;
  while (i < pats.size()) {
    // grow the group [i, j) while its automaton fits; doubling steps, then bisection, so a large
    // column costs O(log n) compilations per DFA rather than one per pattern
    std::vector<Pattern> group{pats[i]};
    Dfa best;
    if (!compile_dfa(group, &best, err, max_states)) return false;
    size_t good = 1, step = 1;
    auto try_n = [&](size_t n, Dfa* d) {
      std::vector<Pattern> g(pats.begin() + (long)i, pats.begin() + (long)(i + n));
      std::string e2;
      return compile_dfa(g, d, &e2, max_states) && d->table_bytes() <= max_bytes;
    };
    size_t bad = 0;  // smallest known size that does not fit (0 = none)
    while (i + good < pats.size()) {
      const size_t n = std::min(pats.size() - i, good + step);
      Dfa d;
      if (try_n(n, &d)) {
        good = n;
        best = std::move(d);
        step *= 2;
      } else {
        bad = n;
        break;
      }
    }
    while (bad && bad - good > 1) {
      const size_t n = good + (bad - good) / 2;
      Dfa d;
      if (try_n(n, &d)) {
        good = n;
        best = std::move(d);
      } else {
        bad = n;
      }
    }
    // local pattern k of the group is column pattern i + k
    if (firsts) firsts->push_back((uint32_t)i);
    for (auto& c : best.classes)
      for (auto& p : c) p += (uint32_t)i;
    out->push_back(std::move(best));
    i += good;
  }
  return true;
}

}  // namespace kw
