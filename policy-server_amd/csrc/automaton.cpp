// automaton.cpp — glob / literal / regex pattern sets -> minimised multi-pattern DFA.
// See automaton.hpp for semantics. Construction: each pattern becomes an NFA fragment (glob
// chain or Thompson construction), all fragments share one start; subset construction with
// beginning-of-string assertions followed only from the initial closure and end-of-string
// assertions followed only when computing a state's accept mask; byte classes from the partition
// of all edge sets; Moore minimisation.
#include "automaton.hpp"

#include <cstring>

#include "kwdev.hpp"
#include "unicode_data.hpp"

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
  std::vector<std::pair<uint32_t, uint32_t>> tr;    // (set id, target)
  std::vector<uint32_t> eps;
  // (allowed (prev, next) kinds: a 16-bit mask, | kAssertUni when the kinds are those of the code
  // points around the position (Unicode word boundaries), target)
  std::vector<std::pair<uint32_t, uint32_t>> asrt;
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
const char* const kStateLimitError = "automaton exceeds the state limit";

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
// fnmatch(3) without flags, over characters (a UTF-8 locale's multibyte matching): `*` any string
// ('/' included), `?` one character, `[...]` / `[!...]` / `[^...]` one character of a set with
// ranges (code point order), `[:class:]` (ASCII classes) and `\` escapes, `\x` the character x; an
// unterminated `[` is an ordinary character and a trailing `\` never matches (glibc).
enum class GTok : uint8_t { Set, Star };
struct GItem {
  GTok t;
  std::vector<std::pair<uint32_t, uint32_t>> cs;  // code point ranges (sorted, disjoint)
};

// next UTF-8 character of s at *i (advances), -1 when the bytes there are not valid UTF-8
int64_t utf8_next(const std::string& s, size_t* i) {
  const unsigned char c = (unsigned char)s[*i];
  const int n = c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
  if (n == 0 || *i + (size_t)n > s.size()) return -1;
  uint32_t v = n == 1 ? c : c & (0x7Fu >> n);
  for (int k = 1; k < n; ++k) {
    const unsigned char d = (unsigned char)s[*i + (size_t)k];
    if ((d & 0xC0) != 0x80) return -1;
    v = (v << 6) | (d & 0x3F);
  }
  static const uint32_t min_of[5] = {0, 0, 0x80, 0x800, 0x10000};
  if (v < min_of[n] || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return -1;
  *i += (size_t)n;
  return v;
}

// Returns false on unsupported syntax; *never = true if glibc would never match (trailing '\').
bool parse_glob(const std::string& p, std::vector<GItem>* out, bool* never, std::string* err) {
  *never = false;
  size_t i = 0, n = p.size();
  for (size_t k = 0; k < n;)
    if (utf8_next(p, &k) < 0) {
      *err = "glob '" + p + "' is not valid UTF-8";
      return false;
    }
  auto one = [](uint32_t c) {
    GItem g{GTok::Set, {}};
    g.cs.push_back({c, c});
    return g;
  };
  while (i < n) {
    const unsigned char c = (unsigned char)p[i];
    if (c == '*') {
      out->push_back({GTok::Star, {}});
      ++i;
      continue;
    }
    if (c == '?') {
      GItem g{GTok::Set, {}};
      g.cs = {{0, 0xD7FF}, {0xE000, 0x10FFFF}};
      out->push_back(g);
      ++i;
      continue;
    }
    if (c == '\\') {
      if (i + 1 >= n) {
        *never = true;  // glibc: "Trailing \ loses."
        return true;
      }
      ++i;
      out->push_back(one((uint32_t)utf8_next(p, &i)));
      continue;
    }
    if (c == '[') {
      size_t j = i + 1;
      bool neg = false;
      if (j < n && (p[j] == '!' || p[j] == '^')) {
        neg = true;
        ++j;
      }
      std::vector<std::pair<uint32_t, uint32_t>> s;
      bool first = true, closed = false;
      while (j < n) {
        const unsigned char x = (unsigned char)p[j];
        if (x == ']' && !first) {
          closed = true;
          ++j;
          break;
        }
        first = false;
        if (x == '[' && j + 1 < n && p[j + 1] == ':') {
          // glibc: a class name is lowercase letters a-y up to ":]"; anything else makes this '['
          // an ordinary member of the set
          size_t e = j + 2;
          while (e < n && p[e] >= 'a' && p[e] < 'z') ++e;
          if (!(e + 1 < n && p[e] == ':' && p[e + 1] == ']')) {
            s.push_back({'[', '['});
            ++j;
            continue;
          }
          BSet cls;
          if (!class_set(p.substr(j + 2, e - j - 2), &cls)) {
            *err = "unsupported character class in glob '" + p + "'";
            return false;
          }
          for (unsigned b = 0; b < 128; ++b)
            if (cls.has(b)) s.push_back({b, b});
          j = e + 2;
          continue;
        }
        if (x == '[' && j + 1 < n && (p[j + 1] == '.' || p[j + 1] == '=')) {
          *err = "collating elements are not supported in glob '" + p + "'";
          return false;
        }
        if (x == '\\') {
          if (j + 1 >= n) break;  // unterminated
          ++j;
        }
        const uint32_t lo = (uint32_t)utf8_next(p, &j);
        if (j < n && p[j] == '-' && (j + 1 >= n || p[j + 1] != ']')) {
          ++j;
          if (j < n && p[j] == '\\') ++j;
          if (j >= n) {  // glibc: a range without its upper end fails the match
            *never = true;
            return true;
          }
          const uint32_t hi = (uint32_t)utf8_next(p, &j);
          if (lo <= hi) s.push_back({lo, hi});
        } else {
          s.push_back({lo, lo});
        }
      }
      if (!closed) {  // glibc: unterminated '[' is an ordinary character
        out->push_back(one('['));
        ++i;
        continue;
      }
      std::sort(s.begin(), s.end());
      std::vector<std::pair<uint32_t, uint32_t>> m;
      for (const auto& r : s) {
        if (!m.empty() && r.first <= m.back().second + 1) m.back().second = std::max(m.back().second, r.second);
        else m.push_back(r);
      }
      if (neg) {  // the complement within the Unicode scalar values
        std::vector<std::pair<uint32_t, uint32_t>> c2;
        uint32_t at = 0;
        for (const auto& r : m) {
          if (r.first > at) c2.push_back({at, r.first - 1});
          at = r.second + 1;
        }
        if (at <= 0x10FFFF) c2.push_back({at, 0x10FFFF});
        m.clear();
        for (const auto& r : c2) {
          if (r.second < 0xD800 || r.first > 0xDFFF) {
            m.push_back(r);
          } else {
            if (r.first < 0xD800) m.push_back({r.first, 0xD7FF});
            if (r.second > 0xDFFF) m.push_back({0xE000, r.second});
          }
        }
      }
      out->push_back({GTok::Set, m});
      i = j;
      continue;
    }
    out->push_back(one((uint32_t)utf8_next(p, &i)));
  }
  return true;
}

// ---------------------------------------------------------------- regex (Rust `regex` crate dialect)
// The label-constraint regexes are Rust `regex` patterns (the upstream safe-labels policy compiles
// them with `Regex::new` and tests them with `is_match`: search semantics). The dialect here:
//   syntax   alternation, concatenation, `(...)`, `(?:...)`, `(?P<name>...)` / `(?<name>...)`,
//            flag groups `(?imsxUu-imsxUu)` and `(?flags:...)`, `* + ? {n} {n,} {n,m}` with an
//            optional lazy `?` (no effect on is_match), `.`, `[...]` classes with ranges, nesting,
//            `&&` `--` `~~`, `[:name:]` / `[:^name:]` ASCII classes, escapes `\d \D \w \W \s \S`,
//            `\a \f \t \n \r \v`, `\xHH \x{H..} \uHHHH \u{H..} \UHHHHHHHH \U{H..}`, escaped ASCII
//            punctuation and space, assertions `^ $ \A \z \b \B \< \> \b{start} \b{end}
//            \b{start-half} \b{end-half}`;
//   matching over Unicode scalar values encoded as UTF-8 (`.` and negated classes consume one whole
//            character); `\d \w \s`, `\b` and case folding (`i`) are ASCII (as with `(?-u:...)`
//            for those four; the only difference from Rust's Unicode defaults is on non-ASCII
//            digits / letters / spaces, which valid label values never contain);
//   refused  (a syntax error: the policy becomes an init error) `\p{..}` / `\P{..}` Unicode
//            property classes, back-references, look-around, the `R` (CRLF) flag, and, with `u`
//            off, any construct that could match a non-ASCII byte (as Rust refuses for str regexes).
// Assertions are conditions on the kinds of the bytes before and after a position
// (EDGE = start / end of the string, NL = '\n', WORD = [0-9A-Za-z_], OTHER), a 4 x 4 bit mask.
enum : uint32_t { BK_EDGE = 0, BK_NL = 1, BK_WORD = 2, BK_OTHER = 3 };
inline uint32_t byte_kind(unsigned c) {
  if (c == '\n') return BK_NL;
  const bool w = (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
  return w ? BK_WORD : BK_OTHER;
}
template <class F>
uint16_t kind_mask(F f) {
  uint16_t m = 0;
  for (uint32_t p = 0; p < 4; ++p)
    for (uint32_t n = 0; n < 4; ++n)
      if (f(p, n)) m |= (uint16_t)(1u << (p * 4 + n));
  return m;
}
inline bool kw_word(uint32_t k) { return k == BK_WORD; }

struct CRange {
  uint32_t lo, hi;
};
typedef std::vector<CRange> CSet;  // sorted, disjoint, non-adjacent code point ranges

CSet cs_norm(CSet v) {
  std::sort(v.begin(), v.end(), [](const CRange& a, const CRange& b) { return a.lo < b.lo; });
  CSet o;
  for (const CRange& r : v) {
    if (!o.empty() && r.lo <= o.back().hi + 1) o.back().hi = std::max(o.back().hi, r.hi);
    else o.push_back(r);
  }
  return o;
}
CSet cs_valid() { return {{0, 0xD7FF}, {0xE000, 0x10FFFF}}; }
CSet cs_inter(const CSet& a, const CSet& b) {
  CSet o;
  for (const CRange& x : a)
    for (const CRange& y : b) {
      const uint32_t lo = std::max(x.lo, y.lo), hi = std::min(x.hi, y.hi);
      if (lo <= hi) o.push_back({lo, hi});
    }
  return cs_norm(o);
}
CSet cs_neg(const CSet& a) {  // complement within the Unicode scalar values
  CSet o;
  uint32_t at = 0;
  for (const CRange& r : a) {
    if (r.lo > at) o.push_back({at, r.lo - 1});
    at = r.hi + 1;
  }
  if (at <= 0x10FFFF) o.push_back({at, 0x10FFFF});
  return cs_inter(o, cs_valid());
}
CSet cs_union(CSet a, const CSet& b) {
  a.insert(a.end(), b.begin(), b.end());
  return cs_norm(a);
}
CSet cs_diff(const CSet& a, const CSet& b) { return cs_inter(a, cs_neg(b)); }
CSet cs_sym(const CSet& a, const CSet& b) { return cs_union(cs_diff(a, b), cs_diff(b, a)); }
void cs_fold_ascii(CSet* s) {  // close under ASCII case folding
  CSet add;
  for (const CRange& r : *s) {
    const uint32_t ulo = std::max(r.lo, (uint32_t)'A'), uhi = std::min(r.hi, (uint32_t)'Z');
    if (ulo <= uhi) add.push_back({ulo + 32, uhi + 32});
    const uint32_t llo = std::max(r.lo, (uint32_t)'a'), lhi = std::min(r.hi, (uint32_t)'z');
    if (llo <= lhi) add.push_back({llo - 32, lhi - 32});
  }
  *s = cs_union(*s, add);
}
bool cs_nonascii(const CSet& s) { return !s.empty() && s.back().hi >= 0x80; }
// close under Unicode simple case folding (every member of a code point's fold orbit)
void cs_fold_unicode(CSet* s) {
  CSet add;
  for (const CRange& r : *s) {
    const UniFold* b = std::lower_bound(kUniFold, kUniFold + kUniFoldN, r.lo,
                                        [](const UniFold& f, uint32_t v) { return f.cp < v; });
    for (const UniFold* f = b; f < kUniFold + kUniFoldN && f->cp <= r.hi; ++f)
      for (uint32_t c = f->next; c != f->cp;) {
        add.push_back({c, c});
        const UniFold* g = std::lower_bound(kUniFold, kUniFold + kUniFoldN, c,
                                            [](const UniFold& x, uint32_t v) { return x.cp < v; });
        c = g->next;
      }
  }
  *s = cs_union(*s, add);
}
// (?i): Unicode simple case folding in Unicode mode, ASCII folding with `u` off (regex-syntax)
void cs_fold(CSet* s, bool unicode) {
  if (unicode) cs_fold_unicode(s);
  else cs_fold_ascii(s);
}
CSet cs_table(const UniRange* t, uint32_t n) {
  CSet o;
  for (uint32_t k = 0; k < n; ++k) o.push_back({t[k].lo, t[k].hi});
  return o;
}
// White_Space (PropList.txt), Rust's Unicode \s
CSet cs_uni_space() {
  return {{9, 13}, {0x20, 0x20}, {0x85, 0x85}, {0xA0, 0xA0}, {0x1680, 0x1680}, {0x2000, 0x200A},
          {0x2028, 0x2029}, {0x202F, 0x202F}, {0x205F, 0x205F}, {0x3000, 0x3000}};
}
constexpr uint32_t kAssertUni = 1u << 16;  // an assertion over the kinds of code points

// \p{..} / \P{..} (r06): the General_Category values of regex-syntax, by their short
// and long names and aliases, matched loosely (UAX44-LM3 as regex-syntax's symbolic_name_normalize:
// ASCII case, ' ', '_' and '-' ignored, an "is" prefix dropped), bare or as gc= / general_category=
// (':' and '!=' too); plus Any, ASCII, Assigned and the White_Space property. Script and the other
// properties are refused by name: this image's Unicode data has no Script property.
std::string uni_name_normalize(const std::string& x) {
  size_t start = 0;
  const bool is = x.size() >= 2 && (x[0] == 'i' || x[0] == 'I') && (x[1] == 's' || x[1] == 'S');
  if (is) start = 2;
  std::string o;
  for (size_t k = start; k < x.size(); ++k) {
    const unsigned char b = (unsigned char)x[k];
    if (b == ' ' || b == '_' || b == '-' || b >= 0x80) continue;
    o.push_back((char)(b >= 'A' && b <= 'Z' ? b + 32 : b));
  }
  if (is && o == "c") o = "isc";  // (regex-syntax: ISO_Comment's 'isc', not Other)
  return o;
}
// the set of a General_Category value (normalized name), false when it is none
bool uni_gencat(const std::string& v, CSet* out) {
  static const std::map<std::string, std::string> alias = {
      {"lu", "Lu"}, {"uppercaseletter", "Lu"}, {"ll", "Ll"}, {"lowercaseletter", "Ll"}, {"lt", "Lt"},
      {"titlecaseletter", "Lt"}, {"lc", "LC"}, {"casedletter", "LC"}, {"l&", "LC"}, {"lm", "Lm"},
      {"modifierletter", "Lm"}, {"lo", "Lo"}, {"otherletter", "Lo"}, {"l", "L"}, {"letter", "L"},
      {"mn", "Mn"}, {"nonspacingmark", "Mn"}, {"mc", "Mc"}, {"spacingmark", "Mc"}, {"me", "Me"},
      {"enclosingmark", "Me"}, {"m", "M"}, {"mark", "M"}, {"combiningmark", "M"}, {"nd", "Nd"},
      {"decimalnumber", "Nd"}, {"digit", "Nd"}, {"nl", "Nl"}, {"letternumber", "Nl"}, {"no", "No"},
      {"othernumber", "No"}, {"n", "N"}, {"number", "N"}, {"pc", "Pc"}, {"connectorpunctuation", "Pc"},
      {"pd", "Pd"}, {"dashpunctuation", "Pd"}, {"ps", "Ps"}, {"openpunctuation", "Ps"}, {"pe", "Pe"},
      {"closepunctuation", "Pe"}, {"pi", "Pi"}, {"initialpunctuation", "Pi"}, {"pf", "Pf"},
      {"finalpunctuation", "Pf"}, {"po", "Po"}, {"otherpunctuation", "Po"}, {"p", "P"}, {"punctuation", "P"},
      {"punct", "P"}, {"sm", "Sm"}, {"mathsymbol", "Sm"}, {"sc", "Sc"}, {"currencysymbol", "Sc"}, {"sk", "Sk"},
      {"modifiersymbol", "Sk"}, {"so", "So"}, {"othersymbol", "So"}, {"s", "S"}, {"symbol", "S"},
      {"zs", "Zs"}, {"spaceseparator", "Zs"}, {"zl", "Zl"}, {"lineseparator", "Zl"}, {"zp", "Zp"},
      {"paragraphseparator", "Zp"}, {"z", "Z"}, {"separator", "Z"}, {"cc", "Cc"}, {"control", "Cc"},
      {"cntrl", "Cc"}, {"cf", "Cf"}, {"format", "Cf"}, {"cs", "Cs"}, {"surrogate", "Cs"}, {"co", "Co"},
      {"privateuse", "Co"}, {"cn", "Cn"}, {"unassigned", "Cn"}, {"c", "C"}, {"other", "C"},
      {"any", "Any"}, {"ascii", "ASCII"}, {"assigned", "Assigned"}};
  auto it = alias.find(v);
  if (it == alias.end()) return false;
  const std::string& g = it->second;
  if (g == "Any") {
    *out = {{0, 0x10FFFF}};
  } else if (g == "ASCII") {
    *out = {{0, 0x7F}};
  } else {
    // a value names the categories whose two-letter names it prefixes (L: Lu Ll Lt Lm Lo; LC: Lu Ll
    // Lt); Cn and Assigned are the code points outside / inside the runs
    auto member = [&](const char* name) {
      if (g == "LC") return !strcmp(name, "Lu") || !strcmp(name, "Ll") || !strcmp(name, "Lt");
      if (g.size() == 1) return name[0] == g[0];
      return g == name;
    };
    CSet assigned, hit;
    for (uint32_t k = 0; k < kUniGcN; ++k) {
      assigned.push_back({kUniGc[k].lo, kUniGc[k].hi});
      if (g != "Assigned" && member(kUniGcNames[kUniGc[k].gc])) hit.push_back({kUniGc[k].lo, kUniGc[k].hi});
    }
    assigned = cs_union(assigned, {});
    if (g == "Assigned") hit = assigned;
    else if (g == "Cn" || g == "C") hit = cs_union(hit, cs_neg(assigned));
    else hit = cs_union(hit, {});
    *out = hit;
  }
  CSet noncs;  // (surrogates are no scalar values: never matched)
  for (const CRange& r : *out) {
    if (r.hi < 0xD800 || r.lo > 0xDFFF) noncs.push_back(r);
    else {
      if (r.lo < 0xD800) noncs.push_back({r.lo, 0xD7FF});
      if (r.hi > 0xDFFF) noncs.push_back({0xE000, r.hi});
    }
  }
  *out = noncs;
  return true;
}
bool uni_property(const std::string& body, CSet* out, bool* negate, std::string* err) {
  size_t eq = body.find('=');
  const size_t colon = body.find(':');
  if (eq == std::string::npos) eq = colon;
  std::string value = body;
  if (eq != std::string::npos) {
    std::string prop = body.substr(0, eq);
    if (!prop.empty() && prop.back() == '!') {  // name!=value
      prop.pop_back();
      *negate = !*negate;
    }
    value = body.substr(eq + 1);
    const std::string np = uni_name_normalize(prop);
    if (np != "gc" && np != "generalcategory") {
      *err = std::string("unsupported by this engine: the Unicode property \\p{") + body + "}" +
             (np == "sc" || np == "script" || np == "scx" || np == "scriptextensions" ? " (scripts)" : "");
      return false;
    }
  }
  const std::string nv = uni_name_normalize(value);
  if (eq == std::string::npos && (nv == "whitespace" || nv == "wspace" || nv == "space")) {
    *out = cs_uni_space();
    return true;
  }
  if (uni_gencat(nv, out)) return true;
  *err = std::string("unsupported by this engine: the Unicode property \\p{") + body +
         "} (only General_Category values and White_Space)";
  return false;
}

// ASCII classes: [:name:] and the \d \w \s escapes
bool ascii_class(const std::string& name, CSet* s) {
  static const std::map<std::string, CSet> k = {
      {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
      {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
      {"ascii", {{0, 0x7F}}},
      {"blank", {{'\t', '\t'}, {' ', ' '}}},
      {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
      {"digit", {{'0', '9'}}},
      {"graph", {{'!', '~'}}},
      {"lower", {{'a', 'z'}}},
      {"print", {{' ', '~'}}},
      {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
      {"space", {{'\t', '\r'}, {' ', ' '}}},
      {"upper", {{'A', 'Z'}}},
      {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
      {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
  };
  auto it = k.find(name);
  if (it == k.end()) return false;
  *s = it->second;
  return true;
}

struct RNode {
  enum K : uint8_t { Empty, Set, Cat, Alt, Star, Plus, Opt, Rep, Assert } k = Empty;
  CSet cs;
  uint32_t mask = 0;  // Assert: allowed (prev kind, next kind) pairs | kAssertUni
  int a = -1, b = -1;
  int lo = 0, hi = 0;  // Rep; hi < 0 = unbounded
};

struct RFlags {
  bool i = false, m = false, s = false, x = false, u = true;
};

struct RParser {
  const std::string& p;
  size_t i = 0;
  std::vector<RNode> nodes;
  std::vector<std::string> names;
  std::string err;
  RFlags f;
  int depth = 0;
  explicit RParser(const std::string& s) : p(s) {}
  int mk(RNode n) {
    nodes.push_back(std::move(n));
    return (int)nodes.size() - 1;
  }
  int fail(const std::string& e) {
    if (err.empty()) err = e;
    return -1;
  }
  bool eof() const { return i >= p.size(); }
  // one UTF-8 encoded character of the pattern at i (advances); -1 on malformed UTF-8
  int64_t getc_() {
    const unsigned char c = (unsigned char)p[i];
    if (c < 0x80) {
      ++i;
      return c;
    }
    int n = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 0;
    if (!n || c > 0xF4 || i + (size_t)n > p.size()) return -1;
    uint32_t v = c & (0x7Fu >> n);
    for (int k = 1; k < n; ++k) {
      const unsigned char d = (unsigned char)p[i + (size_t)k];
      if ((d & 0xC0) != 0x80) return -1;
      v = (v << 6) | (d & 0x3F);
    }
    static const uint32_t min_of[5] = {0, 0, 0x80, 0x800, 0x10000};
    if (v < min_of[n] || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return -1;
    i += (size_t)n;
    return v;
  }
  bool is_space(uint32_t c) const {
    return (c >= 9 && c <= 13) || c == ' ' || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
           c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
  }
  // verbose mode: skip white space and `#` comments
  void skip_x() {
    if (!f.x) return;
    while (!eof()) {
      const size_t at = i;
      const int64_t c = getc_();
      if (c >= 0 && is_space((uint32_t)c)) continue;
      if (c == '#') {
        while (!eof() && p[i] != '\n') ++i;
        continue;
      }
      i = at;
      return;
    }
  }
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
    for (;;) {
      skip_x();
      if (eof() || p[i] == '|' || p[i] == ')') break;
      int r = rep();
      if (r == -2) continue;  // a flag directive: nothing to concatenate
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
    skip_x();
    size_t s = i;
    int64_t x = 0;
    while (!eof() && p[i] >= '0' && p[i] <= '9') {
      x = x * 10 + (p[i] - '0');
      if (x > 100000) return false;
      ++i;
    }
    *v = (int)x;
    skip_x();
    return i > s;
  }
  int rep() {
    int a = atom();
    if (a < 0) return a;
    for (;;) {
      skip_x();
      if (eof()) break;
      const char c = p[i];
      RNode n;
      n.a = a;
      if (c == '*') n.k = RNode::Star;
      else if (c == '+') n.k = RNode::Plus;
      else if (c == '?') n.k = RNode::Opt;
      else if (c == '{') {
        ++i;
        int lo, hi;
        if (!number(&lo)) return fail("invalid counted repetition");
        hi = lo;
        if (!eof() && p[i] == ',') {
          ++i;
          skip_x();
          if (!eof() && p[i] == '}') hi = -1;
          else if (!number(&hi)) return fail("invalid counted repetition");
          else if (hi < lo) return fail("invalid counted repetition range");
        }
        if (eof() || p[i] != '}') return fail("unclosed counted repetition");
        n.k = RNode::Rep;
        n.lo = lo;
        n.hi = hi;
      } else {
        break;
      }
      ++i;
      if (!eof() && p[i] == '?') ++i;  // lazy: the same language
      a = mk(n);
    }
    return a;
  }
  int set_node(CSet cs) {
    RNode n;
    n.k = RNode::Set;
    if (f.i) cs_fold(&cs, f.u);
    cs = cs_inter(cs, cs_valid());
    if (!f.u && cs_nonascii(cs)) return fail("pattern can match invalid UTF-8 (Unicode mode is off)");
    n.cs = std::move(cs);
    return mk(n);
  }
  int assert_node(uint32_t mask) {
    RNode n;
    n.k = RNode::Assert;
    n.mask = mask;
    return mk(n);
  }
  // a word-boundary assertion just set in *mask: over the kinds of code points in Unicode mode
  uint32_t* cur_mask = nullptr;
  void uni_word(int64_t c) {
    if (f.u && c != 'A' && c != 'z' && cur_mask) *cur_mask |= kAssertUni;
  }
  // hex digits of \x / \u / \U: exactly `fixed` digits, or {1-8 digits}
  bool hex_escape(int fixed, uint32_t* v) {
    uint64_t x = 0;
    int nd = 0;
    if (!eof() && p[i] == '{') {
      ++i;
      while (!eof() && p[i] != '}') {
        const char c = p[i];
        const int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
        if (d < 0 || ++nd > 8) return false;
        x = x * 16 + (uint64_t)d;
        ++i;
      }
      if (eof() || nd == 0) return false;
      ++i;
    } else {
      for (int k = 0; k < fixed; ++k) {
        if (eof()) return false;
        const char c = p[i];
        const int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
        if (d < 0) return false;
        x = x * 16 + (uint64_t)d;
        ++i;
      }
    }
    if (x > 0x10FFFF || (x >= 0xD800 && x <= 0xDFFF)) return false;
    *v = (uint32_t)x;
    return true;
  }
  // An escape after '\' (i at the escaped character). Literal / class escapes set *cs and return 1;
  // assertions set *mask and return 2 (not in classes); errors return 0.
  int escape(bool in_class, CSet* cs, uint32_t* mask) {
    if (eof()) {
      err = "incomplete escape sequence";
      return 0;
    }
    const size_t at = i;
    cur_mask = mask;
    const int64_t c = getc_();
    if (c < 0) {
      err = "invalid UTF-8 in pattern";
      return 0;
    }
    // \d \w \s: Unicode (Nd; Alphabetic + M + Nd + Pc + Join_Control; White_Space), ASCII with `u` off
    auto cls = [&](const char* name, bool neg) {
      if (!f.u) ascii_class(name, cs);
      else if (name[0] == 'd') *cs = cs_table(kUniDigit, kUniDigitN);
      else if (name[0] == 'w') *cs = cs_table(kUniWord, kUniWordN);
      else *cs = cs_uni_space();
      if (neg) *cs = cs_neg(*cs);
      return 1;
    };
    switch (c) {
      case 'd': return cls("digit", false);
      case 'D': return cls("digit", true);
      case 'w': return cls("word", false);
      case 'W': return cls("word", true);
      case 's': return cls("space", false);
      case 'S': return cls("space", true);
      case 'a': *cs = {{7, 7}}; return 1;
      case 'f': *cs = {{12, 12}}; return 1;
      case 't': *cs = {{9, 9}}; return 1;
      case 'n': *cs = {{10, 10}}; return 1;
      case 'r': *cs = {{13, 13}}; return 1;
      case 'v': *cs = {{11, 11}}; return 1;
      case 'x':
      case 'u':
      case 'U': {
        uint32_t v = 0;
        if (!hex_escape(c == 'x' ? 2 : c == 'u' ? 4 : 8, &v)) {
          err = "invalid hexadecimal escape";
          return 0;
        }
        if (!f.u && v >= 0x80) {
          err = "pattern can match invalid UTF-8 (Unicode mode is off)";
          return 0;
        }
        *cs = {{v, v}};
        return 1;
      }
      case 'p':
      case 'P': {
        if (!f.u) {
          err = "Unicode classes are not allowed with Unicode mode off";
          return 0;
        }
        std::string body;
        if (!eof() && p[i] == '{') {
          const size_t e = p.find('}', i);
          if (e == std::string::npos) {
            err = "unclosed Unicode class";
            return 0;
          }
          body = p.substr(i + 1, e - i - 1);
          i = e + 1;
        } else {
          const int64_t n = eof() ? -1 : getc_();
          if (n < 0) {
            err = "incomplete Unicode class";
            return 0;
          }
          body = std::string(1, n < 0x80 ? (char)n : '?');  // (a one-letter name is ASCII)
        }
        bool negate = c == 'P';
        if (!uni_property(body, cs, &negate, &err)) return 0;
        // regex-syntax folds a Unicode class under (?i) before negating it
        if (f.i) cs_fold(cs, true);
        if (negate) *cs = cs_neg(*cs);
        return 1;
      }
      default: break;
    }
    if (!in_class) {
      switch (c) {
        case 'A': *mask = kind_mask([](uint32_t p_, uint32_t) { return p_ == BK_EDGE; }); return uni_word(c), 2;
        case 'z': *mask = kind_mask([](uint32_t, uint32_t n) { return n == BK_EDGE; }); return uni_word(c), 2;
        case 'B':
          if (!f.u) {  // (regex-syntax: an ASCII \B can match inside a code point, InvalidUtf8)
            err = "pattern can match invalid UTF-8 (Unicode mode is off)";
            return 0;
          }
          *mask = kind_mask([](uint32_t p_, uint32_t n) { return kw_word(p_) == kw_word(n); });
          return uni_word(c), 2;
        case '<': *mask = kind_mask([](uint32_t p_, uint32_t n) { return !kw_word(p_) && kw_word(n); }); return uni_word(c), 2;
        case '>': *mask = kind_mask([](uint32_t p_, uint32_t n) { return kw_word(p_) && !kw_word(n); }); return uni_word(c), 2;
        case 'b': {
          if (!eof() && p[i] == '{') {
            const size_t e = p.find('}', i);
            const std::string w = e == std::string::npos ? std::string() : p.substr(i + 1, e - i - 1);
            if (w == "start") *mask = kind_mask([](uint32_t p_, uint32_t n) { return !kw_word(p_) && kw_word(n); });
            else if (w == "end") *mask = kind_mask([](uint32_t p_, uint32_t n) { return kw_word(p_) && !kw_word(n); });
            else if (w == "start-half") *mask = kind_mask([](uint32_t p_, uint32_t) { return !kw_word(p_); });
            else if (w == "end-half") *mask = kind_mask([](uint32_t, uint32_t n) { return !kw_word(n); });
            else {
              err = "unrecognized word boundary assertion";
              return 0;
            }
            i = e + 1;
            return uni_word(c), 2;
          }
          *mask = kind_mask([](uint32_t p_, uint32_t n) { return kw_word(p_) != kw_word(n); });
          return uni_word(c), 2;
        }
        default: break;
      }
    }
    if (c >= '0' && c <= '9') {
      err = c == '0' ? "octal escapes are not supported" : "back-references are not supported";
      return 0;
    }
    // any other ASCII character but letters, digits and '<' '>' may be escaped (regex-syntax
    // is_escapeable_character); letters are unknown escapes
    if (c < 0x80 && !((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '<' || c == '>')) {
      *cs = {{(uint32_t)c, (uint32_t)c}};
      return 1;
    }
    i = at;
    err = "unrecognized escape sequence";
    return 0;
  }
  // flags after "(?" : returns 1 for "(?flags)" (applied to the rest of the group), 2 for
  // "(?flags:" (a group with its own flags, *scoped set), 0 on error
  int flags(RFlags* scoped) {
    RFlags g = f;
    bool neg = false, any = false, after_neg = false;
    std::string seen;
    while (!eof() && p[i] != ':' && p[i] != ')') {
      const char c = p[i++];
      if (c == '-') {
        if (neg) return fail("repeated negation in flags"), 0;
        neg = true;
        after_neg = false;
        continue;
      }
      if (seen.find(c) != std::string::npos) return fail("duplicate flag"), 0;
      seen += c;
      const bool v = !neg;
      switch (c) {
        case 'i': g.i = v; break;
        case 'm': g.m = v; break;
        case 's': g.s = v; break;
        case 'x': g.x = v; break;
        case 'u': g.u = v; break;
        case 'U': break;  // swap greed: the same language
        case 'R': return fail("the CRLF flag (R) is not supported"), 0;
        default: return fail("unrecognized flag"), 0;
      }
      any = true;
      if (neg) after_neg = true;
    }
    if (eof()) return fail("unclosed group"), 0;
    if (neg && !after_neg) return fail("dangling flag negation"), 0;
    if (!any) return fail("empty flag group"), 0;
    *scoped = g;
    return p[i++] == ')' ? 1 : 2;
  }
  int group_body(const RFlags& inner) {
    const RFlags saved = f;
    f = inner;
    if (++depth > 250) return fail("nesting too deep");
    int a = alt();
    --depth;
    f = saved;
    if (a < 0) return -1;
    if (eof() || p[i] != ')') return fail("unclosed group");
    ++i;
    return a;
  }
  int atom() {
    const char c = p[i];
    if (c == '(') {
      ++i;
      if (!eof() && p[i] == '?') {
        ++i;
        if (!eof() && (p[i] == 'P' || p[i] == '<')) {
          if (p[i] == 'P') {
            ++i;
            if (eof() || p[i] != '<') return fail("invalid group");
          }
          ++i;
          const size_t s0 = i;
          while (!eof() && p[i] != '>') {
            const char x = p[i];
            const bool first = i == s0;
            const bool ok = x == '_' || (x >= 'a' && x <= 'z') || (x >= 'A' && x <= 'Z') ||
                            (!first && ((x >= '0' && x <= '9') || x == '.' || x == '[' || x == ']'));
            if (!ok) return fail("invalid capture group name");
            ++i;
          }
          if (eof() || i == s0) return fail("invalid capture group name");
          const std::string nm = p.substr(s0, i - s0);
          if (std::find(names.begin(), names.end(), nm) != names.end()) return fail("duplicate capture group name");
          names.push_back(nm);
          ++i;
          return group_body(f);
        }
        if (!eof() && p[i] == ':') {  // (?:...) non-capturing
          ++i;
          return group_body(f);
        }
        RFlags g;
        const int k = flags(&g);
        if (k == 0) return -1;
        if (k == 1) {  // applies to the rest of the enclosing group
          f = g;
          return -2;
        }
        return group_body(g);
      }
      return group_body(f);
    }
    if (c == '*' || c == '+' || c == '?' || c == '{') return fail("repetition operator missing expression");
    if (c == '^') {
      ++i;
      return assert_node(f.m ? kind_mask([](uint32_t p_, uint32_t) { return p_ == BK_EDGE || p_ == BK_NL; })
                             : kind_mask([](uint32_t p_, uint32_t) { return p_ == BK_EDGE; }));
    }
    if (c == '$') {
      ++i;
      return assert_node(f.m ? kind_mask([](uint32_t, uint32_t n) { return n == BK_EDGE || n == BK_NL; })
                             : kind_mask([](uint32_t, uint32_t n) { return n == BK_EDGE; }));
    }
    if (c == '.') {
      ++i;
      if (!f.u) return fail("pattern can match invalid UTF-8 (Unicode mode is off)");
      return set_node(f.s ? cs_valid() : cs_diff(cs_valid(), {{'\n', '\n'}}));
    }
    if (c == '[') {
      ++i;
      CSet cs;
      if (!bracket(&cs)) return -1;
      RNode n;
      n.k = RNode::Set;
      cs = cs_inter(cs, cs_valid());
      if (!f.u && cs_nonascii(cs)) return fail("pattern can match invalid UTF-8 (Unicode mode is off)");
      n.cs = std::move(cs);
      return mk(n);
    }
    if (c == '\\') {
      ++i;
      CSet cs;
      uint32_t mask = 0;
      const int k = escape(false, &cs, &mask);
      if (k == 0) return -1;
      if (k == 2) return assert_node(mask);
      return set_node(cs);
    }
    const int64_t ch = getc_();
    if (ch < 0) return fail("invalid UTF-8 in pattern");
    // a literal character; with `u` off a non-ASCII one is still its UTF-8 bytes (allowed)
    CSet cs{{(uint32_t)ch, (uint32_t)ch}};
    if (f.i) cs_fold(&cs, f.u);
    RNode n;
    n.k = RNode::Set;
    n.cs = cs;
    return mk(n);
  }
  // ---- bracket classes: i just past '['. Items fold (flag i) before the set operations;
  // negation applies last (regex-syntax order).
  void skip_cx() { skip_x(); }  // verbose mode skips white space and comments inside classes too
  bool bracket(CSet* out) {
    bool neg = false;
    skip_cx();
    if (!eof() && p[i] == '^') {
      neg = true;
      ++i;
    }
    CSet acc;
    if (!class_ops(&acc, true)) return false;
    if (eof() || p[i] != ']') {
      err = "unclosed character class";
      return false;
    }
    ++i;
    *out = neg ? cs_neg(acc) : acc;
    return true;
  }
  static int op_at(const std::string& s, size_t k) {
    if (k + 1 >= s.size()) return 0;
    if (s[k] == '&' && s[k + 1] == '&') return 1;
    if (s[k] == '-' && s[k + 1] == '-') return 2;
    if (s[k] == '~' && s[k + 1] == '~') return 3;
    return 0;
  }
  // union (juxtaposition) of items, then left-to-right &&, --, ~~ of such unions
  bool class_ops(CSet* out, bool first_literal_bracket) {
    CSet acc;
    if (!class_union(&acc, first_literal_bracket)) return false;
    for (;;) {
      skip_cx();
      const int op = op_at(p, i);
      if (!op) break;
      i += 2;
      CSet rhs;
      if (!class_union(&rhs, false)) return false;
      acc = op == 1 ? cs_inter(acc, rhs) : op == 2 ? cs_diff(acc, rhs) : cs_sym(acc, rhs);
    }
    *out = acc;
    return true;
  }
  bool class_union(CSet* out, bool first_literal_bracket) {
    CSet acc;
    bool any = false;
    for (;;) {
      skip_cx();
      if (eof()) {
        err = "unclosed character class";
        return false;
      }
      if (p[i] == ']' && !(first_literal_bracket && !any)) break;
      if (any && op_at(p, i)) break;
      CSet item;
      if (!class_item(&item, first_literal_bracket && !any)) return false;
      acc = cs_union(acc, item);
      any = true;
    }
    if (!any) {
      err = "empty character class";
      return false;
    }
    *out = acc;
    return true;
  }
  // one primitive of a class: a character, an escape; returns its code point in *cp when it
  // can start a range (-1 otherwise)
  bool class_prim(CSet* s, int64_t* cp, bool first) {
    *cp = -1;
    const char c = p[i];
    if (c == '[') {
      if (i + 1 < p.size() && p[i + 1] == ':') {
        const size_t e = p.find(":]", i + 2);
        if (e != std::string::npos) {
          std::string name = p.substr(i + 2, e - i - 2);
          bool neg = false;
          if (!name.empty() && name[0] == '^') {
            neg = true;
            name = name.substr(1);
          }
          if (ascii_class(name, s)) {
            i = e + 2;
            if (f.i) cs_fold(s, f.u);
            if (neg) *s = cs_neg(*s);
            return true;
          }
        }
      }
      ++i;  // a nested class
      return bracket(s);
    }
    if (c == '\\') {
      ++i;
      uint32_t mask = 0;
      const size_t at = i;
      const int k = escape(true, s, &mask);
      if (k == 0) return false;
      if (s->size() == 1 && (*s)[0].lo == (*s)[0].hi) {
        const char e = p[at];
        if (e != 'd' && e != 'D' && e != 'w' && e != 'W' && e != 's' && e != 'S') *cp = (*s)[0].lo;
      }
      if (f.i) cs_fold(s, f.u);
      return true;
    }
    (void)first;
    const int64_t ch = getc_();
    if (ch < 0) {
      err = "invalid UTF-8 in pattern";
      return false;
    }
    *s = {{(uint32_t)ch, (uint32_t)ch}};
    *cp = ch;
    if (f.i) cs_fold(s, f.u);
    return true;
  }
  bool class_item(CSet* out, bool first) {
    const size_t at = i;
    CSet s;
    int64_t lo;
    if (first && p[i] == ']') {  // a leading ']' is literal
      ++i;
      s = {{']', ']'}};
      lo = ']';
    } else if (!class_prim(&s, &lo, first)) {
      return false;
    }
    (void)at;
    skip_cx();
    // a range: prim '-' prim, unless the '-' ends the class or starts an operator
    if (lo >= 0 && !eof() && p[i] == '-' && i + 1 < p.size() && p[i + 1] != ']' && !op_at(p, i)) {
      ++i;
      skip_cx();
      CSet hs;
      int64_t hi;
      if (eof() || p[i] == '[') {
        err = "invalid range in character class";
        return false;
      }
      if (!class_prim(&hs, &hi, false)) return false;
      if (hi < 0 || hi < lo) {
        err = "invalid range in character class";
        return false;
      }
      s = {{(uint32_t)lo, (uint32_t)hi}};
      if (f.i) cs_fold(&s, f.u);
    }
    *out = s;
    return true;
  }
};

// UTF-8 byte-range sequences of code points [lo, hi] (each sequence: one byte range per position)
void utf8_seqs(uint32_t lo, uint32_t hi, std::vector<std::vector<std::pair<uint8_t, uint8_t>>>* out) {
  if (lo > hi) return;
  static const uint32_t lim[3] = {0x7F, 0x7FF, 0xFFFF};
  for (uint32_t L : lim)
    if (lo <= L && hi > L) {
      utf8_seqs(lo, L, out);
      utf8_seqs(L + 1, hi, out);
      return;
    }
  if (hi <= 0x7F) {
    out->push_back({{(uint8_t)lo, (uint8_t)hi}});
    return;
  }
  const int n = hi <= 0x7FF ? 2 : hi <= 0xFFFF ? 3 : 4;
  for (int k = 1; k < n; ++k) {
    const uint32_t m = (1u << (6 * k)) - 1;
    if ((lo & ~m) != (hi & ~m)) {
      if (lo & m) {
        utf8_seqs(lo, lo | m, out);
        utf8_seqs((lo | m) + 1, hi, out);
        return;
      }
      if ((hi & m) != m) {
        utf8_seqs(lo, (hi & ~m) - 1, out);
        utf8_seqs(hi & ~m, hi, out);
        return;
      }
    }
  }
  auto enc = [n](uint32_t v, uint8_t* b) {
    if (n == 2) {
      b[0] = (uint8_t)(0xC0 | (v >> 6));
      b[1] = (uint8_t)(0x80 | (v & 0x3F));
    } else if (n == 3) {
      b[0] = (uint8_t)(0xE0 | (v >> 12));
      b[1] = (uint8_t)(0x80 | ((v >> 6) & 0x3F));
      b[2] = (uint8_t)(0x80 | (v & 0x3F));
    } else {
      b[0] = (uint8_t)(0xF0 | (v >> 18));
      b[1] = (uint8_t)(0x80 | ((v >> 12) & 0x3F));
      b[2] = (uint8_t)(0x80 | ((v >> 6) & 0x3F));
      b[3] = (uint8_t)(0x80 | (v & 0x3F));
    }
  };
  uint8_t a[4], b[4];
  enc(lo, a);
  enc(hi, b);
  std::vector<std::pair<uint8_t, uint8_t>> seq;
  for (int k = 0; k < n; ++k) seq.push_back({a[k], b[k]});
  out->push_back(seq);
}

struct Frag {
  uint32_t s, e;
};

struct Thompson {
  Nfa& nfa;
  const std::vector<RNode>& t;
  bool overflow = false;
  Frag set_frag(const CSet& cs) {
    uint32_t a = nfa.add(), b = nfa.add();
    BSet ascii;
    bool any_ascii = false;
    std::vector<std::vector<std::pair<uint8_t, uint8_t>>> seqs;
    for (const CRange& r : cs) {
      if (r.lo < 0x80) {
        ascii.range(r.lo, std::min<uint32_t>(r.hi, 0x7F));
        any_ascii = true;
      }
      if (r.hi >= 0x80) utf8_seqs(std::max<uint32_t>(r.lo, 0x80), r.hi, &seqs);
    }
    if (any_ascii) nfa.edge(a, ascii, b);
    for (const auto& sq : seqs) {
      uint32_t cur = a;
      for (size_t k = 0; k < sq.size(); ++k) {
        BSet s;
        s.range(sq[k].first, sq[k].second);
        const uint32_t nx = k + 1 == sq.size() ? b : nfa.add();
        nfa.edge(cur, s, nx);
        cur = nx;
      }
    }
    return {a, b};
  }
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
      case RNode::Set: return set_frag(n.cs);
      case RNode::Assert: {
        uint32_t a = nfa.add(), b = nfa.add();
        nfa.st[a].asrt.push_back({n.mask, b});
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
        for (int k = 0; k < n.lo && !overflow; ++k) {
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
        for (int k = n.lo; k < n.hi && !overflow; ++k) {
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

// Closure of `set` under epsilon edges and, when next >= 0, the assertion edges that hold between
// a previous byte of kind `prev` and a next byte of kind `next` (BK_*; EDGE = start / end).
void closure(const Nfa& nfa, std::vector<uint32_t>* set, int prev, int next, std::vector<uint32_t>* mark,
             uint32_t stamp) {
  std::vector<uint32_t> stack(set->begin(), set->end());
  for (uint32_t x : *set) (*mark)[x] = stamp;
  const uint32_t bit = next >= 0 ? 1u << (prev * 4 + next) : 0u;
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
    if (bit)
      for (const auto& a : nfa.st[x].asrt)
        if (a.first & bit) push(a.second);
  }
  std::sort(set->begin(), set->end());
}

// The combined NFA of a pattern list: state 0 is the root, pattern k's accepting state has acc = k.
// Literals and globs match the whole string; a regex searches (an unanchored prefix loop before it,
// a sticky accepting state after it: Rust's Regex::is_match).
bool build_nfa(const std::vector<Pattern>& pats, Nfa* out, std::string* err) {
  Nfa& nfa = *out;
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
        if (g.t == GTok::Star) {  // any bytes: a valid UTF-8 string's characters, whatever they are
          uint32_t nx = nfa.add();
          nfa.eps(cur, nx);
          nfa.edge(nx, any, nx);
          cur = nx;
        } else {  // one character of the set (its UTF-8 byte sequences)
          CSet cs;
          for (const auto& r : g.cs) cs.push_back({r.first, r.second});
          Thompson th{nfa, {}};
          const Frag f = th.set_frag(cs);
          nfa.eps(cur, f.s);
          cur = f.e;
        }
      }
      nfa.st[cur].acc = (int)k;
    } else {
      RParser rp(P.text);
      int r = rp.alt();
      if (r >= 0 && !rp.eof()) {
        rp.err = "unopened group";
        r = -1;
      }
      if (r < 0) {
        *err = "invalid regular expression '" + P.text + "': " + rp.err;
        return false;
      }
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
  return true;
}

// Which byte kinds the assertions of an NFA tell apart (a kind no assertion distinguishes from
// OTHER is merged into it, so patterns without such assertions keep their DFA size).
void assertion_kinds(const Nfa& nfa, bool* need_nl, bool* need_word) {
  *need_nl = *need_word = false;
  for (const NState& st : nfa.st)
    for (const auto& a : st.asrt) {
      auto bit = [&](uint32_t p, uint32_t n) { return (a.first >> (p * 4 + n)) & 1u; };
      for (uint32_t x = 0; x < 4; ++x) {
        if (bit(BK_NL, x) != bit(BK_OTHER, x) || bit(x, BK_NL) != bit(x, BK_OTHER)) *need_nl = true;
        if (bit(BK_WORD, x) != bit(BK_OTHER, x) || bit(x, BK_WORD) != bit(x, BK_OTHER)) *need_word = true;
      }
    }
}

}  // namespace

bool regex_ok(const std::string& re, std::string* err) {
  RParser rp(re);
  int root = rp.alt();
  if (root >= 0 && !rp.eof()) {
    rp.err = "unopened group";
    root = -1;
  }
  if (root < 0) {
    if (err) *err = rp.err;
    return false;
  }
  return true;
}

bool pattern_ok(const Pattern& p, std::string* err) {
  Nfa nfa;
  return build_nfa({p}, &nfa, err);
}

bool compile_nfa(const Pattern& p, Dfa* out, std::string* err) {
  Nfa nfa;
  if (!build_nfa({p}, &nfa, err)) return false;
  // flatten: per node its byte-set, epsilon and assertion edges; the sets as 256-bit maps
  std::vector<uint32_t> first, edges;
  uint32_t accept = 0xffffffffu;
  for (uint32_t x = 0; x < (uint32_t)nfa.st.size(); ++x) {
    first.push_back((uint32_t)(edges.size() / 2));
    const NState& S = nfa.st[x];
    if (S.acc >= 0) accept = x;
    for (const auto& e : S.tr) {
      edges.push_back(NE_BYTE | (e.first << 8));
      edges.push_back(e.second);
    }
    for (uint32_t y : S.eps) {
      edges.push_back(NE_EPS);
      edges.push_back(y);
    }
    for (const auto& a : S.asrt) {
      edges.push_back(NE_ASSERT | ((uint32_t)a.first << 8));
      edges.push_back(a.second);
    }
  }
  first.push_back((uint32_t)(edges.size() / 2));
  DevNfa R;
  memset(&R, 0, sizeof(R));
  R.nnodes = (uint32_t)nfa.st.size();
  R.nedges = (uint32_t)(edges.size() / 2);
  R.nsets = (uint32_t)nfa.sets.size();
  R.start = 0;
  R.accept = accept;
  R.search = p.kind == Pattern::Regex ? 1u : 0u;
  auto a16 = [](size_t x) { return (uint32_t)((x + 15) & ~(size_t)15); };
  R.first_off = a16(sizeof(DevNfa));
  R.edge_off = a16(R.first_off + first.size() * 4);
  R.set_off = a16(R.edge_off + edges.size() * 4);
  R.bytes = a16(R.set_off + (size_t)R.nsets * 32);
  bool uni = false;
  for (const NState& S : nfa.st)
    for (const auto& a : S.asrt) uni = uni || (a.first & kAssertUni);
  if (uni) {  // the Unicode \w ranges the assertions' code-point kinds are read from
    R.uni_off = R.bytes;
    R.uni_n = kUniWordN;
    R.bytes = a16(R.uni_off + (size_t)kUniWordN * 8);
  }
  std::vector<uint8_t>& b = out->prog;
  b.assign(R.bytes, 0);
  if (uni) memcpy(b.data() + R.uni_off, kUniWord, (size_t)kUniWordN * 8);
  memcpy(b.data(), &R, sizeof(R));
  memcpy(b.data() + R.first_off, first.data(), first.size() * 4);
  memcpy(b.data() + R.edge_off, edges.data(), edges.size() * 4);
  for (uint32_t k = 0; k < R.nsets; ++k) memcpy(b.data() + R.set_off + 32u * k, nfa.sets[k].w, 32);
  out->nfa = true;
  out->nstates = 0;
  out->ncls = 0;
  out->start = 0;
  out->abs_lo = 0;
  out->trans.clear();
  out->acc.clear();
  out->classes = {{}, {0}};
  return true;
}

bool run_nfa_record(const uint8_t* rec, const uint8_t* s, size_t n) {
  const DevNfa& R = *(const DevNfa*)rec;
  std::vector<uint32_t> scratch((size_t)nfa_scratch_words(R), 0u);
  uint32_t gen = 0;
  return nfa_run(rec, s, (uint32_t)n, scratch.data(), &gen);
}

uint32_t Dfa::run(const uint8_t* s, size_t n) const {
  if (nfa) return run_nfa_record(prog.data(), s, n) ? 1u : 0u;
  uint32_t st = start;
  for (size_t i = 0; i < n && st != 0; ++i) st = trans[(size_t)st * ncls + cls[s[i]]];
  return acc[st];
}

// Subset construction. A DFA state is (a set of NFA states closed under epsilon edges, the kind of
// the byte before the position); the assertion edges are followed when the next byte (or the end)
// is known: on a transition, and for the accept class.
bool compile_dfa(const std::vector<Pattern>& pats, Dfa* out, std::string* err, uint32_t max_states) {
  Nfa nfa;
  if (!build_nfa(pats, &nfa, err)) return false;
  // a Unicode word boundary reads the code points around a position, not the bytes: such a
  // pattern runs as an NFA element (compile_column), whose Pike VM decodes them
  for (const NState& st : nfa.st)
    for (const auto& a : st.asrt)
      if (a.first & kAssertUni) {
        *err = kStateLimitError;
        return false;
      }
  const uint32_t root = 0;
  bool need_nl, need_word;
  assertion_kinds(nfa, &need_nl, &need_word);
  auto canon = [&](uint32_t k) -> uint32_t {
    if ((k == BK_NL && !need_nl) || (k == BK_WORD && !need_word)) return BK_OTHER;
    return k;
  };

  // byte classes: refine the single class by every edge set (and the byte kinds assertions read)
  std::vector<BSet> refine = nfa.sets;
  if (need_nl) {
    BSet s;
    s.set('\n');
    refine.push_back(s);
  }
  if (need_word) {
    BSet s;
    for (unsigned c = 0; c < 256; ++c)
      if (byte_kind(c) == BK_WORD) s.set(c);
    refine.push_back(s);
    // (?-u) word assertions could hold inside a UTF-8 sequence (lead and continuation bytes are
    // both non-word), where Rust never reports an empty match: a position whose next byte is a
    // continuation byte passes no assertion (NL / edge anchors never hold there anyway)
    BSet cont;
    for (unsigned c = 0x80; c < 0xC0; ++c) cont.set(c);
    refine.push_back(cont);
  }
  std::array<uint16_t, 256> cl{};
  uint32_t ncl = 1;
  for (const BSet& s : refine) {
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
  std::vector<uint32_t> kind_of(ncl);
  std::vector<int> next_of(ncl);  // the kind a class shows as the next byte (-1: no assertion holds)
  for (uint32_t c = 0; c < ncl; ++c) {
    kind_of[c] = canon(byte_kind(rep[c]));
    next_of[c] = need_word && rep[c] >= 0x80 && rep[c] < 0xC0 ? -1 : (int)kind_of[c];
  }
  // per NFA set: membership per class
  std::vector<std::vector<uint8_t>> set_has(nfa.sets.size(), std::vector<uint8_t>(ncl));
  for (size_t s = 0; s < nfa.sets.size(); ++s)
    for (uint32_t c = 0; c < ncl; ++c) set_has[s][c] = nfa.sets[s].has(rep[c]);

  std::vector<uint32_t> mark(nfa.st.size(), 0);
  uint32_t stamp = 0;
  // key: the NFA set followed by 0x80000000 | prev kind (the dead state: the empty key)
  std::unordered_map<std::vector<uint32_t>, uint32_t, SetHash> ids;
  std::vector<std::vector<uint32_t>> dstates;
  std::vector<uint32_t> dprev;
  std::vector<uint32_t> trans;
  std::vector<uint32_t> acc;  // accept class per DFA state
  std::map<std::vector<uint32_t>, uint32_t> class_ids;
  std::vector<std::vector<uint32_t>> classes;
  class_ids[{}] = 0;
  classes.push_back({});
  auto accept_of = [&](const std::vector<uint32_t>& set, uint32_t prev) {
    std::vector<uint32_t> e = set;
    closure(nfa, &e, (int)prev, BK_EDGE, &mark, ++stamp);
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
  auto key_of = [](const std::vector<uint32_t>& set, uint32_t prev) {
    std::vector<uint32_t> k = set;
    if (!k.empty()) k.push_back(0x80000000u | prev);
    return k;
  };
  // dead state 0
  dstates.push_back({});
  dprev.push_back(BK_OTHER);
  ids[{}] = 0;
  acc.push_back(0);
  std::vector<uint32_t> s0 = {root};
  closure(nfa, &s0, 0, -1, &mark, ++stamp);
  ids[key_of(s0, BK_EDGE)] = 1;
  dstates.push_back(s0);
  dprev.push_back(BK_EDGE);
  acc.push_back(accept_of(s0, BK_EDGE));
  std::vector<uint32_t> work = {1};
  trans.assign((size_t)2 * ncl, 0);
  while (!work.empty()) {
    uint32_t d = work.back();
    work.pop_back();
    for (uint32_t c = 0; c < ncl; ++c) {
      const uint32_t k = kind_of[c];
      std::vector<uint32_t> cur = dstates[d];
      closure(nfa, &cur, (int)dprev[d], next_of[c], &mark, ++stamp);
      std::vector<uint32_t> nx;
      ++stamp;
      for (uint32_t x : cur)
        for (auto& e : nfa.st[x].tr)
          if (set_has[e.first][c] && mark[e.second] != stamp) {
            mark[e.second] = stamp;
            nx.push_back(e.second);
          }
      closure(nfa, &nx, 0, -1, &mark, ++stamp);
      const std::vector<uint32_t> key = key_of(nx, k);
      uint32_t id;
      auto it = ids.find(key);
      if (it != ids.end()) {
        id = it->second;
      } else {
        id = (uint32_t)dstates.size();
        if (id >= max_states) {
          *err = kStateLimitError;
          return false;
        }
        ids.emplace(key, id);
        dstates.push_back(nx);
        dprev.push_back(k);
        acc.push_back(accept_of(nx, k));
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
    *err = kStateLimitError;
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
    if (!compile_dfa(group, &best, err, max_states)) {
      // alone beyond the state budget: the pattern becomes an NFA element of the chain
      if (*err != kStateLimitError || !compile_nfa(pats[i], &best, err)) return false;
      if (firsts) firsts->push_back((uint32_t)i);
      for (auto& c : best.classes)
        for (auto& p : c) p += (uint32_t)i;
      out->push_back(std::move(best));
      ++i;
      continue;
    }
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
