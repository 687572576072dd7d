// json.cpp — see json.hpp.
#include "json.hpp"

#include <emmintrin.h>

#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>

namespace kw {

// serde_json's recursion limit: 128 levels of remaining depth, the 128th nested array/object fails
// (Deserializer::remaining_depth).
static constexpr uint32_t kMaxDepth = 127;

void JDoc::clear() {
  nodes_.clear();
  arena_.clear();
}

namespace {

inline bool is_ws(char c) {  // one compare rejects every non-blank byte
  return (unsigned char)c <= ' ' && (c == ' ' || c == '\n' || c == '\r' || c == '\t');
}

// First byte in [p, e) that is '"', '\\' or a control character (< 0x20), or e.
inline const char* scan_string(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), c1f = _mm_set1_epi8(0x1f);
  while (e - p >= 16) {
    const __m128i x = _mm_loadu_si128((const __m128i*)p);
    const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)),
                                   _mm_cmpeq_epi8(_mm_min_epu8(x, c1f), x));
    const int mask = _mm_movemask_epi8(m);
    if (mask) return p + __builtin_ctz((unsigned)mask);
    p += 16;
  }
  while (p < e && *p != '"' && *p != '\\' && (unsigned char)*p >= 0x20) ++p;
  return p;
}

void put_utf8(std::string* s, uint32_t cp) {
  if (cp < 0x80) {
    s->push_back((char)cp);
  } else if (cp < 0x800) {
    s->push_back((char)(0xC0 | (cp >> 6)));
    s->push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    s->push_back((char)(0xE0 | (cp >> 12)));
    s->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    s->push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    s->push_back((char)(0xF0 | (cp >> 18)));
    s->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    s->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    s->push_back((char)(0x80 | (cp & 0x3F)));
  }
}

int hex4(const char* p, uint32_t* v) {
  uint32_t x = 0;
  for (int k = 0; k < 4; ++k) {
    const char c = p[k];
    x <<= 4;
    if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
    else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
    else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
    else return 0;
  }
  *v = x;
  return 1;
}

inline bool digit(char c) { return c >= '0' && c <= '9'; }

}  // namespace

// p_ at the opening quote. A string without escapes stays in the source text; the first escape
// moves it to the arena (unescaped).
inline __attribute__((always_inline)) bool JDoc::string_into(uint32_t* off, uint32_t* len, bool* arena) {
  const char* s = ++p_;
  const char* q = scan_string(s, e_);
  if (__builtin_expect(q < e_ && *q == '"', 1)) {
    *off = (uint32_t)(s - src_);
    *len = (uint32_t)(q - s);
    *arena = false;
    p_ = q + 1;
    return true;
  }
  *arena = true;
  return string_escaped(s, q, off, len);
}

// The slow path: from the first escape (or error) on, the string is unescaped into the arena.
bool JDoc::string_escaped(const char* s, const char* q, uint32_t* off, uint32_t* len) {
  *off = (uint32_t)arena_.size();
  for (;;) {
    arena_.append(s, (size_t)(q - s));
    if (q >= e_) {
      *err_ = "EOF while parsing a string";
      return false;
    }
    const char c = *q;
    if (c == '"') {
      p_ = q + 1;
      break;
    }
    if (c != '\\') {
      *err_ = "control character (\\u0000-\\u001F) found while parsing a string";
      return false;
    }
    if (q + 1 >= e_) {
      *err_ = "EOF while parsing a string";
      return false;
    }
    const char x = q[1];
    p_ = q + 2;
    switch (x) {
      case '"': arena_.push_back('"'); break;
      case '\\': arena_.push_back('\\'); break;
      case '/': arena_.push_back('/'); break;
      case 'b': arena_.push_back('\b'); break;
      case 'f': arena_.push_back('\f'); break;
      case 'n': arena_.push_back('\n'); break;
      case 'r': arena_.push_back('\r'); break;
      case 't': arena_.push_back('\t'); break;
      case 'u': {
        uint32_t cp;
        if (e_ - p_ < 4 || !hex4(p_, &cp)) {
          *err_ = "invalid escape";
          return false;
        }
        p_ += 4;
        if (cp >= 0xD800 && cp < 0xDC00) {
          uint32_t lo;
          if (e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u' && hex4(p_ + 2, &lo) && lo >= 0xDC00 && lo < 0xE000) {
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else {
            *err_ = "lone leading surrogate in hex escape";
            return false;
          }
        } else if (cp >= 0xDC00 && cp < 0xE000) {
          *err_ = "lone trailing surrogate in hex escape";
          return false;
        }
        put_utf8(&arena_, cp);
        break;
      }
      default: *err_ = "invalid escape"; return false;
    }
    s = p_;
    q = scan_string(s, e_);
  }
  *len = (uint32_t)arena_.size() - *off;
  return true;
}

// RFC 8259 §6 number grammar: -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?. A float beyond f64
// is "number out of range" (serde_json); integers beyond i64/u64 become f64 there and are accepted.
bool JDoc::number() {
  const char* s = p_;
  bool is_float = false;
  if (p_ < e_ && *p_ == '-') ++p_;
  if (p_ >= e_ || !digit(*p_)) {
    *err_ = "invalid number";
    return false;
  }
  if (*p_ == '0') {
    ++p_;
    if (p_ < e_ && digit(*p_)) {
      *err_ = "invalid number";
      return false;
    }
  } else {
    while (p_ < e_ && digit(*p_)) ++p_;
  }
  if (p_ < e_ && *p_ == '.') {
    is_float = true;
    ++p_;
    if (p_ >= e_ || !digit(*p_)) {
      *err_ = "invalid number";
      return false;
    }
    while (p_ < e_ && digit(*p_)) ++p_;
  }
  if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
    is_float = true;
    ++p_;
    if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
    if (p_ >= e_ || !digit(*p_)) {
      *err_ = "invalid number";
      return false;
    }
    while (p_ < e_ && digit(*p_)) ++p_;
  }
  JNode& n = nodes_.back();
  n.t = is_float ? JType::Float : JType::Int;
  if (is_float) {
    char buf[64];
    const size_t k = (size_t)(p_ - s);
    std::string big;
    const char* z;
    if (k < sizeof(buf)) {
      memcpy(buf, s, k);
      buf[k] = 0;
      z = buf;
    } else {
      big.assign(s, k);
      z = big.c_str();
    }
    if (std::isinf(strtod(z, nullptr))) {
      *err_ = "number out of range";
      return false;
    }
  }
  return true;
}

bool JDoc::value(uint32_t depth) {
  while (p_ < e_ && is_ws(*p_)) ++p_;
  if (p_ >= e_) {
    *err_ = "EOF while parsing a value";
    return false;
  }
  const uint32_t me = (uint32_t)nodes_.size();
  nodes_.emplace_back();
  nodes_.back().next = me + 1;
  const char c = *p_;
  if (c == '{' || c == '[') {
    if (depth >= kMaxDepth) {
      *err_ = "recursion limit exceeded";
      return false;
    }
    const bool obj = c == '{';
    const char close = obj ? '}' : ']';
    ++p_;
    uint32_t count = 0;
    while (p_ < e_ && is_ws(*p_)) ++p_;
    if (p_ < e_ && *p_ == close) {
      ++p_;
    } else {
      for (;;) {
        uint32_t koff = 0, klen = 0;
        bool kar = false;
        if (obj) {
          while (p_ < e_ && is_ws(*p_)) ++p_;
          if (p_ >= e_ || *p_ != '"') {
            *err_ = p_ >= e_ ? "EOF while parsing an object" : "key must be a string";
            return false;
          }
          if (!string_into(&koff, &klen, &kar)) return false;
          while (p_ < e_ && is_ws(*p_)) ++p_;
          if (p_ >= e_ || *p_ != ':') {
            *err_ = p_ >= e_ ? "EOF while parsing an object" : "expected `:`";
            return false;
          }
          ++p_;
        }
        const uint32_t kid = (uint32_t)nodes_.size();
        while (p_ < e_ && is_ws(*p_)) ++p_;
        if (p_ < e_ && *p_ == '"') {  // string member: the common case, no recursion
          nodes_.emplace_back();
          JNode& n = nodes_.back();
          n.t = JType::Str;
          n.next = kid + 1;
          uint32_t off, len;
          bool ar;
          if (!string_into(&off, &len, &ar)) return false;
          JNode& m = nodes_[kid];
          m.a = off;
          m.c = len;
          m.arena = ar;
        } else if (!value(depth + 1)) {
          return false;
        }
        if (obj) {
          JNode& k = nodes_[kid];
          k.key_off = koff;
          k.key_len = klen;
          k.key_arena = kar;
        }
        ++count;
        while (p_ < e_ && is_ws(*p_)) ++p_;
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == close) {
          ++p_;
          break;
        }
        *err_ = p_ >= e_ ? (obj ? "EOF while parsing an object" : "EOF while parsing a list")
                         : (obj ? "expected `,` or `}`" : "expected `,` or `]`");
        return false;
      }
    }
    JNode& n = nodes_[me];
    n.t = obj ? JType::Obj : JType::Arr;
    n.c = count;
    n.next = (uint32_t)nodes_.size();
    return true;
  }
  if (c == '"') {
    uint32_t off, len;
    bool ar;
    if (!string_into(&off, &len, &ar)) return false;
    JNode& n = nodes_[me];
    n.t = JType::Str;
    n.a = off;
    n.c = len;
    n.arena = ar;
    return true;
  }
  if (c == 't' && e_ - p_ >= 4 && memcmp(p_, "true", 4) == 0) {
    p_ += 4;
    nodes_[me].t = JType::Bool;
    nodes_[me].b = true;
    return true;
  }
  if (c == 'f' && e_ - p_ >= 5 && memcmp(p_, "false", 5) == 0) {
    p_ += 5;
    nodes_[me].t = JType::Bool;
    return true;
  }
  if (c == 'n' && e_ - p_ >= 4 && memcmp(p_, "null", 4) == 0) {
    p_ += 4;
    return true;
  }
  if (c == '-' || digit(c)) return number();
  *err_ = "expected value";
  return false;
}

bool JDoc::parse(const char* text, size_t len, std::string* err) {
  clear();
  src_ = text;
  p_ = text;
  e_ = text + len;
  std::string scratch;
  err_ = err ? err : &scratch;
  if (len >= 0x7fffffffu) {
    *err_ = "document too large";
    return false;
  }
  if (!value(0)) return false;
  while (p_ < e_ && is_ws(*p_)) ++p_;
  if (p_ != e_) {
    *err_ = "trailing characters";
    return false;
  }
  return true;
}

int64_t JDoc::get(uint32_t obj, std::string_view k) const {
  const JNode& n = nodes_[obj];
  if (n.t != JType::Obj) return -1;
  int64_t found = -1;
  uint32_t m = obj + 1;
  for (uint32_t j = 0; j < n.c; ++j, m = nodes_[m].next)
    if (nodes_[m].key_len == k.size() && key(m) == k) found = m;
  return found;
}

void JDoc::pick(uint32_t obj, const std::string_view* keys, int nkeys, int64_t* out) const {
  for (int q = 0; q < nkeys; ++q) out[q] = -1;
  const JNode& n = nodes_[obj];
  if (n.t != JType::Obj) return;
  uint32_t m = obj + 1;
  for (uint32_t j = 0; j < n.c; ++j, m = nodes_[m].next) {
    const uint32_t kl = nodes_[m].key_len;
    for (int q = 0; q < nkeys; ++q) {
      if (keys[q].size() != kl) continue;
      if (key(m) == keys[q]) {
        out[q] = m;
        break;
      }
    }
  }
}

int JDoc::dup_field(uint32_t obj, const std::string_view* keys, int nkeys) const {
  const JNode& n = nodes_[obj];
  if (n.t != JType::Obj) return -1;
  uint32_t seen = 0;
  uint32_t m = obj + 1;
  for (uint32_t j = 0; j < n.c; ++j, m = nodes_[m].next) {
    const uint32_t kl = nodes_[m].key_len;
    for (int q = 0; q < nkeys; ++q) {
      if (keys[q].size() != kl || key(m) != keys[q]) continue;
      if (seen & (1u << q)) return q;
      seen |= 1u << q;
      break;
    }
  }
  return -1;
}

void json_escape(std::string* out, std::string_view s) {
  static const char* hexd = "0123456789abcdef";
  out->push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out->append("\\\""); break;
      case '\\': out->append("\\\\"); break;
      case '\n': out->append("\\n"); break;
      case '\r': out->append("\\r"); break;
      case '\t': out->append("\\t"); break;
      case '\b': out->append("\\b"); break;
      case '\f': out->append("\\f"); break;
      default:
        if (c < 0x20) {
          out->append("\\u00");
          out->push_back(hexd[c >> 4]);
          out->push_back(hexd[c & 15]);
        } else {
          out->push_back((char)c);
        }
    }
  }
  out->push_back('"');
}

}  // namespace kw
