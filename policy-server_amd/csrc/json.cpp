// json.cpp — see json.hpp.
#include "json.hpp"

#include <cerrno>
#include <cstddef>
#include <cstdlib>
#include <cstring>

namespace kw {

static constexpr uint32_t kMaxDepth = 256;

void JDoc::clear() {
  nodes_.clear();
  kids_.clear();
  stack_.clear();
  strs_.clear();
}

void JDoc::ws() {
  while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
}

static void put_utf8(std::string* s, uint32_t cp) {
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

static int hex4(const char* p, uint32_t* v) {
  uint32_t x = 0;
  for (int k = 0; k < 4; ++k) {
    char c = p[k];
    x <<= 4;
    if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
    else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
    else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
    else return 0;
  }
  *v = x;
  return 1;
}

bool JDoc::string_into(uint32_t* off, uint32_t* len) {
  // p_ at opening quote
  ++p_;
  *off = (uint32_t)strs_.size();
  const char* run = p_;
  while (true) {
    if (p_ >= e_) {
      *err_ = "EOF while parsing a string";
      return false;
    }
    char c = *p_;
    if (c == '"') {
      strs_.append(run, (size_t)(p_ - run));
      ++p_;
      break;
    }
    if ((unsigned char)c < 0x20) {
      *err_ = "control character while parsing a string";
      return false;
    }
    if (c == '\\') {
      strs_.append(run, (size_t)(p_ - run));
      if (p_ + 1 >= e_) {
        *err_ = "EOF while parsing a string";
        return false;
      }
      char x = p_[1];
      p_ += 2;
      switch (x) {
        case '"': strs_.push_back('"'); break;
        case '\\': strs_.push_back('\\'); break;
        case '/': strs_.push_back('/'); break;
        case 'b': strs_.push_back('\b'); break;
        case 'f': strs_.push_back('\f'); break;
        case 'n': strs_.push_back('\n'); break;
        case 'r': strs_.push_back('\r'); break;
        case 't': strs_.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (e_ - p_ < 4 || !hex4(p_, &cp)) {
            *err_ = "invalid \\u escape";
            return false;
          }
          p_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00) {
            uint32_t lo;
            if (e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u' && hex4(p_ + 2, &lo) && lo >= 0xDC00 &&
                lo < 0xE000) {
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
          put_utf8(&strs_, cp);
          break;
        }
        default: *err_ = "invalid escape"; return false;
      }
      run = p_;
      continue;
    }
    ++p_;
  }
  *len = (uint32_t)strs_.size() - *off;
  return true;
}

bool JDoc::value(uint32_t depth) {
  if (depth > kMaxDepth) {
    *err_ = "recursion limit exceeded";
    return false;
  }
  ws();
  if (p_ >= e_) {
    *err_ = "EOF while parsing a value";
    return false;
  }
  uint32_t me = (uint32_t)nodes_.size();
  nodes_.emplace_back();
  char c = *p_;
  if (c == '{') {
    ++p_;
    size_t base = stack_.size();
    ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
    } else {
      while (true) {
        ws();
        if (p_ >= e_ || *p_ != '"') {
          *err_ = "key must be a string";
          return false;
        }
        JKid k;
        if (!string_into(&k.key_off, &k.key_len)) return false;
        ws();
        if (p_ >= e_ || *p_ != ':') {
          *err_ = "expected `:`";
          return false;
        }
        ++p_;
        k.node = (uint32_t)nodes_.size();
        stack_.push_back(k);
        if (!value(depth + 1)) return false;
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == '}') {
          ++p_;
          break;
        }
        *err_ = "expected `,` or `}`";
        return false;
      }
    }
    JNode& n = nodes_[me];
    n.t = JType::Obj;
    n.k_begin = (uint32_t)kids_.size();
    n.k_count = (uint32_t)(stack_.size() - base);
    kids_.insert(kids_.end(), stack_.begin() + (ptrdiff_t)base, stack_.end());
    stack_.resize(base);
    return true;
  }
  if (c == '[') {
    ++p_;
    size_t base = stack_.size();
    ws();
    if (p_ < e_ && *p_ == ']') {
      ++p_;
    } else {
      while (true) {
        JKid k;
        k.node = (uint32_t)nodes_.size();
        stack_.push_back(k);
        if (!value(depth + 1)) return false;
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == ']') {
          ++p_;
          break;
        }
        *err_ = "expected `,` or `]`";
        return false;
      }
    }
    JNode& n = nodes_[me];
    n.t = JType::Arr;
    n.k_begin = (uint32_t)kids_.size();
    n.k_count = (uint32_t)(stack_.size() - base);
    kids_.insert(kids_.end(), stack_.begin() + (ptrdiff_t)base, stack_.end());
    stack_.resize(base);
    return true;
  }
  if (c == '"') {
    uint32_t off, len;
    if (!string_into(&off, &len)) return false;
    JNode& n = nodes_[me];
    n.t = JType::Str;
    n.s_off = off;
    n.s_len = len;
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
  if (c == '-' || (c >= '0' && c <= '9')) {
    const char* s = p_;
    bool is_float = false;
    if (*p_ == '-') ++p_;
    if (p_ >= e_ || !(*p_ >= '0' && *p_ <= '9')) {
      *err_ = "invalid number";
      return false;
    }
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                       *p_ == '+' || *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') is_float = true;
      ++p_;
    }
    std::string tmp(s, (size_t)(p_ - s));
    JNode& n = nodes_[me];
    char* endp = nullptr;
    if (!is_float) {
      errno = 0;
      long long v = strtoll(tmp.c_str(), &endp, 10);
      if (*endp == 0 && errno == 0) {
        n.t = JType::Int;
        n.i = v;
        n.d = (double)v;
        return true;
      }
    }
    n.t = JType::Float;
    n.d = strtod(tmp.c_str(), &endp);
    if (*endp != 0) {
      *err_ = "invalid number";
      return false;
    }
    return true;
  }
  *err_ = "expected value";
  return false;
}

bool JDoc::parse(const char* text, size_t len, std::string* err) {
  clear();
  p_ = text;
  e_ = text + len;
  std::string scratch;
  err_ = err ? err : &scratch;
  if (!value(0)) return false;
  ws();
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
  for (uint32_t j = 0; j < n.k_count; ++j) {
    const JKid& kid = kids_[n.k_begin + j];
    if (key(kid) == k) found = kid.node;
  }
  return found;
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
