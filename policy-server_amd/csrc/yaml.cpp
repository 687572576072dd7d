// yaml.cpp — the policies.yml reader of the native host: YAML -> JSON text (yaml.hpp).
//
// The reference reads policies.yml with serde_yaml (read_policies_file, src/config.rs:449-453) into
// HashMap<String, PolicyOrPolicyGroup> and converts every policy's settings from YAML to JSON
// (convert_yaml_map_to_json, config.rs:419-443) before handing them to the policy. Here the whole
// document is converted to JSON once and the JSON schema checks of env.cpp (config.rs:287-415)
// apply unchanged. Supported YAML: block mappings and sequences (including "- key: value" items and
// sequences at their key's indentation), flow sequences and mappings, plain / single- / double-
// quoted scalars, literal and folded block scalars with chomping indicators, comments, "---" / "...".
// Scalars resolve as YAML 1.2 core schema (serde_yaml): null (~, null, Null, NULL, empty), bool
// (true / True / TRUE, false / ...), integers (decimal, 0x, 0o), floats (incl. .inf / .nan), else
// strings. Anchors, aliases, tags and multi-document streams are rejected with an error.
#include "yaml.hpp"

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "json.hpp"

namespace kw {
namespace {

struct Line {
  int indent;
  std::string text;  // without indentation and trailing comment / whitespace
  int no;
};

// Strips a comment ('#' at the start or after whitespace, outside quotes) and trailing blanks.
std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (dq) {
      if (c == '\\') ++i;
      else if (c == '"') dq = false;
    } else if (sq) {
      if (c == '\'') sq = false;
    } else if (c == '"' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == '{' || s[i - 1] == ',' || s[i - 1] == ':' || s[i - 1] == '-')) {
      dq = true;
    } else if (c == '\'' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == '{' || s[i - 1] == ',' || s[i - 1] == ':' || s[i - 1] == '-')) {
      sq = true;
    } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
      std::string r = s.substr(0, i);
      while (!r.empty() && (r.back() == ' ' || r.back() == '\t')) r.pop_back();
      return r;
    }
  }
  std::string r = s;
  while (!r.empty() && (r.back() == ' ' || r.back() == '\t' || r.back() == '\r')) r.pop_back();
  return r;
}

struct Parser {
  std::vector<std::string> raw;  // physical lines (block scalars read them verbatim)
  std::vector<Line> lines;       // logical lines (blank / comment-only lines dropped)
  std::vector<size_t> raw_of;    // logical line -> physical line
  size_t i = 0;
  std::string err;

  bool fail(const std::string& m, int no) {
    if (err.empty()) err = m + " (line " + std::to_string(no) + ")";
    return false;
  }

  bool load(const char* s, size_t n) {
    std::string cur;
    for (size_t k = 0; k <= n; ++k) {
      if (k == n || s[k] == '\n') {
        if (k < n || !cur.empty()) raw.push_back(cur);  // text ending in a newline: no empty last line
        cur.clear();
      } else {
        cur.push_back(s[k]);
      }
    }
    bool started = false;
    for (size_t k = 0; k < raw.size(); ++k) {
      const std::string& r = raw[k];
      size_t ind = 0;
      while (ind < r.size() && r[ind] == ' ') ++ind;
      if (ind < r.size() && r[ind] == '\t') return fail("tabs are not allowed for indentation", (int)k + 1);
      std::string t = strip_comment(r.substr(ind));
      if (t.empty()) continue;
      if (ind == 0 && (t == "---" || t.rfind("--- ", 0) == 0)) {
        if (started) return fail("multi-document streams are not supported", (int)k + 1);
        started = true;
        t = t.size() > 4 ? t.substr(4) : std::string();
        if (t.empty()) continue;
      }
      if (ind == 0 && t == "...") break;
      if (t[0] == '%') return fail("directives are not supported", (int)k + 1);
      started = true;
      lines.push_back({(int)ind, t, (int)k + 1});
      raw_of.push_back(k);
    }
    return true;
  }

  // ---- scalars
  static void put_str(std::string* o, const std::string& s) { json_escape(o, s); }

  static bool is_int(const std::string& s, long long* v) {
    if (s.empty()) return false;
    size_t k = 0;
    if (s[0] == '+' || s[0] == '-') k = 1;
    if (k >= s.size()) return false;
    if (s.compare(k, 2, "0x") == 0 || s.compare(k, 2, "0o") == 0) {
      const int base = s[k + 1] == 'x' ? 16 : 8;
      if (k + 2 >= s.size()) return false;
      for (size_t j = k + 2; j < s.size(); ++j)
        if (!(base == 16 ? isxdigit((unsigned char)s[j]) : (s[j] >= '0' && s[j] <= '7'))) return false;
      *v = strtoll(s.c_str() + k + 2, nullptr, base) * (s[0] == '-' ? -1 : 1);
      return true;
    }
    for (size_t j = k; j < s.size(); ++j)
      if (!isdigit((unsigned char)s[j])) return false;
    errno = 0;
    *v = strtoll(s.c_str(), nullptr, 10);
    return errno != ERANGE;  // beyond i64: the exact digits instead (plain())
  }
  // A decimal integer beyond i64 as its exact JSON number text (no '+', no leading zeros); the
  // hexadecimal / octal forms must fit i64.
  static bool big_decimal(const std::string& s, std::string* out) {
    size_t k = (s[0] == '+' || s[0] == '-') ? 1 : 0;
    if (k >= s.size() || s.compare(k, 2, "0x") == 0 || s.compare(k, 2, "0o") == 0) return false;
    for (size_t j = k; j < s.size(); ++j)
      if (!isdigit((unsigned char)s[j])) return false;
    while (k + 1 < s.size() && s[k] == '0') ++k;
    *out = (s[0] == '-' ? "-" : "") + s.substr(k);
    return true;
  }
  static bool is_float(const std::string& s) {
    size_t k = 0;
    if (k < s.size() && (s[k] == '+' || s[k] == '-')) ++k;
    const size_t b = k;
    bool digits = false, dot = false;
    while (k < s.size() && isdigit((unsigned char)s[k])) ++k, digits = true;
    if (k < s.size() && s[k] == '.') {
      dot = true;
      ++k;
      while (k < s.size() && isdigit((unsigned char)s[k])) ++k, digits = true;
    }
    if (!digits || k == b) return false;
    bool exp = false;
    if (k < s.size() && (s[k] == 'e' || s[k] == 'E')) {
      exp = true;
      ++k;
      if (k < s.size() && (s[k] == '+' || s[k] == '-')) ++k;
      const size_t e0 = k;
      while (k < s.size() && isdigit((unsigned char)s[k])) ++k;
      if (k == e0) return false;
    }
    return k == s.size() && (dot || exp);
  }

  // A plain scalar as JSON (core-schema resolution).
  static std::string plain(const std::string& s) {
    if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return "null";
    if (s == "true" || s == "True" || s == "TRUE") return "true";
    if (s == "false" || s == "False" || s == "FALSE") return "false";
    long long v;
    if (is_int(s, &v)) return std::to_string(v);
    std::string big;
    if (big_decimal(s, &big)) return big;
    if (is_float(s)) {
      std::string t = s;
      if (t[0] == '+') t = t.substr(1);
      const size_t dot = t.find('.');
      if (dot != std::string::npos && (dot + 1 == t.size() || !isdigit((unsigned char)t[dot + 1])))
        t.insert(dot + 1, "0");  // "1." -> "1.0"
      if (t[0] == '.' || (t[0] == '-' && t.size() > 1 && t[1] == '.')) t.insert(t[0] == '-' ? 1 : 0, "0");
      return t;
    }
    std::string o;
    put_str(&o, s);  // .inf / .nan have no JSON form: strings, as serde_json would refuse them
    return o;
  }

  // Quoted scalar starting at s[k] (k at the quote); returns the decoded text, k past the quote.
  bool quoted(const std::string& s, size_t* k, std::string* out, int no) {
    const char q = s[*k];
    size_t j = *k + 1;
    out->clear();
    while (j < s.size()) {
      const char c = s[j];
      if (q == '\'') {
        if (c == '\'') {
          if (j + 1 < s.size() && s[j + 1] == '\'') {
            out->push_back('\'');
            j += 2;
            continue;
          }
          *k = j + 1;
          return true;
        }
        out->push_back(c);
        ++j;
      } else {
        if (c == '"') {
          *k = j + 1;
          return true;
        }
        if (c == '\\' && j + 1 < s.size()) {
          const char e = s[j + 1];
          j += 2;
          switch (e) {
            case 'n': out->push_back('\n'); break;
            case 't': out->push_back('\t'); break;
            case 'r': out->push_back('\r'); break;
            case '0': out->push_back('\0'); break;
            case '\\': out->push_back('\\'); break;
            case '"': out->push_back('"'); break;
            case '/': out->push_back('/'); break;
            case ' ': out->push_back(' '); break;
            case 'x':
            case 'u':
            case 'U': {
              const int nd = e == 'x' ? 2 : e == 'u' ? 4 : 8;
              if (j + nd > s.size()) return fail("bad escape", no);
              const unsigned long cp = strtoul(s.substr(j, nd).c_str(), nullptr, 16);
              j += nd;
              if (cp < 0x80) out->push_back((char)cp);
              else if (cp < 0x800) {
                out->push_back((char)(0xC0 | (cp >> 6)));
                out->push_back((char)(0x80 | (cp & 0x3F)));
              } else if (cp < 0x10000) {
                out->push_back((char)(0xE0 | (cp >> 12)));
                out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                out->push_back((char)(0x80 | (cp & 0x3F)));
              } else {
                out->push_back((char)(0xF0 | (cp >> 18)));
                out->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
                out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                out->push_back((char)(0x80 | (cp & 0x3F)));
              }
              break;
            }
            default: return fail(std::string("unknown escape \\") + e, no);
          }
          continue;
        }
        out->push_back(c);
        ++j;
      }
    }
    return fail("unterminated quoted scalar", no);
  }

  // ---- flow collections (may span lines: the caller joins them)
  bool flow(const std::string& s, size_t* k, std::string* o, int no) {
    auto ws = [&]() {
      while (*k < s.size() && (s[*k] == ' ' || s[*k] == '\t')) ++*k;
    };
    ws();
    if (*k >= s.size()) return fail("unexpected end of flow collection", no);
    const char c = s[*k];
    if (c == '[' || c == '{') {
      const bool map = c == '{';
      const char close = map ? '}' : ']';
      ++*k;
      o->push_back(map ? '{' : '[');
      bool first = true;
      for (;;) {
        ws();
        if (*k >= s.size()) return fail("unterminated flow collection", no);
        if (s[*k] == close) {
          ++*k;
          break;
        }
        if (!first) o->push_back(',');
        first = false;
        if (map) {
          std::string key;
          if (!flow_key(s, k, &key, no)) return false;
          put_str(o, key);
          o->push_back(':');
          ws();
          if (*k < s.size() && s[*k] == ':') {
            ++*k;
            ws();
            if (*k < s.size() && (s[*k] == ',' || s[*k] == '}')) o->append("null");
            else if (!flow(s, k, o, no)) return false;
          } else {
            o->append("null");
          }
        } else if (!flow(s, k, o, no)) {
          return false;
        }
        ws();
        if (*k < s.size() && s[*k] == ',') ++*k;
        else if (*k < s.size() && s[*k] == close) continue;
        else if (*k >= s.size()) return fail("unterminated flow collection", no);
        else return fail("expected ',' in flow collection", no);
      }
      o->push_back(map ? '}' : ']');
      return true;
    }
    if (c == '"' || c == '\'') {
      std::string t;
      if (!quoted(s, k, &t, no)) return false;
      put_str(o, t);
      return true;
    }
    const size_t b = *k;
    while (*k < s.size() && s[*k] != ',' && s[*k] != ']' && s[*k] != '}' &&
           !(s[*k] == ':' && (*k + 1 >= s.size() || s[*k + 1] == ' ')))
      ++*k;
    std::string t = s.substr(b, *k - b);
    while (!t.empty() && t.back() == ' ') t.pop_back();
    o->append(plain(t));
    return true;
  }
  bool flow_key(const std::string& s, size_t* k, std::string* key, int no) {
    if (s[*k] == '"' || s[*k] == '\'') return quoted(s, k, key, no);
    const size_t b = *k;
    while (*k < s.size() && s[*k] != ':' && s[*k] != ',' && s[*k] != '}') ++*k;
    *key = s.substr(b, *k - b);
    while (!key->empty() && key->back() == ' ') key->pop_back();
    return true;
  }

  // ---- block structure
  // Position of the ": " (or trailing ":") that makes line text a mapping key, npos if none.
  static size_t key_colon(const std::string& t) {
    size_t k = 0;
    if (!t.empty() && (t[0] == '"' || t[0] == '\'')) {
      const char q = t[0];
      k = 1;
      while (k < t.size()) {
        if (t[k] == q) {
          if (q == '\'' && k + 1 < t.size() && t[k + 1] == '\'') {
            k += 2;
            continue;
          }
          break;
        }
        if (q == '"' && t[k] == '\\') ++k;
        ++k;
      }
      ++k;
      while (k < t.size() && t[k] == ' ') ++k;
      return (k < t.size() && t[k] == ':' && (k + 1 == t.size() || t[k + 1] == ' ')) ? k : std::string::npos;
    }
    if (!t.empty() && (t[0] == '[' || t[0] == '{')) return std::string::npos;
    for (; k < t.size(); ++k)
      if (t[k] == ':' && (k + 1 == t.size() || t[k + 1] == ' ')) return k;
    return std::string::npos;
  }
  static bool is_seq(const std::string& t) { return t == "-" || t.rfind("- ", 0) == 0; }

  // Inline value text of a key or sequence item (flow collection, block scalar, quoted or plain).
  bool inline_value(const std::string& v, int indent, int no, std::string* o) {
    if (v[0] == '&' || v[0] == '*' || v[0] == '!') return fail("anchors, aliases and tags are not supported", no);
    if (v[0] == '|' || v[0] == '>') return block_scalar(v, indent, no, o);
    if (v[0] == '[' || v[0] == '{') {
      std::string text = v;
      // join continuation lines until the brackets balance
      auto balanced = [](const std::string& s) {
        int d = 0;
        bool sq = false, dq = false;
        for (size_t k = 0; k < s.size(); ++k) {
          const char c = s[k];
          if (dq) {
            if (c == '\\') ++k;
            else if (c == '"') dq = false;
          } else if (sq) {
            if (c == '\'') sq = false;
          } else if (c == '"') dq = true;
          else if (c == '\'') sq = true;
          else if (c == '[' || c == '{') ++d;
          else if (c == ']' || c == '}') --d;
        }
        return d <= 0;
      };
      while (!balanced(text) && i < lines.size()) text += " " + lines[i++].text;
      size_t k = 0;
      if (!flow(text, &k, o, no)) return false;
      while (k < text.size() && text[k] == ' ') ++k;
      if (k != text.size()) return fail("trailing characters after a flow collection", no);
      return true;
    }
    if (v[0] == '"' || v[0] == '\'') {
      size_t k = 0;
      std::string t;
      if (!quoted(v, &k, &t, no)) return false;
      while (k < v.size() && v[k] == ' ') ++k;
      if (k != v.size()) return fail("trailing characters after a quoted scalar", no);
      put_str(o, t);
      return true;
    }
    // plain scalar, possibly continued on more-indented lines (folded with spaces). ": " inside it
    // would start a mapping where none may begin (`key: a: b`): an error, as in libyaml/serde_yaml.
    std::string t = v;
    while (i < lines.size() && lines[i].indent > indent && key_colon(lines[i].text) == std::string::npos &&
           !is_seq(lines[i].text))
      t += " " + lines[i++].text;
    if (t.find(": ") != std::string::npos || t.back() == ':') return fail("mapping values are not allowed in this context", no);
    o->append(plain(t));
    return true;
  }

  // Literal (|) / folded (>) block scalar read from the physical lines after the header line.
  bool block_scalar(const std::string& hdr, int indent, int no, std::string* o) {
    const bool folded = hdr[0] == '>';
    char chomp = 'c';  // clip
    for (size_t k = 1; k < hdr.size(); ++k) {
      if (hdr[k] == '-') chomp = 's';
      else if (hdr[k] == '+') chomp = 'k';
      else if (!isdigit((unsigned char)hdr[k])) return fail("bad block scalar header", no);
    }
    const size_t start = (size_t)no;  // physical index of the first content line
    size_t k = start;
    int bi = -1;
    std::vector<std::string> body;
    for (; k < raw.size(); ++k) {
      const std::string& r = raw[k];
      size_t ind = 0;
      while (ind < r.size() && r[ind] == ' ') ++ind;
      const bool blank = ind == r.size() || (r.size() == ind + 1 && r[ind] == '\r');
      if (!blank) {
        if (bi < 0) bi = (int)ind;
        if ((int)ind < bi || (int)ind <= indent) break;
      }
      std::string line = blank ? std::string() : r.substr((size_t)bi);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      body.push_back(line);
    }
    // skip the logical lines consumed
    while (i < lines.size() && raw_of[i] < k) ++i;
    size_t trailing = 0;
    while (!body.empty() && body.back().empty()) {
      body.pop_back();
      ++trailing;
    }
    // Line breaks between content lines L1 and L2 with e empty lines between them: literal keeps
    // e + 1 of them; folded (YAML 1.2 §8.1.3) turns the break after L1 into a space when e = 0 and
    // drops it otherwise (the e empty lines give e newlines), unless L1 or L2 is more indented
    // (starts with a space), whose breaks are kept. Leading empty lines are kept as newlines.
    std::string s;
    size_t q = 0, empties = 0;
    while (q < body.size() && body[q].empty()) {
      s.push_back('\n');
      ++q;
    }
    const std::string* prev = nullptr;
    for (; q < body.size(); ++q) {
      if (body[q].empty()) {
        ++empties;
        continue;
      }
      if (prev) {
        const bool more = body[q][0] == ' ', prev_more = (*prev)[0] == ' ';
        if (folded && !more && !prev_more) s.append(empties ? std::string(empties, '\n') : std::string(" "));
        else s.append(std::string(empties + 1, '\n'));
      }
      empties = 0;
      s += body[q];
      prev = &body[q];
    }
    if (chomp == 'c' && !body.empty()) s.push_back('\n');
    if (chomp == 'k') s.append(std::string(trailing + (body.empty() ? 0 : 1), '\n'));
    put_str(o, s);
    return true;
  }

  bool node(int min_indent, std::string* o) {
    if (i >= lines.size() || lines[i].indent < min_indent) {
      o->append("null");
      return true;
    }
    const Line& L = lines[i];
    if (is_seq(L.text)) return seq(L.indent, o);
    if (key_colon(L.text) != std::string::npos) return map(L.indent, o);
    ++i;
    return inline_value(L.text, L.indent, L.no, o);
  }

  bool seq(int indent, std::string* o) {
    o->push_back('[');
    bool first = true;
    while (i < lines.size() && lines[i].indent == indent && is_seq(lines[i].text)) {
      if (!first) o->push_back(',');
      first = false;
      Line& L = lines[i];
      std::string item = L.text.size() > 2 ? L.text.substr(2) : std::string();
      size_t pad = 0;
      while (pad < item.size() && item[pad] == ' ') ++pad;
      item = item.substr(pad);
      if (item.empty()) {
        ++i;
        if (!node(indent + 1, o)) return false;
        continue;
      }
      if (is_seq(item) || key_colon(item) != std::string::npos) {
        // "- key: v" / "- - x": the item's node starts at its text column on this line
        L.indent = indent + 2 + (int)pad;
        L.text = item;
        if (!node(L.indent, o)) return false;
        continue;
      }
      ++i;
      if (!inline_value(item, indent, L.no, o)) return false;
    }
    o->push_back(']');
    return true;
  }

  bool map(int indent, std::string* o) {
    o->push_back('{');
    bool first = true;
    while (i < lines.size() && lines[i].indent == indent) {
      const Line& L = lines[i];
      const size_t c = key_colon(L.text);
      if (c == std::string::npos) return fail("expected a mapping key", L.no);
      std::string key = L.text.substr(0, c);
      while (!key.empty() && key.back() == ' ') key.pop_back();
      if (!key.empty() && (key[0] == '"' || key[0] == '\'')) {
        size_t k = 0;
        std::string t;
        if (!quoted(key, &k, &t, L.no)) return false;
        key = t;
      } else if (key == "?" || key.rfind("? ", 0) == 0) {
        return fail("complex mapping keys are not supported", L.no);
      }
      if (!first) o->push_back(',');
      first = false;
      put_str(o, key);
      o->push_back(':');
      std::string v = c + 1 < L.text.size() ? L.text.substr(c + 1) : std::string();
      size_t pad = 0;
      while (pad < v.size() && v[pad] == ' ') ++pad;
      v = v.substr(pad);
      const int no = L.no;
      ++i;
      if (v.empty()) {
        // nested block: deeper lines, or a sequence at the key's own indentation
        if (i < lines.size() && lines[i].indent == indent && is_seq(lines[i].text)) {
          if (!seq(indent, o)) return false;
        } else if (!node(indent + 1, o)) {
          return false;
        }
      } else if (!inline_value(v, indent, no, o)) {
        return false;
      }
    }
    o->push_back('}');
    return true;
  }
};

}  // namespace

bool yaml_to_json(const char* text, size_t len, std::string* json, std::string* err) {
  Parser p;
  if (!p.load(text, len)) {
    *err = p.err;
    return false;
  }
  json->clear();
  if (p.lines.empty()) {
    json->assign("null");
    return true;
  }
  const int top = p.lines[0].indent;
  if (!p.node(top, json)) {
    *err = p.err;
    return false;
  }
  if (p.i < p.lines.size()) {
    *err = "unexpected content (line " + std::to_string(p.lines[p.i].no) + ")";
    return false;
  }
  return true;
}

}  // namespace kw
