// json.hpp — minimal DOM JSON parser and writer for the kwgpu host side.
//
// Used to deserialize AdmissionReview / RawReview bodies (the serde step of validate_handler,
// src/api/handlers.rs:120-141, and AdmissionReviewRequest, src/api/admission_review.rs:4-14), the
// policies document (src/config.rs:449-453) and to serialize AdmissionReviewResponse
// (admission_review.rs:16-36). Strings are unescaped into one arena; nodes and object members live
// in flat vectors, so a parsed document is three allocations.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace kw {

enum class JType : uint8_t { Null, Bool, Int, Float, Str, Arr, Obj };

struct JNode {
  JType t = JType::Null;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  uint32_t s_off = 0, s_len = 0;    // Str: unescaped bytes in JDoc::strs
  uint32_t k_begin = 0, k_count = 0;  // Arr/Obj: members in JDoc::kids
};

struct JKid {
  uint32_t key_off = 0, key_len = 0;  // Obj member key (unescaped), empty for Arr
  uint32_t node = 0;
};

class JDoc {
 public:
  // Parses `text`; returns false and sets err on malformed input (trailing garbage included).
  bool parse(const char* text, size_t len, std::string* err);
  uint32_t root() const { return 0; }
  const JNode& n(uint32_t i) const { return nodes_[i]; }
  std::string_view str(uint32_t i) const {
    const JNode& x = nodes_[i];
    return std::string_view(strs_.data() + x.s_off, x.s_len);
  }
  std::string_view key(const JKid& k) const { return std::string_view(strs_.data() + k.key_off, k.key_len); }
  const JKid* kids(uint32_t i) const { return kids_.data() + nodes_[i].k_begin; }
  uint32_t count(uint32_t i) const { return nodes_[i].k_count; }
  // Object member lookup (first match, as serde takes the last duplicate we take the last too).
  int64_t get(uint32_t obj, std::string_view key) const;
  bool is(uint32_t i, JType t) const { return nodes_[i].t == t; }
  void clear();

 private:
  bool value(uint32_t depth);
  bool string_into(uint32_t* off, uint32_t* len);
  void ws();
  const char* p_ = nullptr;
  const char* e_ = nullptr;
  std::string* err_ = nullptr;
  std::vector<JNode> nodes_;
  std::vector<JKid> kids_;
  std::vector<JKid> stack_;
  std::string strs_;
};

// JSON string escaping for response bodies.
void json_escape(std::string* out, std::string_view s);

}  // namespace kw
