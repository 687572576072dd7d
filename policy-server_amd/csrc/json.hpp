// json.hpp — DOM JSON parser and writer for the kwgpu host side.
//
// Used to deserialize AdmissionReview / RawReview bodies (the serde step of validate_handler,
// src/api/handlers.rs:120-141, and AdmissionReviewRequest, src/api/admission_review.rs:4-14), the
// policies document (src/config.rs:449-453) and to serialize AdmissionReviewResponse
// (admission_review.rs:16-36).
//
// Built for the serving path (kw_batch_from_json): strings without escapes are not copied — a node
// points into the parsed text, which must outlive the queries — and only escaped strings are
// unescaped into an arena; string bodies are scanned 16 bytes at a time (SSE2); numbers are checked
// against the JSON grammar without conversion (RFC 8259 §6: no leading zeros, digits after '.' and
// 'e'), a float that overflows f64 is "number out of range" as in serde_json. Values form one
// tape of 24-byte nodes in a vector reused across documents (thread_local JDoc).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace kw {

enum class JType : uint8_t { Null, Bool, Int, Float, Str, Arr, Obj };

// One value in document order (a tape): a container's members follow it, the first at index i+1,
// each member's `next` is the index after its own subtree, and the container's `next` the index after
// all of them, so members are walked without a member array and nothing is copied after parsing.
struct JNode {
  JType t = JType::Null;
  bool b = false;         // Bool value
  bool arena = false;     // Str: bytes in JDoc's arena (unescaped), else in the source text
  bool key_arena = false; // object member: key bytes in the arena
  uint32_t a = 0, c = 0;  // Str: offset, length; Arr/Obj: member count in c
  uint32_t key_off = 0, key_len = 0;  // object member: its key
  uint32_t next = 0;      // index after this value's subtree
};

class JDoc {
 public:
  // Parses `text` (which must stay alive while the document is queried); returns false and sets
  // err on malformed input (trailing garbage included).
  bool parse(const char* text, size_t len, std::string* err);
  uint32_t root() const { return 0; }
  const JNode& n(uint32_t i) const { return nodes_[i]; }
  std::string_view str(uint32_t i) const {
    const JNode& x = nodes_[i];
    return std::string_view((x.arena ? arena_.data() : src_) + x.a, x.c);
  }
  // key of object member m (a node index from members())
  std::string_view key(uint32_t m) const {
    const JNode& x = nodes_[m];
    return std::string_view((x.key_arena ? arena_.data() : src_) + x.key_off, x.key_len);
  }
  uint32_t count(uint32_t i) const { return nodes_[i].t == JType::Arr || nodes_[i].t == JType::Obj ? nodes_[i].c : 0; }
  // The members (array items, object values) of container i as node indices, in document order.
  struct Members {
    const JNode* nodes;
    uint32_t first, n;
    struct It {
      const JNode* nodes;
      uint32_t at, left;
      uint32_t operator*() const { return at; }
      It& operator++() {
        at = nodes[at].next;
        --left;
        return *this;
      }
      bool operator!=(const It& o) const { return left != o.left; }
    };
    It begin() const { return {nodes, first, n}; }
    It end() const { return {nodes, 0, 0}; }
  };
  Members members(uint32_t i) const { return {nodes_.data(), i + 1, count(i)}; }
  // Object member lookup; serde_json::Value keeps the last of duplicate keys, so does this.
  int64_t get(uint32_t obj, std::string_view key) const;
  // One pass over an object's members: out[k] = node of the last member named keys[k], or -1.
  void pick(uint32_t obj, const std::string_view* keys, int nkeys, int64_t* out) const;
  // Index of the first of keys[0..nkeys) (nkeys <= 32) that object obj holds more than once, -1 if
  // none: serde's derived structs refuse a repeated known field ("duplicate field").
  int dup_field(uint32_t obj, const std::string_view* keys, int nkeys) const;
  bool is(uint32_t i, JType t) const { return nodes_[i].t == t; }
  void clear();

 private:
  bool value(uint32_t depth);
  inline bool string_into(uint32_t* off, uint32_t* len, bool* arena);
  bool string_escaped(const char* s, const char* q, uint32_t* off, uint32_t* len);
  bool number();
  const char* src_ = nullptr;
  const char* p_ = nullptr;
  const char* e_ = nullptr;
  std::string* err_ = nullptr;
  std::vector<JNode> nodes_;
  std::string arena_;
};

// JSON string escaping for response bodies.
void json_escape(std::string* out, std::string_view s);

}  // namespace kw
