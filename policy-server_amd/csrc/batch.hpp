// batch.hpp — host-side columnar request batch (kw_soa owner) and the JSON flattener.
//
// The reference deserializes each AdmissionReview body with serde (JsonExtractor,
// src/api/handlers.rs:29-39; AdmissionReviewRequest, src/api/admission_review.rs:4-14) and hands
// the whole AdmissionRequest to a Wasm guest per (request, policy). Here a micro-batch of bodies is
// flattened once into SoA columns (include/kwgpu.h kw_soa) that the device streams from HBM.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/kwgpu.h"
#include "kwdev.hpp"

namespace kw {

// Copies n bytes without a library call for the short strings of a request (two overlapping
// loads / stores of the largest power of two <= n; memcpy above 16 bytes). Never reads or writes
// outside [src, src + n) / [dst, dst + n).
inline void copy_small(uint8_t* dst, const uint8_t* src, size_t n) {
  if (n >= 8) {
    if (n > 16) {
      memcpy(dst, src, n);
      return;
    }
    uint64_t a, b;
    memcpy(&a, src, 8);
    memcpy(&b, src + n - 8, 8);
    memcpy(dst, &a, 8);
    memcpy(dst + n - 8, &b, 8);
  } else if (n >= 4) {
    uint32_t a, b;
    memcpy(&a, src, 4);
    memcpy(&b, src + n - 4, 4);
    memcpy(dst, &a, 4);
    memcpy(dst + n - 4, &b, 4);
  } else if (n) {
    dst[0] = src[0];
    dst[n / 2] = src[n / 2];
    dst[n - 1] = src[n - 1];
  }
}

struct StrCol {
  std::vector<uint32_t> off{0};
  std::vector<uint8_t> bytes;
  // Appends one string. The pool grows geometrically and may hold zeroed slack past off.back()
  // (and device padding after finalize()); off.back() is the byte count, pad() trims.
  void push(std::string_view s) {
    const size_t o = off.back(), n = s.size();
    if (bytes.size() < o + n) bytes.resize(std::max(o + n, bytes.size() * 2 + 256));
    copy_small(bytes.data() + o, (const uint8_t*)s.data(), n);
    off.push_back((uint32_t)(o + n));
  }
  size_t n() const { return off.size() - 1; }
  // string i, or "" when i is out of range (callers that must tell the difference use get())
  std::string_view at(size_t i) const {
    if (i + 1 >= off.size()) return std::string_view();
    return std::string_view((const char*)bytes.data() + off[i], off[i + 1] - off[i]);
  }
  bool get(size_t i, std::string_view* s) const {
    if (i + 1 >= off.size()) return false;
    *s = at(i);
    return true;
  }
  void reserve(size_t ns, size_t nb) {
    off.reserve(ns + 1);
    bytes.reserve(nb + 16);
  }
  void pad() { bytes.resize(((size_t)off.back() + 31) & ~(size_t)15, 0); }  // >=16 B zero tail
  kw_strcol view() const {
    kw_strcol c;
    c.off = off.data();
    c.bytes = bytes.data();
    c.n = n();
    return c;
  }
  void clear() {
    off.assign(1, 0);
    bytes.clear();
  }
  void append(const StrCol& o) {  // o unpadded or padded: only its strings are copied
    if (bytes.size() != off.back()) bytes.resize(off.back());
    const uint32_t base = off.back();
    bytes.insert(bytes.end(), o.bytes.begin(), o.bytes.begin() + o.off.back());
    for (size_t i = 1; i < o.off.size(); ++i) off.push_back(base + o.off[i]);
  }
};

struct DeviceBatch;  // capi.cpp

// Host copy of a pass's side data (kernels.hpp WideRec): the values of verdict words whose ARG is
// kArgWide. Filled by kw_batch_verdicts.
struct WideData {
  struct Rec {
    uint64_t row;
    int32_t policy;
    uint32_t value;
  };
  std::vector<Rec> recs;             // entity indices >= 65535 (sorted by row, policy)
  std::vector<uint64_t> groups;      // dense [row][nwide] cause masks of > 15-member groups
  uint32_t nwide = 0;
  std::vector<int32_t> wide_policy;  // wide index -> group policy (all-pairs mode)
  bool rows_mode = false;
  // cause bitsets of wide groups (> 64 members or deep stacks, kernels.hpp WideGroupPass):
  // [row][big_stride] u64, the group `policy` at words [off, off + words) of its row
  struct BigRef {
    int32_t policy;
    uint32_t off, words;
  };
  std::vector<uint64_t> big;
  uint32_t big_stride = 0;
  std::vector<BigRef> big_ref;
  bool lookup(uint64_t row, int32_t policy, uint64_t* v) const;
  // the cause words of wide group `policy` at `row`, nullptr when the pass recorded none
  const uint64_t* lookup_big(uint64_t row, int32_t policy, uint32_t* words) const {
    for (const BigRef& r : big_ref)
      if (r.policy == policy && (row + 1) * big_stride <= big.size()) {
        *words = r.words;
        return big.data() + row * big_stride + r.off;
      }
    return nullptr;
  }
  void clear() {
    recs.clear();
    groups.clear();
    nwide = 0;
    wide_policy.clear();
    rows_mode = false;
    big.clear();
    big_stride = 0;
    big_ref.clear();
  }
};

struct Batch {
  uint64_t n = 0;
  std::vector<uint8_t> req_flags;
  std::vector<uint32_t> ctr_off{0}, lbl_off{0};
  StrCol uid, ns, op, kind;
  StrCol rkind;  // request.requestKind.kind, "" when absent (host only: metrics resource_kind)
  std::vector<uint8_t> ctr_flags;
  std::vector<uint32_t> capadd_off{0}, capdrop_off{0};
  StrCol ctr_name, ctr_image, ctr_aa, cap_add, cap_drop, lbl_key, lbl_val;
  DeviceBatch* dev = nullptr;
  WideData wide;  // side data of the last pass (kw_batch_verdicts)
  uint64_t containers() const { return ctr_flags.size(); }
  uint64_t labels() const { return lbl_key.n(); }
  void view(kw_soa* s) const;
  void finalize();  // pads every byte pool (device loads may read 16 B past a string)
  void append(const Batch& o);  // o's rows after this batch's (multi-threaded flatten)
};

class JDoc;
// The PodSpec of a request's object (Pod: /spec; Deployment, ReplicaSet, StatefulSet, DaemonSet, Job,
// ReplicationController: /spec/template/spec; CronJob: /spec/jobTemplate/spec/template/spec), its
// template metadata and that JSON Pointer (relative to the object). spec = -1: none.
struct PodSpecRef {
  bool has_obj = false;
  int64_t spec = -1, meta = -1;
  const char* pointer = "";
};
PodSpecRef find_podspec(const JDoc& d, int64_t req);

// Flattens one document (AdmissionReview or RawReview) and appends it as a row. On a
// deserialization error returns false with the 422 rejection text.
bool flatten_document(const char* doc, size_t len, int doc_kind, Batch* b, std::string* err);
// Copies a caller SoA into the batch.
bool batch_from_soa(const kw_soa& s, Batch* b, std::string* err);

}  // namespace kw
