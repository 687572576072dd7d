// kwdev.hpp — layout of the compiled-table blob shared by the host compiler (env.cpp) and the
// HIP kernels (kernels.hip). The blob is position independent (offsets from its start), so the
// same bytes are uploaded to every GPU and broadcast over RCCL.
#pragma once
#include <cstdint>

namespace kw {

constexpr uint32_t kBlobMagic = 0x4b574731;  // "KWG1"
constexpr uint32_t kBlobVersion = 2;

// request columns that carry strings classified by a DFA
enum Col : uint32_t {
  COL_NS = 0,   // request namespace
  COL_REG = 1,  // image registry (normalised)
  COL_TAG = 2,  // image effective tag
  COL_IMG = 3,  // normalised image reference
  COL_CAP = 4,  // capability names (add and drop lists)
  COL_AA = 5,   // AppArmor profile
  COL_LK = 6,   // label key
  COL_LV = 7,   // label value
  NCOL = 8
};

enum Family : uint8_t {
  FAM_NONE = 0,
  FAM_PRIVILEGED = 1,
  FAM_NAMESPACE = 2,
  FAM_TRUSTED_REPOS = 3,
  FAM_CAPABILITIES = 4,
  FAM_APPARMOR = 5,
  FAM_LABELS = 6,
  FAM_GROUP = 7
};

enum PolicyFlag : uint8_t {
  PF_SKIP_INIT = 1,
  PF_SKIP_EPHEMERAL = 2,
  PF_ALLOW_ALL = 4,     // psp-capabilities allowed_capabilities contains "*"
  PF_INIT_ERROR = 8,    // PolicyInitialization recorded (continue_on_errors)
  PF_EXPR_ERROR = 16,   // group expression does not evaluate to a bool
  PF_REGISTERED = 32
};

// group program opcodes (postfix, bool stack with evaluated-member masks)
enum GOp : uint8_t { G_CONST0 = 0, G_CONST1 = 1, G_CALL = 2, G_NOT = 3, G_AND = 4, G_OR = 5, G_EQ = 6, G_NE = 7 };
constexpr int kMaxGroupStack = 16;
constexpr int kMaxGroupMembers = 16;
constexpr int kMaxListIdx = 16;
constexpr size_t kKvDfaBytes = 3072;  // u16 table bytes of one per-key label-value DFA before the key chains

#if defined(__HIPCC__)
#define KW_HD __host__ __device__
#else
#define KW_HD
#endif

// Compact DFA of the per-key label-value region (every offset region-relative, region < 64 KB):
// u8 transitions (nstates <= 256), accept masks deduplicated (a u8 index per state into u64
// accv[]), byte-class maps shared between DFAs and cut to 128 entries when every non-ASCII byte
// falls in one class (`hi`). The region is staged whole in LDS by the slot kernel, so its size is
// occupancy: these cuts take the C4 region from 16.8 KB of DevDfa records to about 7 KB.
struct alignas(16) KvDfa {
  uint16_t cls_off;    // u8 class of bytes [0, cls_len)
  uint16_t trans_off;  // u8 [nstates][ncls]
  uint16_t acc_off;    // u8 [nstates]: index into accv
  uint16_t accv_off;   // u64 [nacc] (8-B aligned): accepted pattern bits (the column's global bits)
  uint16_t next;       // next DFA of the key's chain, 0 = last
  uint8_t ncls, start, hi, wide;  // hi: class of bytes >= 128 when !wide; wide: 256-entry map
  uint16_t nstates;
};
static_assert(sizeof(KvDfa) == 16, "KvDfa layout");

// One byte through a KvDfa (r: the region, LDS or blob).
inline KW_HD uint32_t kv_step(const uint8_t* r, const KvDfa& d, uint32_t st, uint32_t c) {
  const uint32_t k = (c < 128u || d.wide) ? r[d.cls_off + c] : d.hi;
  return r[d.trans_off + st * d.ncls + k];
}

struct alignas(16) DevDfa {
  uint32_t nstates, ncls, start, trans_off;  // trans_off: blob offset of u16 [nstates][ncls]
  uint32_t acc_off;                          // blob offset of u64 [nstates]
  uint32_t bytes;                            // bytes of this DFA's record + tables (for LDS staging)
  uint32_t next;                             // blob offset of the next DFA of the column chain, 0 = last
  uint32_t chain_bytes;                      // bytes of this DFA and all that follow it in the chain
  uint8_t cls[256];
};

// Literal column: a perfect hash over the column's literal patterns (every pattern of the column
// is a Literal). A string matches at most one pattern; lookup = hash of its canonical little-endian
// dwords -> slot -> one verify against the pattern's words. Record layout (offsets from its start):
//   DevLit | u32 slot[nslots] | u32 words[]
// slot: 0 = empty, else (pattern index + 1) | len << 7 | word index << 19 (len < 4096, word
// index < 8192), so a probe reads the slot and then the pattern words, two dependent loads.
// words: each pattern zero-padded to whole dwords, followed by 32 zero bytes (batched verify reads).
struct alignas(16) DevLit {
  uint32_t nslots, seed, npat, bytes;      // bytes: whole record, multiple of 16
  uint32_t slot_off, word_off, pad0, pad1;
};
constexpr uint32_t lit_slot_pat(uint32_t s) { return s & 127u; }  // pattern index + 1
constexpr uint32_t lit_slot_len(uint32_t s) { return (s >> 7) & 4095u; }
constexpr uint32_t lit_slot_word(uint32_t s) { return s >> 19; }

// hash shared by the host table builder (env.cpp) and the kernels
inline KW_HD uint32_t lit_init(uint32_t seed, uint32_t len) { return seed ^ (len * 0x9E3779B1u); }
inline KW_HD uint32_t lit_mix(uint32_t h, uint32_t w) {
  h ^= w;
  h *= 0x85EBCA6Bu;
  return h ^ (h >> 13);
}
inline KW_HD uint32_t lit_final(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  return h ^ (h >> 15);
}

// One policy (or group member) — 192 bytes. Mask meaning per family (env.cpp):
//   NAMESPACE:     m[0] valid-namespace bit (COL_NS)
//   TRUSTED_REPOS: m[0] registry allow, m[1] registry reject (COL_REG), m[2] tag reject (COL_TAG),
//                  m[3] image allow, m[4] image reject (COL_IMG); nl[k] = list length
//   CAPABILITIES:  m[0] allowed U default_add, m[1] required_drop, m[2] default_add, m[3] "ALL" (COL_CAP)
//   APPARMOR:      m[0] allowed profiles (COL_AA)
//   LABELS:        m[0] denied keys, m[1] mandatory keys (COL_LK); idx[0..16) mandatory key bits,
//                  idx[16..32) constrained key bits, idx[32..48) constrained value-regex bits (COL_LV)
//   GROUP:         prog_off/prog_len postfix program, member_off/nmembers member policy indices
struct alignas(16) DevPolicy {
  uint8_t family, mode, a2m, flags;
  uint8_t nl[6];
  uint8_t n_mand, n_constr;
  uint32_t prog_off, prog_len, member_off, nmembers;
  uint32_t pad0;
  uint64_t m[6];
  uint8_t idx[48];
  uint8_t pad1[64];
};
static_assert(sizeof(DevPolicy) == 192, "DevPolicy layout");

struct alignas(16) DevHeader {
  uint32_t magic, version, npolicies, blob_bytes;
  uint32_t dfa_off[NCOL];  // head of the column's DFA chain, 0 = no patterns for this column
  uint32_t lit_off[NCOL];  // DevLit record of an all-literal column, 0 = none
  // per-key label-value DFAs: region = u16 idx[64] (region-relative offset of the first KvDfa for
  // label-key bit k over the value regexes constrained on that key, 0 = none) + shared byte-class
  // maps + the KvDfa records and tables; a key's DFAs form a chain through KvDfa.next
  uint32_t kv_off, kv_bytes;  // 0 = none (the COL_LV chain is used)
  int32_t bypass_bit;      // COL_NS bit of the always-accept namespace, -1 = none
  uint32_t policy_off;     // DevPolicy[npolicies]
  uint32_t prog_off;       // group programs (bytes)
  uint32_t member_off;     // group member indices (i32)
};

}  // namespace kw
