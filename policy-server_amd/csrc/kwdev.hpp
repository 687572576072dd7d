// kwdev.hpp — layout of the compiled-table blob shared by the host compiler (env.cpp) and the
// HIP kernels (kernels.hip). The blob is position independent (offsets from its start), so the
// same bytes are uploaded to every GPU and broadcast over RCCL.
//
// The blob holds only *classifiers*: for every request column, the tables that turn a string into
// a small integer class (a literal perfect hash, a DFA chain with an accept class per state, and
// for label values one DFA chain per constrained label key). Which policies a class violates is a
// property of the policy list a pass answers, so those tables live in the slot-plan records
// (slots.hpp), compiled per policy list. No table is indexed by pattern bits, so nothing bounds the
// number of patterns a policy set may name.
#pragma once
#include <cstdint>

namespace kw {

constexpr uint32_t kBlobMagic = 0x4b574733;  // "KWG3"
constexpr uint32_t kBlobVersion = 8;  // 8: S_FN u8 fid u8 nargs|mut, the script char table (r06)

// request columns that carry strings classified by a DFA or a literal table
enum Col : uint32_t {
  COL_NS = 0,   // request namespace                                   (literal table)
  COL_REG = 1,  // image registry (normalised)                         (literal table + DFA chain)
  COL_TAG = 2,  // image effective tag                                 (literal table + DFA chain)
  COL_IMG = 3,  // normalised image reference                          (DFA chain)
  COL_CAP = 4,  // capability names (add and drop lists)               (literal table)
  COL_AA = 5,   // AppArmor profile                                    (literal table)
  COL_LK = 6,   // label key                                           (literal table)
  COL_LV = 7,   // label value, against the regexes of its key         (per-key DFA chains)
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
  PF_ALLOW_ALL = 4,  // psp-capabilities allowed_capabilities contains "*"
};

// Group programs: short-circuit jump code over the member results (expr.cpp emits it, slots.hpp
// run_group_prog runs it). The value stack is a bit stack in one u64; a member call records the
// member as evaluated, exactly as rhai's lazy || and && call members (evaluation_environment.rs:979-1042).
//   G_CONST0 / G_CONST1     push false / true
//   G_CALL s                push ok(s); s is the member slot (one byte)
//   G_NOT                   negate the top
//   G_JT t / G_JF t         (||, &&) top true / false: jump to byte t (u16 LE), keeping it; else pop
//   G_EQ / G_NE             pop b, pop a, push a == b / a != b
//   G_CALL16 s              (wide programs) push ok(s), s a u16 member index; in wide programs the
//                           G_JT / G_JF targets are u32
enum GOp : uint8_t { G_CONST0 = 0, G_CONST1 = 1, G_CALL = 2, G_NOT = 3, G_JT = 4, G_JF = 5, G_EQ = 6, G_NE = 7, G_CALL16 = 8 };
// Script bytecode (groups beyond the bool-only subset that no truth table covers; expr.cpp emits
// it, slots.hpp run_script_prog runs it). Header (32 B): u32 depth (value stack bound), nvars
// (variable slots of every frame a run can hold), arena (bytes of strings and arrays a run may
// build), code_len, nframes (script-function frames: 0 or kMaxCallDepth), type_of names offset,
// char table offset and entry count; then the code, then the string pool, then the char table.
// The char table (r06) holds, for every non-ASCII code point a run can ever hold (those of the
// script's string literals, closed under the case mappings), 32-B entries sorted by code point:
// u32 cp, u32 flags (bit 0 White_Space, bit 1 Cased and not Case_Ignorable, bit 2 Case_Ignorable,
// bits 8-9 / 10-11 the lengths of the lower / upper mappings), u32 lower[3], u32 upper[3]. Values are 16 B: word 0 = type (0 unit, 1 bool, 2 i64, 3 string,
// 4 array) | 256 when the bytes are in the arena | length << 32 (string bytes, array elements);
// word 1 = the bool / i64 value, or the byte offset of the string (program-relative, or
// arena-relative with 256) or of the array's 16-B cells (arena-relative). Values are immutable:
// every operation that changes an array or builds a string writes a new arena block, charged
// against kMaxScriptAlloc exactly as the host interpreter charges it. Operands little-endian.
//   S_UNIT | S_BOOL u8 | S_INT i64 | S_STR u32 off u32 len (pool, program-relative)
//   S_LOAD u16 / S_STORE u16 (pops)          variable slot of the current frame
//   S_CALL u32                                push ok(member), the member counts as called
//   S_FAIL                                    an evaluation error found at compile time (unknown
//                                             function or variable, ...): the host words it
//   S_NOT / S_NEG / S_POS                     unary (type-checked, -i64::MIN overflows)
//   S_BIN u8                                  SBin (checked; string + any concatenates)
//   S_AND u32 / S_OR u32                      top must be bool; short circuit: jump keeping it, else pop
//   S_CHKB                                    the right side of && / || must be bool
//   S_IF u32                                  pop the condition (bool), false: jump
//   S_JMP u32 | S_POP | S_END (the result must be a bool)
//   S_ARR u16 n                               pop n values, push an array of them
//   S_INDEX                                   pop index, pop array: push the element (rhai's
//                                             negative indices count from the end)
//   S_SETIDX u16 slot                         pop value, pop index: slot's array with that element set
//   S_FN u8 fid u8 nargs | mut << 7           built-in function (SFn) over its nargs arguments: pushes
//                                             its result, or for a function rhai gives a `&mut`
//                                             first parameter (mut) the receiver as changed and
//                                             then the result (S_XSTORE / S_DROPKEEP 1 follow)
//   S_XSTORE u16 slot                         store the value under the top into a variable slot
//                                             and drop it, keeping the top
//   S_COAL u32                                ??: top not (): jump keeping it, else pop
//   S_INRANGE u8 incl                         pop hi, lo, x: x in lo..hi (all i64, else an error)
//   S_RCASE i64 lo i64 hi u8 incl             pop x: push x is an i64 in the range (switch cases)
//   S_TICK                                    one loop iteration: counts against kMaxScriptOps
//   S_FORR u16 i u16 e u8 incl u32 exit       range loop: slots i / e hold the cursor and the end;
//                                             done: jump to exit, else push the cursor, advance it
//   S_FORA u16 a u16 i u8 with_index u32 exit array loop over slot a's array, cursor slot i;
//                                             push the element (and its index)
//   S_RANGECHK                                the two range bounds on the top must be i64
//   S_CALLF u32 at u8 nargs u16 caller_slots  call a script function (counts against
//                                             kMaxScriptOps; more than kMaxCallDepth frames: error)
//   S_RET                                     return the top value to the caller
//   S_DROP u16 n / S_DROPKEEP u16 n           drop n values / n values under the top (break, continue)
enum SOp : uint8_t { S_UNIT = 0, S_BOOL, S_INT, S_STR, S_LOAD, S_STORE, S_CALL, S_FAIL, S_NOT, S_NEG, S_POS, S_BIN,
                     S_AND, S_OR, S_CHKB, S_IF, S_JMP, S_POP, S_END, S_ARR, S_INDEX, S_SETIDX, S_FN, S_COAL,
                     S_INRANGE, S_RCASE, S_TICK, S_FORR, S_FORA, S_RANGECHK, S_CALLF, S_RET, S_DROP, S_DROPKEEP,
                     S_XSTORE };
// | ^ & == != < <= > >= + - * / %, then the compound assignments that differ from their operator:
// `+=` (an array pushes / appends; otherwise `+`) and the `x op= y` forms whose errors name `op=`
enum SBin : uint8_t { SB_OR = 0, SB_XOR, SB_AND, SB_EQ, SB_NE, SB_LT, SB_LE, SB_GT, SB_GE, SB_ADD, SB_SUB, SB_MUL, SB_DIV,
                      SB_MOD, SB_ADDA, SB_POW, SB_SHL, SB_SHR };  // (r06: ** << >>)
// Built-in functions (method or function-call style; `x in y` is contains(y, x)). r06: rhai's
// standard packages over the engine's values (i64, string, array), one id per
// (name, arity); the argument types are dispatched at run time as rhai's overloads are.
enum SFn : uint8_t {
  F_LEN = 0, F_IS_EMPTY, F_CONTAINS, F_TO_STRING, F_TYPE_OF, F_STARTS_WITH, F_ENDS_WITH, F_PUSH, F_IN,
  // integers
  F_ABS, F_SIGN, F_IS_ZERO, F_IS_ODD, F_IS_EVEN, F_MAX, F_MIN, F_TO_HEX, F_TO_OCTAL, F_TO_BINARY, F_PARSE_INT,
  F_PARSE_INT_R,
  // strings
  F_TO_UPPER, F_TO_LOWER, F_MAKE_UPPER, F_MAKE_LOWER, F_TRIM, F_SUB_STRING, F_SUB_STRING_N, F_CROP, F_CROP_N,
  F_INDEX_OF, F_INDEX_OF_FROM, F_REPLACE, F_SPLIT_WS, F_SPLIT, F_SPLIT_N, F_SPLIT_REV, F_SPLIT_REV_N, F_BYTES,
  // arrays (and the string forms of append / remove / clear / truncate)
  F_APPEND, F_INSERT, F_POP, F_SHIFT, F_REMOVE, F_REVERSE, F_SORT, F_CLEAR, F_TRUNCATE, F_CHOP, F_GET, F_SET,
  F_EXTRACT, F_EXTRACT_N, F_DRAIN, F_RETAIN, F_SPLICE, F_DEDUP, F_PAD,
  F_COUNT
};
// char table flags (script programs, above)
constexpr uint32_t kChWs = 1u, kChCased = 2u, kChIgnorable = 4u;
constexpr uint32_t kChEntry = 32;
// Engine limits of one run of a group expression (host interpreter, device bytecode and the oracle
// apply them identically; each is named in the run's error message)
constexpr uint32_t kMaxScriptAlloc = 16384;   // bytes of strings and array cells a run may build
constexpr uint32_t kMaxScriptOps = 100000;    // loop iterations + script-function calls
constexpr uint32_t kMaxCallDepth = 64;        // nested script-function calls ("Stack overflow")
constexpr uint32_t kMaxCompareDepth = 16;     // array nesting inside one comparison
constexpr uint32_t kScriptHeader = 32;
constexpr int kMaxGroupStack = 64;    // value-stack depth (only == / != nest it)
constexpr int kMaxGroupMembers = 64;  // members evaluate as slots of one slot-plan chunk
constexpr int kMaxLocalBits = 64;     // per chunk: distinct mandatory label keys / mutation capabilities

#if defined(__HIPCC__)
#define KW_HD __host__ __device__
#else
#define KW_HD
#endif

// Compact DFA of the per-key label-value region (offsets region-relative). A label value is only
// ever tested against the regexes constrained on its own key, so each constrained key has a chain
// of small DFAs over just those regexes. acc[state] is the DFA's local accept class; the value's
// global COL_LV class is kbase[key] + cbase + acc[state] (kbase: the region's per-key table), so a
// chain shared by keys with the same regexes still gives each key its own classes.
struct alignas(16) KvDfa {
  uint32_t cls_off;    // u8 byte class of bytes [0, 128) and entry 128 = hi (all 256 when wide)
  uint32_t trans_off;  // [nstates][ncls]: u8 (t16 = 0) or u16 (t16 = 1) next state
  uint32_t acc_off;    // u16 [nstates]: local accept class
  uint32_t next;       // next KvDfa of the key's chain, 0 = last
  uint32_t start;
  uint16_t cbase, nstates, ncls;
  uint16_t abs_lo;                // states [abs_lo, nstates) and 0 are absorbing: a walk stops there
  uint8_t hi, wide, t16;          // hi: class of bytes >= 128 when !wide
  uint8_t nfa;                    // 1: an NFA element (DevNfa): trans_off is the program's blob offset,
                                  // acc_off its u16 [2] local classes (no match, match); no table
};
static_assert(sizeof(KvDfa) == 32, "KvDfa layout");

// One byte through a KvDfa (r: the region, LDS or blob).
inline KW_HD uint32_t kv_step(const uint8_t* r, const KvDfa& d, uint32_t st, uint32_t c) {
  const uint32_t k = (c < 128u || d.wide) ? r[d.cls_off + c] : d.hi;
  const uint32_t i = st * d.ncls + k;
  return d.t16 ? ((const uint16_t*)(r + d.trans_off))[i] : r[d.trans_off + i];
}

// One DFA of a column chain. acc: u16 [nstates] global class of the column (0 = no pattern).
struct alignas(16) DevDfa {
  uint32_t nstates, ncls, start, trans_off;  // trans_off: blob offset of u16 [nstates][ncls]
  uint32_t acc_off;                          // blob offset of u16 [nstates]
  uint32_t bytes;                            // bytes of this DFA's record + tables (for LDS staging)
  uint32_t next;                             // blob offset of the next DFA of the column chain, 0 = last
  uint32_t chain_bytes;                      // bytes of this DFA and all that follow it in the chain
  uint32_t abs_lo;                           // states [abs_lo, nstates) and 0 are absorbing (walks stop)
  // states after the constant prefixes of image normalisation, from `start` (an implicit registry
  // costs no walk): pre0 = "docker.io" | "docker.io/" << 16, pre1 = "docker.io/library/" | "latest" << 16
  uint32_t pre0, pre1;
  uint32_t kind;  // 0 a DFA; 1 an NFA element (DevNfa at blob offset trans_off; acc: u16 [2] classes no match / match)
  uint8_t cls[256];
};
// A walk may stop at state 0 (dead) and at states >= abs_lo (absorbing): `live` is st in [1, abs_lo).
inline KW_HD bool dfa_live(uint32_t st, uint32_t abs_lo) { return st - 1u < abs_lo - 1u; }

// Literal column part: a minimal-probe perfect hash over the column's literal patterns. A string
// matches at most one of them; lookup = hash g of its canonical little-endian dwords -> (bucket
// displacement) -> slot -> one verify against the pattern's words. Small sets use one bucket (no
// displacement table: g alone is collision-free for the seed); large ones hash-and-displace
// (bucket = top nb_log2 bits of g, slot = (g ^ lit_disp(disp[bucket])) mod nslots). Record layout
// (offsets from its start): DevLit | u32x2 slot[nslots] | u16 disp[1 << nb_log2] | u32 words[]
// slot.x: 0 = empty, else literal class (1 + literal index, < 65536) | len << 16 (len < 65536);
// slot.y: word index of the pattern. words: each pattern zero-padded to whole dwords, followed by
// 32 zero bytes (batched verify reads).
struct alignas(16) DevLit {
  uint32_t nslots, seed, npat, bytes;  // bytes: whole record, multiple of 16
  uint32_t slot_off, word_off, disp_off, nb_log2;
};
constexpr uint32_t lit_slot_cls(uint32_t x) { return x & 0xffffu; }
constexpr uint32_t lit_slot_len(uint32_t x) { return x >> 16; }

// hash shared by the host table builder (env.cpp) and the kernels
inline KW_HD uint32_t lit_init(uint32_t seed, uint32_t len) { return seed ^ (len * 0x9E3779B1u); }
// per-word step without a 32-bit multiply (a quarter-rate VALU op on CDNA): rotate, times 5, add
// (bijective in h for a fixed word, so strings differing in one word never collide before
// lit_final's avalanche)
inline KW_HD uint32_t lit_mix(uint32_t h, uint32_t w) {
  h ^= w;
  h = (h << 13) | (h >> 19);
  return h * 5u + 0xE6546B64u;  // (an inline-asm v_lshl_add_u32 form lost at C4 in r03: DESIGN.md §10)
}
inline KW_HD uint32_t lit_final(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  return h ^ (h >> 15);
}
inline KW_HD uint32_t lit_disp(uint32_t d) { return d; }  // the builder tries every xor mask below nslots
inline KW_HD uint32_t lit_slot_index(uint32_t g, uint32_t d, uint32_t nslots) { return (g ^ lit_disp(d)) & (nslots - 1u); }

// Classifier of one column. Global classes: 0 = no pattern, [1, 1 + nlit) the literal patterns,
// then the DFA chain's accept classes (each DevDfa.acc holds global ids). A string's pattern set is
// the union of its literal class and its class in every DFA of the chain.
struct alignas(16) DevCol {
  uint32_t lit_off;    // DevLit record, 0 = none
  uint32_t dfa_off;    // head of the DFA chain, 0 = none
  uint32_t nclass;     // global classes of the column (COL_LV: of the per-key region)
  uint32_t nlit;       // literal patterns
  uint32_t ndfa;       // DFAs in the chain (COL_LV: the longest per-key chain)
  uint32_t dfa_bytes;  // bytes of the whole chain (COL_LV: of the per-key region)
  uint32_t lit_bytes;
  uint32_t flags;      // bit 0: the chain has NFA elements (DevDfa::kind / KvDfa::nfa)
};

// ---- Patterns whose DFA exceeds the state budget (kMaxDfaStates: e.g. `a[a-z]{14}b` searched
// anywhere, or the glob `*a?????????????????`) run as their Thompson NFA instead (a Pike VM: one
// list of live states per position, linear in the string), so no valid pattern ever fails the
// environment (evaluation_environment.rs:216-225, 256-262, 472-510 build any regex the policy
// accepts). Such a pattern is an element of its column's DFA chain (DevDfa::kind / KvDfa::nfa = 1)
// that holds no table: nfa_classify_kernel runs the program for every entity of the batch before
// the tile kernel, which reads the element's class from that pass's HBM array.
//
// Record (16-B aligned, offsets from the record start): DevNfa | u32 first[nnodes + 1] (edges of
// node k: [first[k], first[k + 1])) | u32x2 edge[nedges] | 32-B byte sets[nsets].
// edge.x = kind (0 byte set, 1 epsilon, 2 assertion) | arg << 8 (set id, or the assertion's 16-bit
// mask over (previous, next) kinds, bit prev * 4 + next, kinds below, | kNfaUni when the kinds are
// those of the code points before and after the position: Unicode word boundaries); edge.y =
// target node. A record with such assertions carries the Unicode \w ranges (u32 lo, hi pairs) at
// uni_off.
struct alignas(16) DevNfa {
  uint32_t nnodes, nedges, nsets, start;
  uint32_t first_off, edge_off, set_off;
  uint32_t accept;  // the accepting node
  uint32_t search;  // 1: a regex (Regex::is_match: the accepting node is sticky, a walk may stop there)
  uint32_t bytes;   // whole record
  uint32_t uni_off, uni_n;  // Unicode \w ranges (0, 0: the record has no code-point assertions)
};
constexpr uint32_t kNfaUni = 1u << 16;
enum NfaEdge : uint32_t { NE_BYTE = 0, NE_EPS = 1, NE_ASSERT = 2 };
// byte kinds of the assertion masks: EDGE = before the first / after the last byte
enum : uint32_t { NK_EDGE = 0, NK_NL = 1, NK_WORD = 2, NK_OTHER = 3 };
inline KW_HD uint32_t nfa_kind(uint32_t c) {
  if (c == '\n') return NK_NL;
  const bool w = (c - '0' < 10u) || (c - 'A' < 26u) || (c - 'a' < 26u) || c == '_';
  return w ? NK_WORD : NK_OTHER;
}
// the kind of code point c for a Unicode assertion: NL, WORD (the Unicode \w ranges), OTHER
inline KW_HD uint32_t nfa_uni_kind(uint32_t c, const uint32_t* word, uint32_t n) {
  if (c < 0x80) return nfa_kind(c);
  uint32_t lo = 0, hi = n;  // first range whose hi >= c
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (word[2 * m + 1] < c) lo = m + 1;
    else hi = m;
  }
  return lo < n && word[2 * lo] <= c ? NK_WORD : NK_OTHER;
}
// the code point that starts at byte i / ends at byte i (lenient: a malformed sequence reads as a
// non-word code point; positions inside a character never carry an assertion)
inline KW_HD uint32_t nfa_cp_at(const uint8_t* s, uint32_t i, uint32_t n) {
  const uint32_t c = s[i];
  const uint32_t len = c < 0x80 ? 1u : c >= 0xF0 ? 4u : c >= 0xE0 ? 3u : c >= 0xC0 ? 2u : 0u;
  if (len == 0 || i + len > n) return 0xFFFFFFFFu;
  if (len == 1) return c;
  uint32_t v = c & (0x7Fu >> len);
  for (uint32_t k = 1; k < len; ++k) v = (v << 6) | (s[i + k] & 0x3Fu);
  return v;
}
inline KW_HD uint32_t nfa_cp_before(const uint8_t* s, uint32_t i, uint32_t n) {
  uint32_t j = i - 1;
  for (uint32_t k = 0; k < 3 && j > 0 && (s[j] & 0xC0u) == 0x80u; ++k) --j;
  return nfa_cp_at(s, j, n);
}
// Scratch a walk of `r` needs, in u32 words: mark[nnodes], two lists[nnodes], stack[nedges + 1].
inline KW_HD uint64_t nfa_scratch_words(const DevNfa& r) { return 3ull * r.nnodes + r.nedges + 1; }

// The Pike VM: 1 if the string s[0, n) is accepted. `scratch`: nfa_scratch_words(r) u32 words;
// `gen`: the caller's generation counter (mark[] entries equal to a generation the walk uses must not
// exist: the caller zeroes mark[] once, then keeps passing the same counter).
inline KW_HD bool nfa_run(const uint8_t* rec, const uint8_t* s, uint32_t n, uint32_t* scratch, uint32_t* gen) {
  const DevNfa& R = *(const DevNfa*)rec;
  const uint32_t* first = (const uint32_t*)(rec + R.first_off);
  const uint32_t* edge = (const uint32_t*)(rec + R.edge_off);
  const uint32_t* sets = (const uint32_t*)(rec + R.set_off);
  uint32_t* mark = scratch;
  uint32_t* cur = scratch + R.nnodes;
  uint32_t* nxt = cur + R.nnodes;
  uint32_t* stack = nxt + R.nnodes;
  uint32_t ncur = 0, nnxt = 0;
  bool hit = false;
  const uint32_t* uword = (const uint32_t*)(rec + R.uni_off);
  // kinds of the code points around position i (a record with Unicode word boundaries only)
  auto uni_bit = [&](uint32_t i) -> uint32_t {
    if (!R.uni_n) return 0u;
    const uint32_t p = i == 0 ? NK_EDGE : nfa_uni_kind(nfa_cp_before(s, i, n), uword, R.uni_n);
    const uint32_t q = i >= n ? NK_EDGE : nfa_uni_kind(nfa_cp_at(s, i, n), uword, R.uni_n);
    return 1u << (p * 4u + q);
  };
  // the closure of `node` at a position into list L; bit: the position's byte kinds (p, q) as a mask
  // bit, ubit: its code-point kinds (assertions flagged kNfaUni test that one); both 0 inside a
  // UTF-8 sequence, where Rust never reports an empty match
  auto add = [&](uint32_t node, uint32_t bit, uint32_t ubit, uint32_t* L, uint32_t* cnt) {
    const uint32_t g = *gen;
    uint32_t sp = 0;
    stack[sp++] = node;
    while (sp) {
      const uint32_t x = stack[--sp];
      if (mark[x] == g) continue;
      mark[x] = g;
      if (x == R.accept) hit = true;
      bool stepping = false;
      for (uint32_t e = first[x], e1 = first[x + 1]; e < e1; ++e) {
        const uint32_t k = edge[2 * e] & 0xffu, arg = edge[2 * e] >> 8, y = edge[2 * e + 1];
        if (k == NE_BYTE) stepping = true;
        else if (k == NE_EPS || (arg & ((arg & kNfaUni) ? ubit : bit))) stack[sp++] = y;
      }
      if (stepping) L[(*cnt)++] = x;
    }
  };
  ++*gen;
  add(R.start, 1u << (NK_EDGE * 4u + (n ? nfa_kind(s[0]) : NK_EDGE)), uni_bit(0), cur, &ncur);
  for (uint32_t i = 0; i < n; ++i) {
    if (hit && R.search) return true;
    hit = false;
    const uint32_t c = s[i], p = nfa_kind(c), q = i + 1 < n ? nfa_kind(s[i + 1]) : NK_EDGE;
    ++*gen;
    nnxt = 0;
    const bool inside = i + 1 < n && (s[i + 1] & 0xC0u) == 0x80u;
    const uint32_t ub = inside ? 0u : uni_bit(i + 1), bb = inside ? 0u : 1u << (p * 4u + q);
    for (uint32_t t = 0; t < ncur; ++t) {
      const uint32_t x = cur[t];
      for (uint32_t e = first[x], e1 = first[x + 1]; e < e1; ++e) {
        if ((edge[2 * e] & 0xffu) != NE_BYTE) continue;
        const uint32_t set = edge[2 * e] >> 8;
        if ((sets[set * 8u + (c >> 5)] >> (c & 31u)) & 1u) add(edge[2 * e + 1], bb, ub, nxt, &nnxt);
      }
    }
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
    ncur = nnxt;
    if (!ncur && !hit) return false;  // no live state: nothing can match any more
  }
  return hit;
}

struct alignas(16) DevHeader {
  uint32_t magic, version, blob_bytes, npatterns;
  DevCol col[NCOL];
  // per-key label-value region: u32 kidx[nlk] (region-relative offset of the first KvDfa of label
  // key class k, 0 = the key has no constraints) | u32 kbase[nlk] (COL_LV class base of key k) |
  // byte-class maps | KvDfa records and tables; nlk = col[COL_LK].nclass
  uint32_t kv_off, kv_bytes;
  uint32_t bypass_cls;     // COL_NS class of the always-accept namespace, 0 = none
  uint32_t docker_io_cls;  // COL_REG literal class of "docker.io" (implicit registry), 0 = none
  uint32_t latest_cls;     // COL_TAG literal class of "latest" (implicit tag), 0 = none
  uint32_t nfa_words;      // the largest NFA element's scratch in u32 words (nfa_scratch_words), 0 = none
  uint32_t pad[2];
};

}  // namespace kw
