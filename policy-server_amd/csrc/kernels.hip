// kernels.hip — the MI355X (gfx950) hot path of EvaluationEnvironment::validate for the
// declarative policy class (src/evaluation/evaluation_environment.rs:546-594) fused with the
// service::evaluate epilogue (src/api/service.rs:40-116, 160-208).
//
// Kernels:
//  evaluate_tiles_kernel — the hot path (kw_validate_batch, kw_validate_rows). Persistent 256-thread
//      workgroups, several per CU, each owning a tile of up to 64 requests at a time: stage the
//      tile's columns into LDS, classify every string into its column class (literal perfect hash,
//      DFA chains, per-key label-value DFAs; kwdev.hpp), then for each slot-plan chunk of the policy
//      list derive every entity's violation set from the chunk's class tables, find each slot's first
//      violation entity-parallel, and write the verdict words with coalesced 16-B stores.
//  overflow_classify_kernel / overflow_eval_kernel — requests whose entities exceed the tile
//      capacities even alone: classes into HBM, then the sequential walks of slots.hpp per request.
// The verdict word (include/kwgpu.h) carries the vanilla response and the service-level result.
// Integer / byte work only: no MFMA. Bound: HBM streaming of request bytes in and verdict words
// out.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstddef>
#include <mutex>

#include "../../include/kwgpu.h"
#include "imgscan.hpp"
#include "kernels.hpp"

// The measured-and-dropped variants of r01-r04 (A/B knobs) are gone from the source; git history
// and DESIGN.md §10 keep what each measured. KW_PREFETCH (kernels.hpp) stays: the next-tile L2
// prefetch is a documented diagnostic (KW_L2_PREFETCH=1 runs it).

namespace kw {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// Classification (LDS or global tables; `bytes` may be LDS-staged strings or an HBM pool, both
// padded so the dword reads below never leave their buffer)
// ------------------------------------------------------------------------------------------
__device__ inline uint32_t lit_word(const uint32_t* base, uint32_t i, uint32_t sh, uint32_t len) {
  const uint32_t w = align_bytes(base[i + 1], base[i], sh);
  const uint32_t rem = len - 4u * i;
  return rem >= 4u ? w : (w & ((1u << (8u * rem)) - 1u));
}

// Literal class of bytes [b, e) (DevLit, kwdev.hpp), 0 = no literal pattern. BATCH: the first 32
// bytes of the string and of the candidate pattern are read in one batch each (up to 36 bytes past
// the string start: LDS staging slack); otherwise word by word (<= 7 bytes past the end).
template <bool BATCH, int N = 8>
__device__ inline uint32_t lit_lookup(const uint8_t* rec, const uint8_t* bytes, uint32_t b, uint32_t e) {
  const DevLit* L = (const DevLit*)rec;
  const uint32_t len = e - b, sh = b & 3u, nw = (len + 3u) >> 2;
  const uint32_t* base = (const uint32_t*)(bytes + (b & ~3u));
  uint32_t h = lit_init(L->seed, len);
  uint32_t w[N];
  if (BATCH) {
    uint32_t raw[N + 1];
#pragma unroll
    for (int i = 0; i < N + 1; ++i) raw[i] = base[i];
    // only the last word (nw - 1) is partial: one tail mask (len % 4 == 0: shift 0, all bytes);
    // words past it are neither hashed nor compared
    const uint32_t last = nw - 1u, tm = 0xffffffffu >> ((32u - 8u * (len & 3u)) & 31u);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint32_t x = align_bytes(raw[i + 1], raw[i], sh);
      w[i] = (uint32_t)i < last ? x : (x & tm);
      if ((uint32_t)i < nw) h = lit_mix(h, w[i]);
    }
    for (uint32_t i = N; i < nw; ++i) h = lit_mix(h, lit_word(base, i, sh, len));
  } else {
    for (uint32_t i = 0; i < nw; ++i) h = lit_mix(h, lit_word(base, i, sh, len));
  }
  const uint32_t g = lit_final(h);
  const uint32_t d = L->nb_log2 ? ((const uint16_t*)(rec + L->disp_off))[g >> (32u - L->nb_log2)] : 0u;
  const uint2 sl = ((const uint2*)(rec + L->slot_off))[lit_slot_index(g, d, L->nslots)];
  if (!sl.x || lit_slot_len(sl.x) != len) return 0u;
  const uint32_t* pw = (const uint32_t*)(rec + L->word_off) + sl.y;
  bool eq = true;
  if (BATCH) {
    uint32_t pv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) pv[i] = pw[i];  // zero tail of the words section covers short patterns
#pragma unroll
    for (int i = 0; i < N; ++i) eq = eq && ((uint32_t)i >= nw || w[i] == pv[i]);
    for (uint32_t i = N; i < nw && eq; ++i) eq = lit_word(base, i, sh, len) == pw[i];
  } else {
    for (uint32_t i = 0; i < nw && eq; ++i) eq = lit_word(base, i, sh, len) == pw[i];
  }
  return eq ? lit_slot_cls(sl.x) : 0u;
}

// lit_lookup with the smallest word batch that covers every string of the wave (the words past the
// batch are read one by one, so any choice is exact); registry and tag parts are mostly <= 8 bytes.
template <bool BATCH>
__device__ inline uint32_t lit_lookup_short(const uint8_t* rec, const uint8_t* bytes, uint32_t b, uint32_t e) {
  if (BATCH) {
    if (!__ballot(e - b > 8u)) return lit_lookup<true, 2>(rec, bytes, b, e);
    if (!__ballot(e - b > 16u)) return lit_lookup<true, 4>(rec, bytes, b, e);
  }
  return lit_lookup<BATCH>(rec, bytes, b, e);
}

// A column's DFA chain, staged contiguously (LDS) or read from the blob: element at blob offset
// `off` lives at base + (off - head).
struct Chain {
  const uint8_t* base;
  uint32_t head;
};
struct DfaView {
  const uint8_t* cls;     // 256
  const uint16_t* trans;  // [state][ncls]
  const uint16_t* acc;    // [state] global class
  uint32_t ncls, start, abs_lo;
  uint32_t pre0, pre1;    // states after the normalisation prefixes (DevDfa)
};
__device__ inline DfaView chain_view(const Chain& c, uint32_t off) {
  const uint8_t* base = c.base + (off - c.head);
  const DevDfa* h = (const DevDfa*)base;
  DfaView v;
  v.cls = h->cls;
  v.ncls = h->ncls;
  v.start = h->start;
  v.abs_lo = h->abs_lo;
  v.pre0 = h->pre0;
  v.pre1 = h->pre1;
  v.trans = (const uint16_t*)(base + (h->trans_off - off));
  v.acc = (const uint16_t*)(base + (h->acc_off - off));
  return v;
}
__device__ inline uint32_t chain_next(const Chain& c, uint32_t off) { return ((const DevDfa*)(c.base + (off - c.head)))->next; }
__device__ inline uint32_t chain_kind(const Chain& c, uint32_t off) { return ((const DevDfa*)(c.base + (off - c.head)))->kind; }

// Byte offset of transition (st, class) in a [state][ncls] table of 2^sh-byte entries, with the class
// pre-shifted (cq = class << sh): one 24-bit multiply-add on the transition chain (states and class
// counts are < 65536, DevDfa / KvDfa), instead of a quarter-rate 32-bit multiply plus shifts.
__device__ inline uint32_t trans_at(uint32_t st, uint32_t ncls_sh, uint32_t cq) { return (uint32_t)__umul24(st, ncls_sh) + cq; }
// u16 transition at `at`: a byte offset from the table (global or generic tables), or, for tables
// staged in LDS (L), the entry's LDS address itself (tr_base folded into the pre-shifted classes)
template <bool L>
__device__ inline uint32_t tr16(const uint16_t* trans, uint32_t at) {
  if constexpr (L) return *(const __attribute__((address_space(3))) uint16_t*)(uintptr_t)at;
  return *(const uint16_t*)((const uint8_t*)trans + at);
}
template <bool L>
__device__ inline uint32_t tr_base(const uint16_t* trans) {
  return L ? (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint16_t*)trans : 0u;
}

template <bool L>
__device__ inline uint32_t step(const DfaView& d, uint32_t st, uint32_t byte) {
  return tr16<L>(d.trans, trans_at(st, d.ncls << 1, tr_base<L>(d.trans) + ((uint32_t)d.cls[byte] << 1)));
}

// Walk bytes [b, e) in 8-byte windows: the window's dwords, then its 8 byte classes load as batches;
// only the transitions form a dependent chain (aligned dword reads up to 11 bytes past the window
// start: pools and staged strings carry a zero tail). A walk ends at the first window that starts
// in the dead state or an absorbing one (kwdev.hpp dfa_live).
template <bool L>
__device__ inline uint32_t feed(const DfaView& d, uint32_t st, const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e) {
  const uint32_t nc2 = d.ncls << 1, tb = tr_base<L>(d.trans);
  for (uint32_t p = b; p < e && dfa_live(st, d.abs_lo); p += 8u) {
    const uint32_t* q = (const uint32_t*)(bytes + (p & ~3u));
    const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], sh = p & 3u;
    const uint32_t x0 = align_bytes(q1, q0, sh), x1 = align_bytes(q2, q1, sh);
    uint32_t c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = tb + ((uint32_t)d.cls[((i < 4 ? x0 : x1) >> (8 * (i & 3))) & 0xffu] << 1);
    // materialised here, after all eight loads and ahead of the masked steps: otherwise the
    // compiler sinks the shift and base add into each step (three VALU on the chain, not one)
    if constexpr (L) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(c[i]));
    }
    const uint32_t lim = min(8u, e - p);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if ((uint32_t)i < lim) st = tr16<L>(d.trans, trans_at(st, nc2, c[i]));
  }
  return st;
}

template <bool L, int N>
__device__ inline uint32_t feed_const(const DfaView& d, uint32_t st, const char (&s)[N]) {
  if (!dfa_live(st, d.abs_lo)) return st;  // dead or absorbing: the constant cannot change it
#pragma unroll
  for (int i = 0; i < N - 1; ++i) st = step<L>(d, st, (uint8_t)s[i]);  // state 0 is absorbing
  return st;
}

// Registry (k=0), effective tag (k=1) or normalised image (k=2) through one DFA: its class.
template <bool L>
__device__ uint32_t image_part(int k, const DfaView& d, const uint8_t* __restrict__ bytes, const ImageRef& r) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t st = d.start;
  // an implicit registry ("docker.io", then "/" and "library/" for a one-segment path) and the
  // implicit tag start from the precomputed prefix states (DevDfa pre0 / pre1): no walk
  if (k == 0) {
    st = r.is_reg ? feed<L>(d, st, bytes, r.b, r.slash0) : (d.pre0 & 0xffffu);
  } else if (k == 1) {
    if (r.colon != NONE) st = feed<L>(d, st, bytes, r.colon + 1, r.name_end);
    else if (r.at == NONE) st = d.pre1 >> 16;
    else return 0u;  // digest only: no tag
  } else {
    if (r.is_reg) {
      st = feed<L>(d, st, bytes, r.b, r.slash0);
      if (dfa_live(st, d.abs_lo)) st = step<L>(d, st, '/');
      if (r.is_docker && !r.path_slash) st = feed_const<L>(d, st, kLibrary);
    } else {
      st = r.path_slash ? (d.pre0 >> 16) : (d.pre1 & 0xffffu);
    }
    st = feed<L>(d, st, bytes, r.rest_b, r.path_end);
    if (r.eff_tag) {
      if (dfa_live(st, d.abs_lo)) st = step<L>(d, st, ':');
      st = r.colon != NONE ? feed<L>(d, st, bytes, r.colon + 1, r.name_end) : feed_const<L>(d, st, kLatest);
    }
    if (r.at != NONE) st = feed<L>(d, st, bytes, r.at, r.e);
  }
  return d.acc[st];
}

// The classifiers of one launch, resolved to LDS or blob pointers.
struct Classifiers {
  const uint8_t* lit[NCOL];  // DevLit records, nullptr = none
  Chain dfa[NCOL];           // head 0 = none
  const uint8_t* kv;         // per-key label-value region, nullptr = none
  uint32_t nlk, docker_io_cls, latest_cls;
};

// All classes of one image reference: il.nreg COL_REG entries (literal, DFAs), il.ntag COL_TAG
// entries, il.nimg COL_IMG entries.
// dbg (diagnostics, TileArgs::debug): 32768 skips the DFA chains, 65536 the literal lookups (class 0).
// NFA (instantiations with NFA elements): an element of kind 1 takes its class from nfa_row[j] (the
// pass's nfa_classify_kernel output for this container) instead of a walk.
template <bool BATCH, bool L, bool NFA = false, class Out>
__device__ inline void classify_image(const Classifiers& C, const ImgLayout& il, const uint8_t* __restrict__ bytes,
                                      uint32_t b, uint32_t e, Out out, uint32_t dbg = 0,
                                      const uint16_t* __restrict__ nfa_row = nullptr) {
  const uint32_t NONE = 0xffffffffu;
  const ImageRef r = parse_image(bytes, b, e);
  const bool nodfa = (dbg & 32768u) != 0, nolit = (dbg & 65536u) != 0;
  uint32_t j = 0;
  auto part = [&](int k, Col c, uint32_t o) -> uint32_t {
    if (NFA && chain_kind(C.dfa[c], o)) return nfa_row[j];
    return image_part<L>(k, chain_view(C.dfa[c], o), bytes, r);
  };
  if (C.lit[COL_REG])
    out(j++, nolit ? 0u : r.is_reg ? lit_lookup_short<BATCH>(C.lit[COL_REG], bytes, r.b, r.slash0) : C.docker_io_cls);
  for (uint32_t o = C.dfa[COL_REG].head; o; o = chain_next(C.dfa[COL_REG], o)) {
    out(j, nodfa ? 0u : part(0, COL_REG, o));
    ++j;
  }
  if (C.lit[COL_TAG])
    out(j++, nolit ? 0u : r.colon != NONE ? lit_lookup_short<BATCH>(C.lit[COL_TAG], bytes, r.colon + 1, r.name_end)
                                          : (r.at == NONE ? C.latest_cls : 0u));
  for (uint32_t o = C.dfa[COL_TAG].head; o; o = chain_next(C.dfa[COL_TAG], o)) {
    out(j, nodfa ? 0u : part(1, COL_TAG, o));
    ++j;
  }
  for (uint32_t o = C.dfa[COL_IMG].head; o; o = chain_next(C.dfa[COL_IMG], o)) {
    out(j, nodfa ? 0u : part(2, COL_IMG, o));
    ++j;
  }
}

// The region pointer carries its address space (3: LDS, 1: global), so the walk compiles to ds_read /
// global_load rather than flat loads.
template <int AS>
using as_ptr = const __attribute__((address_space(AS))) uint8_t*;

// A label-value chain record (two 16-B loads: a struct copy cannot bind an address-space-qualified
// reference).
template <int AS>
__device__ inline KvDfa kv_record(as_ptr<AS> R, uint32_t rel) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(AS))) v4* v4p;
  KvDfa d;
  const v4 lo = ((v4p)(R + rel))[0], hi = ((v4p)(R + rel))[1];
  __builtin_memcpy(&d, &lo, 16);
  __builtin_memcpy((uint8_t*)&d + 16, &hi, 16);
  return d;
}

// One DFA of a chain over bytes [b, e) from d.start: the final state. 8-byte windows: the window's
// dwords, then its 8 byte classes, load as two batches; only the transitions form a dependent chain
// (bytes past the string read the zero tail, unused); the walk ends at a window starting in the dead
// state or an absorbing one.
template <int AS>
__device__ inline uint32_t kv_walk(as_ptr<AS> R, const KvDfa& d, const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e) {
  typedef const __attribute__((address_space(AS))) uint16_t* u16p;
  uint32_t st = d.start;
  for (uint32_t p = b; p < e && dfa_live(st, d.abs_lo); p += 8u) {
    const uint32_t* q = (const uint32_t*)(bytes + (p & ~3u));
    const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], sh = p & 3u;
    const uint32_t x0 = align_bytes(q1, q0, sh), x1 = align_bytes(q2, q1, sh);
    uint32_t c[8];
    const uint32_t lim = min(8u, e - p);
    if constexpr (AS == 3) {
      // LDS region: branch-free (every class load and step of the window runs; `fin` keeps the
      // state after the lane's last byte; a step no lane of the wave needs ends the window). The
      // global-table form below keeps its masked steps: extra lanes' gathers cost L2 bandwidth.
      // Classes come out as LDS byte addresses of their column in the transition table (tb +
      // class << t16), so a step is one 24-bit multiply-add and the load (trans_at).
      const uint32_t t16 = d.t16, tb = (uint32_t)(uintptr_t)(R + d.trans_off), ncs = (uint32_t)d.ncls << t16;
      const uint32_t bm = 128u + (uint32_t)d.wide * 127u;  // narrow maps: entry 128 is the class of bytes >= 128 (wide: 0 / 1)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t by = ((i < 4 ? x0 : x1) >> (8 * (i & 3))) & 0xffu;
        c[i] = tb + ((uint32_t)R[d.cls_off + min(by, bm)] << t16);
      }
      uint32_t fin = st;
      if (t16) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i > 0 && !__any((uint32_t)i < lim)) break;
          st = *(u16p)(uintptr_t)trans_at(st, ncs, c[i]);
          fin = (uint32_t)i < lim ? st : fin;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i > 0 && !__any((uint32_t)i < lim)) break;
          st = *(as_ptr<AS>)(uintptr_t)trans_at(st, ncs, c[i]);
          fin = (uint32_t)i < lim ? st : fin;
        }
      }
      st = fin;
      continue;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t by = ((i < 4 ? x0 : x1) >> (8 * (i & 3))) & 0xffu;
      c[i] = R[d.cls_off + min(by, 128u + (uint32_t)d.wide * 127u)];
    }
    const as_ptr<AS> tr = R + d.trans_off;
    if (d.t16) {
      const uint32_t nc2 = (uint32_t)d.ncls << 1;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((uint32_t)i < lim) st = *(u16p)(tr + trans_at(st, nc2, c[i] << 1));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((uint32_t)i < lim) st = tr[trans_at(st, d.ncls, c[i])];
    }
  }
  return st;
}

template <int AS, bool NFA, class Out>
__device__ inline uint32_t classify_value_as(as_ptr<AS> R, uint32_t nlk, uint32_t k, const uint8_t* __restrict__ bytes,
                                             uint32_t b, uint32_t e, Out out, const uint16_t* __restrict__ nfa_row) {
  typedef const __attribute__((address_space(AS))) uint32_t* u32p;
  typedef const __attribute__((address_space(AS))) uint16_t* u16p;
  uint32_t j = 0;
  const uint32_t kbase = ((u32p)R)[nlk + k];
  for (uint32_t rel = ((u32p)R)[k]; rel;) {
    const KvDfa d = kv_record<AS>(R, rel);
    if (NFA && d.nfa) {  // an NFA element: its class from the pass's nfa_classify_kernel
      out(j, (uint32_t)nfa_row[j]);
      ++j;
      rel = d.next;
      continue;
    }
    const uint32_t st = kv_walk<AS>(R, d, bytes, b, e);
    out(j++, kbase + d.cbase + ((u16p)(R + d.acc_off))[st]);
    rel = d.next;
  }
  return j;
}

// COL_LV classes of a label value under label-key class k: one per DFA of the key's chain, 0xffff
// fills the rest of the nlv entries. kv_lds: the region is staged in LDS (else the blob in HBM).
template <bool NFA = false, class Out>
__device__ inline void classify_value(const Classifiers& C, bool kv_lds, uint32_t k, uint32_t nlv, const uint8_t* __restrict__ bytes,
                                      uint32_t b, uint32_t e, Out out, const uint16_t* __restrict__ nfa_row = nullptr) {
  uint32_t j = 0;
  if (C.kv && k)
    j = kv_lds ? classify_value_as<3, NFA>((as_ptr<3>)C.kv, C.nlk, k, bytes, b, e, out, nfa_row)
               : classify_value_as<1, NFA>((as_ptr<1>)C.kv, C.nlk, k, bytes, b, e, out, nfa_row);
  for (; j < nlv; ++j) out(j, 0xffffu);
}

// ------------------------------------------------------------------------------------------
// Per-chunk violation sets (slots.hpp tables) from stored classes
// ------------------------------------------------------------------------------------------
__device__ inline uint64_t dv_label(const SlotView& sv, uint32_t k, const uint16_t* lv, uint32_t nlv) {
  if (!sv.h->lbl || !k) return 0ull;
  uint64_t v = sv.row(T_DENY, k);
  for (uint32_t j = 0; j < nlv; ++j) {
    const uint32_t c = lv[j];
    if (c != 0xffffu) v |= sv.row(T_FAIL, c);
  }
  return v;
}

__device__ inline uint64_t dv_image(const SlotView& sv, const ImgLayout& il, uint32_t fl, const uint16_t* ic) {
  if (!sv.h->trs || !(fl & KW_CTR_HAS_IMAGE)) return 0ull;
  uint64_t why[5];
  trs_whys(sv, il, [&](uint32_t j) { return (uint32_t)ic[j]; }, why);
  return (why[0] | why[1] | why[2] | why[3] | why[4]) & sv.h->trs;
}

// OR of a[lo, hi), four loads a round issued together (guarded: a short range costs one round, not
// one dependent loop trip per element). Used for a container's predecessors when tiles carry many containers per request
// (TileArgs::ctr_ranges: C5's skewed counts, -6 %; C4 +0.8 % with this form, so not there).
__device__ inline uint64_t or_range(const uint64_t* a, uint32_t lo, uint32_t hi) {
  uint64_t r = 0;
  for (uint32_t j = lo; j < hi; j += 4u) {
    uint64_t x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = a[j + (uint32_t)u < hi ? j + (uint32_t)u : lo];
#pragma unroll
    for (int u = 0; u < 4; ++u) r |= j + (uint32_t)u < hi ? x[u] : 0ull;
  }
  return r;
}

// A 64-bit value from another lane by DPP (CTRL: row_shr:n 0x110+n, row_bcast:15 0x142, row_bcast:31
// 0x143, wave_shr:1 0x138; rows outside ROWS and lanes with no source read 0). The move must run
// on every lane (a disabled source lane reads as no source), so the volatile asm keeps the
// compiler from folding the caller's select into the move's EXEC mask.
template <int CTRL, int ROWS>
__device__ inline uint64_t dpp64(uint64_t v) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROWS, 0xf, false);
  uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROWS, 0xf, false);
  asm volatile("" : "+v"(lo), "+v"(hi));
  return ((uint64_t)hi << 32) | lo;
}

// Segmented exclusive OR-scan over the wave's 64 lanes (all active): lane l, item i = base + l, gets
// the OR of x over the lanes l' < l whose item is >= first (the first item of l's segment). Row
// shifts within 16 lanes, then the row broadcasts of lanes 15 / 31 (GFX9 DPP), then one wave shift.
__device__ inline uint64_t seg_or_scan_excl(uint64_t x, uint32_t lane, uint32_t i, uint32_t first) {
  const uint32_t r = lane & 15u;
  uint64_t y;
  y = dpp64<0x111, 0xf>(x);
  x |= (first + 1u <= i) ? y : 0ull;
  y = dpp64<0x112, 0xf>(x);
  x |= (first + 2u <= i) ? y : 0ull;
  y = dpp64<0x114, 0xf>(x);
  x |= (first + 4u <= i) ? y : 0ull;
  y = dpp64<0x118, 0xf>(x);
  x |= (first + 8u <= i) ? y : 0ull;
  y = dpp64<0x142, 0xa>(x);  // rows 1, 3: lane 16 row - 1
  x |= (first + r + 1u <= i) ? y : 0ull;
  y = dpp64<0x143, 0xc>(x);  // rows 2, 3: lane 31
  x |= (lane >= 32u && first + lane - 31u <= i) ? y : 0ull;
  y = dpp64<0x138, 0xf>(x);
  return (first + 1u <= i) ? y : 0ull;
}

// ------------------------------------------------------------------------------------------
// The tile kernel
// ------------------------------------------------------------------------------------------
template <class T>
__device__ inline const __attribute__((address_space(1))) T* gp(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}

__device__ inline uint32_t rup64(uint32_t n) { return (n + 63u) & ~63u; }

// First global entity index of string column m within a tile.
__device__ inline uint32_t str_g0(int m, uint32_t r0, uint32_t cb, uint32_t kab, uint32_t kdb, uint32_t lb) {
  return m == S_NS ? r0 : m == S_CAPADD ? kab : m == S_CAPDROP ? kdb : (m == S_LK || m == S_LV) ? lb : cb;
}
__device__ inline uint32_t str_n(int m, uint32_t nr, uint32_t nc, uint32_t nka, uint32_t nkd, uint32_t nl) {
  return m == S_NS ? nr : m == S_CAPADD ? nka : m == S_CAPDROP ? nkd : (m == S_LK || m == S_LV) ? nl : nc;
}

// LDS-DMA copies (global_load_lds) issued by every wave of the workgroup: the LDS image is
// wave-linear (wave-uniform base + lane x size), so lane l of the wave whose first element is i - l
// lands at dst + i. Tails are masked by the loop bound.
__device__ inline void glds_dwords(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t tid) {
  const uint32_t lane = tid & 63u;
  for (uint32_t i = tid; i < n; i += kSlotThreads)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i),
                                     (__attribute__((address_space(3))) void*)(dst + (i - lane)), 4, 0, 0);
}
__device__ inline void glds_x4(const u32x4* src, u32x4* dst, uint32_t n, uint32_t tid) {
  const uint32_t lane = tid & 63u;
  for (uint32_t i = tid; i < n; i += kSlotThreads)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i),
                                     (__attribute__((address_space(3))) void*)(dst + (i - lane)), 16, 0, 0);
}
// The same copies issued by one wave alone (lane l of the wave lands at dst + i for element i).
__device__ inline void wglds_dwords(const uint32_t* src, uint32_t* dst, uint32_t n, uint32_t lane) {
  for (uint32_t i = lane; i < n; i += 64u)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i),
                                     (__attribute__((address_space(3))) void*)(dst + (i - lane)), 4, 0, 0);
}
__device__ inline void wglds_x4(const u32x4* src, u32x4* dst, uint32_t n, uint32_t lane) {
  for (uint32_t i = lane; i < n; i += 64u)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i),
                                     (__attribute__((address_space(3))) void*)(dst + (i - lane)), 16, 0, 0);
}
#ifndef KW_DESC_EARLY
#define KW_DESC_EARLY 1
#endif
#ifndef KW_TABLE_DMA  // the workgroup's table staging by LDS-DMA (below)
#define KW_TABLE_DMA 1
#endif
#ifndef KW_P0_SPREAD  // P0 copy jobs spread over the waves (below)
#define KW_P0_SPREAD 1
#endif
__device__ inline void copy_x4(const uint8_t* src, uint8_t* dst, uint32_t bytes, uint32_t tid) {
  const auto* s = gp((const u32x4*)src);
  u32x4* d = (u32x4*)dst;
  for (uint32_t i = tid; i < bytes / 16; i += kSlotThreads) d[i] = s[i];
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations,
// not for its outstanding global stores — the verdict stores of a tile drain under the next tile
// instead of stalling every wave at the barrier (__syncthreads waits vmcnt(0)). Used where no
// global load result is consumed across the barrier; the staging barrier (LDS-DMA, counted by
// vmcnt) stays __syncthreads.
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// L2 prefetch of `bytes` at `src`: one dword per 128-B line, by LDS-DMA from lanes 0..kPfLanes-1 of
// each wave into a 4 x kPfLanes-byte scratch line shared by the waves (never read; a DMA lane lands at base + 4 x lane), so
// no VGPR waits for the data and no barrier but the next staging barrier (vmcnt) covers it; the next
// tile's staging loads then hit L2.
__device__ inline void prefetch_l2(const void* src, uint32_t bytes, uint8_t* scratch, uint32_t tid) {
  const uint8_t* p = (const uint8_t*)src;
  if ((tid & 63u) >= kPfLanes) return;
  const uint32_t q = (tid >> 6) * kPfLanes + (tid & (kPfLanes - 1u));  // kPfLanes lanes per wave
  for (uint32_t off = q * 128u; off < bytes; off += (kSlotThreads / 64u) * kPfLanes * 128u)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + off),
                                     (__attribute__((address_space(3))) void*)scratch, 4, 0, 0);
}

// TIMING: the diagnostics instantiation (EvalArgs::phase) — phase clocks add registers, so the
// product kernel is compiled without them.
template <bool LDST, bool TIMING, uint32_t F>
__global__ void __launch_bounds__(kSlotThreads, 1)
    evaluate_tiles_kernel(EvalArgs a, const TileArgs* __restrict__ tp, const TileDesc* __restrict__ desc) {
  // TileArgs lives in device memory: its fields are scalar-loaded where used instead of all being
  // hoisted from the kernarg segment into SGPRs at entry.
  const TileArgs& t = *tp;
  // families compiled into this instantiation (TileArgs::feat): images / trusted-repos, labels,
  // container families (pod-privileged, psp-capabilities, psp-apparmor), group columns
  constexpr bool IMG = (F & kFeatImg) != 0, LBL = (F & kFeatLbl) != 0, CTR = (F & kFeatCtr) != 0, GRP = (F & kFeatGrp) != 0;
  constexpr bool NFA = (F & kFeatNfa) != 0;  // classifiers with NFA elements (their classes precomputed in HBM)
  constexpr bool RNG = (F & kFeatRng) != 0;  // many containers per request: predecessor sets by wave scan
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* __restrict__ out = a.out;

  // phase clocks (diagnostics): thread 0 reads the shader clock right after each barrier
  constexpr bool timing = TIMING;
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tk = timing ? clock64() : 0;
  const uint64_t t_begin = tk;
  auto mark = [&](int k) {
    if (timing && tid == 0) {
      const uint64_t now = clock64();
      ph[k] += now - tk;
      tk = now;
    }
  };
  // per-wave segment clocks (diagnostics, kPhaseWords layout in kernels.hpp): the item loops of P1
  // and P2 are wave-uniform per iteration, so each wave charges an iteration to its segment
  // (lane 0 adds to the workgroup's counters in HBM: returnless atomics, no registers held)
  auto sg_add = [&](uint32_t k, uint64_t d) {
    if (timing && lane == 0) atomicAdd((unsigned long long*)&a.phase[(uint64_t)blockIdx.x * kPhaseWords + 8u + k], (unsigned long long)d);
  };
  if (timing && tid == 0) a.phase[(uint64_t)blockIdx.x * kPhaseWords + 8u + SG_START] = __builtin_amdgcn_s_memrealtime();
  uint64_t sg_t = 0;
  int sg_k = -1;
  auto seg = [&](int k) {
    if (timing) {
      const uint64_t now = clock64();
      if (sg_k >= 0) sg_add((uint32_t)sg_k, now - sg_t);
      sg_t = now;
      sg_k = __builtin_amdgcn_readfirstlane(k);
    }
  };

  const uint32_t npol = a.npol;
  // Tile schedule (capi.cpp sched_dynamic picks one per launch). Workgroup b runs on XCD b % 8 and
  // serves that XCD's contiguous range of tiles. Static: the range strided by the XCD's
  // workgroups. Dynamic (a.sched): the tiles one at a time from the XCD's own
  // counter (a 128-B line each, so no counter is shared between XCDs); the atomic for the next tile
  // is issued when the current tile starts and its result is read only at the tile's end, so its
  // latency hides behind the tile. The XCD's last workgroup to finish zeroes the counter again.
  // The schedule runs two tiles ahead: while a tile is evaluated, the index of the next one is
  // already known, so its descriptor is copied into LDS under this tile's staging (the next tile's
  // P0 and its L2 prefetch read it there, with no dependent global load), and the counter fetch
  // issued now names the tile after next.
  const bool dyn = a.sched != nullptr;
  const uint32_t nx = min(8u, gridDim.x);
  const uint32_t xcd = blockIdx.x % nx;
  // both schedules serve the XCD's contiguous range (adjacent tiles share the cache lines at their
  // boundaries, so they stay in one L2)
  const uint64_t t_lo = a.ndesc * xcd / nx, t_hi = a.ndesc * (xcd + 1) / nx;
  uint32_t* cnt = dyn ? a.sched + xcd * 32u : nullptr;
  uint32_t* l_nx = (uint32_t*)(lds + t.o_nx);  // the tile after next, double-buffered
  TileDesc* l_desc = (TileDesc*)(lds + t.o_desc);
  // descriptor `i` into LDS slot `s`: 32 lanes of wave 0, one dword each (LDS-DMA, counted by vmcnt)
  auto fetch_desc = [&](uint64_t i, uint32_t s) {
    if (tid < 32u)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)((const uint32_t*)(desc + i) + tid),
                                       (__attribute__((address_space(3))) void*)(l_desc + s), 4, 0, 0);
  };
  auto sfield = [](const uint32_t& f) -> uint32_t { return __builtin_amdgcn_readfirstlane(f); };
  // P1 / P2 item blocks (64 items, one wave each, costliest segments first). DYNB (the instantiations
  // without image code: C4, C5): a wave's first block is its own, each further one comes from the
  // phase's LDS counter (l_nx[2] / l_nx[3]), so a wave that drew cheap blocks takes more instead of
  // waiting at the barrier for one that drew costly ones (C5 -8 %, C4 flat). The image
  // instantiations keep blocks strided by the waves (C2 +1.6 %, C3 +3.6 % with the counters;
  // profiles/r05_dyn_blocks_ab.txt).
  constexpr bool DYNB = !IMG;
  auto next_block = [&](uint32_t k) -> uint32_t {
    uint32_t v = 0;
    if (lane == 0u) v = atomicAdd(&l_nx[2u + k], 1u);
    return (kSlotThreads >> 6) + __builtin_amdgcn_readfirstlane(v);
  };
  // Dynamic: a workgroup's first two tiles are static (the XCD's range in workgroup order), so a
  // launch does not open with every workgroup's counter fetches queued on one L2 line; the counter
  // hands out the range from its third tile-set on (value v = tile dbase + v). r05: the opening
  // fetches cost a 1M C4 pass 2.4 % and a 64k-request shard 57 % (profiles/r05_sched_ab.txt).
  const uint32_t wpx = (gridDim.x - xcd + nx - 1u) / nx;  // workgroups b < gridDim.x with b % nx == xcd
  const uint64_t dbase = t_lo + 2ull * wpx;
  uint64_t tile = t_lo + blockIdx.x / nx, next = tile + wpx;
  // the first tile's descriptor goes out with the table staging below (r06: one memory round trip
  // fewer before the first tile, which a small shard's ~2 tiles a workgroup feel; KW_DESC_EARLY=0
  // restores the separate fetch and barrier for A/B)
  // (LDS-table instantiations only: the global-table one, C6, stages no tables and runs 1.2 % slower
  // with the early fetch, profiles/r06_c6_desc_early_ab.txt)
  constexpr bool desc_early = KW_DESC_EARLY && LDST;
  if (desc_early && tile < t_hi) fetch_desc(tile, 0);
  // ---- once per workgroup: the column classifiers and the chunks' staged record prefixes
  if (LDST) {
#if KW_TABLE_DMA
    // LDS-DMA: every 16-B piece of the tables in flight at once, one memory latency before the barrier
    // (a copy through VGPRs waits a latency per loop trip: ~3 trips of 256 x 16 B for C4's 12 KB)
    for (uint32_t s = 0; s < t.nstage; ++s)
      glds_x4((const u32x4*)(a.blob + t.stage_blob[s]), (u32x4*)(lds + t.stage_lds[s]), t.stage_bytes[s] / 16u, tid);
    for (uint32_t c = 0; c < t.nchunk; ++c)
      glds_x4((const u32x4*)t.chunk[c].rec, (u32x4*)(lds + t.chunk[c].o_lds), ((const SlotHdr*)t.chunk[c].rec)->staged / 16u, tid);
#else
    for (uint32_t s = 0; s < t.nstage; ++s) copy_x4(a.blob + t.stage_blob[s], lds + t.stage_lds[s], t.stage_bytes[s], tid);
    for (uint32_t c = 0; c < t.nchunk; ++c)
      copy_x4(t.chunk[c].rec, lds + t.chunk[c].o_lds, ((const SlotHdr*)t.chunk[c].rec)->staged, tid);
#endif
  }
  __syncthreads();
  mark(7);
  const uint8_t* tb = LDST ? (const uint8_t*)lds : a.blob;
  Classifiers C;
#pragma unroll
  for (int c = 0; c < (int)NCOL; ++c) {
    uint32_t lo = LDST ? t.lit_lds[c] : t.lit_blob[c];
    // the label-key and capability literal tables, probed in C4's hottest P1 loops
    if constexpr (!IMG && !GRP && LDST)
      if (c == COL_LK || c == COL_CAP) asm("" : "+v"(lo));
    C.lit[c] = t.lit_blob[c] ? tb + lo : nullptr;
    C.dfa[c].head = t.dfa_blob[c];
    C.dfa[c].base = tb + (LDST ? t.dfa_lds[c] : t.dfa_blob[c]);
  }
  uint32_t kvo = t.kv_lds;
  C.kv = t.kv_blob ? ((LDST && t.kv_lds) ? (const uint8_t*)lds + kvo : a.blob + t.kv_blob) : nullptr;  // kv_lds 0: global
  C.nlk = t.nlk;
  C.docker_io_cls = t.docker_io_cls;
  C.latest_cls = t.latest_cls;
  auto chunk_view = [&](uint32_t c) {
    SlotView sv;
    sv.base = LDST ? (const uint8_t*)lds + t.chunk[c].o_lds : t.chunk[c].rec;
    sv.h = (const SlotHdr*)sv.base;
    return sv;
  };

  // The tile's LDS regions. Where the instantiation's occupancy is bound by LDS with VGPRs to spare
  // (the label / container families, C4 / C5 at <= 4 workgroups per CU), their offsets
  // are held in VGPRs: otherwise they are 24 more uniform values competing for the 102 SGPRs, and
  // the compiler spills SGPRs to VGPR lanes, each reload a v_readlane_b32 in the hot loops.
  auto region = [&](uint32_t off) -> uint8_t* {
    if constexpr (!IMG && !GRP && LDST) asm("" : "+v"(off));
    return lds + off;
  };
  uint8_t* l_rf = region(t.o_rf);
  uint32_t* l_coff = (uint32_t*)region(t.o_coff);
  uint32_t* l_loff = (uint32_t*)region(t.o_loff);
  uint8_t* l_cflags = region(t.o_cflags);
  uint32_t* l_cadd = (uint32_t*)region(t.o_cadd);
  uint32_t* l_cdrop = (uint32_t*)region(t.o_cdrop);
  uint16_t* c_ns = (uint16_t*)region(t.o_ns);
  uint16_t* c_aa = (uint16_t*)region(t.o_aa);
  uint16_t* c_img = (uint16_t*)region(t.o_img);
  uint16_t* c_add = (uint16_t*)region(t.o_capadd);
  uint16_t* c_drop = (uint16_t*)region(t.o_capdrop);
  uint16_t* c_lk = (uint16_t*)region(t.o_lk);
  uint16_t* c_lv = (uint16_t*)region(t.o_lv);
  uint64_t* l_rej = (uint64_t*)region(t.o_rej);
  uint64_t* l_mut = (uint64_t*)region(t.o_mut);
  uint8_t* l_byp = region(t.o_byp);
  uint32_t* l_sa = (uint32_t*)region(t.o_sa);
  uint64_t* l_vadd = (uint64_t*)region(t.o_vadd);
  uint64_t* l_vl = (uint64_t*)region(t.o_vl);
  uint64_t* l_vc = (uint64_t*)region(t.o_vc);
  uint64_t* l_vtr = (uint64_t*)region(t.o_vtr);
  uint32_t* l_vw = (uint32_t*)region(t.o_vw);
  uint8_t* own_c = region(t.o_own_c);  // tile-local request of each staged container / label
  uint8_t* own_l = region(t.o_own_l);
  const ImgLayout il = t.il;
  const uint32_t nim = il.n(), nlv = t.nlv;
  const uint32_t need = t.need;

  if (!desc_early) {
    if (tile < t_hi) fetch_desc(tile, 0);
    __syncthreads();
  }
  mark(4);
  for (uint32_t it = 0; tile < t_hi; ++it) {
    const uint64_t p0_t0 = timing ? clock64() : 0;
    const uint32_t cur = it & 1u;
    uint32_t nxt2 = 0;
    if (dyn && tid == 0) nxt2 = atomicAdd(cnt, 1u);  // the tile after next (read after the staging barrier)
    if (next < t_hi) fetch_desc(next, cur ^ 1u);      // the next tile's descriptor (slot free since its last read)
    const TileDesc& d = l_desc[cur];
#define KW_DF(x) sfield(x)
    if (!KW_DF(d.fits)) {  // queued for the overflow kernels by the host (uniform: no barrier skipped unevenly)
      if (dyn && tid == 0) l_nx[cur] = nxt2;
      __syncthreads();  // also waits for the next descriptor
      tile = next;
      next = dyn ? dbase + l_nx[cur] : next + wpx;
      continue;
    }
    const uint64_t r0 = ((uint64_t)KW_DF(d.r0hi) << 32) | KW_DF(d.r0lo);
    const uint32_t nr = KW_DF(d.nr);
    const uint32_t cb = KW_DF(d.cb), ce = KW_DF(d.ce), lb = KW_DF(d.lb), le = KW_DF(d.le);
    const uint32_t kab = KW_DF(d.kab), kae = KW_DF(d.kae), kdb = KW_DF(d.kdb), kde = KW_DF(d.kde);
    const uint32_t nc = ce - cb, nl = le - lb;
    uint64_t p0_t1 = 0, p0_t2 = 0;
    if (timing) {
      p0_t1 = clock64();
      sg_add(SG_P0_TOP, p0_t1 - p0_t0);
    }

    // ---- P0: stage request headers, container offsets and the tile's strings. Every copy is an
    //      LDS-DMA (global_load_lds: no VGPR round trip), so all of a tile's loads are in flight
    //      together and the barrier waits for one memory latency, not one per array.
    // Label / container instantiations (several staged string columns): each copy job runs on one
    // wave (job j on wave j % 4). A job's setup is a chain of dependent round trips (the column's
    // addresses are scalar loads from TileArgs, its span descriptor fields LDS reads, each waited
    // for before the copy can issue); spread over the waves, each wave waits for a quarter of them,
    // and the copies take a few more trips of a cheap loop. r06 (profiles/r06_p0_spread_ab.txt):
    // C4 -3.2 %, C6 -0.7 %; the image-only ones (C2 / C3: one string column) +0.5-1 %, so they
    // keep the workgroup-wide copies.
    constexpr bool p0_spread = KW_P0_SPREAD && (LBL || CTR);
    if constexpr (p0_spread) {
      auto job = [&](uint32_t j) { return wave == (j & 3u); };
      if (job(0)) wglds_dwords((const uint32_t*)(a.req_flags + r0), (uint32_t*)l_rf, (nr + 3u) >> 2, lane);
      if (job(1)) wglds_dwords(a.ctr_off + r0, l_coff, nr + 1, lane);
      if (job(2)) wglds_dwords(a.lbl_off + r0, l_loff, nr + 1, lane);
      if (job(3)) wglds_dwords((const uint32_t*)a.ctr_flags + (cb >> 2), (uint32_t*)l_cflags, ((ce + 3u) >> 2) - (cb >> 2), lane);
      if (job(4)) wglds_dwords(a.capadd_off + cb, l_cadd, nc + 1, lane);
      if (job(5)) wglds_dwords(a.capdrop_off + cb, l_cdrop, nc + 1, lane);
      if (timing) {
        p0_t2 = clock64();
        sg_add(SG_P0_REQ, p0_t2 - p0_t1);
      }
#pragma unroll
      for (int m = 0; m < (int)NSTR; ++m) {
        const uint32_t jo = 6u + 2u * (uint32_t)m, jb = jo + 1u;
        if (!(job(jo) || job(jb)) || !t.o_sb[m]) continue;
        if (job(jo)) {
          const uint32_t g0 = str_g0(m, (uint32_t)r0, cb, kab, kdb, lb);
          const uint32_t n = str_n(m, nr, nc, kae - kab, kde - kdb, nl);
          wglds_dwords(t.s_off[m] + g0, (uint32_t*)(lds + t.o_so[m]), n + 1, lane);  // absolute: rebased by l_sa
        } else {
          wglds_x4((const u32x4*)(t.s_bytes[m] + KW_DF(d.sa[m])), (u32x4*)(lds + t.o_sb[m]), KW_DF(d.nv[m]), lane);
        }
      }
    } else {
      glds_dwords((const uint32_t*)(a.req_flags + r0), (uint32_t*)l_rf, (nr + 3u) >> 2, tid);
      glds_dwords(a.ctr_off + r0, l_coff, nr + 1, tid);
      glds_dwords(a.lbl_off + r0, l_loff, nr + 1, tid);
      glds_dwords((const uint32_t*)a.ctr_flags + (cb >> 2), (uint32_t*)l_cflags, ((ce + 3u) >> 2) - (cb >> 2), tid);
      glds_dwords(a.capadd_off + cb, l_cadd, nc + 1, tid);
      glds_dwords(a.capdrop_off + cb, l_cdrop, nc + 1, tid);
      if (timing) {
        p0_t2 = clock64();
        sg_add(SG_P0_REQ, p0_t2 - p0_t1);
      }
#pragma unroll
      for (int m = 0; m < (int)NSTR; ++m) {
        if (!t.o_sb[m]) continue;
        const uint32_t g0 = str_g0(m, (uint32_t)r0, cb, kab, kdb, lb);
        const uint32_t n = str_n(m, nr, nc, kae - kab, kde - kdb, nl);
        glds_dwords(t.s_off[m] + g0, (uint32_t*)(lds + t.o_so[m]), n + 1, tid);  // absolute: rebased by l_sa
        glds_x4((const u32x4*)(t.s_bytes[m] + KW_DF(d.sa[m])), (u32x4*)(lds + t.o_sb[m]), KW_DF(d.nv[m]), tid);
      }
    }
    if (timing) sg_add(SG_P0_STR, clock64() - p0_t2);
    for (uint32_t i = tid; i < nr; i += kSlotThreads) l_rej[i] = l_mut[i] = 0;
    if (DYNB && tid == 0) l_nx[2] = l_nx[3] = 0;  // P1 / P2 block counters (below)
    if (tid < NSTR) l_sa[tid] = d.sa[tid];
#undef KW_DF
    const uint64_t p0_end = timing ? clock64() : 0;
    __syncthreads();  // staged tile, the next descriptor and the counter fetch have landed
    if (timing) sg_add(SG_P0_WAIT, clock64() - p0_end);
    mark(0);
    if (timing && tid == 0) ++ph[5];
    if (dyn && tid == 0) l_nx[cur] = nxt2;  // read after this tile's last barrier
    // the next tile's staged ranges into L2 (covered by this tile's classification, walk and stores),
    // from its descriptor in LDS
    auto prefetch_next = [&]() {
      // (compiled only into the LDS-table image instantiations: its presence, never run, changes
      // their register allocation — C2 -3.3 %, C3 -1.7 % against builds without it — while r05's
      // label / container instantiations are 1.1-1.3 % faster without it and the global-table
      // ones 2 % (r04); profiles/r05_prefetch_code_ab.txt)
      if (KW_PREFETCH && LDST && IMG && t.prefetch && next < t_hi) {
        const TileDesc& dn = l_desc[cur ^ 1u];
        if (sfield(dn.fits)) {
          const uint64_t q0 = ((uint64_t)sfield(dn.r0hi) << 32) | sfield(dn.r0lo);
          const uint32_t qn = sfield(dn.nr), qcb = sfield(dn.cb), qc = sfield(dn.ce) - qcb;
          const uint32_t qlb = sfield(dn.lb), qkab = sfield(dn.kab), qkdb = sfield(dn.kdb);
          uint8_t* scratch = lds + t.o_pf;
          prefetch_l2(a.req_flags + q0, qn, scratch, tid);
          prefetch_l2(a.ctr_off + q0, (qn + 1) * 4u, scratch, tid);
          prefetch_l2(a.lbl_off + q0, (qn + 1) * 4u, scratch, tid);
          prefetch_l2(a.ctr_flags + qcb, qc, scratch, tid);
          prefetch_l2(a.capadd_off + qcb, (qc + 1) * 4u, scratch, tid);
          prefetch_l2(a.capdrop_off + qcb, (qc + 1) * 4u, scratch, tid);
#pragma unroll
          for (int m = 0; m < (int)NSTR; ++m) {
            if (!t.o_sb[m]) continue;
            const uint32_t g0 = str_g0(m, (uint32_t)q0, qcb, qkab, qkdb, qlb);
            const uint32_t n = str_n(m, qn, qc, sfield(dn.kae) - qkab, sfield(dn.kde) - qkdb, sfield(dn.le) - qlb);
            prefetch_l2(t.s_off[m] + g0, (n + 1) * 4u, scratch, tid);
            prefetch_l2(t.s_bytes[m] + sfield(dn.sa[m]), sfield(dn.nv[m]) * 16u, scratch, tid);
          }
        }
      }
    };
    const uint8_t* cfl = l_cflags + (cb & 3u);  // staged from the dword holding flag cb
    const bool classify = !(t.debug & 1u);  // diagnostics: skip classification (entities match nothing)
    auto str = [&](int m, uint32_t i, uint32_t* b, uint32_t* e) {
      const uint32_t* so = (const uint32_t*)(lds + t.o_so[m]);
      const uint32_t sa = l_sa[m];
      *b = so[i] - sa;
      *e = so[i + 1] - sa;
    };
    auto lit = [&](Col c, int m, uint32_t i) -> uint32_t {
      if (!classify || !C.lit[c]) return 0u;
      uint32_t b, e;
      str(m, i, &b, &e);
      // every string of the wave within 16 bytes (the common case): the 4-word batch
      if (!__ballot(e - b > 16u)) return lit_lookup<true, 4>(C.lit[c], lds + t.o_sb[m], b, e);
      return lit_lookup<true>(C.lit[c], lds + t.o_sb[m], b, e);
    };

    // ---- P1: classify the staged strings entity-parallel, and derive chunk 0's violation sets.
    //      Items come in segments padded to whole waves, ordered by cost: labels (key literal,
    //      value DFAs -> V_l), containers (AppArmor, added / dropped capabilities -> V_c, V_add),
    //      images (registry / tag / image classes -> V_tr), requests (namespace, owner maps, bypass).
    {
      const SlotView sv0 = chunk_view(0);
      const SlotHdr& h0 = *sv0.h;
      const uint32_t n3 = (LBL && (need & (1u << S_LK))) ? nl : 0u;
      const uint32_t nka = kae - kab, nkd = kde - kdb;
      const uint32_t nk = (CTR && (need & (1u << S_CAPADD))) ? nka + nkd : 0u;
      const uint32_t n2 = CTR ? nc : 0u;
      const uint32_t n1 = (IMG && (need & (1u << S_IMG))) ? nc : 0u;
      const uint32_t n0 = nr;
      const uint32_t ek = rup64(n3), e0 = ek + rup64(nk), e1 = e0 + rup64(n2), e2 = e1 + rup64(n1), e3 = e2 + rup64(n0);
      // helper lanes for second label-value DFAs (below): LDS tables, chains of at most two DFAs, and
      // one chunk (its class array, unused then, holds the 4 waves' 128-B mailboxes: lmax * nlv * 2
      // bytes with nlv == 2, so lmax >= 128 holds them only while a workgroup is 4 waves)
      static_assert(kSlotThreads == 256u && (kSlotThreads / 64u) * 128u == 128u * 2u * 2u,
                    "the label-pair mailboxes assume 4 waves and a class array of >= 128 labels x 2 x u16");
      const bool label_pairs = LDST && C.kv && t.kv_lds && nlv == 2u && t.nchunk == 1u && t.lmax >= 128u && classify &&
                               t.o_sb[S_LV] && !(t.debug & 2048u);
      const uint64_t p1_t0 = timing ? clock64() : 0;
      for (uint32_t w = tid; w < e3; w = DYNB ? next_block(0u) * 64u + lane : w + kSlotThreads) {
        seg(w < ek ? SG_P1_LABEL : w < e0 ? SG_P1_CAPSTR : w < e1 ? SG_P1_CTR : w < e2 ? SG_P1_IMAGE : SG_P1_REQ);
        if (LBL && w < ek) {  // label
          const uint32_t i = w;
          if (!NFA && LDST && label_pairs) {
            // Two-DFA chains, single-chunk pass: a wave walks one DFA per lane, not two. A label whose
            // key's chain has a second DFA hands that walk to a lane with nothing to walk (a key
            // without value constraints, or past the tile's labels): the n-th such label to the
            // n-th idle lane, matched through a per-wave mailbox in the (here unused) class array;
            // the task and its class cross lanes by ds_bpermute. Labels left without a helper walk
            // their second DFA themselves.
            const bool act = i < n3;
            uint32_t k = 0;
            if (act) {
              k = lit(COL_LK, S_LK, i);
              c_lk[i] = (uint16_t)k;
            }
            const as_ptr<3> R = (as_ptr<3>)C.kv;
            typedef const __attribute__((address_space(3))) uint32_t* u32l;
            typedef const __attribute__((address_space(3))) uint16_t* u16l;
            uint32_t b = 0, e = 0, rel1 = 0, rel2 = 0, kbase = 0;
            if (k) {
              str(S_LV, i, &b, &e);
              rel1 = ((u32l)R)[k];
              kbase = ((u32l)R)[C.nlk + k];
            }
            if (rel1) rel2 = kv_record<3>(R, rel1).next;
            const uint64_t needm = __ballot(rel2 != 0u), idlem = __ballot(rel1 == 0u);
            uint32_t wrel = rel1, wb = b, we = e, wkb = kbase, helper = 64u;
            if (needm) {
              uint8_t* mb = (uint8_t*)c_lv + wave * 128u;
              const uint32_t rn = __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
              const uint32_t ri = __builtin_amdgcn_mbcnt_hi((uint32_t)(idlem >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idlem, 0u));
              const uint32_t nidle = (uint32_t)__popcll(idlem), nneed = (uint32_t)__popcll(needm);
              if (rel1 == 0u) mb[ri] = (uint8_t)lane;
              if (rel2) mb[64u + rn] = (uint8_t)lane;
              // (a wave's LDS operations complete in order: the reads below see these writes; the
              // empty asm keeps the compiler from moving a read above another lane's write)
              asm volatile("" ::: "memory");
              helper = (rel2 && rn < nidle) ? mb[rn] : 64u;
              const uint32_t served = (rel1 == 0u && ri < nneed) ? mb[64u + ri] : lane;
              const int sa = (int)(served * 4u);
              const uint32_t t_rel = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)rel2);
              const uint32_t t_b = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)b);
              const uint32_t t_e = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)e);
              const uint32_t t_kb = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)kbase);
              if (served != lane) {
                wrel = t_rel;
                wb = t_b;
                we = t_e;
                wkb = t_kb;
              }
            }
            // walk 0: the lane's first DFA (or its served lane's second); walk 1: second DFAs no
            // idle lane took
            uint32_t res[2] = {0xffffu, 0xffffu};
#pragma nounroll
            for (uint32_t it = 0; it < 2u; ++it) {
              const bool self2 = rel2 && helper == 64u;
              if (it == 1u && !__any(self2)) break;
              const uint32_t r = it == 0u ? wrel : (self2 ? rel2 : 0u);
              if (r) {
                const KvDfa d = kv_record<3>(R, r);
                const uint32_t st = kv_walk<3>(R, d, lds + t.o_sb[S_LV], it == 0u ? wb : b, it == 0u ? we : e);
                res[it] = (it == 0u ? wkb : kbase) + d.cbase + ((u16l)(R + d.acc_off))[st];
              }
            }
            const uint32_t hc = needm ? (uint32_t)__builtin_amdgcn_ds_bpermute((int)((helper < 64u ? helper : lane) * 4u), (int)res[0]) : 0u;
            if (act) {
              const uint32_t c1 = rel1 ? res[0] : 0xffffu;
              const uint32_t c2 = rel2 ? (helper < 64u ? hc : res[1]) : 0xffffu;
              uint64_t v = 0;
              if (h0.lbl && k) {
                v = sv0.row(T_DENY, k);
                if (c1 != 0xffffu) v |= sv0.row(T_FAIL, c1);
                if (c2 != 0xffffu) v |= sv0.row(T_FAIL, c2);
              }
              l_vl[i] = v;
            }
            continue;
          }
          if (i >= n3) continue;
          const uint32_t k = lit(COL_LK, S_LK, i);
          c_lk[i] = (uint16_t)k;
          uint16_t* lv = c_lv + i * nlv;
          // chunk 0's failed-constraint slots folded in as the walk yields each value class; the
          // classes themselves are stored only for a pass whose later chunks rederive l_vl (D)
          const bool keep = t.nchunk > 1u;
          uint64_t vf = 0;
          auto out = [&](uint32_t j, uint32_t c) {
            if (keep) lv[j] = (uint16_t)c;
            if (h0.lbl && c != 0xffffu) vf |= sv0.row(T_FAIL, c);
          };
          if (k && classify && t.o_sb[S_LV] && !(t.debug & 2048u)) {
            uint32_t b, e;
            str(S_LV, i, &b, &e);
            classify_value<NFA>(C, LDST && t.kv_lds, k, nlv, lds + t.o_sb[S_LV], b, e, out,
                                NFA ? a.nfa_lv + (uint64_t)(lb + i) * nlv : nullptr);
          } else if (keep) {
            for (uint32_t j = 0; j < nlv; ++j) lv[j] = 0xffffu;
          }
          l_vl[i] = (h0.lbl && k) ? sv0.row(T_DENY, k) | vf : 0ull;  // (dv_label's sets)
        } else if (CTR && w < e0) {  // capability string: added ones first, then dropped ones
          const uint32_t k = w - ek;
          if (k >= nk) continue;
          if (k < nka) {
            const uint32_t cc = lit(COL_CAP, S_CAPADD, k);
            // single-chunk pass: the capability's mutation bit itself (P2 reads no class table)
            c_add[k] = (uint16_t)cc;
            l_vadd[k] = (h0.caps && h0.caps_strict) ? sv0.row(T_NACAP, cc) : 0ull;
          } else {
            const uint32_t dc = lit(COL_CAP, S_CAPDROP, k - nka);
            c_drop[k - nka] = (uint16_t)dc;
          }
        } else if (CTR && w < e1) {  // container (its added capabilities' sets stay in l_vadd: P2 ORs them)
          const uint32_t i = w - e0;
          if (i >= n2) continue;
          const uint32_t fl = cfl[i];
          uint64_t v = priv_viol(h0, fl);
          if (need & (1u << S_AA)) {
            const uint32_t ac = (fl & KW_CTR_HAS_APPARMOR) ? lit(COL_AA, S_AA, i) : 0u;
            c_aa[i] = (uint16_t)ac;
            if (h0.aa && (fl & KW_CTR_HAS_APPARMOR)) v |= sv0.row(T_NAAA, ac);
          }
          l_vc[i] = v;
        } else if (IMG && w < e2) {  // image reference: one parse feeds the registry, tag and image classes
          const uint32_t i = w - e1;
          if (i >= n1) continue;
          uint16_t* ic = c_img + i * nim;
          const uint32_t fl = cfl[i];
          if (classify && (fl & KW_CTR_HAS_IMAGE)) {
            uint32_t b, e;
            str(S_IMG, i, &b, &e);
            classify_image<true, LDST, NFA>(C, il, lds + t.o_sb[S_IMG], b, e, [&](uint32_t j, uint32_t c) { ic[j] = (uint16_t)c; },
                                 t.debug, NFA ? a.nfa_img + (uint64_t)(cb + i) * nim : nullptr);
          } else {
            for (uint32_t j = 0; j < nim; ++j) ic[j] = 0;
          }
          l_vtr[i] = dv_image(sv0, il, fl, ic);
        } else if (w >= e2) {  // request: namespace class, owner maps, bypass
          const uint32_t i = w - e2;
          if (i >= n0) continue;
          const uint32_t nsc = (need & (1u << S_NS)) ? lit(COL_NS, S_NS, i) : 0u;
          c_ns[i] = (uint16_t)nsc;
          if (CTR || IMG)
            for (uint32_t c = l_coff[i] - cb, c1 = l_coff[i + 1] - cb; c < c1; ++c) own_c[c] = (uint8_t)i;
          if (LBL)
            for (uint32_t l = l_loff[i] - lb, l1 = l_loff[i + 1] - lb; l < l1; ++l) own_l[l] = (uint8_t)i;
          l_byp[i] = is_bypass(l_rf[i], nsc, t.bypass_cls) ? 1 : 0;
        }
      }
      seg(-1);
      if (timing) sg_add(SG_P1_BUSY, clock64() - p1_t0);
    }
    const uint64_t p1_end = timing ? clock64() : 0;
    lds_barrier();
    if (timing) sg_add(SG_P1_WAIT, clock64() - p1_end);
    mark(1);
    prefetch_next();

    for (uint32_t ck = 0; ck < t.nchunk; ++ck) {
      const SlotView sv = chunk_view(ck);
      const SlotHdr& SH = *sv.h;
      if (ck > 0) {
        // ---- D: this chunk's violation sets from the stored classes
        const uint32_t n3 = (LBL && SH.lbl) ? nl : 0u, nk = (CTR && SH.caps) ? kae - kab : 0u, n2 = CTR ? nc : 0u,
                       n1 = (IMG && SH.trs) ? nc : 0u;
        const uint32_t ek = rup64(n3), e0 = ek + rup64(nk), e1 = e0 + rup64(n2), e2 = e1 + rup64(n1), e3 = e2 + rup64(nr);
        for (uint32_t w = tid; w < e3; w += kSlotThreads) {
          if (LBL && w < ek) {
            const uint32_t i = w;
            if (i < n3) l_vl[i] = dv_label(sv, c_lk[i], c_lv + i * nlv, nlv);
          } else if (CTR && w < e0) {  // added capability (read by P2 only when this chunk has caps slots)
            const uint32_t k = w - ek;
            if (k < nk) l_vadd[k] = SH.caps_strict ? sv.row(T_NACAP, c_add[k]) : 0ull;
          } else if (CTR && w < e1) {
            const uint32_t i = w - e0;
            if (i >= n2) continue;
            const uint32_t fl = cfl[i];
            uint64_t v = priv_viol(SH, fl);
            if (SH.aa && (fl & KW_CTR_HAS_APPARMOR)) v |= sv.row(T_NAAA, c_aa[i]);
            l_vc[i] = v;  // (l_vtr is read only by chunks with trusted-repos slots, which rewrite it below)
          } else if (IMG && w < e2) {
            const uint32_t i = w - e1;
            if (i < n1) l_vtr[i] = dv_image(sv, il, cfl[i], c_img + i * nim);
          } else if (w >= e2) {
            const uint32_t i = w - e2;
            if (i < nr) l_rej[i] = l_mut[i] = 0;
          }
        }
        lds_barrier();
        mark(2);
      }

      // ---- P2: first violations, entity-parallel. A slot's first violation is the first entity
      //      of the request (object order) whose violation set holds it: each entity thread ORs the
      //      sets of its predecessors in the request (independent LDS loads) and writes the words of
      //      the slots it violates first; within an entity the family's own order applies
      //      (capabilities in list order, trusted-repos reasons in precedence). Request items add
      //      the namespace and mandatory-label slots. Rejected / mutated slots merge with ds_or_b64.
      //      (Sequential form of the same walk: slots.hpp walk_*.)
      if (!(t.debug & 2u)) {
        const uint64_t privany = SH.priv[0] | SH.priv[1] | SH.priv[2] | SH.priv[3];
        const bool trs = IMG && SH.trs != 0;
        const bool ctr_fam = (CTR && (privany | SH.caps | SH.aa) != 0) || trs;
        const uint32_t n1 = ctr_fam ? nc : 0u, n2 = (LBL && SH.lbl) ? nl : 0u;
        // a container's violation set: its own families' (V_c) and its image's (V_tr)
        auto vset = [&](uint32_t j) -> uint64_t { return (CTR ? l_vc[j] : 0ull) | (trs ? l_vtr[j] : 0ull); };
        // item order: containers, labels, requests; DYNB: containers, requests, labels (the costly
        // request block drawn before the label blocks, most of whose items end at once)
        const uint32_t f0 = rup64(n1), f1 = f0 + rup64(DYNB ? nr : n2), f2 = f1 + rup64(DYNB ? n2 : nr);
        const uint64_t p2_t0 = timing ? clock64() : 0;
        for (uint32_t w = tid; w < f2; w = DYNB ? next_block(1u) * 64u + lane : w + kSlotThreads) {
          seg(w < f0 ? SG_P2_CTR : (w < f1) == DYNB ? SG_P2_REQ : SG_P2_LABEL);
          if (w < f0) {  // container
            const uint32_t i = w;
            const bool capv = CTR && SH.caps != 0;
            uint32_t q, c0, ka0, ka, ka1;
            uint64_t pre = 0, own;
            if constexpr (RNG) {
              // many containers per request: a container's set X = its own families', its image's and
              // its added capabilities'; the predecessors' union is a segmented exclusive OR-scan of X
              // over the wave's lanes (a segment = one request's containers), plus, for a request
              // that began before this wave's first container, the OR of that part from LDS.
              const bool act = i < n1;
              q = act ? own_c[i] : 0u;
              c0 = act ? l_coff[q] - cb : i;
              ka = act ? l_cadd[i] - kab : 0u;
              ka1 = act ? l_cadd[i + 1] - kab : 0u;
              own = act ? vset(i) : 0ull;
              if (capv) own |= or_range(l_vadd, ka, ka1);
              // lane 0 adds the part of its request before this wave (c0 < i): the scan hands it on
              uint64_t carry = 0;
              if (lane == 0u && c0 < i) {
                carry = (CTR ? or_range(l_vc, c0, i) : 0ull) | (trs ? or_range(l_vtr, c0, i) : 0ull);
                if (capv) carry |= or_range(l_vadd, l_cadd[c0] - kab, ka);
              }
              pre = seg_or_scan_excl(own | carry, lane, i, c0) | carry;
              if (t.debug & 4096u) pre = 0;  // (ablation bit 4096: no predecessor ORs, in every form)
              if (!act || !(l_rf[q] & KW_REQ_HAS_PODSPEC)) continue;
            } else {
            if (i >= n1) continue;
            q = own_c[i];
            if (!(l_rf[q] & KW_REQ_HAS_PODSPEC)) continue;
            c0 = l_coff[q] - cb;
            // predecessors' sets: their own families' and images', and their added capabilities'
            // (a contiguous range of l_vadd); the same for this container
            ka0 = l_cadd[c0] - kab, ka = l_cadd[i] - kab, ka1 = l_cadd[i + 1] - kab;
            own = vset(i);
            if (t.ctr_ranges) {  // many containers per request: the ranges four loads a round
              if (!(t.debug & 4096u)) {  // (ablation bit 4096: no predecessor ORs, in both forms)
                pre = (CTR ? or_range(l_vc, c0, i) : 0ull) | (trs ? or_range(l_vtr, c0, i) : 0ull);
                if (capv) pre |= or_range(l_vadd, ka0, ka);
              }
              if (capv) own |= or_range(l_vadd, ka, ka1);
            } else {
              if (!(t.debug & 4096u)) {
                for (uint32_t j = c0; j < i; ++j) pre |= vset(j);
                if (capv)
                  for (uint32_t k = ka0; k < ka; ++k) pre |= l_vadd[k];
              }
              if (capv)
                for (uint32_t k = ka; k < ka1; ++k) own |= l_vadd[k];
            }
            }
            const uint64_t nv = own & ~pre;
            const uint32_t ci = i - c0;
            uint32_t* vw = l_vw + q * t.vw_stride;
            if (nv && !(t.debug & 16384u)) {
              ViolSink vs{vw, nullptr};
              if (CTR) {
                vs.put(nv & privany, KW_R_PRIVILEGED, ci);
                vs.put(nv & SH.aa, KW_R_APPARMOR, ci);
              }
              uint64_t cn = CTR ? (nv & SH.caps) : 0ull;  // capability slots: the first added capability of the list
              const uint32_t kfirst = l_cadd[c0] - kab;
              for (uint32_t k = l_cadd[i] - kab, k1 = l_cadd[i + 1] - kab; k < k1 && cn; ++k) {
                const uint64_t nw = l_vadd[k] & cn;
                vs.put(nw, KW_R_CAP_NOT_ALLOWED, k - kfirst);
                cn &= ~nw;
              }
              uint64_t tn = IMG ? (nv & SH.trs) : 0ull;  // trusted-repos slots: reasons in precedence order
              if (tn) {
                uint64_t why[5];
                const uint16_t* ic = c_img + i * nim;
                trs_whys(sv, il, [&](uint32_t j) { return (uint32_t)ic[j]; }, why);
                for (uint32_t k = 0; k < 5; ++k) {
                  const uint64_t nw = why[k] & tn;
                  vs.put(nw, KW_R_REG_NOT_ALLOWED + k, ci);
                  tn &= ~nw;
                }
              }
              atomicOr((unsigned long long*)&l_rej[q], (unsigned long long)nv);
            }
            if (CTR && SH.caps && !(t.debug & 8192u)) {  // mutation: required drops missing, default adds neither added nor dropped
              uint64_t addm = 0, dropm = 0;
              for (uint32_t k = ka; k < ka1; ++k) addm |= bit_of(sv.capmb(c_add[k]));
              for (uint32_t k = l_cdrop[i] - kdb, k1 = l_cdrop[i + 1] - kdb; k < k1; ++k) dropm |= bit_of(sv.capmb(c_drop[k]));
              const uint64_t mut = caps_mutation(sv, addm, dropm);
              if (mut) atomicOr((unsigned long long*)&l_mut[q], (unsigned long long)mut);
            }
          } else if (LBL && (DYNB ? w >= f1 : w < f1)) {  // label
            const uint32_t i = w - (DYNB ? f1 : f0);
            if (i >= n2) continue;
            const uint64_t v = l_vl[i];
            if (!v) continue;
            const uint32_t q = own_l[i];
            const uint32_t l0 = l_loff[q] - lb;
            uint64_t pre = 0;
            for (uint32_t j = l0; j < i; ++j) pre |= l_vl[j];
            const uint64_t nv = v & ~pre;
            if (!nv || (t.debug & 16384u)) continue;
            const uint64_t den = sv.row(T_DENY, c_lk[i]);
            const uint32_t li = i - l0;
            ViolSink vs{l_vw + q * t.vw_stride, nullptr};
            vs.put(nv & den, KW_R_LABEL_DENIED, li);
            vs.put(nv & ~den, KW_R_LABEL_CONSTRAINT, li);
            atomicOr((unsigned long long*)&l_rej[q], (unsigned long long)nv);
          } else if (DYNB ? w < f1 : w >= f1) {  // request: namespace, mandatory labels
            const uint32_t i = w - (DYNB ? f0 : f1);
            if (i >= nr) continue;
            const uint32_t rf = l_rf[i];
            ViolSink vs{l_vw + i * t.vw_stride, nullptr};
            uint64_t rej = 0;
            if (SH.ns) {
              const uint64_t ok = (rf & KW_REQ_HAS_NAMESPACE) ? sv.row(T_NSOK, c_ns[i]) : 0ull;
              rej = SH.ns & ~ok;
              vs.put(rej, KW_R_NAMESPACE, 0);
            }
            if (LBL && SH.lbl && SH.mand_union && !(t.debug & 1024u)) {
              uint64_t present = 0, lrej = 0;
              for (uint32_t l = l_loff[i] - lb, l1 = l_loff[i + 1] - lb; l < l1; ++l) {
                present |= bit_of(sv.lkmb(c_lk[l]));
                lrej |= l_vl[l];
              }
              // slots missing a mandatory key: rows of the missing local bits, four loads per round
              uint64_t miss = SH.mand_union & ~present, nw = 0;
              const uint64_t* mt = sv.mand();
              while (miss) {
                uint32_t bb[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  bb[u] = miss ? kw_ctz64(miss) : 64u;
                  miss &= miss - 1;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) nw |= bb[u] < 64u ? mt[bb[u]] : 0ull;
              }
              nw &= ~lrej;
              rej |= nw;
              vs.put(nw & SH.mand_one, KW_R_LABEL_MANDATORY, 0);  // single-key lists: index 0, no list read
              nw &= ~SH.mand_one;
              while (nw) {  // the first missing mandatory key of each such slot (settings order), four per round
                uint32_t ss[4];
                uint64_t pk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  ss[u] = nw ? kw_ctz64(nw) : 64u;
                  nw &= nw - 1;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) pk[u] = ss[u] < 64u ? sv.mpack(ss[u]) : 0ull;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                  if (ss[u] < 64u) vs.vw[ss[u]] = vword(KW_R_LABEL_MANDATORY, first_missing_packed(sv, ss[u], pk[u], present));
              }
            }
            if (rej) atomicOr((unsigned long long*)&l_rej[i], (unsigned long long)rej);
          }
        }
        seg(-1);
        if (timing) sg_add(SG_P2_BUSY, clock64() - p2_t0);
      }
      const uint64_t p2_end = timing ? clock64() : 0;
      lds_barrier();
      if (timing) sg_add(SG_P2_WAIT, clock64() - p2_end);
      mark(3);

      // ---- P3: verdict words. All-pairs: items = (request, 4 columns), 16 lanes per 256-B row,
      //      column records from LDS (group / constant columns from the record's global copy).
      //      Rows mode: one word per request, its own column.
      const uint64_t p3_t0 = timing ? clock64() : 0;
      if (!(t.debug & 4u)) {
        const ChunkArgs& CA = t.chunk[ck];
        const uint64_t init = CA.init;
        const ColInfo* cols = (const ColInfo*)(CA.rec + SH.o_cols);
        const uint32_t ncols = CA.ncols;
        auto word = [&](uint32_t rr, uint32_t j) -> uint32_t {
          if (!GRP) {  // no group column in this launch: plain or constant columns only
            const ColInfo& ci = cols[j];
            if (ci.kind != CK_PLAIN) return ci.okw;
            if ((l_rej[rr] >> ci.slot) & 1ull) return ci.rejb | l_vw[rr * t.vw_stride + ci.slot];
            return ((l_mut[rr] >> ci.slot) & 1ull) ? ci.mutw : ci.okw;
          }
          uint64_t wide = 0;
          const uint32_t w = column_word(cols[j], l_rej[rr], l_mut[rr], init, l_vw + rr * t.vw_stride, CA.rec, &wide);
          if (cols[j].wide != ~0u && KW_REASON(w) == KW_R_GROUP) a.wide_groups[(r0 + rr) * a.nwide + cols[j].wide] = wide;
          return w;
        };
        if (t.rows_mode) {
          for (uint32_t rr = tid; rr < nr; rr += kSlotThreads) {
            const uint32_t rc = a.rowcol[r0 + rr];
            if ((rc >> 16) != ck) continue;
            out[r0 + rr] = l_byp[rr] ? kBypassWord : word(rr, rc & 0xffffu);
          }
        } else if (CA.vec4) {
          const uint32_t* cs = (const uint32_t*)(sv.base + SH.o_csoa);
          const uint32_t cs_n = (ncols + 3u) & ~3u;
          const uint32_t G = ncols >> 2;
          // the 4-column group g of request rr: one 16-B non-temporal store. Column data (kind,
          // slot, ok / mutated / rejected words) comes from the chunk's column arrays.
          struct Cols4 {
            uint4 ks, ok, mu, rj;
          };
          auto load4 = [&](uint32_t g) -> Cols4 {
            return {*(const uint4*)(cs + 4 * g), *(const uint4*)(cs + cs_n + 4 * g), *(const uint4*)(cs + 2 * cs_n + 4 * g),
                    *(const uint4*)(cs + 3 * cs_n + 4 * g)};
          };
          auto emit = [&](uint32_t rr, uint32_t g, const Cols4& c4, uint32_t* dst) {
            uint4 wv;
            if (l_byp[rr]) {
              wv = make_uint4(kBypassWord, kBypassWord, kBypassWord, kBypassWord);
            } else {
              const uint64_t rej = l_rej[rr], mut = l_mut[rr];
              const uint32_t* vw = l_vw + rr * t.vw_stride;
              auto pw = [&](uint32_t k, uint32_t okw, uint32_t mutw, uint32_t rejb, uint32_t j) -> uint32_t {
                if ((k & 0xffu) != CK_PLAIN) return GRP ? word(rr, j) : okw;  // (no group: a constant column)
                const uint32_t s = k >> 8;
                if ((rej >> s) & 1ull) return rejb | vw[s];
                return ((mut >> s) & 1ull) ? mutw : okw;
              };
              wv.x = pw(c4.ks.x, c4.ok.x, c4.mu.x, c4.rj.x, 4 * g + 0);
              wv.y = pw(c4.ks.y, c4.ok.y, c4.mu.y, c4.rj.y, 4 * g + 1);
              wv.z = pw(c4.ks.z, c4.ok.z, c4.mu.z, c4.rj.z, 4 * g + 2);
              wv.w = pw(c4.ks.w, c4.ok.w, c4.mu.w, c4.rj.w, 4 * g + 3);
            }
            const u32x4 nv4 = {wv.x, wv.y, wv.z, wv.w};
            __builtin_nontemporal_store(nv4, (u32x4*)dst);  // streamed once
          };
          if ((G & (G - 1u)) == 0 && G <= kSlotThreads) {
            // G a power of two dividing the workgroup: each thread keeps one column group for every
            // request it writes, so the column data is loaded once and no division is needed
            const uint32_t lg = (uint32_t)__builtin_ctz(G), g = tid & (G - 1u), step = kSlotThreads >> lg;
            const Cols4 c4 = load4(g);
            uint32_t* dst = out + (r0 + (tid >> lg)) * npol + CA.col0 + 4 * g;
            const uint64_t dstep = (uint64_t)step * npol;
            // (not in image-only instantiations: two more VGPRs there cross C2's 6-wave boundary, +8 %)
            if (!GRP && (LBL || CTR)) {
              // branch-free words from 32-bit halves: per column, the slot's rejected / mutated bits
              // as 0 / -1 masks (v_bfe_i32 of the half holding the slot), then two bit-selects
              // (v_bitop3_b32 0xCA: S0 ? S1 : S2). A constant column keeps okw: its rejected field
              // has width 0 (mask 0) and its mutated word is okw.
              const uint32_t ks[4] = {c4.ks.x, c4.ks.y, c4.ks.z, c4.ks.w};
              const uint32_t okc[4] = {c4.ok.x, c4.ok.y, c4.ok.z, c4.ok.w};
              const uint32_t muc[4] = {c4.mu.x, c4.mu.y, c4.mu.z, c4.mu.w};
              const uint32_t rjc[4] = {c4.rj.x, c4.rj.y, c4.rj.z, c4.rj.w};
              uint32_t cs[4], bs[4], wd[4], muw[4];
              bool hi[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const bool pl = (ks[k] & 0xffu) == CK_PLAIN;
                cs[k] = (ks[k] >> 8) & 63u;
                bs[k] = cs[k] & 31u;
                hi[k] = cs[k] >= 32u;
                wd[k] = pl ? 1u : 0u;
                muw[k] = pl ? muc[k] : okc[k];
              }
              for (uint32_t rr = tid >> lg; rr < nr; rr += step, dst += dstep) {
                const uint2 rj = *(const uint2*)&l_rej[rr], mu = *(const uint2*)&l_mut[rr];
                const uint32_t byp = l_byp[rr];
                const uint32_t* vw = l_vw + rr * t.vw_stride;
                uint32_t av[4], wk[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) av[k] = vw[cs[k]];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  const uint32_t rb = (uint32_t)__builtin_amdgcn_sbfe((int)(hi[k] ? rj.y : rj.x), bs[k], wd[k]);
                  const uint32_t mb = (uint32_t)__builtin_amdgcn_sbfe((int)(hi[k] ? mu.y : mu.x), bs[k], 1u);
                  const uint32_t tw = __builtin_amdgcn_bitop3_b32(mb, muw[k], okc[k], 0xCA);
                  wk[k] = __builtin_amdgcn_bitop3_b32(rb, rjc[k] | av[k], tw, 0xCA);
                }
                u32x4 wv = {wk[0], wk[1], wk[2], wk[3]};
                if (byp) wv = u32x4{kBypassWord, kBypassWord, kBypassWord, kBypassWord};
                __builtin_nontemporal_store(wv, (u32x4*)dst);  // streamed once
              }
            } else
            if (!GRP) {
              // branch-free words: the thread's four columns are loop-invariant; every row reads its
              // four violation words whether or not the slot rejected, then selects
              const uint32_t cs0 = (c4.ks.x >> 8) & 63u, cs1 = (c4.ks.y >> 8) & 63u, cs2 = (c4.ks.z >> 8) & 63u,
                             cs3 = (c4.ks.w >> 8) & 63u;
              const bool pl0 = (c4.ks.x & 0xffu) == CK_PLAIN, pl1 = (c4.ks.y & 0xffu) == CK_PLAIN,
                         pl2 = (c4.ks.z & 0xffu) == CK_PLAIN, pl3 = (c4.ks.w & 0xffu) == CK_PLAIN;
              for (uint32_t rr = tid >> lg; rr < nr; rr += step, dst += dstep) {
                const uint64_t rej = l_rej[rr], mut = l_mut[rr];
                const uint32_t byp = l_byp[rr];
                const uint32_t* vw = l_vw + rr * t.vw_stride;
                const uint32_t a0 = vw[cs0], a1 = vw[cs1], a2 = vw[cs2], a3 = vw[cs3];
                auto one = [&](bool pl, uint32_t cs, uint32_t av, uint32_t okw, uint32_t mutw, uint32_t rejb) -> uint32_t {
                  const uint32_t rb = (uint32_t)(rej >> cs) & 1u, mb = (uint32_t)(mut >> cs) & 1u;
                  const uint32_t w = rb ? (rejb | av) : (mb ? mutw : okw);
                  return pl ? w : okw;  // (not plain: a constant column)
                };
                u32x4 wv = {one(pl0, cs0, a0, c4.ok.x, c4.mu.x, c4.rj.x), one(pl1, cs1, a1, c4.ok.y, c4.mu.y, c4.rj.y),
                            one(pl2, cs2, a2, c4.ok.z, c4.mu.z, c4.rj.z), one(pl3, cs3, a3, c4.ok.w, c4.mu.w, c4.rj.w)};
                if (byp) wv = u32x4{kBypassWord, kBypassWord, kBypassWord, kBypassWord};
                __builtin_nontemporal_store(wv, (u32x4*)dst);  // streamed once
              }
            } else {
              for (uint32_t rr = tid >> lg; rr < nr; rr += step, dst += dstep) emit(rr, g, c4, dst);
            }
          } else {
            for (uint32_t q = tid; q < nr * G; q += kSlotThreads) {
              const uint32_t rr = q / G, g = q - rr * G;
              emit(rr, g, load4(g), out + (r0 + rr) * npol + CA.col0 + 4 * g);
            }
          }
        } else {
          for (uint32_t q = tid; q < nr * ncols; q += kSlotThreads) {
            const uint32_t rr = q / ncols, g = q - rr * ncols;
            out[(r0 + rr) * npol + CA.col0 + g] = l_byp[rr] ? kBypassWord : word(rr, g);
          }
        }
      }
      if (timing) sg_add(SG_P3_BUSY, clock64() - p3_t0);
      if (ck + 1 < t.nchunk) {
        if (DYNB && tid == 0) l_nx[3] = 0;  // the next chunk's P2 block counter
        lds_barrier();  // the next chunk rewrites the violation sets and words
        mark(4);
      }
    }
    const uint64_t p3_end = timing ? clock64() : 0;
    lds_barrier();  // the next tile restages LDS (its strings alias this tile's violation words)
    if (timing) sg_add(SG_P3_WAIT, clock64() - p3_end);
    mark(4);
    tile = next;
    next = dyn ? dbase + l_nx[cur] : next + wpx;
  }
  if (timing && tid == 0) {  // one lane's vector stores
    ph[6] = clock64() - t_begin;
    for (int k = 0; k < 8; ++k) a.phase[(uint64_t)blockIdx.x * kPhaseWords + (uint32_t)k] = ph[k];
  }
  if (dyn && tid == 0) {  // the XCD's last workgroup (every other one has taken its last tile) resets
    uint32_t* done = a.sched + 256u + xcd * 32u;
    __threadfence();  // this workgroup's last counter fetch is ordered before its done count
    if (atomicAdd(done, 1u) == wpx - 1u) {
      atomicExch(cnt, 0u);
      atomicExch(done, 0u);
    }
  }
  (void)lane;
  (void)wave;
}

// ------------------------------------------------------------------------------------------
// Overflow: requests whose entity counts or string bytes exceed the tile capacities even alone
// (listed by the host with the tile descriptors: [count, request indices...]). Two launches:
// overflow_classify_kernel classifies their strings into the HBM class arrays (tables read from the
// blob, one workgroup per request), then overflow_eval_kernel walks each request sequentially
// (slots.hpp walk_*, one lane per request) over every chunk of the launch.
// ------------------------------------------------------------------------------------------
constexpr int kOverflowThreads = 256;

__device__ inline Classifiers blob_classifiers(const EvalArgs& a, const TileArgs& t) {
  Classifiers C;
  for (int c = 0; c < (int)NCOL; ++c) {
    C.lit[c] = t.lit_blob[c] ? a.blob + t.lit_blob[c] : nullptr;
    C.dfa[c].head = t.dfa_blob[c];
    C.dfa[c].base = a.blob + t.dfa_blob[c];
  }
  C.kv = t.kv_blob ? a.blob + t.kv_blob : nullptr;
  C.nlk = t.nlk;
  C.docker_io_cls = t.docker_io_cls;
  C.latest_cls = t.latest_cls;
  return C;
}

__global__ void __launch_bounds__(kOverflowThreads)
    overflow_classify_kernel(EvalArgs a, const TileArgs* __restrict__ tp, const uint32_t* __restrict__ overflow) {
  const TileArgs& t = *tp;
  const uint32_t count = overflow[0];
  const uint32_t tid = threadIdx.x;
  const Classifiers C = blob_classifiers(a, t);
  const ImgLayout il = t.il;
  const uint32_t nim = il.n(), nlv = t.nlv;
  for (uint32_t q = blockIdx.x; q < count; q += gridDim.x) {
    const uint64_t r = overflow[1 + q];
    const uint32_t cb = a.ctr_off[r], ce = a.ctr_off[r + 1];
    const uint32_t lb = a.lbl_off[r], le = a.lbl_off[r + 1];
    const uint32_t kab = a.capadd_off[cb], kae = a.capadd_off[ce];
    const uint32_t kdb = a.capdrop_off[cb], kde = a.capdrop_off[ce];
    auto lit = [&](Col c, int m, uint32_t i) -> uint32_t {
      return C.lit[c] ? lit_lookup<false>(C.lit[c], t.s_bytes[m], t.s_off[m][i], t.s_off[m][i + 1]) : 0u;
    };
    if (tid == 0) a.g_ns[r] = (uint16_t)((t.need & (1u << S_NS)) ? lit(COL_NS, S_NS, (uint32_t)r) : 0u);
    for (uint32_t c = cb + tid; c < ce; c += kOverflowThreads) {
      const uint32_t fl = a.ctr_flags[c];
      if (t.need & (1u << S_AA)) a.g_aa[c] = (uint16_t)((fl & KW_CTR_HAS_APPARMOR) ? lit(COL_AA, S_AA, c) : 0u);
      if (t.need & (1u << S_IMG)) {
        uint16_t* ic = a.g_img + (uint64_t)c * nim;
        if (fl & KW_CTR_HAS_IMAGE)
          classify_image<false, false, true>(C, il, t.s_bytes[S_IMG], t.s_off[S_IMG][c], t.s_off[S_IMG][c + 1],
                                [&](uint32_t j, uint32_t cl) { ic[j] = (uint16_t)cl; }, 0u,
                                a.nfa_img ? a.nfa_img + (uint64_t)c * nim : nullptr);
        else
          for (uint32_t j = 0; j < nim; ++j) ic[j] = 0;
      }
    }
    if (t.need & (1u << S_CAPADD)) {
      for (uint32_t k = kab + tid; k < kae; k += kOverflowThreads) a.g_capadd[k] = (uint16_t)lit(COL_CAP, S_CAPADD, k);
      for (uint32_t k = kdb + tid; k < kde; k += kOverflowThreads) a.g_capdrop[k] = (uint16_t)lit(COL_CAP, S_CAPDROP, k);
    }
    if (t.need & (1u << S_LK))
      for (uint32_t l = lb + tid; l < le; l += kOverflowThreads) {
        const uint32_t k = lit(COL_LK, S_LK, l);
        a.g_lk[l] = (uint16_t)k;
        uint16_t* lv = a.g_lv + (uint64_t)l * nlv;
        classify_value<true>(C, false, k, nlv, t.s_bytes[S_LV], t.s_off[S_LV][l], t.s_off[S_LV][l + 1],
                             [&](uint32_t j, uint32_t c) { lv[j] = (uint16_t)c; }, a.nfa_lv ? a.nfa_lv + (uint64_t)l * nlv : nullptr);
      }
  }
}

// Accessor of the sequential walks over the HBM class arrays (absolute entity indices).
struct GlobalSrc {
  const EvalArgs* a;
  ImgLayout il;
  uint32_t nlv_;
  __device__ uint32_t rf(uint64_t r) const { return a->req_flags[r]; }
  __device__ uint32_t coff(uint64_t r) const { return a->ctr_off[r]; }
  __device__ uint32_t loff(uint64_t r) const { return a->lbl_off[r]; }
  __device__ uint32_t cflags(uint32_t c) const { return a->ctr_flags[c]; }
  __device__ uint32_t cadd(uint32_t c) const { return a->capadd_off[c]; }
  __device__ uint32_t cdrop(uint32_t c) const { return a->capdrop_off[c]; }
  __device__ uint32_t ns(uint64_t r) const { return a->g_ns[r]; }
  __device__ uint32_t aa(uint32_t c) const { return a->g_aa[c]; }
  __device__ uint32_t capadd(uint32_t k) const { return a->g_capadd[k]; }
  __device__ uint32_t capdrop(uint32_t k) const { return a->g_capdrop[k]; }
  __device__ uint32_t lk(uint32_t l) const { return a->g_lk ? a->g_lk[l] : 0u; }
  __device__ uint32_t nlv() const { return nlv_; }
  __device__ uint32_t lv(uint32_t l, uint32_t j) const { return a->g_lv[(uint64_t)l * nlv_ + j]; }
  __device__ uint32_t img(uint32_t c, uint32_t j) const { return a->g_img[(uint64_t)c * il.n() + j]; }
};

__global__ void __launch_bounds__(kOverflowThreads)
    overflow_eval_kernel(EvalArgs a, const TileArgs* __restrict__ tp, const uint32_t* __restrict__ overflow) {
  const TileArgs& t = *tp;
  const uint32_t count = overflow[0];
  GlobalSrc src{&a, t.il, t.nlv};
  for (uint32_t q = blockIdx.x * kOverflowThreads + threadIdx.x; q < count; q += gridDim.x * kOverflowThreads) {
    const uint64_t r = overflow[1 + q];
    const bool byp = is_bypass(a.req_flags[r], a.g_ns[r], t.bypass_cls);
    for (uint32_t ck = 0; ck < t.nchunk; ++ck) {
      const ChunkArgs& CA = t.chunk[ck];
      SlotView sv;
      sv.base = CA.rec;
      sv.h = (const SlotHdr*)CA.rec;
      uint32_t vw[kSlots], va[kSlots];
      const ViolSink vs{vw, va};
      uint64_t mut = 0, rej = 0;
      if (!byp) {
        rej = walk_privileged_caps(src, sv, r, vs, &mut);
        rej |= walk_apparmor_images(src, sv, r, vs);
        if (a.g_lk) rej |= walk_labels(src, sv, r, vs);
        rej |= walk_namespace(src, sv, r, vs);
      }
      const ColInfo* cols = (const ColInfo*)(CA.rec + sv.h->o_cols);
      auto emit = [&](uint32_t j, uint32_t* dst) {
        if (byp) {
          *dst = kBypassWord;
          return;
        }
        uint64_t wide = 0;
        const ColInfo& ci = cols[j];
        const uint32_t w = column_word(ci, rej, mut, CA.init, vw, CA.rec, &wide);
        *dst = w;
        if (KW_REASON(w) == 0 || KW_ARG(w) != kArgWide) return;
        if (KW_REASON(w) == KW_R_GROUP) {
          a.wide_groups[r * a.nwide + ci.wide] = wide;
        } else if (ci.kind == CK_PLAIN && ((rej >> ci.slot) & 1ull)) {  // entity index >= 65535
          const uint32_t at = atomicAdd(a.wide_count, 1u);
          if (at < a.wide_cap) {
            WideRec wr;
            wr.row_lo = (uint32_t)r;
            wr.row_hi = (uint32_t)(r >> 32);
            wr.policy = ci.policy;
            wr.value = va[ci.slot];
            a.wide_rec[at] = wr;
          }
        }
      };
      if (t.rows_mode) {
        const uint32_t rc = a.rowcol[r];
        if ((rc >> 16) == ck) emit(rc & 0xffffu, a.out + r);
      } else {
        for (uint32_t j = 0; j < CA.ncols; ++j) emit(j, a.out + r * a.npol + CA.col0 + j);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// NFA elements (kwdev.hpp DevNfa): patterns whose DFA exceeds the state budget. Before the tile
// kernel, one thread per entity runs every NFA element of its classifier chains (a Pike VM over the
// string, lists in the thread's scratch) and stores the element's class where the tile kernel's
// classification reads it: label values under their key's chain ([label][nlv]), image references
// under the registry / tag / normalised-image chains ([container][il.n()]). Rare (a pattern has to
// blow a DFA past kMaxDfaStates), so it is simple rather than fast.
// ------------------------------------------------------------------------------------------
constexpr int kNfaThreads = 256;

__global__ void __launch_bounds__(kNfaThreads) nfa_classify_kernel(EvalArgs a, const TileArgs* __restrict__ tp, NfaPass np) {
  const TileArgs& t = *tp;
  const uint64_t nthreads = (uint64_t)gridDim.x * kNfaThreads;
  const uint64_t gtid = (uint64_t)blockIdx.x * kNfaThreads + threadIdx.x;
  uint32_t* scratch = np.scratch + gtid * np.words_per_thread;
  uint8_t* subj = (uint8_t*)(scratch + np.nfa_words);
  for (uint32_t k = 0; k < np.nfa_words; ++k) scratch[k] = 0u;  // marks: generation 0 is never used
  uint32_t gen = 0;
  const uint8_t* blob = a.blob;
  const uint32_t NONE = 0xffffffffu;
  const uint64_t items = (np.do_lv ? np.nlabels : 0ull) + (np.do_img ? np.nctrs : 0ull);
  for (uint64_t q = gtid; q < items; q += nthreads) {
    if (np.do_lv && q < np.nlabels) {
      const uint64_t l = q;
      if (!t.kv_blob || !t.lit_blob[COL_LK]) continue;
      const uint32_t kb = t.s_off[S_LK][l], ke = t.s_off[S_LK][l + 1];
      const uint32_t k = lit_lookup<false>(blob + t.lit_blob[COL_LK], t.s_bytes[S_LK], kb, ke);
      if (!k) continue;
      const uint8_t* R = blob + t.kv_blob;
      const uint32_t kbase = ((const uint32_t*)R)[t.nlk + k];
      const uint32_t vb = t.s_off[S_LV][l], ve = t.s_off[S_LV][l + 1];
      uint32_t j = 0;
      for (uint32_t rel = ((const uint32_t*)R)[k]; rel; ++j) {
        const KvDfa& d = *(const KvDfa*)(R + rel);
        if (d.nfa) {
          const bool m = nfa_run(blob + d.trans_off, t.s_bytes[S_LV] + vb, ve - vb, scratch, &gen);
          np.lv[l * np.nlv + j] = (uint16_t)(kbase + d.cbase + (m ? 1u : 0u));
        }
        rel = d.next;
      }
      continue;
    }
    const uint64_t c = np.do_lv ? q - np.nlabels : q;
    if (!(a.ctr_flags[c] & KW_CTR_HAS_IMAGE)) continue;
    const uint8_t* bytes = t.s_bytes[S_IMG];
    const ImageRef r = parse_image(bytes, t.s_off[S_IMG][c], t.s_off[S_IMG][c + 1]);
    uint16_t* row = np.img + c * np.nim;
    auto put = [&](const uint8_t* src, uint32_t n, uint32_t at) {
      for (uint32_t x = 0; x < n; ++x) subj[at + x] = src[x];
      return at + n;
    };
    auto put_c = [&](const char* src, uint32_t at) {
      for (; *src; ++src) subj[at++] = (uint8_t)*src;
      return at;
    };
    auto run_chain = [&](Col col, uint32_t j, int part) {
      const uint32_t head = t.dfa_blob[col];
      for (uint32_t o = head; o; o = ((const DevDfa*)(blob + o))->next, ++j) {
        const DevDfa& d = *(const DevDfa*)(blob + o);
        if (d.kind != 1) continue;
        const uint16_t* acc = (const uint16_t*)(blob + d.acc_off);
        uint32_t n = 0;
        if (part == 0) {  // registry (implicit: docker.io)
          n = r.is_reg ? put(bytes + r.b, r.slash0 - r.b, 0) : put_c("docker.io", 0);
        } else if (part == 1) {  // effective tag (implicit: latest); a digest-only reference has none
          if (r.colon != NONE) n = put(bytes + r.colon + 1, r.name_end - r.colon - 1, 0);
          else if (r.at == NONE) n = put_c("latest", 0);
          else {
            row[j] = 0;
            continue;
          }
        } else {  // normalised reference: registry/[library/]path[:tag][@digest]
          n = r.is_reg ? put(bytes + r.b, r.slash0 - r.b, 0) : put_c("docker.io", 0);
          subj[n++] = '/';
          if (r.is_docker && !r.path_slash) n = put_c("library/", n);
          n = put(bytes + r.rest_b, r.path_end - r.rest_b, n);
          if (r.eff_tag) {
            subj[n++] = ':';
            n = r.colon != NONE ? put(bytes + r.colon + 1, r.name_end - r.colon - 1, n) : put_c("latest", n);
          }
          if (r.at != NONE) n = put(bytes + r.at, r.e - r.at, n);
        }
        row[j] = acc[nfa_run(blob + d.trans_off, subj, n, scratch, &gen) ? 1 : 0];
      }
      return j;
    };
    uint32_t j = t.lit_blob[COL_REG] ? 1u : 0u;
    j = run_chain(COL_REG, j, 0);
    j += t.lit_blob[COL_TAG] ? 1u : 0u;
    j = run_chain(COL_TAG, j, 1);
    run_chain(COL_IMG, j, 2);
  }
}

uint32_t nfa_threads(uint64_t items, uint64_t words_per_thread) {
  constexpr uint64_t kBudget = 256ull << 20;  // scratch bytes
  uint64_t n = std::min<uint64_t>(std::max<uint64_t>(items, 1), 256ull * 1024);
  n = std::min<uint64_t>(n, std::max<uint64_t>(kNfaThreads, kBudget / (4 * std::max<uint64_t>(words_per_thread, 1))));
  return (uint32_t)((n + kNfaThreads - 1) / kNfaThreads * kNfaThreads);
}

hipError_t launch_nfa_classify(const EvalArgs& a, const TileArgs* d_t, const NfaPass& np, uint32_t threads, hipStream_t s) {
  if (!np.do_lv && !np.do_img) return hipSuccess;
  hipLaunchKernelGGL(nfa_classify_kernel, dim3(threads / kNfaThreads), dim3(kNfaThreads), 0, s, a, d_t, np);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Wide policy groups: the members' verdict words of a separate pass -> each group's jump code per
// row (slots.hpp run_wide_prog), its value stack in this thread's scratch words and its causes in
// the per-row side data. A row the main pass answered with the bypass word keeps it.
// ------------------------------------------------------------------------------------------
constexpr int kWideThreads = 256;

__global__ void __launch_bounds__(kWideThreads) wide_groups_kernel(WideGroupPass w) {
  const uint64_t nthreads = (uint64_t)gridDim.x * kWideThreads;
  const uint64_t gtid = (uint64_t)blockIdx.x * kWideThreads + threadIdx.x;
  uint64_t* stack = w.stack + gtid * w.stack_words;
  const uint64_t pairs = w.nrows * w.ngroups;
  for (uint64_t q = gtid; q < pairs; q += nthreads) {
    const uint64_t r = q / w.ngroups;
    const WideGroupArgs& g = w.groups[q - r * w.ngroups];
    uint32_t* dst;
    if (w.rowcol) {
      if (w.rowcol[r] != g.col) continue;
      dst = w.out + r;
    } else {
      dst = w.out + r * w.npol + g.col;
    }
    if (*dst == kBypassWord) continue;
    uint64_t* cz = w.causes + r * w.cause_stride + g.cause_off;
    for (uint32_t k = 0; k < g.cause_words; ++k) cz[k] = 0;
    const uint32_t* mw = w.member_words + r * w.nmw;
    const uint32_t* midx = w.midx + g.midx_off;
    auto ok = [&](uint32_t s) {
      const uint32_t c = midx[s];
      uint32_t x;
      if (c & kSplitMember) {  // a split member: its word from its parts' words
        const WideGroupArgs& a = w.groups[w.ngroups + (c & ~kSplitMember)];
        const uint32_t* am = w.midx + a.midx_off;
        x = combine_parts(a, (const uint32_t*)(w.progs + a.prog_off), [&](uint32_t t) { return mw[am[t]]; });
      } else {
        x = mw[c];
      }
      return (x & KW_V_ALLOWED) && !(x & KW_V_MUTATED);
    };
    auto cause = [&](uint32_t s) { cz[s >> 6] |= 1ull << (s & 63u); };
    // a group of at most 15 members carries its causes in ARG, as column_word's forms do
    // (a group without members has no cause words: cz then points past its own range)
    auto rej = [&]() {
      const uint32_t c0 = g.cause_words ? (uint32_t)cz[0] : 0u;
      return g.nmem <= 15 ? (g.rejb & 0xffffu) | (c0 << 16) : g.rejb;
    };
    if (g.kind == 1) {  // script bytecode: true, false or an evaluation error
      const int v = run_script_prog(w.progs + g.prog_off, stack, ok, cause);
      *dst = v == 1 ? g.okw : v == 0 ? rej() : g.errw;
      continue;
    }
    if (g.kind >= 2) {  // a split plain policy: its parts' words
      *dst = combine_parts(g, (const uint32_t*)(w.progs + g.prog_off), [&](uint32_t s) { return mw[midx[s]]; });
      continue;
    }
    const bool v = run_wide_prog(w.progs + g.prog_off, g.prog_len, stack, ok, cause);
    *dst = v ? g.okw : rej();
  }
}

hipError_t launch_wide_groups(const WideGroupPass& w, uint32_t grid, hipStream_t s) {
  if (w.nrows == 0 || w.ngroups == 0) return hipSuccess;
  hipLaunchKernelGGL(wide_groups_kernel, dim3(grid), dim3(kWideThreads), 0, s, w);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------
namespace {
// hipFuncSetAttribute is per device: set once per device, thread-safe (std::call_once).
constexpr int kMaxDevices = 64;
std::once_flag g_attr_once[kMaxDevices];
hipError_t g_attr_err[kMaxDevices];

// The instantiation of a launch: LDS or global tables, phase clocks (diagnostics), image support
// (passes whose policies read no image reference run a kernel without that code: fewer registers,
// a tighter schedule for the rest).
template <bool LDST, uint32_t... Fs>
constexpr std::array<const void*, sizeof...(Fs)> tile_fns() {
  return {(const void*)evaluate_tiles_kernel<LDST, false, Fs>...};
}
const void* tile_fn(bool ldst, bool timing, uint32_t feat) {
  static const auto g = tile_fns<false, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15>();
  static const auto l = tile_fns<true, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15>();
  if (feat & kFeatNfa)  // the one instantiation with NFA elements: every family (timing runs it too)
    return ldst ? (const void*)evaluate_tiles_kernel<true, false, kFeatAll | kFeatNfa>
                : (const void*)evaluate_tiles_kernel<false, false, kFeatAll | kFeatNfa>;
  if ((feat & kFeatRng) && ldst && !timing && (feat & kFeatAll) == (kFeatLbl | kFeatCtr))
    return (const void*)evaluate_tiles_kernel<true, false, kFeatLbl | kFeatCtr | kFeatRng>;
  if (timing) {  // diagnostics: the C2 / C3 / C4 family sets with LDS tables (same registers as the product), else every family
    if (ldst && (feat & kFeatAll) == kFeatImg) return (const void*)evaluate_tiles_kernel<true, true, kFeatImg>;
    if (ldst && (feat & kFeatAll) == (kFeatImg | kFeatGrp)) return (const void*)evaluate_tiles_kernel<true, true, kFeatImg | kFeatGrp>;
    if (ldst && (feat & kFeatAll) == (kFeatLbl | kFeatCtr)) return (const void*)evaluate_tiles_kernel<true, true, kFeatLbl | kFeatCtr>;
    return ldst ? (const void*)evaluate_tiles_kernel<true, true, kFeatAll> : (const void*)evaluate_tiles_kernel<false, true, kFeatAll>;
  }
  return ldst ? l[feat & kFeatAll] : g[feat & kFeatAll];
}
uint32_t tile_feat(const TileArgs& t) { return t.feat & (kFeatAll | kFeatNfa | kFeatRng); }

hipError_t ensure_attrs() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::call_once(g_attr_once[dev], [dev] {
    // allow > 64 KB of dynamic LDS per workgroup (gfx950: 160 KB per CU)
    hipError_t e = hipSuccess;
    for (int k = 0; k < 70; ++k) {  // (LDS tables, timing, families; the two NFA instantiations; the scan one at k = 69)
      const uint32_t feat = k < 64 ? (uint32_t)(k >> 2) & kFeatAll : k < 68 ? (kFeatAll | kFeatNfa) : (kFeatLbl | kFeatCtr | kFeatRng);
      const hipError_t ek =
          hipFuncSetAttribute(tile_fn(k & 1, (k & 2) != 0, feat), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e == hipSuccess) e = ek;
    }
    g_attr_err[dev] = e;
  });
  return g_attr_err[dev];
}
}  // namespace

hipError_t launch_evaluate_tiles(const EvalArgs& a, const TileArgs& t, const TileArgs* d_t, const TileDesc* d_desc,
                                 uint32_t grid, hipStream_t s) {
  if (a.nrows == 0 || t.nchunk == 0 || a.ndesc == 0) return hipSuccess;
  if (hipError_t e = ensure_attrs(); e != hipSuccess) return e;
  // The grid is persistent (tiles strided by gridDim.x), so it must be co-resident: a workgroup
  // that only starts when another retires doubles the tail. Clamp the planner's grid to the
  // runtime's occupancy for this LDS size (queried once per device and LDS size, per thread).
  {
    thread_local int c_dev = -1, c_ncu = 0, c_occ = 0;
    thread_local uint64_t c_key = ~0ull;
    int dev = 0;
    const uint64_t key = ((uint64_t)t.lds_bytes << 8) | ((uint64_t)tile_feat(t) << 2) | (a.phase ? 2u : 0u) | (t.lds_tables ? 1u : 0u);
    if (hipGetDevice(&dev) == hipSuccess && (dev != c_dev || key != c_key)) {
      int ncu = 0, occ = 0;
      const void* fn = tile_fn(t.lds_tables != 0, a.phase != nullptr, tile_feat(t));
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kSlotThreads, t.lds_bytes) != hipSuccess)
        ncu = occ = 0;
      c_dev = dev;
      c_key = key;
      c_ncu = ncu;
      c_occ = occ;
    }
    // (the API's LDS bound is floor(160 KiB / bytes); the CU allocates 1280-byte granules)
    c_occ = std::min<int>(c_occ, (int)lds_workgroups_per_cu(t.lds_bytes));
    if (c_occ > 0 && c_ncu > 0) grid = std::max<uint32_t>(1u, std::min<uint32_t>(grid, (uint32_t)(c_occ * c_ncu)));
    if (t.debug & 256u)
      fprintf(stderr, "[kw tile] launch grid=%u occupancy=%d wg/cu x %d CUs lds=%u\n", grid, c_occ, c_ncu, t.lds_bytes);
  }
  using TileFn = void (*)(EvalArgs, const TileArgs*, const TileDesc*);
  const TileFn fn = (TileFn)tile_fn(t.lds_tables != 0, a.phase != nullptr, tile_feat(t));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kSlotThreads), t.lds_bytes, s, a, d_t, d_desc);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) scatter_kernel(ScatterArgs a) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x, nt = (uint64_t)gridDim.x * 256u;
  for (uint32_t k = 0; k < a.nseg; ++k) {
    const ScatterSeg g = a.seg[k];
    uint8_t* d = a.dst + g.dst_off;
    const uint8_t* s = a.src + g.src_off;
    const uint64_t head = std::min<uint64_t>(g.bytes, (16u - ((uintptr_t)d & 15u)) & 15u);
    const uint64_t words = (g.bytes - head) / 16u, tail = g.bytes - head - words * 16u;
    if (tid < head) d[tid] = s[tid];
    const u32x4* sw = (const u32x4*)(s + head);
    u32x4* dw = (u32x4*)(d + head);
    for (uint64_t i = tid; i < words; i += nt) __builtin_nontemporal_store(__builtin_nontemporal_load(sw + i), dw + i);
    if (tid < tail) d[head + words * 16u + tid] = s[head + words * 16u + tid];
  }
}

hipError_t launch_scatter(const ScatterArgs& a, hipStream_t s) {
  uint64_t bytes = 0;
  for (uint32_t k = 0; k < a.nseg; ++k) bytes += a.seg[k].bytes;
  if (!bytes) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, bytes / (256u * 64u)));
  hipLaunchKernelGGL(scatter_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_overflow(const EvalArgs& a, const TileArgs* d_t, const uint32_t* d_overflow, uint32_t n_overflow,
                           hipStream_t s) {
  if (n_overflow == 0 || a.nrows == 0) return hipSuccess;
  hipLaunchKernelGGL(overflow_classify_kernel, dim3(std::min<uint32_t>(n_overflow, 1024)), dim3(kOverflowThreads), 0, s,
                     a, d_t, d_overflow);
  const uint32_t blocks = std::min<uint32_t>((n_overflow + kOverflowThreads - 1) / kOverflowThreads, 1024);
  hipLaunchKernelGGL(overflow_eval_kernel, dim3(blocks), dim3(kOverflowThreads), 0, s, a, d_t, d_overflow);
  return hipGetLastError();
}

}  // namespace kw
