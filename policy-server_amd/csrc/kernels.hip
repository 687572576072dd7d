// kernels.hip — the MI355X (gfx950) hot path of EvaluationEnvironment::validate for the
// declarative policy class (src/evaluation/evaluation_environment.rs:546-594) fused with the
// service::evaluate epilogue (src/api/service.rs:40-116, 160-208).
//
// Kernels:
//  evaluate_slots_kernel — the all-pairs hot path (kw_validate_batch). Persistent 256-thread
//                     workgroups, several per CU, each owning a 64-request tile at a time: stage the
//                     tile's columns into LDS, classify every string there (literal perfect hash,
//                     per-key value DFA, image DFA chains), walk each request's entities once with
//                     the bit-parallel slot tables (slots.hpp: one lane per request, one wave per
//                     family group), then write the verdict rows with coalesced 16-B stores.
//  classify_kernel  — two-kernel form for automata too large for LDS: one lane per string, masks
//                     to HBM; the slot kernel then stages the masks instead of the strings.
//  overflow_kernel  — tiles whose entity counts exceed the LDS capacities, from global memory.
//  evaluate_rows_kernel — micro-batch form (kw_validate_rows): one lane per (row, its policy).
// The verdict word (include/kwgpu.h) carries the vanilla response and the service-level result.
// Integer / byte work only: no MFMA. Bound: HBM streaming of request bytes in and verdict words
// out.
#include <hip/hip_runtime.h>

#include <cstddef>

#include "../../include/kwgpu.h"
#include "kernels.hpp"

namespace kw {

// ------------------------------------------------------------------------------------------
// DFA views
// ------------------------------------------------------------------------------------------
struct DfaView {
  const uint8_t* cls;     // 256
  const uint16_t* trans;  // [state][ncls]
  const uint64_t* acc;    // [state]
  uint32_t ncls, start;
  bool valid;
};

__device__ inline DfaView make_view(const uint8_t* base, const uint8_t* blob, uint32_t dfa_off) {
  // base points at the staged copy of the DevDfa record at blob offset dfa_off (LDS or the blob)
  DfaView v;
  const DevDfa* h = (const DevDfa*)base;
  v.cls = h->cls;
  v.ncls = h->ncls;
  v.start = h->start;
  v.trans = (const uint16_t*)(base + (h->trans_off - dfa_off));
  v.acc = (const uint64_t*)(base + (h->acc_off - dfa_off));
  v.valid = true;
  (void)blob;
  return v;
}

__device__ inline uint32_t step(const DfaView& d, uint32_t st, uint32_t byte) {
  return d.trans[st * d.ncls + d.cls[byte]];
}

// Walk bytes [b, e) of a global pool with 4-byte aligned loads (pools carry a 16 B zero tail).
__device__ inline uint32_t feed(const DfaView& d, uint32_t st, const uint8_t* __restrict__ bytes, uint32_t b,
                                uint32_t e) {
  uint32_t p = b;
  while (p < e && st != 0) {
    uint32_t w = *(const uint32_t*)(bytes + (p & ~3u));
    uint32_t k = p & 3u;
    uint32_t lim = min(4u - k, e - p);
    w >>= 8u * k;
    for (uint32_t j = 0; j < lim; ++j) {
      st = step(d, st, w & 0xffu);
      w >>= 8;
    }
    p += lim;
  }
  return st;
}

// Literal fragments of image normalisation; constexpr + unrolled loops turn them into immediates.
constexpr char kDockerIo[] = "docker.io";
constexpr char kLibrary[] = "library/";
constexpr char kLatest[] = "latest";
constexpr char kLocalhost[] = "localhost";

template <int N>
__device__ inline uint32_t feed_const(const DfaView& d, uint32_t st, const char (&s)[N]) {
#pragma unroll
  for (int i = 0; i < N - 1; ++i) st = step(d, st, (uint8_t)s[i]);  // state 0 is absorbing
  return st;
}

__device__ inline uint32_t byte_at(const uint8_t* __restrict__ bytes, uint32_t p) { return bytes[p]; }

template <int N>
__device__ inline bool equals_const(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e, const char (&s)[N]) {
  if ((int)(e - b) != N - 1) return false;
#pragma unroll
  for (int i = 0; i < N - 1; ++i)
    if (byte_at(bytes, b + (uint32_t)i) != (uint8_t)s[i]) return false;
  return true;
}

// Literal-column lookup (DevLit, kwdev.hpp): hash the string's canonical dwords, probe one slot,
// verify against the pattern's words. `rec` and `bytes` may be LDS or global; dwords are read at
// 4-aligned addresses and realigned with v_alignbyte (reads may touch <= 7 bytes past the string,
// inside the pool's zero pad or the staged tile's slack).
__device__ inline uint32_t lit_word(const uint32_t* base, uint32_t i, uint32_t sh, uint32_t len) {
  uint32_t w = __builtin_amdgcn_alignbyte(base[i + 1], base[i], sh);
  const uint32_t rem = len - 4u * i;
  return rem >= 4u ? w : (w & ((1u << (8u * rem)) - 1u));
}
__device__ inline uint64_t lit_lookup(const uint8_t* rec, const uint8_t* bytes, uint32_t b, uint32_t e) {
  // LDS only: the first 32 bytes of the string and of the candidate pattern are read in one batch
  // each (up to 36 bytes past the string: staged slack / other LDS; masked off by len)
  const DevLit* L = (const DevLit*)rec;
  const uint32_t len = e - b, sh = b & 3u, nw = (len + 3u) >> 2;
  const uint32_t* base = (const uint32_t*)(bytes + (b & ~3u));
  uint32_t raw[9], w[8];
#pragma unroll
  for (int i = 0; i < 9; ++i) raw[i] = base[i];
  uint32_t h = lit_init(L->seed, len);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t x = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
    const uint32_t rem = len - 4u * (uint32_t)i;  // >= 4: whole dword
    w[i] = rem >= 4u ? x : (x & ((1u << (8u * rem)) - 1u));
    if ((uint32_t)i < nw) h = lit_mix(h, w[i]);
  }
  for (uint32_t i = 8; i < nw; ++i) h = lit_mix(h, lit_word(base, i, sh, len));
  h = lit_final(h);
  const uint32_t s = ((const uint32_t*)(rec + L->slot_off))[h & (L->nslots - 1u)];
  if (!s || lit_slot_len(s) != len) return 0ull;
  const uint32_t* pw = (const uint32_t*)(rec + L->word_off) + lit_slot_word(s);
  uint32_t pv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) pv[i] = pw[i];  // zero tail of the words section covers short patterns
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq = eq && ((uint32_t)i >= nw || w[i] == pv[i]);
  for (uint32_t i = 8; i < nw && eq; ++i) eq = lit_word(base, i, sh, len) == pw[i];
  return eq ? 1ull << (lit_slot_pat(s) - 1u) : 0ull;
}

// A column's DFA chain, staged contiguously (LDS, or the blob itself): element at blob offset
// `off` lives at base + (off - head).
struct Chain {
  const uint8_t* base;
  uint32_t head;
};

__device__ inline DfaView chain_view(const Chain& c, uint32_t off) { return make_view(c.base + (off - c.head), nullptr, off); }
__device__ inline uint32_t chain_next(const Chain& c, uint32_t off) {
  return ((const DevDfa*)(c.base + (off - c.head)))->next;
}

// Parsed image reference (oracle: orc_image_parts).
struct ImageRef {
  uint32_t b, e, at, slash0, rest_b, colon, path_end, name_end;
  bool is_reg, path_slash, is_docker, eff_tag;
};

__device__ ImageRef parse_image(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t at = NONE, slash0 = NONE, slash1 = NONE, last_colon = NONE;
  bool dotcolon = false;
  uint32_t p = b;
  bool stop = false;
  while (p < e && !stop) {
    uint32_t w = *(const uint32_t*)(bytes + (p & ~3u));
    uint32_t k = p & 3u;
    uint32_t lim = min(4u - k, e - p);
    w >>= 8u * k;
    for (uint32_t j = 0; j < lim; ++j) {
      uint32_t c = w & 0xffu;
      w >>= 8;
      uint32_t q = p + j;
      if (c == '@') {
        at = q;
        stop = true;
        break;
      }
      if (c == '/') {
        if (slash0 == NONE) slash0 = q;
        else if (slash1 == NONE) slash1 = q;
      } else if (c == ':') {
        last_colon = q;
        if (slash0 == NONE) dotcolon = true;
      } else if (c == '.') {
        if (slash0 == NONE) dotcolon = true;
      }
    }
    p += lim;
  }
  ImageRef r;
  r.b = b;
  r.e = e;
  r.at = at;
  r.slash0 = slash0;
  r.name_end = at != NONE ? at : e;
  r.is_reg = slash0 != NONE && (dotcolon || equals_const(bytes, b, slash0, kLocalhost));
  r.rest_b = r.is_reg ? slash0 + 1 : b;
  r.colon = (last_colon != NONE && last_colon >= r.rest_b) ? last_colon : NONE;
  r.path_end = r.colon != NONE ? r.colon : r.name_end;
  uint32_t first_slash_rest = r.is_reg ? slash1 : slash0;
  r.path_slash = first_slash_rest != NONE && first_slash_rest < r.path_end;
  r.is_docker = !r.is_reg || equals_const(bytes, b, slash0, kDockerIo);
  r.eff_tag = r.colon != NONE || at == NONE;
  return r;
}

// Registry (k=0), effective tag (k=1) or normalised image (k=2) through one DFA.
__device__ uint64_t image_part(int k, const DfaView& d, const uint8_t* __restrict__ bytes, const ImageRef& r) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t st = d.start;
  if (k == 0) {
    st = r.is_reg ? feed(d, st, bytes, r.b, r.slash0) : feed_const(d, st, kDockerIo);
  } else if (k == 1) {
    if (r.colon != NONE) st = feed(d, st, bytes, r.colon + 1, r.name_end);
    else if (r.at == NONE) st = feed_const(d, st, kLatest);
    else return 0ull;  // digest only: no tag
  } else {
    st = r.is_reg ? feed(d, st, bytes, r.b, r.slash0) : feed_const(d, st, kDockerIo);
    if (st) st = step(d, st, '/');
    if (r.is_docker && !r.path_slash) st = feed_const(d, st, kLibrary);
    st = feed(d, st, bytes, r.rest_b, r.path_end);
    if (r.eff_tag) {
      if (st) st = step(d, st, ':');
      st = r.colon != NONE ? feed(d, st, bytes, r.colon + 1, r.name_end) : feed_const(d, st, kLatest);
    }
    if (r.at != NONE) st = feed(d, st, bytes, r.at, r.e);
  }
  return d.acc[st];
}

template <bool USE_LDS>
__global__ void __launch_bounds__(kClassifyThreads) classify_kernel(const uint8_t* __restrict__ blob, ClassifyJobs jobs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t bid = blockIdx.x;
  int jx = 0;
  for (int k = 1; k < jobs.n; ++k)
    if (bid >= jobs.j[k].block_begin) jx = k;
  const ClassifyJob& J = jobs.j[jx];

  Chain ch[3];
  if (USE_LDS) {
    // stage this job's DFA chains into LDS (16 B per lane per step, coalesced)
    for (int k = 0; k < 3; ++k) {
      if (!J.dfa[k]) continue;
      const DevDfa* h = (const DevDfa*)(blob + J.dfa[k]);
      uint32_t nbytes = h->chain_bytes;
      const uint4* src = (const uint4*)(blob + J.dfa[k]);
      uint4* dst = (uint4*)(lds + J.lds_pos[k]);
      for (uint32_t i = threadIdx.x; i < nbytes / 16; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();
  }
  for (int k = 0; k < 3; ++k) {
    ch[k].head = J.dfa[k];
    ch[k].base = USE_LDS ? lds + J.lds_pos[k] : blob + J.dfa[k];
  }

  const uint32_t lb = bid - J.block_begin;
  const uint32_t stride = J.nblocks * kClassifyThreads;
  const uint32_t* __restrict__ off = J.off;
  const uint8_t* __restrict__ bytes = J.bytes;
  for (uint32_t i = lb * kClassifyThreads + threadIdx.x; i < J.n; i += stride) {
    const uint32_t b = off[i], e = off[i + 1];
    if (J.mode == 0) {
      uint64_t m = 0;
      for (uint32_t o = ch[0].head; o; o = chain_next(ch[0], o)) {
        DfaView v = chain_view(ch[0], o);
        m |= v.acc[feed(v, v.start, bytes, b, e)];
      }
      J.out[0][i] = m;
    } else {
      const ImageRef r = parse_image(bytes, b, e);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (!ch[k].head) continue;
        uint64_t m = 0;
        for (uint32_t o = ch[k].head; o; o = chain_next(ch[k], o)) m |= image_part(k, chain_view(ch[k], o), bytes, r);
        J.out[k][i] = m;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Policy evaluation
// ------------------------------------------------------------------------------------------
// Policy fields are read as whole dwords: with wave-uniform policy indices and __restrict__ kernel
// parameters the loads become scalar (s_load, K$), the bytes are extracted with SALU ops.
__device__ inline uint32_t pword(const DevPolicy& P, uint32_t w) { return ((const uint32_t*)&P)[w]; }
__device__ inline uint32_t pbyte(const DevPolicy& P, uint32_t off) { return (pword(P, off >> 2) >> (8u * (off & 3u))) & 0xffu; }
// byte offsets within DevPolicy (kwdev.hpp)
constexpr uint32_t PB_FAMILY = 0, PB_MODE = 1, PB_A2M = 2, PB_FLAGS = 3, PB_NL = 4, PB_NMAND = 10, PB_NCONSTR = 11, PB_IDX = 80;
static_assert(offsetof(DevPolicy, nl) == PB_NL && offsetof(DevPolicy, n_mand) == PB_NMAND &&
                  offsetof(DevPolicy, n_constr) == PB_NCONSTR && offsetof(DevPolicy, idx) == PB_IDX,
              "DevPolicy byte offsets");

struct FamOut {
  uint32_t reason, arg;
  bool mutated;
};

// Column accessors of the overflow and row kernels: the HBM arrays, absolute indices.
struct GlobalSrc {
  const EvalArgs* a;
  __device__ uint8_t rf(uint64_t r) const { return a->req_flags[r]; }
  __device__ uint32_t coff(uint64_t r) const { return a->ctr_off[r]; }
  __device__ uint32_t loff(uint64_t r) const { return a->lbl_off[r]; }
  __device__ uint8_t cflags(uint32_t c) const { return a->ctr_flags[c]; }
  __device__ uint32_t cadd(uint32_t c) const { return a->capadd_off[c]; }
  __device__ uint32_t cdrop(uint32_t c) const { return a->capdrop_off[c]; }
  template <int K>
  __device__ uint64_t m(uint64_t i) const { return a->m[K] ? a->m[K][i] : 0ull; }
};

template <class S>
__device__ FamOut eval_family(const S& src, const DevPolicy& P, uint64_t r) {
  FamOut o{0, 0, false};
  const uint8_t rf = src.rf(r);
  const uint32_t cb = src.coff(r), ce = src.coff(r + 1);
  switch (pbyte(P, PB_FAMILY)) {
    case FAM_PRIVILEGED: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        uint8_t f = src.cflags(c);
        bool skip = ((pbyte(P, PB_FLAGS) & PF_SKIP_INIT) && (f & KW_CTR_INIT)) || ((pbyte(P, PB_FLAGS) & PF_SKIP_EPHEMERAL) && (f & KW_CTR_EPHEMERAL));
        if (!skip && (f & KW_CTR_PRIVILEGED)) {
          o.reason = KW_R_PRIVILEGED;
          o.arg = pack1(c - cb);
          break;
        }
      }
      break;
    }
    case FAM_NAMESPACE: {
      bool ok = (rf & KW_REQ_HAS_NAMESPACE) && pbyte(P, PB_NL + (0)) && (src.template m<M_NS>(r) & P.m[0]);
      if (!ok) o.reason = KW_R_NAMESPACE;
      break;
    }
    case FAM_TRUSTED_REPOS: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        if (!(src.cflags(c) & KW_CTR_HAS_IMAGE)) continue;
        uint64_t reg = src.template m<M_REG>(c), tag = src.template m<M_TAG>(c), img = src.template m<M_IMG>(c);
        uint32_t why = 0;
        if (pbyte(P, PB_NL + (0)) && !(reg & P.m[0])) why = KW_R_REG_NOT_ALLOWED;
        else if (pbyte(P, PB_NL + (1)) && (reg & P.m[1])) why = KW_R_REG_REJECTED;
        else if (pbyte(P, PB_NL + (2)) && (tag & P.m[2])) why = KW_R_TAG_REJECTED;
        else if (pbyte(P, PB_NL + (3)) && !(img & P.m[3])) why = KW_R_IMG_NOT_ALLOWED;
        else if (pbyte(P, PB_NL + (4)) && (img & P.m[4])) why = KW_R_IMG_REJECTED;
        if (why) {
          o.reason = why;
          o.arg = pack1(c - cb);
          break;
        }
      }
      break;
    }
    case FAM_CAPABILITIES: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        const uint32_t kb = src.cadd(c), ke = src.cadd(c + 1);
        uint64_t addm = 0, dropm = 0;
        for (uint32_t k = kb; k < ke; ++k) {
          uint64_t mk = src.template m<M_CAPADD>(k);
          addm |= mk;
          if (!(pbyte(P, PB_FLAGS) & PF_ALLOW_ALL) && !(mk & P.m[0])) {
            o.reason = KW_R_CAP_NOT_ALLOWED;
            o.arg = pack2(c - cb, k - kb);
            break;
          }
        }
        if (o.reason) break;
        for (uint32_t k = src.cdrop(c); k < src.cdrop(c + 1); ++k) dropm |= src.template m<M_CAPDROP>(k);
        if (!(dropm & P.m[3]) && (P.m[1] & ~dropm)) o.mutated = true;
        if (P.m[2] & ~(addm | dropm)) o.mutated = true;
      }
      if (o.reason) o.mutated = false;
      break;
    }
    case FAM_APPARMOR: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        if ((src.cflags(c) & KW_CTR_HAS_APPARMOR) && !(src.template m<M_AA>(c) & P.m[0])) {
          o.reason = KW_R_APPARMOR;
          o.arg = pack1(c - cb);
          break;
        }
      }
      break;
    }
    case FAM_LABELS: {
      const uint32_t lb = src.loff(r), le = src.loff(r + 1);
      uint64_t present = 0;
      for (uint32_t l = lb; l < le && !o.reason; ++l) {
        uint64_t km = src.template m<M_LK>(l);
        present |= km;
        if (km & P.m[0]) {
          o.reason = KW_R_LABEL_DENIED;
          o.arg = pack1(l - lb);
          break;
        }
        if (km) {
          const uint64_t vm = src.template m<M_LV>(l);
          for (uint32_t i = 0; i < pbyte(P, PB_NCONSTR); ++i) {
            if (((km >> pbyte(P, PB_IDX + (16 + i))) & 1ull) && !((vm >> pbyte(P, PB_IDX + (32 + i))) & 1ull)) {
              o.reason = KW_R_LABEL_CONSTRAINT;
              o.arg = pack2(l - lb, i);
              break;
            }
          }
        }
      }
      if (o.reason) break;
      for (uint32_t i = 0; i < pbyte(P, PB_NMAND); ++i)
        if (!((present >> pbyte(P, PB_IDX + (i))) & 1ull)) {
          o.reason = KW_R_LABEL_MANDATORY;
          o.arg = i;
          break;
        }
      break;
    }
    default: break;
  }
  return o;
}

// EvaluationEnvironment::validate + service::evaluate constraints for one (request, policy).
template <class S>
__device__ uint32_t verdict(const S& src, const EvalArgs& a, const DevHeader& H, const DevPolicy* __restrict__ pols,
                            const DevPolicy& P, uint64_t r, uint16_t* gstk, uint32_t gstride) {
  const uint8_t rf = src.rf(r);
  // namespace bypass (service.rs:40-71), AdmissionRequest only
  if (H.bypass_bit >= 0 && !(rf & KW_REQ_RAW) && (rf & KW_REQ_HAS_NAMESPACE) &&
      ((src.template m<M_NS>(r) >> H.bypass_bit) & 1ull))
    return KW_V_ALLOWED | KW_F_ALLOWED | KW_BYPASS;
  // PolicyInitialization -> reject 500 before any constraint (service.rs:78-91)
  if (pbyte(P, PB_FLAGS) & PF_INIT_ERROR) return ((uint32_t)KW_FST_INIT_ERROR << KW_F_STATUS_SHIFT) | ((uint32_t)KW_R_INIT_ERROR << 8);
  uint32_t reason = 0, arg = 0;
  bool mutated = false;
  if (pbyte(P, PB_FAMILY) == FAM_GROUP) {
    if (pbyte(P, PB_FLAGS) & PF_EXPR_ERROR) {
      reason = KW_R_GROUP_EXPR;
    } else {
      const int32_t* mem = (const int32_t*)(a.blob + H.member_off) + P.member_off;
      uint32_t ok = 0;
      for (uint32_t s = 0; s < P.nmembers; ++s) {
        const DevPolicy& Q = pols[mem[s]];
        if (pbyte(Q, PB_FLAGS) & PF_INIT_ERROR) continue;
        FamOut fo = eval_family(src, Q, r);
        if (fo.reason == 0 && !fo.mutated) ok |= 1u << s;
      }
      uint32_t causes;
      if (!run_group_prog(a.blob + H.prog_off + P.prog_off, P.prog_len, ok, gstk, gstride, &causes)) {
        reason = KW_R_GROUP;
        arg = causes;
      }
    }
  } else {
    FamOut fo = eval_family(src, P, r);
    reason = fo.reason;
    arg = fo.arg;
    mutated = fo.mutated;
  }
  return finish_word(pbyte(P, PB_MODE), pbyte(P, PB_A2M), a.origin, reason, arg, mutated);
}

// Micro-batch form (kw_validate_rows): one lane per row, each row with its own policy.
__global__ void __launch_bounds__(kEvalThreads) evaluate_rows_kernel(EvalArgs a) {
  __shared__ uint16_t gstk[kMaxGroupStack * kEvalThreads];
  const DevHeader H = *(const DevHeader*)a.blob;
  const DevPolicy* __restrict__ pols = (const DevPolicy*)(a.blob + H.policy_off);
  GlobalSrc src{&a};
  const uint64_t stride = (uint64_t)gridDim.x * kEvalThreads;
  for (uint64_t r = (uint64_t)blockIdx.x * kEvalThreads + threadIdx.x; r < a.nrows; r += stride) {
    const DevPolicy& P = pols[a.row_policy[r]];
    a.out[r] = verdict(src, a, H, pols, P, r, gstk + threadIdx.x, kEvalThreads);
  }
}

// ------------------------------------------------------------------------------------------
// All-pairs slot kernel (evaluate_slots_kernel). A workgroup owns a tile of 64 consecutive
// requests at a time (persistent grid, several workgroups per CU so one tile's staging latency hides
// under another's walk). Per tile:
//  P0 stage the tile's request headers, container offsets and string bytes into LDS (coalesced
//     16-B loads; byte ranges come from the host-built TileDesc, so there is no dependent
//     global-load chain);
//  P1 classify every staged string from LDS-resident tables (literal perfect hash, per-key label
//     value DFA, image DFA chains);
//  P2 walk each request's entities once with the slot tables (slots.hpp), lane = request, one wave
//     per family group;
//  P3 write the verdict rows (ABI layout, row-major) with coalesced 16-B stores.
// A tile whose entity counts exceed the LDS capacities is left to overflow_kernel.
// ------------------------------------------------------------------------------------------
template <int K>
__device__ inline uint64_t classify_one(const Chain& ch, const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e) {
  uint64_t m = 0;
  for (uint32_t o = ch.head; o; o = chain_next(ch, o)) {
    DfaView v = chain_view(ch, o);
    m |= v.acc[feed(v, v.start, bytes, b, e)];
  }
  return m;
}

__device__ inline void classify_image_all(const Chain cr, const Chain ct, const Chain ci, const uint8_t* __restrict__ bytes,
                                          uint32_t b, uint32_t e, uint64_t* mr, uint64_t* mt, uint64_t* mi) {
  const ImageRef r = parse_image(bytes, b, e);
  uint64_t m0 = 0, m1 = 0, m2 = 0;
  for (uint32_t o = cr.head; o; o = chain_next(cr, o)) m0 |= image_part(0, chain_view(cr, o), bytes, r);
  for (uint32_t o = ct.head; o; o = chain_next(ct, o)) m1 |= image_part(1, chain_view(ct, o), bytes, r);
  for (uint32_t o = ci.head; o; o = chain_next(ci, o)) m2 |= image_part(2, chain_view(ci, o), bytes, r);
  *mr = m0;
  *mt = m1;
  *mi = m2;
}

// Pointers read from TileArgs are generic to the compiler; these casts make their loads global_load
// (not flat) in the staging loops.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <class T>
__device__ inline const __attribute__((address_space(1))) T* gp(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}

// First global entity index and entity count of mask m's string column within a tile.
__device__ inline uint32_t tile_g0(int m, uint32_t r0, uint32_t cb, uint32_t kab, uint32_t kdb, uint32_t lb) {
  return m == M_NS ? r0 : m == M_CAPADD ? kab : m == M_CAPDROP ? kdb : (m == M_LK || m == M_LV) ? lb : cb;
}
__device__ inline uint32_t tile_n(int m, uint32_t nr, uint32_t nc, uint32_t nka, uint32_t nkd, uint32_t nl) {
  return m == M_NS ? nr : m == M_CAPADD ? nka : m == M_CAPDROP ? nkd : (m == M_LK || m == M_LV) ? nl : nc;
}

// Literal pattern index of a one-bit mask (0xff: no pattern).
__device__ inline uint8_t lit_index(uint64_t r) { return r ? (uint8_t)__builtin_ctzll(r) : (uint8_t)0xffu; }

// A label value against the value regexes constrained on its key (label-key mask km): the key's
// per-key DFA chain, else the whole label-value column chain.
__device__ inline uint64_t classify_value(const TileArgs& t, const uint8_t* lds, uint64_t km, const uint8_t* bytes,
                                          uint32_t b, uint32_t e) {
  uint64_t vm = 0;
  if (t.kv_lds) {
    const uint8_t* R = lds + t.kv_lds;
    for (uint32_t rel = ((const uint16_t*)R)[__builtin_ctzll(km)]; rel;) {
      const KvDfa d = *(const KvDfa*)(R + rel);  // one ds_read_b128
      uint32_t st = d.start;
      // 8-byte windows: the window's dwords, then its 8 byte classes, load as two batches; only the
      // transitions form a dependent chain (bytes past the string read the staged slack, unused)
      for (uint32_t p = b; p < e && st != 0; p += 8u) {
        const uint32_t* q = (const uint32_t*)(bytes + (p & ~3u));
        const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], sh = p & 3u;
        const uint32_t x0 = __builtin_amdgcn_alignbyte(q1, q0, sh), x1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t by = ((j < 4 ? x0 : x1) >> (8 * (j & 3))) & 0xffu;
          c[j] = (by < 128u || d.wide) ? R[d.cls_off + by] : d.hi;
        }
        const uint32_t lim = min(8u, e - p);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((uint32_t)j < lim) st = R[d.trans_off + st * d.ncls + c[j]];
      }
      vm |= ((const uint64_t*)(R + d.accv_off))[R[d.acc_off + st]];
      rel = d.next;
    }
  } else {
    Chain c;
    c.head = t.dfa_head[M_LV];
    c.base = lds + t.dfa_lds[M_LV];
    for (uint32_t o = c.head; o; o = chain_next(c, o)) {
      const DfaView v = chain_view(c, o);
      vm |= v.acc[feed(v, v.start, bytes, b, e)];
    }
  }
  return vm;
}

__device__ inline uint32_t rup64(uint32_t n) { return (n + 63u) & ~63u; }
__device__ inline uint64_t idx_mask(uint32_t v) { return v < 64u ? 1ull << v : 0ull; }

// Trusted-repos reasons of staged container i, in precedence order (registry not allowed, registry
// rejected, tag rejected, image not allowed, image rejected; oracle fam_trusted).
__device__ inline void trs_whys(const SlotView& sv, const uint8_t* lds, const TileArgs& t, uint32_t i, uint64_t why[5]) {
  const SlotHdr& h = *sv.h;
  const uint64_t reg = t.o_m[M_REG] ? ((const uint64_t*)(lds + t.o_m[M_REG]))[i] : 0ull;
  const uint64_t tag = t.o_m[M_TAG] ? ((const uint64_t*)(lds + t.o_m[M_TAG]))[i] : 0ull;
  const uint64_t img = t.o_m[M_IMG] ? ((const uint64_t*)(lds + t.o_m[M_IMG]))[i] : 0ull;
  why[0] = h.has_ra & ~tab_or(sv.tab(ST_RA), reg);
  why[1] = tab_or(sv.tab(ST_RR), reg);
  why[2] = tab_or(sv.tab(ST_TR), tag);
  why[3] = h.has_ia & ~tab_or(sv.tab(ST_IA), img);
  why[4] = tab_or(sv.tab(ST_IR), img);
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

template <bool FUSED>
__global__ void __launch_bounds__(kSlotThreads)
    evaluate_slots_kernel(EvalArgs a, const TileArgs* __restrict__ tp, const TileDesc* __restrict__ desc,
                          const uint8_t* __restrict__ blob, uint32_t* __restrict__ out) {
  // TileArgs lives in device memory: its fields are scalar-loaded where used instead of all being
  // hoisted from the kernarg segment into SGPRs at entry.
  const TileArgs& t = *tp;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const DevHeader H = *(const DevHeader*)blob;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- once per workgroup: this chunk's slot plan and (FUSED) the column tables
  {
    const auto* src = gp((const u32x4*)t.slot_plan);
    u32x4* dst = (u32x4*)(lds + t.o_slot);
    for (uint32_t i = tid; i < t.slot_bytes / 16; i += kSlotThreads) dst[i] = src[i];
  }
  Chain ch[NMASK];
  if (FUSED) {
    for (uint32_t s = 0; s < t.nstage; ++s) {
      const auto* src = gp((const u32x4*)(blob + t.stage_blob[s]));
      u32x4* dst = (u32x4*)(lds + t.stage_lds[s]);
      for (uint32_t i = tid; i < t.stage_bytes[s] / 16; i += kSlotThreads) dst[i] = src[i];
    }
#pragma unroll
    for (int k = 0; k < (int)NMASK; ++k) {
      ch[k].head = t.dfa_head[k];
      ch[k].base = lds + t.dfa_lds[k];
    }
  }
  __syncthreads();
  SlotView sv;
  sv.h = (const SlotHdr*)(lds + t.o_slot);
  sv.base = lds + t.o_slot;
  // the column records as four u32 arrays (kind | slot << 8, okw, mutw, rejb; slotplan.cpp emit):
  // P3 items read the words of 4 consecutive columns with one conflict-free ds_read_b128 per array
  const uint32_t* cs = (const uint32_t*)(sv.base + sv.h->o_csoa);
  const uint32_t cs_n = (t.ncols + 3u) & ~3u;

  uint8_t* l_rf = lds + t.o_rf;
  uint32_t* l_coff = (uint32_t*)(lds + t.o_coff);
  uint32_t* l_loff = (uint32_t*)(lds + t.o_loff);
  uint8_t* l_cflags = lds + t.o_cflags;
  uint32_t* l_cadd = (uint32_t*)(lds + t.o_cadd);
  uint32_t* l_cdrop = (uint32_t*)(lds + t.o_cdrop);
  uint64_t* l_rej = (uint64_t*)(lds + t.o_rej);
  uint64_t* l_mut = (uint64_t*)(lds + t.o_mut);
  uint8_t* l_byp = lds + t.o_byp;
  uint32_t* l_sa = (uint32_t*)(lds + t.o_sa);
  uint64_t* l_vadd = (uint64_t*)(lds + t.o_vadd);
  uint64_t* l_vl = (uint64_t*)(lds + t.o_vl);
  uint32_t* l_vw = (uint32_t*)(lds + t.o_vw);
  uint16_t* gstk = t.o_gstk ? (uint16_t*)(lds + t.o_gstk) : nullptr;
  uint64_t* l_vc = (uint64_t*)(lds + t.o_vc);  // V_c per staged container
  uint8_t* own_c = lds + t.o_own_c;            // tile-local request of each staged container / label
  uint8_t* own_l = lds + t.o_own_l;

  const uint32_t npol = a.npol;
  // Tile schedule. Static: tiles strided by the grid. Dynamic (a.sched): workgroup b runs on XCD
  // b % 8 and takes the tiles of that XCD's contiguous range one at a time from the XCD's own
  // counter (a 128-B line each, so no counter is shared between XCDs); the atomic for the next tile
  // is issued when the current tile starts and its result is read only at the tile's end, so its
  // latency hides behind the tile. The XCD's last workgroup to finish zeroes the counter again.
  const bool dyn = a.sched != nullptr;
  const uint32_t nx = min(8u, gridDim.x);
  const uint32_t xcd = blockIdx.x % nx;
  const uint64_t t_lo = dyn ? a.ndesc * xcd / nx : 0ull, t_hi = dyn ? a.ndesc * (xcd + 1) / nx : a.ndesc;
  uint32_t* cnt = dyn ? a.sched + xcd * 32u : nullptr;
  uint32_t* l_nx = (uint32_t*)(lds + t.o_nx);
  uint64_t tile = blockIdx.x;
  if (dyn) {
    if (tid == 0) l_nx[0] = atomicAdd(cnt, 1u);
    __syncthreads();
    tile = t_lo + l_nx[0];
  }
  uint32_t nxt = 0, it = 1;
  // next tile: the strided one, or the counter value thread 0 fetched (double-buffered in LDS: a
  // slot is rewritten only two barriers after every thread read it)
  auto advance = [&]() -> uint64_t {
    if (!dyn) return tile + gridDim.x;
    if (tid == 0) l_nx[it & 1u] = nxt;
    __syncthreads();  // also: the next tile restages LDS (its strings alias this tile's violation words)
    const uint64_t nt = t_lo + l_nx[it & 1u];
    ++it;
    return nt;
  };
  for (; tile < t_hi; tile = advance()) {
    if (dyn && tid == 0) nxt = atomicAdd(cnt, 1u);
    const TileDesc& d = desc[tile];
    if (!d.fits) continue;  // queued for the overflow kernels by the host (uniform: no barrier skipped unevenly)
    const uint64_t r0 = ((uint64_t)d.r0hi << 32) | d.r0lo;
    const uint32_t nr = d.nr;
    const uint32_t cb = d.cb, ce = d.ce, lb = d.lb, le = d.le;
    const uint32_t kab = d.kab, kae = d.kae, kdb = d.kdb, kde = d.kde;
    const uint32_t nc = ce - cb;

    // ---- P0: stage request headers, container offsets and (FUSED) the tile's strings. Every copy is
    //      an LDS-DMA (global_load_lds: no VGPR round trip), so all of a tile's loads are in flight
    //      together and the barrier waits for one memory latency, not one per array.
    glds_dwords((const uint32_t*)(a.req_flags + r0), (uint32_t*)l_rf, (nr + 3u) >> 2, tid);
    glds_dwords(a.ctr_off + r0, l_coff, nr + 1, tid);
    glds_dwords(a.lbl_off + r0, l_loff, nr + 1, tid);
    glds_dwords((const uint32_t*)a.ctr_flags + (cb >> 2), (uint32_t*)l_cflags, ((ce + 3u) >> 2) - (cb >> 2), tid);
    glds_dwords(a.capadd_off + cb, l_cadd, nc + 1, tid);
    glds_dwords(a.capdrop_off + cb, l_cdrop, nc + 1, tid);
    if (FUSED) {
#pragma unroll
      for (int m = 0; m < (int)NMASK; ++m) {
        if (!t.o_sb[m]) continue;
        const uint32_t g0 = tile_g0(m, (uint32_t)r0, cb, kab, kdb, lb);
        const uint32_t n = tile_n(m, nr, nc, kae - kab, kde - kdb, le - lb);
        glds_dwords(t.s_off[m] + g0, (uint32_t*)(lds + t.o_so[m]), n + 1, tid);  // absolute: rebased by l_sa
        glds_x4((const u32x4*)(t.s_bytes[m] + d.sa[m]), (u32x4*)(lds + t.o_sb[m]), d.nv[m], tid);
      }
    }
    for (uint32_t i = tid; i < nr; i += kSlotThreads) l_rej[i] = l_mut[i] = 0;
    if (tid < NMASK) l_sa[tid] = d.sa[tid];
    __syncthreads();
    const uint8_t* cfl = l_cflags + (cb & 3u);  // staged from the dword holding flag cb

    // ---- P1: classify the staged strings (FUSED) or take the classify kernel's masks (two-kernel
    //      form), and derive each entity's violation set from the slot tables, entity-parallel:
    //      request items (namespace; owner maps of the tile's containers and labels), image items
    //      (registry / tag / image masks), container items (privileged candidates, added and
    //      dropped capabilities, AppArmor profile -> V_c) and label items (key, value -> V_l).
    const SlotHdr& SH = *sv.h;
    const uint64_t privany = SH.priv[0] | SH.priv[1] | SH.priv[2] | SH.priv[3];
    const bool ctr_fam = (privany | SH.caps | SH.aa | SH.trs) != 0;
    const bool classify = !(t.debug & 1u);  // diagnostics: skip classification (entities match nothing)
    // pattern mask of string i of literal column m: the staged strings (FUSED) or the classify
    // kernel's masks (entity index relative to the mask's tile base `g0`)
    auto lit = [&](int m, uint32_t i, uint32_t g0) -> uint64_t {
      if (!classify) return 0ull;
      if (!FUSED) return a.m[m][g0 + i];
      const uint32_t* so = (const uint32_t*)(lds + t.o_so[m]);
      const uint32_t sa = l_sa[m];
      return lit_lookup(lds + t.lit_lds[m], lds + t.o_sb[m], so[i] - sa, so[i + 1] - sa);
    };
    {
      const uint32_t n0 = nr;
      const uint32_t n1 = (t.use_mask & ((1u << M_REG) | (1u << M_TAG) | (1u << M_IMG))) ? nc : 0u;
      const uint32_t n2 = ctr_fam ? nc : 0u;
      const uint32_t n3 = t.o_m[M_LK] ? le - lb : 0u;
      // item segments in falling cost order, each padded to whole waves: a wave's 64 items are one
      // kind (no divergence between kinds) and the round-robin of waves over segments balances
      const uint32_t e0 = rup64(n3), e1 = e0 + rup64(n2), e2 = e1 + rup64(n1), e3 = e2 + rup64(n0);
      for (uint32_t w = tid; w < e3; w += kSlotThreads) {
        if (w < e0) {  // label: key, value -> V_l = denied | constrained-and-failed slots
          const uint32_t i = w;
          if (i >= n3) continue;
          const uint64_t r = lit(M_LK, i, lb);
          uint64_t vm = 0;
          if (!r) {
          } else if (FUSED) {
            if (t.o_sb[M_LV] && !(t.debug & 512u)) {
              const uint32_t* vo = (const uint32_t*)(lds + t.o_so[M_LV]);
              const uint32_t vsa = l_sa[M_LV];
              vm = classify_value(t, lds, r, lds + t.o_sb[M_LV], vo[i] - vsa, vo[i + 1] - vsa);
            }
          } else {
            vm = a.m[M_LV] ? a.m[M_LV][lb + i] : 0ull;
          }
          lds[t.o_m[M_LK] + i] = lit_index(r);
          l_vl[i] = (r && SH.lbl) ? derive_label(sv, r, vm) | sv.tab(ST_DENY)[kw_ctz64(r)] : 0ull;
        } else if (w < e1) {  // container: V_c over the privileged, capability and AppArmor slots
          const uint32_t i = w - e0;
          if (i >= n2) continue;
          const uint32_t fl = cfl[i];
          uint64_t v = 0;
          if ((fl & KW_CTR_PRIVILEGED) && privany) {
            v |= SH.priv[0];
            if (!(fl & KW_CTR_INIT)) v |= SH.priv[1];
            if (!(fl & KW_CTR_EPHEMERAL)) v |= SH.priv[2];
            if (!(fl & (KW_CTR_INIT | KW_CTR_EPHEMERAL))) v |= SH.priv[3];
          }
          if (SH.aa && (t.use_mask & (1u << M_AA)) && (fl & KW_CTR_HAS_APPARMOR)) {
            v |= derive_apparmor(sv, lit(M_AA, i, cb));
          }
          if (t.o_m[M_CAPADD]) {
            for (uint32_t k = l_cadd[i] - kab, k1 = l_cadd[i + 1] - kab; k < k1; ++k) {
              const uint64_t r = lit(M_CAPADD, k, kab);
              lds[t.o_m[M_CAPADD] + k] = lit_index(r);
              const uint64_t va = derive_capadd(sv, r);
              l_vadd[k] = va;
              v |= va;
            }
          }
          if (t.o_m[M_CAPDROP]) {
            for (uint32_t k = l_cdrop[i] - kdb, k1 = l_cdrop[i + 1] - kdb; k < k1; ++k)
              lds[t.o_m[M_CAPDROP] + k] = lit_index(lit(M_CAPDROP, k, kdb));
          }
          l_vc[i] = v;
        } else if (w < e2) {  // image reference: one parse feeds the registry, tag and image chains
          const uint32_t i = w - e1;
          if (i >= n1) continue;
          uint64_t mr = 0, mt = 0, mi = 0;
          if (!classify) {
          } else if (FUSED) {
            if (cfl[i] & KW_CTR_HAS_IMAGE) {
              const uint32_t* so = (const uint32_t*)(lds + t.o_so[M_IMG]);
              const uint32_t sa = l_sa[M_IMG];
              classify_image_all(ch[M_REG], ch[M_TAG], ch[M_IMG], lds + t.o_sb[M_IMG], so[i] - sa, so[i + 1] - sa, &mr,
                                 &mt, &mi);
            }
          } else {
            if (a.m[M_REG]) mr = a.m[M_REG][cb + i];
            if (a.m[M_TAG]) mt = a.m[M_TAG][cb + i];
            if (a.m[M_IMG]) mi = a.m[M_IMG][cb + i];
          }
          if (t.o_m[M_REG]) ((uint64_t*)(lds + t.o_m[M_REG]))[i] = mr;
          if (t.o_m[M_TAG]) ((uint64_t*)(lds + t.o_m[M_TAG]))[i] = mt;
          if (t.o_m[M_IMG]) ((uint64_t*)(lds + t.o_m[M_IMG]))[i] = mi;
        } else {  // request: namespace and the owner maps
          const uint32_t i = w - e2;
          if (i >= n0) continue;
          if (t.o_m[M_NS]) lds[t.o_m[M_NS] + i] = lit_index(lit(M_NS, i, (uint32_t)r0));
          for (uint32_t c = l_coff[i] - cb, c1 = l_coff[i + 1] - cb; c < c1; ++c) own_c[c] = (uint8_t)i;
          for (uint32_t l = l_loff[i] - lb, l1 = l_loff[i + 1] - lb; l < l1; ++l) own_l[l] = (uint8_t)i;
        }
      }
    }
    __syncthreads();

    // ---- P2: first violations, entity-parallel. A slot's first violation is the first entity of
    //      the request (object order) whose violation set holds it: each entity thread ORs the sets
    //      of its predecessors in the request (independent LDS loads) and writes the words of the
    //      slots it violates first; within an entity the family's own order applies (capabilities
    //      in list order, trusted-repos reasons in precedence). Request items add the namespace and
    //      mandatory-label slots and the bypass flag. Rejected / mutated slots merge with ds_or_b64.
    //      (Sequential form of the same walk: slots.hpp walk_*, the host diagnostic.)
    if (SH.trs && !(t.debug & 2u)) {  // trusted-repos reasons join V_c once the image masks exist
      for (uint32_t i = tid; i < nc; i += kSlotThreads) {
        if (!(cfl[i] & KW_CTR_HAS_IMAGE)) continue;
        uint64_t why[5];
        trs_whys(sv, lds, t, i, why);
        l_vc[i] |= (why[0] | why[1] | why[2] | why[3] | why[4]) & SH.trs;
      }
      __syncthreads();
    }
    if (!(t.debug & 2u)) {
      const uint32_t n0 = nr, n1 = ctr_fam ? nc : 0u, n2 = (SH.lbl && t.o_m[M_LK]) ? le - lb : 0u;
      const uint32_t f0 = rup64(n1), f1 = f0 + rup64(n2), f2 = f1 + rup64(n0);  // as in P1
      for (uint32_t w = tid; w < f2; w += kSlotThreads) {
        if (w < f0) {  // container
          const uint32_t i = w;
          if (i >= n1) continue;
          const uint32_t q = own_c[i];
          if (!(l_rf[q] & KW_REQ_HAS_PODSPEC)) continue;
          const uint32_t c0 = l_coff[q] - cb;
          uint64_t pre = 0;
          for (uint32_t j = c0; j < i; ++j) pre |= l_vc[j];
          const uint64_t nv = l_vc[i] & ~pre;
          const uint32_t ci = i - c0;
          uint32_t* vw = l_vw + q * t.vw_stride;
          if (nv) {
            put_viol(vw, nv & privany, vword(KW_R_PRIVILEGED, pack1(ci)));
            put_viol(vw, nv & SH.aa, vword(KW_R_APPARMOR, pack1(ci)));
            uint64_t cn = nv & SH.caps;  // capability slots: the first added capability of the list
            for (uint32_t k = l_cadd[i] - kab, k0 = k, k1 = l_cadd[i + 1] - kab; k < k1 && cn; ++k) {
              const uint64_t nw = l_vadd[k] & cn;
              put_viol(vw, nw, vword(KW_R_CAP_NOT_ALLOWED, pack2(ci, k - k0)));
              cn &= ~nw;
            }
            uint64_t tn = nv & SH.trs;  // trusted-repos slots: reasons in precedence order
            if (tn) {
              uint64_t why[5];
              trs_whys(sv, lds, t, i, why);
              for (uint32_t k = 0; k < 5; ++k) {
                const uint64_t nw = why[k] & tn;
                put_viol(vw, nw, vword(KW_R_REG_NOT_ALLOWED + k, pack1(ci)));
                tn &= ~nw;
              }
            }
            atomicOr((unsigned long long*)&l_rej[q], (unsigned long long)nv);
          }
          if (SH.caps) {  // mutation: required drops missing, default adds neither added nor dropped
            uint64_t addm = 0, dropm = 0;
            if (t.o_m[M_CAPADD])
              for (uint32_t k = l_cadd[i] - kab, k1 = l_cadd[i + 1] - kab; k < k1; ++k)
                addm |= idx_mask(lds[t.o_m[M_CAPADD] + k]);
            if (t.o_m[M_CAPDROP])
              for (uint32_t k = l_cdrop[i] - kdb, k1 = l_cdrop[i + 1] - kdb; k < k1; ++k)
                dropm |= idx_mask(lds[t.o_m[M_CAPDROP] + k]);
            uint64_t mut = 0;
            if (!(dropm & SH.cap_all)) mut |= tab_or(sv.tab(ST_REQD), SH.reqd_union & ~dropm);
            mut |= tab_or(sv.tab(ST_DEFA), SH.defa_union & ~(addm | dropm));
            mut &= SH.caps;
            if (mut) atomicOr((unsigned long long*)&l_mut[q], (unsigned long long)mut);
          }
        } else if (w < f1) {  // label
          const uint32_t i = w - f0;
          if (i >= n2) continue;
          const uint64_t v = l_vl[i];
          if (!v) continue;
          const uint32_t q = own_l[i];
          const uint32_t l0 = l_loff[q] - lb;
          uint64_t pre = 0;
          for (uint32_t j = l0; j < i; ++j) pre |= l_vl[j];
          const uint64_t nv = v & ~pre;
          if (!nv) continue;
          const uint32_t kb = lds[t.o_m[M_LK] + i];
          const uint64_t den = sv.tab(ST_DENY)[kb];
          const uint32_t li = i - l0;
          uint32_t* vw = l_vw + q * t.vw_stride;
          put_viol(vw, nv & den, vword(KW_R_LABEL_DENIED, pack1(li)));
          put_viol(vw, nv & ~den, vword(KW_R_LABEL_CONSTRAINT, pack2(li, 0)) | kb);
          atomicOr((unsigned long long*)&l_rej[q], (unsigned long long)nv);
        } else {  // request: namespace, mandatory labels, bypass
          const uint32_t i = w - f1;
          if (i >= n0) continue;
          const uint32_t rf = l_rf[i];
          uint32_t* vw = l_vw + i * t.vw_stride;
          const uint64_t nsm = t.o_m[M_NS] ? idx_mask(lds[t.o_m[M_NS] + i]) : 0ull;
          uint64_t rej = 0;
          if (SH.ns) {
            const uint64_t ok = (rf & KW_REQ_HAS_NAMESPACE) ? tab_or(sv.tab(ST_NSOK), nsm) : 0ull;
            rej = SH.ns & ~ok;
            put_viol(vw, rej, vword(KW_R_NAMESPACE, 0));
          }
          if (SH.lbl && SH.mand_union && t.o_m[M_LK]) {
            uint64_t present = 0, lrej = 0;
            for (uint32_t l = l_loff[i] - lb, l1 = l_loff[i + 1] - lb; l < l1; ++l) {
              present |= idx_mask(lds[t.o_m[M_LK] + l]);
              lrej |= l_vl[l];
            }
            uint64_t nw = tab_or(sv.tab(ST_MAND), SH.mand_union & ~present) & ~lrej;
            rej |= nw;
            const uint8_t* mand = sv.base + SH.o_mand;  // staged with the record (LDS)
            while (nw) {  // the first missing mandatory key of each such slot, settings order
              const uint32_t sl = kw_ctz64(nw);
              nw &= nw - 1;
              const uint4 mk = *(const uint4*)(mand + sl * 16u);
              const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
              uint32_t k = 0;
              for (; k < 16; ++k) {
                const uint32_t kb = (mw[k >> 2] >> (8 * (k & 3))) & 0xffu;
                if (kb == 0xffu || !((present >> kb) & 1ull)) break;
              }
              vw[sl] = vword(KW_R_LABEL_MANDATORY, k);
            }
          }
          if (rej) atomicOr((unsigned long long*)&l_rej[i], (unsigned long long)rej);
          // namespace bypass (service.rs:40-71): AdmissionRequest in the always-accept namespace
          l_byp[i] = H.bypass_bit >= 0 && !(rf & KW_REQ_RAW) && (rf & KW_REQ_HAS_NAMESPACE) && ((nsm >> H.bypass_bit) & 1ull);
        }
      }
    } else {
      for (uint32_t i = tid; i < nr; i += kSlotThreads) l_byp[i] = 0;
    }
    __syncthreads();

    // ---- P3: verdict rows. Default: one lane per request, each wave a quarter of the columns; the
    //      column records come from the global copy of the slot plan with wave-uniform indices
    //      (scalar loads) and each lane writes 16-B pieces of its own row. p3_item: items =
    //      (request, 4 columns), 16 lanes per 256-B row, column records from LDS.
    if (!(t.debug & 4u)) {
      const uint64_t init = t.slot_init;
      const uint8_t* cidx = t.slot_plan + t.o_cidx_rec;
      uint16_t* gs = gstk ? gstk + tid : nullptr;
      if (!t.p3_item) {
        if (lane < nr) {
          const ColInfo* gcols = (const ColInfo*)(t.slot_plan + t.o_cols_rec);
          const uint64_t rej = l_rej[lane], mut = l_mut[lane];
          const bool byp = l_byp[lane] != 0;
          const uint32_t* vw = l_vw + lane * t.vw_stride;
          uint32_t* orow = out + (r0 + lane) * npol + t.col0;
          const uint32_t q = ((t.ncols + 15u) >> 4) << 2;
          const uint32_t j0 = min(t.ncols, wave * q), j1 = min(t.ncols, j0 + q);
          if (t.vec4) {
            for (uint32_t j = j0; j < j1; j += 4) {
              uint4 w = make_uint4(kBypassWord, kBypassWord, kBypassWord, kBypassWord);
              if (!byp) {
                w.x = column_word(gcols[j + 0], rej, mut, init, vw, blob, cidx, gs, kSlotThreads);
                w.y = column_word(gcols[j + 1], rej, mut, init, vw, blob, cidx, gs, kSlotThreads);
                w.z = column_word(gcols[j + 2], rej, mut, init, vw, blob, cidx, gs, kSlotThreads);
                w.w = column_word(gcols[j + 3], rej, mut, init, vw, blob, cidx, gs, kSlotThreads);
              }
              *(uint4*)(orow + j) = w;
            }
          } else {
            for (uint32_t j = j0; j < j1; ++j)
              orow[j] = byp ? kBypassWord : column_word(gcols[j], rej, mut, init, vw, blob, cidx, gs, kSlotThreads);
          }
        }
      } else {
        const ColInfo* cols = (const ColInfo*)(t.slot_plan + t.o_cols_rec);  // global: group / constant columns
        if (t.vec4) {
          const uint32_t G = t.ncols >> 2;
          for (uint32_t it = tid; it < nr * G; it += kSlotThreads) {
            const uint32_t rr = it / G, g = it - rr * G;
            uint4 w;
            if (l_byp[rr]) {
              w = make_uint4(kBypassWord, kBypassWord, kBypassWord, kBypassWord);
            } else {
              const uint64_t rej = l_rej[rr], mut = l_mut[rr];
              const uint32_t* vw = l_vw + rr * t.vw_stride;
              const uint4 ks = *(const uint4*)(cs + 4 * g), ok = *(const uint4*)(cs + cs_n + 4 * g),
                          mu = *(const uint4*)(cs + 2 * cs_n + 4 * g), rj = *(const uint4*)(cs + 3 * cs_n + 4 * g);
              auto word = [&](uint32_t k, uint32_t okw, uint32_t mutw, uint32_t rejb, uint32_t j) -> uint32_t {
                if ((k & 0xffu) != CK_PLAIN) return column_word(cols[j], rej, mut, init, vw, blob, cidx, gs, kSlotThreads);
                const uint32_t s = k >> 8;
                if ((rej >> s) & 1ull) {
                  uint32_t v = vw[s];
                  if (((v >> 8) & 0xffu) == KW_R_LABEL_CONSTRAINT)
                    v = (v & ~0xffu) | ((uint32_t)cidx[s * 64u + (v & 63u)] << 16);
                  return rejb | v;
                }
                return ((mut >> s) & 1ull) ? mutw : okw;
              };
              w.x = word(ks.x, ok.x, mu.x, rj.x, 4 * g + 0);
              w.y = word(ks.y, ok.y, mu.y, rj.y, 4 * g + 1);
              w.z = word(ks.z, ok.z, mu.z, rj.z, 4 * g + 2);
              w.w = word(ks.w, ok.w, mu.w, rj.w, 4 * g + 3);
            }
            *(uint4*)(out + (r0 + rr) * npol + t.col0 + 4 * g) = w;
          }
        } else {
          const uint32_t G = t.ncols;
          for (uint32_t it = tid; it < nr * G; it += kSlotThreads) {
            const uint32_t rr = it / G, g = it - rr * G;
            uint32_t w = kBypassWord;
            if (!l_byp[rr])
              w = column_word(cols[g], l_rej[rr], l_mut[rr], init, l_vw + rr * t.vw_stride, blob, cidx, gs, kSlotThreads);
            out[(r0 + rr) * npol + t.col0 + g] = w;
          }
        }
      }
    }
    if (!dyn) __syncthreads();  // the next tile restages LDS (its strings alias this tile's violation words)
  }
  if (dyn && tid == 0) {  // the XCD's last workgroup (every other one has taken its last tile) resets
    uint32_t* done = a.sched + 256u + xcd * 32u;
    const uint32_t nwg = (gridDim.x - xcd + nx - 1u) / nx;  // workgroups b < gridDim.x with b % nx == xcd
    __threadfence();  // this workgroup's last counter fetch is ordered before its done count
    if (atomicAdd(done, 1u) == nwg - 1u) {
      atomicExch(cnt, 0u);
      atomicExch(done, 0u);
    }
  }
}

// Requests whose entity counts or string bytes exceed the LDS capacities even in a tile of their
// own (listed by the host with the tile descriptors in `overflow`: count, then request indices).
// Two launches: overflow_classify_kernel classifies their strings into the global mask arrays (DFA
// chains read from the blob, one workgroup per request), then overflow_eval_kernel evaluates every
// (request, column) pair from global memory, one lane per pair.
constexpr int kOverflowThreads = 256;
__global__ void __launch_bounds__(kOverflowThreads)
    overflow_classify_kernel(EvalArgs a, const TileArgs* __restrict__ tp, const uint32_t* __restrict__ overflow) {
  const TileArgs& t = *tp;
  const uint32_t count = overflow[0];
  const uint32_t tid = threadIdx.x;
  Chain ch[NMASK];
#pragma unroll
  for (int k = 0; k < (int)NMASK; ++k) {
    ch[k].head = t.dfa_head[k];
    ch[k].base = a.blob + t.dfa_head[k];
  }
  for (uint32_t q = blockIdx.x; q < count; q += gridDim.x) {
    const uint64_t r0 = overflow[1 + q];
    const uint32_t nr = 1;
    const uint32_t cb = a.ctr_off[r0], ce = a.ctr_off[r0 + nr];
    const uint32_t lb = a.lbl_off[r0], le = a.lbl_off[r0 + nr];
    const uint32_t kab = a.capadd_off[cb], kae = a.capadd_off[ce];
    const uint32_t kdb = a.capdrop_off[cb], kde = a.capdrop_off[ce];
    const uint32_t nc = ce - cb;
    if (a.m[M_NS])
      for (uint32_t i = tid; i < nr; i += kOverflowThreads)
        ((uint64_t*)a.m[M_NS])[r0 + i] =
            classify_one<M_NS>(ch[M_NS], t.s_bytes[M_NS], t.s_off[M_NS][r0 + i], t.s_off[M_NS][r0 + i + 1]);
    if (a.m[M_REG] || a.m[M_TAG] || a.m[M_IMG])
      for (uint32_t i = tid; i < nc; i += kOverflowThreads) {
        uint64_t mr = 0, mt = 0, mi = 0;
        if (a.ctr_flags[cb + i] & KW_CTR_HAS_IMAGE)
          classify_image_all(ch[M_REG], ch[M_TAG], ch[M_IMG], t.s_bytes[M_IMG], t.s_off[M_IMG][cb + i],
                             t.s_off[M_IMG][cb + i + 1], &mr, &mt, &mi);
        if (a.m[M_REG]) ((uint64_t*)a.m[M_REG])[cb + i] = mr;
        if (a.m[M_TAG]) ((uint64_t*)a.m[M_TAG])[cb + i] = mt;
        if (a.m[M_IMG]) ((uint64_t*)a.m[M_IMG])[cb + i] = mi;
      }
    if (a.m[M_AA])
      for (uint32_t i = tid; i < nc; i += kOverflowThreads)
        ((uint64_t*)a.m[M_AA])[cb + i] =
            (a.ctr_flags[cb + i] & KW_CTR_HAS_APPARMOR)
                ? classify_one<M_AA>(ch[M_AA], t.s_bytes[M_AA], t.s_off[M_AA][cb + i], t.s_off[M_AA][cb + i + 1])
                : 0ull;
    if (a.m[M_CAPADD])
      for (uint32_t i = kab + tid; i < kae; i += kOverflowThreads)
        ((uint64_t*)a.m[M_CAPADD])[i] =
            classify_one<M_CAPADD>(ch[M_CAPADD], t.s_bytes[M_CAPADD], t.s_off[M_CAPADD][i], t.s_off[M_CAPADD][i + 1]);
    if (a.m[M_CAPDROP])
      for (uint32_t i = kdb + tid; i < kde; i += kOverflowThreads)
        ((uint64_t*)a.m[M_CAPDROP])[i] =
            classify_one<M_CAPDROP>(ch[M_CAPDROP], t.s_bytes[M_CAPDROP], t.s_off[M_CAPDROP][i], t.s_off[M_CAPDROP][i + 1]);
    if (a.m[M_LK])
      for (uint32_t i = lb + tid; i < le; i += kOverflowThreads)
        ((uint64_t*)a.m[M_LK])[i] = classify_one<M_LK>(ch[M_LK], t.s_bytes[M_LK], t.s_off[M_LK][i], t.s_off[M_LK][i + 1]);
    if (a.m[M_LV])
      for (uint32_t i = lb + tid; i < le; i += kOverflowThreads)
        ((uint64_t*)a.m[M_LV])[i] = classify_one<M_LV>(ch[M_LV], t.s_bytes[M_LV], t.s_off[M_LV][i], t.s_off[M_LV][i + 1]);
  }
}

__global__ void __launch_bounds__(kOverflowThreads)
    overflow_eval_kernel(EvalArgs a, const TileArgs* __restrict__ tp, const uint32_t* __restrict__ overflow) {
  __shared__ uint16_t gstk[kMaxGroupStack * kOverflowThreads];
  const TileArgs& t = *tp;
  const uint32_t count = overflow[0];
  const DevHeader H = *(const DevHeader*)a.blob;
  const DevPolicy* __restrict__ pols = (const DevPolicy*)(a.blob + H.policy_off);
  const uint32_t npol = a.npol;
  const uint64_t items = (uint64_t)count * npol;
  GlobalSrc src{&a};
  (void)t;
  for (uint64_t it = (uint64_t)blockIdx.x * kOverflowThreads + threadIdx.x; it < items;
       it += (uint64_t)gridDim.x * kOverflowThreads) {
    const uint32_t j = (uint32_t)(it % npol);
    const uint64_t r = overflow[1 + it / npol];
    const DevPolicy& P = pols[a.pols[j]];
    a.out[r * npol + j] = verdict(src, a, H, pols, P, r, gstk + threadIdx.x, kOverflowThreads);
  }
}

hipError_t launch_classify(const uint8_t* d_blob, const ClassifyJobs& jobs, hipStream_t s) {
  if (jobs.n == 0 || jobs.total_blocks == 0) return hipSuccess;
  if (jobs.lds_bytes > 0)
    hipLaunchKernelGGL(classify_kernel<true>, dim3(jobs.total_blocks), dim3(kClassifyThreads), jobs.lds_bytes, s, d_blob,
                       jobs);
  else
    hipLaunchKernelGGL(classify_kernel<false>, dim3(jobs.total_blocks), dim3(kClassifyThreads), 0, s, d_blob, jobs);
  return hipGetLastError();
}

hipError_t launch_evaluate_rows(const EvalArgs& a, hipStream_t s) {
  if (a.nrows == 0) return hipSuccess;
  uint64_t blocks = (a.nrows + kEvalThreads - 1) / kEvalThreads;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(evaluate_rows_kernel, dim3((uint32_t)blocks), dim3(kEvalThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_evaluate_slots(const EvalArgs& a, const TileArgs& t, const TileArgs* d_t, const TileDesc* d_desc,
                                 bool fused, uint32_t grid, hipStream_t s) {
  if (a.nrows == 0 || t.ncols == 0) return hipSuccess;
  static bool attr_set = false;  // allow > 64 KB of dynamic LDS per workgroup (gfx950: 160 KB per CU)
  if (!attr_set) {
    hipError_t e1 = hipFuncSetAttribute((const void*)evaluate_slots_kernel<true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipError_t e2 = hipFuncSetAttribute((const void*)evaluate_slots_kernel<false>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e1 != hipSuccess || e2 != hipSuccess) return e1 != hipSuccess ? e1 : e2;
    attr_set = true;
  }
  // The grid is persistent (tiles strided by gridDim.x), so it must be co-resident: a workgroup
  // that only starts when another retires doubles the tail. Clamp the planner's grid to the
  // runtime's occupancy for this LDS size (queried once per device and LDS size).
  {
    thread_local int c_dev = -1, c_ncu = 0, c_occ = 0;
    thread_local uint64_t c_key = ~0ull;
    int dev = 0;
    const uint64_t key = ((uint64_t)t.lds_bytes << 1) | (fused ? 1u : 0u);
    if (hipGetDevice(&dev) == hipSuccess && (dev != c_dev || key != c_key)) {
      int ncu = 0, occ = 0;
      const void* fn = fused ? (const void*)evaluate_slots_kernel<true> : (const void*)evaluate_slots_kernel<false>;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kSlotThreads, t.lds_bytes) != hipSuccess)
        ncu = occ = 0;
      c_dev = dev;
      c_key = key;
      c_ncu = ncu;
      c_occ = occ;
    }
    if (c_occ > 0 && c_ncu > 0) grid = std::max<uint32_t>(1u, std::min<uint32_t>(grid, (uint32_t)(c_occ * c_ncu)));
    if (t.debug & 256u)
      fprintf(stderr, "[kw tile] launch grid=%u occupancy=%d wg/cu x %d CUs lds=%u\n", grid, c_occ, c_ncu, t.lds_bytes);
  }
  if (fused)
    hipLaunchKernelGGL(evaluate_slots_kernel<true>, dim3(grid), dim3(kSlotThreads), t.lds_bytes, s, a, d_t, d_desc,
                       a.blob, a.out);
  else
    hipLaunchKernelGGL(evaluate_slots_kernel<false>, dim3(grid), dim3(kSlotThreads), t.lds_bytes, s, a, d_t, d_desc,
                       a.blob, a.out);
  return hipGetLastError();
}

hipError_t launch_overflow(const EvalArgs& a, const TileArgs* d_t, const uint32_t* d_overflow, uint32_t n_overflow,
                           hipStream_t s) {
  if (n_overflow == 0 || a.nrows == 0 || a.npol == 0) return hipSuccess;
  hipLaunchKernelGGL(overflow_classify_kernel, dim3(std::min<uint32_t>(n_overflow, 1024)), dim3(kOverflowThreads), 0, s,
                     a, d_t, d_overflow);
  const uint64_t items = (uint64_t)n_overflow * a.npol;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((items + kOverflowThreads - 1) / kOverflowThreads, 4096);
  hipLaunchKernelGGL(overflow_eval_kernel, dim3(blocks), dim3(kOverflowThreads), 0, s, a, d_t, d_overflow);
  return hipGetLastError();
}

}  // namespace kw
