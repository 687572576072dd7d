// kernels.hip — the MI355X (gfx950) hot path of EvaluationEnvironment::validate for the
// declarative policy class (src/evaluation/evaluation_environment.rs:546-594) fused with the
// service::evaluate epilogue (src/api/service.rs:40-116, 160-208).
//
// Two kernels per validate pass:
//  classify_kernel  — every request string that some selected policy reads (namespace, image
//                     reference, capability names, AppArmor profile, label key / value) runs
//                     through its column's multi-pattern DFA, one lane per string. The column DFA
//                     (byte-class map, u16 transitions, u64 accept masks) is staged into LDS once
//                     per workgroup; string bytes stream from HBM with 4-byte aligned loads.
//                     Image references are parsed in-lane (registry / path / tag / digest, with
//                     docker.io / library/ / latest normalisation fed as virtual bytes) and drive
//                     three DFAs. Output: one u64 pattern-match mask per string.
//  evaluate_kernel  — one lane per (request, policy) pair; lanes of a wave share a request in the
//                     all-pairs layout, so entity loads broadcast. Each policy is a few bit tests
//                     over the masks; groups evaluate their members eagerly and run a postfix
//                     program that tracks rhai's short-circuit "called" set per stack entry.
//                     The verdict word (include/kwgpu.h) carries the vanilla response and the
//                     service-level result.
// Integer / byte work only: no MFMA. Bound: HBM streaming of string bytes + masks + verdicts, and
// the dependent LDS chain of the DFA walk.
#include <hip/hip_runtime.h>

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

__constant__ char kDockerIo[9] = {'d', 'o', 'c', 'k', 'e', 'r', '.', 'i', 'o'};
__constant__ char kLibrary[8] = {'l', 'i', 'b', 'r', 'a', 'r', 'y', '/'};
__constant__ char kLatest[6] = {'l', 'a', 't', 'e', 's', 't'};
__constant__ char kLocalhost[9] = {'l', 'o', 'c', 'a', 'l', 'h', 'o', 's', 't'};

__device__ inline uint32_t feed_const(const DfaView& d, uint32_t st, const char* s, int n) {
  for (int i = 0; i < n && st != 0; ++i) st = step(d, st, (uint8_t)s[i]);
  return st;
}

__device__ inline uint32_t byte_at(const uint8_t* __restrict__ bytes, uint32_t p) { return bytes[p]; }

__device__ inline bool equals_const(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e, const char* s,
                                    int n) {
  if ((int)(e - b) != n) return false;
  for (int i = 0; i < n; ++i)
    if (byte_at(bytes, b + (uint32_t)i) != (uint8_t)s[i]) return false;
  return true;
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
  r.is_reg = slash0 != NONE && (dotcolon || equals_const(bytes, b, slash0, kLocalhost, 9));
  r.rest_b = r.is_reg ? slash0 + 1 : b;
  r.colon = (last_colon != NONE && last_colon >= r.rest_b) ? last_colon : NONE;
  r.path_end = r.colon != NONE ? r.colon : r.name_end;
  uint32_t first_slash_rest = r.is_reg ? slash1 : slash0;
  r.path_slash = first_slash_rest != NONE && first_slash_rest < r.path_end;
  r.is_docker = !r.is_reg || equals_const(bytes, b, slash0, kDockerIo, 9);
  r.eff_tag = r.colon != NONE || at == NONE;
  return r;
}

// Registry (k=0), effective tag (k=1) or normalised image (k=2) through one DFA.
__device__ uint64_t image_part(int k, const DfaView& d, const uint8_t* __restrict__ bytes, const ImageRef& r) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t st = d.start;
  if (k == 0) {
    st = r.is_reg ? feed(d, st, bytes, r.b, r.slash0) : feed_const(d, st, kDockerIo, 9);
  } else if (k == 1) {
    if (r.colon != NONE) st = feed(d, st, bytes, r.colon + 1, r.name_end);
    else if (r.at == NONE) st = feed_const(d, st, kLatest, 6);
    else return 0ull;  // digest only: no tag
  } else {
    st = r.is_reg ? feed(d, st, bytes, r.b, r.slash0) : feed_const(d, st, kDockerIo, 9);
    if (st) st = step(d, st, '/');
    if (r.is_docker && !r.path_slash) st = feed_const(d, st, kLibrary, 8);
    st = feed(d, st, bytes, r.rest_b, r.path_end);
    if (r.eff_tag) {
      if (st) st = step(d, st, ':');
      st = r.colon != NONE ? feed(d, st, bytes, r.colon + 1, r.name_end) : feed_const(d, st, kLatest, 6);
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
struct FamOut {
  uint32_t reason, arg;
  bool mutated;
};

__device__ inline uint64_t M(const uint64_t* __restrict__ m, uint64_t i) { return m ? m[i] : 0ull; }
__device__ inline uint32_t pack2(uint32_t a, uint32_t b) { return (min(a, 255u) << 8) | min(b, 255u); }
__device__ inline uint32_t pack1(uint32_t a) { return min(a, 65535u); }

__device__ FamOut eval_family(const EvalArgs& a, const DevPolicy& P, uint64_t r) {
  FamOut o{0, 0, false};
  const uint8_t rf = a.req_flags[r];
  const uint32_t cb = a.ctr_off[r], ce = a.ctr_off[r + 1];
  switch (P.family) {
    case FAM_PRIVILEGED: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        uint8_t f = a.ctr_flags[c];
        bool skip = ((P.flags & PF_SKIP_INIT) && (f & KW_CTR_INIT)) || ((P.flags & PF_SKIP_EPHEMERAL) && (f & KW_CTR_EPHEMERAL));
        if (!skip && (f & KW_CTR_PRIVILEGED)) {
          o.reason = KW_R_PRIVILEGED;
          o.arg = pack1(c - cb);
          break;
        }
      }
      break;
    }
    case FAM_NAMESPACE: {
      bool ok = (rf & KW_REQ_HAS_NAMESPACE) && P.nl[0] && (M(a.m[M_NS], r) & P.m[0]);
      if (!ok) o.reason = KW_R_NAMESPACE;
      break;
    }
    case FAM_TRUSTED_REPOS: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        if (!(a.ctr_flags[c] & KW_CTR_HAS_IMAGE)) continue;
        uint64_t reg = M(a.m[M_REG], c), tag = M(a.m[M_TAG], c), img = M(a.m[M_IMG], c);
        uint32_t why = 0;
        if (P.nl[0] && !(reg & P.m[0])) why = KW_R_REG_NOT_ALLOWED;
        else if (P.nl[1] && (reg & P.m[1])) why = KW_R_REG_REJECTED;
        else if (P.nl[2] && (tag & P.m[2])) why = KW_R_TAG_REJECTED;
        else if (P.nl[3] && !(img & P.m[3])) why = KW_R_IMG_NOT_ALLOWED;
        else if (P.nl[4] && (img & P.m[4])) why = KW_R_IMG_REJECTED;
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
      if (!(P.flags & PF_ALLOW_ALL)) {
        for (uint32_t c = cb; c < ce && !o.reason; ++c) {
          uint32_t kb = a.capadd_off[c], ke = a.capadd_off[c + 1];
          for (uint32_t k = kb; k < ke; ++k)
            if (!(M(a.m[M_CAPADD], k) & P.m[0])) {
              o.reason = KW_R_CAP_NOT_ALLOWED;
              o.arg = pack2(c - cb, k - kb);
              break;
            }
        }
        if (o.reason) break;
      }
      for (uint32_t c = cb; c < ce; ++c) {
        uint64_t addm = 0, dropm = 0;
        for (uint32_t k = a.capadd_off[c]; k < a.capadd_off[c + 1]; ++k) addm |= M(a.m[M_CAPADD], k);
        for (uint32_t k = a.capdrop_off[c]; k < a.capdrop_off[c + 1]; ++k) dropm |= M(a.m[M_CAPDROP], k);
        if (!(dropm & P.m[3]) && (P.m[1] & ~dropm)) o.mutated = true;
        if (P.m[2] & ~(addm | dropm)) o.mutated = true;
      }
      break;
    }
    case FAM_APPARMOR: {
      if (!(rf & KW_REQ_HAS_PODSPEC)) break;
      for (uint32_t c = cb; c < ce; ++c) {
        if ((a.ctr_flags[c] & KW_CTR_HAS_APPARMOR) && !(M(a.m[M_AA], c) & P.m[0])) {
          o.reason = KW_R_APPARMOR;
          o.arg = pack1(c - cb);
          break;
        }
      }
      break;
    }
    case FAM_LABELS: {
      const uint32_t lb = a.lbl_off[r], le = a.lbl_off[r + 1];
      uint64_t present = 0;
      for (uint32_t l = lb; l < le && !o.reason; ++l) {
        uint64_t km = M(a.m[M_LK], l);
        present |= km;
        if (km & P.m[0]) {
          o.reason = KW_R_LABEL_DENIED;
          o.arg = pack1(l - lb);
          break;
        }
        for (uint32_t i = 0; i < P.n_constr; ++i) {
          if (((km >> P.idx[16 + i]) & 1ull) && !((M(a.m[M_LV], l) >> P.idx[32 + i]) & 1ull)) {
            o.reason = KW_R_LABEL_CONSTRAINT;
            o.arg = pack2(l - lb, i);
            break;
          }
        }
      }
      if (o.reason) break;
      for (uint32_t i = 0; i < P.n_mand; ++i)
        if (!((present >> P.idx[i]) & 1ull)) {
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

__device__ uint32_t verdict(const EvalArgs& a, const DevHeader& H, const DevPolicy* __restrict__ pols, int32_t pidx,
                            uint64_t r, uint16_t* gstk) {
  const DevPolicy& P = pols[pidx];
  const uint8_t rf = a.req_flags[r];
  // namespace bypass (service.rs:40-71), AdmissionRequest only
  if (H.bypass_bit >= 0 && !(rf & KW_REQ_RAW) && (rf & KW_REQ_HAS_NAMESPACE) &&
      ((M(a.m[M_NS], r) >> H.bypass_bit) & 1ull))
    return KW_V_ALLOWED | KW_F_ALLOWED | KW_BYPASS;
  // PolicyInitialization -> reject 500 before any constraint (service.rs:78-91)
  if (P.flags & PF_INIT_ERROR) return ((uint32_t)KW_FST_INIT_ERROR << KW_F_STATUS_SHIFT) | ((uint32_t)KW_R_INIT_ERROR << 8);
  uint32_t reason = 0, arg = 0;
  bool mutated = false;
  if (P.family == FAM_GROUP) {
    if (P.flags & PF_EXPR_ERROR) {
      reason = KW_R_GROUP_EXPR;
    } else {
      const int32_t* mem = (const int32_t*)(a.blob + H.member_off) + P.member_off;
      uint32_t ok = 0;
      for (uint32_t s = 0; s < P.nmembers; ++s) {
        const DevPolicy& Q = pols[mem[s]];
        if (Q.flags & PF_INIT_ERROR) continue;
        FamOut fo = eval_family(a, Q, r);
        if (fo.reason == 0 && !fo.mutated) ok |= 1u << s;
      }
      const uint8_t* prog = a.blob + H.prog_off + P.prog_off;
      uint32_t vals = 0;  // bit stack of values
      int sp = 0;
      for (uint32_t pc = 0; pc < P.prog_len; ++pc) {
        uint8_t op = prog[pc];
        if (op <= G_CALL) {
          uint32_t v = op == G_CONST1 ? 1u : 0u, e = 0;
          if (op == G_CALL) {
            uint32_t s = prog[++pc];
            v = (ok >> s) & 1u;
            e = 1u << s;
          }
          vals = (vals & ~(1u << sp)) | (v << sp);
          gstk[sp * kEvalThreads] = (uint16_t)e;
          ++sp;
        } else if (op == G_NOT) {
          vals ^= 1u << (sp - 1);
        } else {
          --sp;
          uint32_t bv = (vals >> sp) & 1u, av = (vals >> (sp - 1)) & 1u;
          uint32_t be = gstk[sp * kEvalThreads], ae = gstk[(sp - 1) * kEvalThreads];
          uint32_t v, e;
          if (op == G_AND) {
            v = av & bv;
            e = ae | (av ? be : 0u);
          } else if (op == G_OR) {
            v = av | bv;
            e = ae | (av ? 0u : be);
          } else if (op == G_EQ) {
            v = (av == bv);
            e = ae | be;
          } else {
            v = (av != bv);
            e = ae | be;
          }
          vals = (vals & ~(1u << (sp - 1))) | (v << (sp - 1));
          gstk[(sp - 1) * kEvalThreads] = (uint16_t)e;
        }
      }
      if (!(vals & 1u)) {
        reason = KW_R_GROUP;
        arg = (uint32_t)gstk[0] & ~ok & 0xffffu;
      }
    }
  } else {
    FamOut fo = eval_family(a, P, r);
    reason = fo.reason;
    arg = fo.arg;
    mutated = fo.mutated;
  }
  uint32_t v = (reason << 8) | ((arg & 0xffffu) << 16);
  const bool allowed = reason == 0;
  if (allowed) v |= KW_V_ALLOWED;
  if (mutated) v |= KW_V_MUTATED;
  // validation_response_with_constraints (service.rs:160-208) for the Validate origin
  uint32_t fst = allowed ? KW_FST_NONE : KW_FST_VANILLA;
  bool fallowed = allowed;
  if (a.origin == KW_ORIGIN_VALIDATE) {
    if (P.mode == KW_MODE_MONITOR) {
      fallowed = true;
      fst = KW_FST_NONE;
    } else if (mutated && !P.a2m) {
      fallowed = false;
      fst = KW_FST_MUTATION_REFUSED;
    }
  }
  if (fallowed) v |= KW_F_ALLOWED;
  if (mutated && fst == KW_FST_NONE && (a.origin == KW_ORIGIN_AUDIT || P.mode == KW_MODE_PROTECT)) v |= KW_F_PATCH;
  v |= fst << KW_F_STATUS_SHIFT;
  return v;
}

__global__ void __launch_bounds__(kEvalThreads) evaluate_kernel(EvalArgs a) {
  __shared__ uint16_t gstk[kMaxGroupStack * kEvalThreads];
  const DevHeader H = *(const DevHeader*)a.blob;
  const DevPolicy* __restrict__ pols = (const DevPolicy*)(a.blob + H.policy_off);
  const uint64_t stride = (uint64_t)gridDim.x * kEvalThreads;
  for (uint64_t pair = (uint64_t)blockIdx.x * kEvalThreads + threadIdx.x; pair < a.npairs; pair += stride) {
    uint64_t r;
    int32_t pidx;
    if (a.row_policy) {
      r = pair;
      pidx = a.row_policy[r];
    } else {
      r = pair / a.npol;
      pidx = a.pols[pair - r * a.npol];
    }
    a.out[pair] = verdict(a, H, pols, pidx, r, gstk + threadIdx.x);
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

hipError_t launch_evaluate(const EvalArgs& a, hipStream_t s) {
  if (a.npairs == 0) return hipSuccess;
  uint64_t blocks = (a.npairs + kEvalThreads - 1) / kEvalThreads;
  if (blocks > 256 * 16) blocks = 256 * 16;  // grid-stride beyond 16 blocks per CU
  hipLaunchKernelGGL(evaluate_kernel, dim3((uint32_t)blocks), dim3(kEvalThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace kw
