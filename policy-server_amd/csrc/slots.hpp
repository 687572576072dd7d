// slots.hpp — bit-parallel evaluation of a policy list against one request.
//
// A validate pass answers a list of policy ids for every request of a batch
// (EvaluationEnvironment::validate, evaluation_environment.rs:546-594). The list compiles into
// chunks of up to 64 *slots* (one per plain policy or group member; equal settings share one) and
// the output columns that read them. A slot is one bit of a u64.
//
// Every string of a request is first classified into a small integer (kwdev.hpp classifiers). A
// chunk record then holds, per column class, the set of slots an entity of that class violates
// (tables below), so an entity's violation set is one table load — however many patterns the
// policies name. A slot's verdict is its *first* violation in object order (containers, then
// labels; the families' own order, DESIGN.md §2, oracle/kworacle.c fam_*), and the cost per request
// is O(entities + violations), not O(policies x entities).
//
// Shared by the device kernels (kernels.hip: entity-parallel in the tile kernel, the sequential
// walks below in the overflow kernel) and the host diagnostic kw_debug_host_walk (capi.cpp), which
// the CPU test suite uses to check the slot compiler against the oracle.
#pragma once
#include <cstdint>

#include "../../include/kwgpu.h"
#include "kwdev.hpp"

namespace kw {

constexpr uint32_t kSlots = 64;
constexpr uint32_t kArgWide = 0xffffu;  // ARG sentinel: the full value is in the pass's side data

// Per-class slot tables, each u64[nclass of its column] indexed by the column class.
enum SlotTab : uint32_t {
  T_NSOK = 0,  // COL_NS:  namespace slots whose valid_namespace is this class
  T_RA,        // COL_REG: trusted-repos slots whose registries.allow matches
  T_RR,        // COL_REG: ... registries.reject
  T_TR,        // COL_TAG: ... tags.reject
  T_IA,        // COL_IMG: ... images.allow
  T_IR,        // COL_IMG: ... images.reject
  T_NACAP,     // COL_CAP: strict psp-capabilities slots that allow neither the capability nor default-add it
  T_NAAA,      // COL_AA:  psp-apparmor slots that do not allow the profile
  T_DENY,      // COL_LK:  safe-labels slots that deny the key
  T_FAIL,      // COL_LV:  safe-labels slots whose constraint on the label's key the value fails
  NTAB
};

struct alignas(16) SlotHdr {
  uint64_t caps_strict;  // psp-capabilities slots without "*" in allowed_capabilities
  uint64_t caps;         // every psp-capabilities slot (mutation)
  uint64_t aa, lbl, ns, trs;
  uint64_t has_ra, has_ia;  // trusted-repos slots with a non-empty registries.allow / images.allow
  uint64_t priv[4];         // pod-privileged slots by (skip_init | skip_ephemeral << 1)
  uint64_t init;            // slots whose policy failed to initialise (group members: never ok)
  // local bits (per chunk): capabilities some slot requires dropped / adds by default ("ALL" always
  // has one when the chunk has psp-capabilities slots), and mandatory label keys
  uint64_t reqd_union, defa_union, all_bit, mand_union;
  uint64_t mand_one;  // slots whose mandatory list is a single key (its absence: index 0)
  uint32_t ncols, nslots, bytes, staged;  // bytes: whole record; staged: prefix the device keeps in LDS
  uint32_t tab_off[NTAB];                 // byte offset of each class table (0 = not emitted)
  uint32_t o_capmb, o_lkmb;               // u8 per COL_CAP / COL_LK class: its local bit, 0xff = none
  uint32_t o_reqd, o_defa, o_mand;        // u64[64] per local bit: the slots that list it
  uint32_t o_mlist;                       // u32 per slot: offset of its mandatory list (local bits in
                                          // settings order, 0xff-terminated), 0 = none
  uint32_t o_csoa;   // column arrays (kind | slot << 8, okw, mutw, rejb), each ncols rounded up to 4 u32
  uint32_t o_cols;   // ColInfo[ncols] (global memory on the device)
  uint32_t o_prog;   // group programs (global memory on the device)
  uint32_t nwide;    // group columns of this chunk with more than 15 members
  uint32_t o_mpack;  // u64 per slot: its first 8 mandatory local bits packed (0xff pad), 0 = none
  uint32_t pad1;
};
static_assert(sizeof(SlotHdr) % 16 == 0, "SlotHdr layout");

enum ColKind : uint32_t { CK_CONST = 0, CK_PLAIN = 1, CK_GROUP = 2, CK_TABLE = 3, CK_WIDE = 4 };

// One output column (a selected policy). PLAIN: verdict of slot `slot`. GROUP: the jump program at
// record offset prog_off over the member slots [slot, slot + nmem). TABLE: the truth table (u32
// entries, expr.hpp kGt*) at record offset prog_off over member slots [slot, slot + nmem), nmem <= 16;
// errw: the word of an evaluation error. WIDE: a wide group's placeholder (okw = 0), written after
// the pass by the wide-group combine kernel (kernels.hpp WideGroupPass). CONST: the word `okw` whatever
// the request (initialisation error, group expression that is not a bool). okw / mutw / rejb: the
// service-level verdict word of an accepted, an accepted-and-mutated and a rejected vanilla response
// (reason/arg bits clear in rejb). wide: index of a > 15-member group in the pass's dense cause
// array (its causes do not fit ARG), else ~0.
struct alignas(16) ColInfo {
  uint32_t kind, slot, nmem, prog_off, prog_len, okw, mutw, rejb, wide, policy, errw, pad;
};
static_assert(sizeof(ColInfo) == 48, "ColInfo layout");

KW_HD inline uint32_t kw_ctz64(uint64_t x) { return (uint32_t)__builtin_ctzll(x); }
KW_HD inline uint32_t sat16(uint32_t a) { return a < kArgWide ? a : kArgWide; }
KW_HD inline uint32_t vword(uint32_t reason, uint32_t arg) { return (reason << 8) | (sat16(arg) << 16); }
KW_HD inline uint64_t bit_of(uint32_t b) { return b < 64u ? 1ull << b : 0ull; }  // 0xff: none

// Verdict word from a family result: the vanilla response plus validation_response_with_constraints
// (service.rs:160-208) for the Validate origin, vanilla for Audit (service.rs:108-116).
KW_HD inline uint32_t finish_word(uint32_t mode, uint32_t a2m, int origin, uint32_t reason, uint32_t arg, bool mutated) {
  uint32_t v = vword(reason, arg);
  const bool allowed = reason == 0;
  if (allowed) v |= KW_V_ALLOWED;
  if (mutated) v |= KW_V_MUTATED;
  uint32_t fst = allowed ? KW_FST_NONE : KW_FST_VANILLA;
  bool fallowed = allowed;
  if (origin == KW_ORIGIN_VALIDATE) {
    if (mode == KW_MODE_MONITOR) {
      fallowed = true;
      fst = KW_FST_NONE;
    } else if (mutated && !a2m) {
      fallowed = false;
      fst = KW_FST_MUTATION_REFUSED;
    }
  }
  if (fallowed) v |= KW_F_ALLOWED;
  if (mutated && fst == KW_FST_NONE && (origin == KW_ORIGIN_AUDIT || mode == KW_MODE_PROTECT)) v |= KW_F_PATCH;
  v |= fst << KW_F_STATUS_SHIFT;
  return v;
}
constexpr uint32_t kInitErrorWord = ((uint32_t)KW_FST_INIT_ERROR << KW_F_STATUS_SHIFT) | ((uint32_t)KW_R_INIT_ERROR << 8);
constexpr uint32_t kBypassWord = KW_V_ALLOWED | KW_F_ALLOWED | KW_BYPASS;

// The record's sections, resolved once (device: LDS or global pointers; host: the record bytes).
struct SlotView {
  const SlotHdr* h;
  const uint8_t* base;
  KW_HD const uint64_t* tab(uint32_t k) const { return (const uint64_t*)(base + h->tab_off[k]); }
  KW_HD uint64_t row(uint32_t k, uint32_t cls) const { return tab(k)[cls]; }
  KW_HD uint32_t capmb(uint32_t cls) const { return base[h->o_capmb + cls]; }
  KW_HD uint32_t lkmb(uint32_t cls) const { return base[h->o_lkmb + cls]; }
  KW_HD const uint64_t* reqd() const { return (const uint64_t*)(base + h->o_reqd); }
  KW_HD const uint64_t* defa() const { return (const uint64_t*)(base + h->o_defa); }
  KW_HD const uint64_t* mand() const { return (const uint64_t*)(base + h->o_mand); }
  KW_HD const uint8_t* mlist(uint32_t s) const { return base + ((const uint32_t*)(base + h->o_mlist))[s]; }
  KW_HD uint64_t mpack(uint32_t s) const { return ((const uint64_t*)(base + h->o_mpack))[s]; }
};

// OR of table rows over the set bits of `bits` (per 32-bit half, two independent row loads a round).
KW_HD inline uint64_t tab_or(const uint64_t* t, uint64_t bits) {
  uint64_t r = 0;
  for (uint32_t h = 0; h < 2; ++h) {
    uint32_t m = (uint32_t)(bits >> (32u * h));
    const uint64_t* th = t + 32u * h;
    while (m) {
      const uint32_t i = (uint32_t)__builtin_ctz(m);
      m &= m - 1u;
      const uint32_t j = m ? (uint32_t)__builtin_ctz(m) : i;
      m &= m - 1u;
      r |= th[i] | th[j];
    }
  }
  return r;
}

// Image classes of one container: the COL_REG entries (literal class, then one per DFA of the
// chain), the COL_TAG entries, the COL_IMG entries, in that order.
struct ImgLayout {
  uint32_t nreg, ntag, nimg;
  KW_HD uint32_t n() const { return nreg + ntag + nimg; }
};

// Trusted-repos reasons of one container (precedence order: registry not allowed, registry
// rejected, tag rejected, image not allowed, image rejected; oracle fam_trusted). `ic(j)`: the
// container's j-th image class.
template <class F>
KW_HD inline void trs_whys(const SlotView& sv, const ImgLayout& L, F ic, uint64_t why[5]) {
  uint64_t ra = 0, rr = 0, tr = 0, ia = 0, ir = 0;
  for (uint32_t j = 0; j < L.nreg; ++j) {
    const uint32_t c = ic(j);
    ra |= sv.row(T_RA, c);
    rr |= sv.row(T_RR, c);
  }
  for (uint32_t j = L.nreg; j < L.nreg + L.ntag; ++j) tr |= sv.row(T_TR, ic(j));
  for (uint32_t j = L.nreg + L.ntag; j < L.n(); ++j) {
    const uint32_t c = ic(j);
    ia |= sv.row(T_IA, c);
    ir |= sv.row(T_IR, c);
  }
  why[0] = sv.h->has_ra & ~ra;
  why[1] = rr;
  why[2] = tr;
  why[3] = sv.h->has_ia & ~ia;
  why[4] = ir;
}

// Privileged slots a container flagged `fl` violates.
KW_HD inline uint64_t priv_viol(const SlotHdr& h, uint32_t fl) {
  if (!(fl & KW_CTR_PRIVILEGED)) return 0ull;
  uint64_t v = h.priv[0];
  if (!(fl & KW_CTR_INIT)) v |= h.priv[1];
  if (!(fl & KW_CTR_EPHEMERAL)) v |= h.priv[2];
  if (!(fl & (KW_CTR_INIT | KW_CTR_EPHEMERAL))) v |= h.priv[3];
  return v;
}

// Mutated psp-capabilities slots of a container from its added / dropped local bits: a required
// drop missing (unless ALL is dropped) or a default add neither added nor dropped.
KW_HD inline uint64_t caps_mutation(const SlotView& sv, uint64_t addm, uint64_t dropm) {
  const SlotHdr& h = *sv.h;
  uint64_t mut = 0;
  if (!(dropm & h.all_bit)) mut |= tab_or(sv.reqd(), h.reqd_union & ~dropm);
  mut |= tab_or(sv.defa(), h.defa_union & ~(addm | dropm));
  return mut & h.caps;
}

// Index (settings order) of slot s's first mandatory key absent from `present` (local bits).
KW_HD inline uint32_t first_missing(const SlotView& sv, uint32_t s, uint64_t present) {
  const uint8_t* m = sv.mlist(s);
  uint32_t i = 0;
  for (;; ++i) {
    const uint32_t b = m[i];
    if (b == 0xffu || !((present >> b) & 1ull)) break;
  }
  return i;
}

// first_missing from the slot's packed list (one u64 load for lists of up to 8 keys; longer lists
// continue in mlist): the same index.
KW_HD inline uint32_t first_missing_packed(const SlotView& sv, uint32_t s, uint64_t packed, uint64_t present) {
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t b = (uint32_t)(packed >> (8u * i)) & 0xffu;
    if (b == 0xffu || !((present >> b) & 1ull)) return i;
  }
  const uint8_t* m = sv.mlist(s);
  uint32_t i = 8;
  while (m[i] != 0xffu && ((present >> m[i]) & 1ull)) ++i;
  return i;
}

// Violation sink of the sequential walks: the word (16-bit ARG, saturated) and the full argument.
struct ViolSink {
  uint32_t* vw;
  uint32_t* va;  // may be null
  // (the mask is walked as two 32-bit halves: one find-first-set and one clear per slot)
  KW_HD void put(uint64_t nw, uint32_t reason, uint32_t arg) const {
    const uint32_t w = vword(reason, arg);
#ifdef KW_PUT64
    while (nw) {
      const uint32_t s = kw_ctz64(nw);
      vw[s] = w;
      if (va) va[s] = arg;
      nw &= nw - 1;
    }
    return;
#endif
#ifndef KW_PUT2  // two slots a loop trip (the second repeats the first when the half runs out: idempotent)
#define KW_PUT2 1
#endif
    for (uint32_t h = 0; h < 2; ++h) {
      uint32_t m = (uint32_t)(nw >> (32u * h));
      while (m) {
        const uint32_t s = 32u * h + (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        uint32_t s2 = s;
        if (KW_PUT2 && m) {
          s2 = 32u * h + (uint32_t)__builtin_ctz(m);
          m &= m - 1u;
        }
        vw[s] = w;
        vw[s2] = w;
        if (va) {
          va[s] = arg;
          va[s2] = arg;
        }
      }
    }
  }
};

// ---- sequential walks over one request (host diagnostic and the overflow kernel). The accessor
// S gives the request's structure (rf / coff / loff / cflags / cadd / cdrop) and the classes of its
// strings (ns / aa / capadd / capdrop / lk / lv(l, j) / img(c, j)) with img layout `il` and nlv()
// classes per label value. Each walk returns the rejected slots of its families.

// walk A: pod-privileged + psp-capabilities (validation, then mutation), containers in order.
// *mut_out gets the mutated-and-not-rejected psp-capabilities slots.
template <class S>
KW_HD uint64_t walk_privileged_caps(const S& src, const SlotView& sv, uint64_t r, const ViolSink& vs, uint64_t* mut_out) {
  const SlotHdr& h = *sv.h;
  uint64_t rej = 0, mut = 0;
  const uint64_t privany = h.priv[0] | h.priv[1] | h.priv[2] | h.priv[3];
  if ((src.rf(r) & KW_REQ_HAS_PODSPEC) && (privany | h.caps)) {
    const uint32_t cb = src.coff(r), ce = src.coff(r + 1);
    const uint32_t kfirst = src.cadd(cb);
    for (uint32_t c = cb; c < ce; ++c) {
      const uint32_t fl = src.cflags(c);
      const uint64_t pv = priv_viol(h, fl) & ~rej;
      vs.put(pv, KW_R_PRIVILEGED, c - cb);
      rej |= pv;
      if (h.caps) {
        const uint32_t k0 = src.cadd(c), k1 = src.cadd(c + 1);
        uint64_t addm = 0, dropm = 0;
        for (uint32_t k = k0; k < k1; ++k) {
          const uint32_t cls = src.capadd(k);
          addm |= bit_of(sv.capmb(cls));
          const uint64_t nw = (h.caps_strict ? sv.row(T_NACAP, cls) : 0ull) & ~rej;
          vs.put(nw, KW_R_CAP_NOT_ALLOWED, k - kfirst);  // index in the request's add lists, flattened
          rej |= nw;
        }
        for (uint32_t k = src.cdrop(c), k1d = src.cdrop(c + 1); k < k1d; ++k) dropm |= bit_of(sv.capmb(src.capdrop(k)));
        mut |= caps_mutation(sv, addm, dropm);
      }
    }
  }
  *mut_out = mut & ~rej;
  return rej;
}

// walk B: psp-apparmor + trusted-repos, containers in order.
template <class S>
KW_HD uint64_t walk_apparmor_images(const S& src, const SlotView& sv, uint64_t r, const ViolSink& vs) {
  const SlotHdr& h = *sv.h;
  uint64_t rej = 0;
  if ((src.rf(r) & KW_REQ_HAS_PODSPEC) && (h.aa | h.trs)) {
    const uint32_t cb = src.coff(r), ce = src.coff(r + 1);
    for (uint32_t c = cb; c < ce; ++c) {
      const uint32_t ci = c - cb;
      const uint32_t fl = src.cflags(c);
      if (h.aa && (fl & KW_CTR_HAS_APPARMOR)) {
        const uint64_t nw = sv.row(T_NAAA, src.aa(c)) & ~rej;
        vs.put(nw, KW_R_APPARMOR, ci);
        rej |= nw;
      }
      if (h.trs && (fl & KW_CTR_HAS_IMAGE)) {
        uint64_t why[5];
        trs_whys(sv, src.il, [&](uint32_t j) { return src.img(c, j); }, why);
        for (uint32_t k = 0; k < 5; ++k) {
          const uint64_t nw = why[k] & h.trs & ~rej;
          vs.put(nw, KW_R_REG_NOT_ALLOWED + k, ci);
          rej |= nw;
        }
      }
    }
  }
  return rej;
}

// V_l of one label: the safe-labels slots that deny its key or whose constraint on it the value fails.
template <class S>
KW_HD uint64_t label_viol(const S& src, const SlotView& sv, uint32_t l) {
  const uint32_t k = src.lk(l);
  if (!k) return 0ull;
  uint64_t v = sv.row(T_DENY, k);
  for (uint32_t j = 0; j < src.nlv(); ++j) {
    const uint32_t c = src.lv(l, j);
    if (c != 0xffffu) v |= sv.row(T_FAIL, c);
  }
  return v;
}

// walk C: safe-labels (denied, then constrained, label by label in object order; then the first
// missing mandatory key, settings order).
template <class S>
KW_HD uint64_t walk_labels(const S& src, const SlotView& sv, uint64_t r, const ViolSink& vs) {
  const SlotHdr& h = *sv.h;
  if (!h.lbl) return 0;
  uint64_t rej = 0, present = 0;
  const uint32_t lb = src.loff(r), le = src.loff(r + 1);
  for (uint32_t l = lb; l < le; ++l) {
    const uint32_t k = src.lk(l);
    if (!k) continue;
    present |= bit_of(sv.lkmb(k));
    const uint64_t den = sv.row(T_DENY, k);
    const uint64_t nv = label_viol(src, sv, l) & ~rej;
    vs.put(nv & den, KW_R_LABEL_DENIED, l - lb);
    vs.put(nv & ~den, KW_R_LABEL_CONSTRAINT, l - lb);
    rej |= nv;
  }
  uint64_t nw = tab_or(sv.mand(), h.mand_union & ~present) & ~rej;
  rej |= nw;
  while (nw) {
    const uint32_t s = kw_ctz64(nw);
    nw &= nw - 1;
    vs.put(1ull << s, KW_R_LABEL_MANDATORY, first_missing(sv, s, present));
  }
  return rej;
}

// walk D: namespace allow-list.
template <class S>
KW_HD uint64_t walk_namespace(const S& src, const SlotView& sv, uint64_t r, const ViolSink& vs) {
  const SlotHdr& h = *sv.h;
  if (!h.ns) return 0;
  const uint64_t ok = (src.rf(r) & KW_REQ_HAS_NAMESPACE) ? sv.row(T_NSOK, src.ns(r)) : 0ull;
  const uint64_t nw = h.ns & ~ok;
  vs.put(nw, KW_R_NAMESPACE, 0);
  return nw;
}

// namespace bypass (service.rs:40-71): an AdmissionRequest in the always-accept namespace
KW_HD inline bool is_bypass(uint32_t rf, uint32_t ns_cls, uint32_t bypass_cls) {
  return bypass_cls != 0 && !(rf & KW_REQ_RAW) && (rf & KW_REQ_HAS_NAMESPACE) && ns_cls == bypass_cls;
}

// Group jump program (kwdev.hpp GOp) over the member results `ok` (bit s: member s accepted and did
// not mutate). Returns the expression's value; *causes = the members rhai would have called that
// rejected (evaluation_environment.rs:979-1042).
KW_HD inline bool run_group_prog(const uint8_t* prog, uint32_t len, uint64_t ok, uint64_t* causes) {
  uint64_t vals = 0, cz = 0;
  uint32_t sp = 0;
  for (uint32_t pc = 0; pc < len;) {
    const uint32_t op = prog[pc++];
    if (op == G_CONST0 || op == G_CONST1 || op == G_CALL) {
      uint64_t v = op == G_CONST1 ? 1ull : 0ull;
      if (op == G_CALL) {
        const uint32_t s = prog[pc++];
        v = (ok >> s) & 1ull;
        if (!v) cz |= 1ull << s;
      }
      vals = (vals & ~(1ull << sp)) | (v << sp);
      ++sp;
    } else if (op == G_NOT) {
      vals ^= 1ull << (sp - 1);
    } else if (op == G_JT || op == G_JF) {
      const uint32_t t = (uint32_t)prog[pc] | ((uint32_t)prog[pc + 1] << 8);
      pc += 2;
      const bool top = (vals >> (sp - 1)) & 1ull;
      if (top == (op == G_JT)) pc = t;
      else --sp;
    } else {  // G_EQ / G_NE
      --sp;
      const uint64_t b = (vals >> sp) & 1ull, a = (vals >> (sp - 1)) & 1ull;
      const uint64_t v = op == G_EQ ? (uint64_t)(a == b) : (uint64_t)(a != b);
      vals = (vals & ~(1ull << (sp - 1))) | (v << (sp - 1));
    }
  }
  *causes = cz;
  return vals & 1ull;
}

// Wide group jump code (G_CALL16 u16 member operands, u32 G_JT / G_JF targets) over any number of
// members and any stack depth: `stack` holds the value bits (u64 words, the caller's scratch),
// ok(s) a member's result, cause(s) records a called member that rejected.
template <class Ok, class Cause>
KW_HD inline bool run_wide_prog(const uint8_t* prog, uint32_t len, uint64_t* stack, Ok ok, Cause cause) {
  uint32_t sp = 0;
  auto put = [&](uint32_t i, uint64_t v) {
    uint64_t& w = stack[i >> 6];
    w = (w & ~(1ull << (i & 63u))) | (v << (i & 63u));
  };
  auto get = [&](uint32_t i) -> uint64_t { return (stack[i >> 6] >> (i & 63u)) & 1ull; };
  for (uint32_t pc = 0; pc < len;) {
    const uint32_t op = prog[pc++];
    if (op == G_CONST0 || op == G_CONST1) {
      put(sp++, op == G_CONST1 ? 1ull : 0ull);
    } else if (op == G_CALL16) {
      const uint32_t s = (uint32_t)prog[pc] | ((uint32_t)prog[pc + 1] << 8);
      pc += 2;
      const uint64_t v = ok(s) ? 1ull : 0ull;
      if (!v) cause(s);
      put(sp++, v);
    } else if (op == G_NOT) {
      put(sp - 1, get(sp - 1) ^ 1ull);
    } else if (op == G_JT || op == G_JF) {
      const uint32_t t = (uint32_t)prog[pc] | ((uint32_t)prog[pc + 1] << 8) | ((uint32_t)prog[pc + 2] << 16) |
                         ((uint32_t)prog[pc + 3] << 24);
      pc += 4;
      const bool top = get(sp - 1) != 0;
      if (top == (op == G_JT)) pc = t;
      else --sp;
    } else {  // G_EQ / G_NE
      --sp;
      const uint64_t b = get(sp), a = get(sp - 1);
      put(sp - 1, op == G_EQ ? (uint64_t)(a == b) : (uint64_t)(a != b));
    }
  }
  return get(0) != 0;
}

// Script bytecode (kwdev.hpp SOp) over the member results: 1 / 0 the bool result, 2 an evaluation
// error (a type mismatch, checked-arithmetic overflow, division by zero, an index out of bounds, an
// unknown name, an engine limit, a non-bool result: the host interpreter words the message).
// `scratch`: run_script_words(prog) u64 words. cause(s) records a called member that rejected.
KW_HD inline uint64_t run_script_words(const uint8_t* prog) {
  const uint32_t* h = (const uint32_t*)prog;  // depth, nvars, arena bytes, code_len, nframes
  return 2ull * h[0] + 2ull * h[1] + 2ull * h[4] + (h[2] + 15u) / 16u * 2u + 1u;
}

namespace sv {
constexpr uint32_t UNIT = 0, BOOL = 1, INT = 2, STR = 3, ARR = 4, ARENA = 256;
}

template <class Ok, class Cause>
KW_HD inline int run_script_prog(const uint8_t* prog, uint64_t* scratch, Ok ok, Cause cause) {
  const uint32_t* h = (const uint32_t*)prog;
  const uint32_t depth = h[0], nvars = h[1], arena_cap = (h[2] + 15u) & ~15u, code_len = h[3], nframes = h[4];
  const uint32_t tnames = h[5];  // program-relative offset of "()booli64stringarray" (type_of)
  const uint8_t* code = prog + kScriptHeader;
  uint64_t* st = scratch;                     // value stack: 2 words a value
  uint64_t* vars = st + 2ull * depth;         // variable slots of every frame
  uint64_t* frames = vars + 2ull * nvars;     // call frames: (return pc | caller fp << 32, sp)
  uint8_t* arena = (uint8_t*)(frames + 2ull * nframes);
  uint32_t sbot = 0, atop = arena_cap;  // strings grow up from 0, array cells down from the cap
  uint32_t alloc = 0, ops = 0, sp = 0, fp = 0, nf = 0;
  auto rd16 = [&](uint32_t pc) { return (uint32_t)code[pc] | ((uint32_t)code[pc + 1] << 8); };
  auto rd32 = [&](uint32_t pc) { return rd16(pc) | (rd16(pc + 2) << 16); };
  auto rd64 = [&](uint32_t pc) { return (uint64_t)rd32(pc) | ((uint64_t)rd32(pc + 4) << 32); };
  auto type = [&](uint32_t i) -> uint32_t { return (uint32_t)(st[2 * i] & 0xffu); };
  auto bytes_of = [&](uint64_t w0, uint64_t w1) -> const uint8_t* { return (w0 & sv::ARENA) ? arena + w1 : prog + w1; };
  auto len_of = [&](uint64_t w0) -> uint32_t { return (uint32_t)(w0 >> 32); };
  auto cells_of = [&](uint64_t w1) -> uint64_t* { return (uint64_t*)(arena + w1); };
  auto set = [&](uint32_t i, uint32_t t, uint64_t v) {
    st[2 * i] = t;
    st[2 * i + 1] = v;
  };
  // charge `n` bytes of a run's kMaxScriptAlloc budget (the host interpreter charges the same)
  auto charge = [&](uint32_t n) {
    if (n > kMaxScriptAlloc - alloc) return false;
    alloc += n;
    return true;
  };
  auto new_str = [&](uint32_t n) -> uint8_t* {  // (charged by the caller)
    if (sbot + n > atop) return nullptr;
    uint8_t* p = arena + sbot;
    sbot += n;
    return p;
  };
  auto new_cells = [&](uint32_t n) -> uint64_t* {
    if (atop < sbot + 16u * n) return nullptr;
    atop -= 16u * n;
    return (uint64_t*)(arena + atop);
  };
  // deep equality: 1 / 0, or -1 when arrays nest deeper than kMaxCompareDepth
  auto veq = [&](uint64_t x0, uint64_t x1, uint64_t y0, uint64_t y1) -> int {
    const uint64_t* fa[kMaxCompareDepth];
    const uint64_t* fb[kMaxCompareDepth];
    uint32_t fn[kMaxCompareDepth];
    uint32_t d = 0;
    for (;;) {
      const uint32_t tx = (uint32_t)(x0 & 0xffu), ty = (uint32_t)(y0 & 0xffu);
      bool eq = tx == ty, descend = false;
      if (eq && (tx == sv::BOOL || tx == sv::INT)) {
        eq = x1 == y1;
      } else if (eq && tx == sv::STR) {
        const uint32_t n = len_of(x0);
        eq = n == len_of(y0);
        const uint8_t *pa = bytes_of(x0, x1), *pb = bytes_of(y0, y1);
        for (uint32_t k = 0; eq && k < n; ++k) eq = pa[k] == pb[k];
      } else if (eq && tx == sv::ARR) {
        const uint32_t n = len_of(x0);
        eq = n == len_of(y0);
        if (eq && n) {
          if (d == kMaxCompareDepth) return -1;
          fa[d] = cells_of(x1);
          fb[d] = cells_of(y1);
          fn[d] = n;
          ++d;
          descend = true;
        }
      }
      if (!eq) return 0;
      (void)descend;
      while (d > 0 && fn[d - 1] == 0) --d;
      if (d == 0) return 1;
      x0 = fa[d - 1][0];
      x1 = fa[d - 1][1];
      y0 = fb[d - 1][0];
      y1 = fb[d - 1][1];
      fa[d - 1] += 2;
      fb[d - 1] += 2;
      --fn[d - 1];
    }
  };
  // decimal text of an i64 into `buf` (20 bytes), returns its length
  auto itoa = [](int64_t v, uint8_t* buf) -> uint32_t {
    uint8_t t[20];
    uint32_t n = 0;
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do {
      t[n++] = (uint8_t)('0' + u % 10u);
      u /= 10u;
    } while (u);
    uint32_t k = 0;
    if (v < 0) buf[k++] = '-';
    while (n) buf[k++] = t[--n];
    return k;
  };
  // to_string of a scalar as (length, bytes in `tmp` or the value's own bytes); false for an array
  auto text_of = [&](uint64_t w0, uint64_t w1, uint8_t* tmp, const uint8_t** p, uint32_t* n) -> bool {
    const uint32_t t = (uint32_t)(w0 & 0xffu);
    if (t == sv::STR) {
      *p = bytes_of(w0, w1);
      *n = len_of(w0);
    } else if (t == sv::UNIT) {
      *p = tmp;
      *n = 0;
    } else if (t == sv::BOOL) {
      const char* s = w1 ? "true" : "false";
      *n = w1 ? 4u : 5u;
      for (uint32_t k = 0; k < *n; ++k) tmp[k] = (uint8_t)s[k];
      *p = tmp;
    } else if (t == sv::INT) {
      *n = itoa((int64_t)w1, tmp);
      *p = tmp;
    } else {
      return false;  // arrays: converting them to text is outside this engine
    }
    return true;
  };
  for (uint32_t pc = 0; pc < code_len;) {
    const uint32_t op = code[pc++];
    switch (op) {
      case S_UNIT: set(sp++, sv::UNIT, 0); break;
      case S_BOOL: set(sp++, sv::BOOL, code[pc++]); break;
      case S_INT:
        set(sp++, sv::INT, rd64(pc));
        pc += 8;
        break;
      case S_STR: {
        const uint32_t off = rd32(pc), len = rd32(pc + 4);
        pc += 8;
        st[2 * sp] = sv::STR | ((uint64_t)len << 32);
        st[2 * sp + 1] = off;
        ++sp;
        break;
      }
      case S_LOAD: {
        const uint32_t v = fp + rd16(pc);
        pc += 2;
        st[2 * sp] = vars[2 * v];
        st[2 * sp + 1] = vars[2 * v + 1];
        ++sp;
        break;
      }
      case S_STORE: {
        const uint32_t v = fp + rd16(pc);
        pc += 2;
        --sp;
        vars[2 * v] = st[2 * sp];
        vars[2 * v + 1] = st[2 * sp + 1];
        break;
      }
      case S_CALL: {
        const uint32_t m = rd32(pc);
        pc += 4;
        const bool v = ok(m);
        if (!v) cause(m);
        set(sp++, sv::BOOL, v ? 1u : 0u);
        break;
      }
      case S_FAIL: return 2;
      case S_NOT:
        if (type(sp - 1) != sv::BOOL) return 2;
        st[2 * (sp - 1) + 1] ^= 1u;
        break;
      case S_NEG:
      case S_POS: {
        if (type(sp - 1) != sv::INT) return 2;
        const int64_t a = (int64_t)st[2 * (sp - 1) + 1];
        if (op == S_NEG) {
          if (a == INT64_MIN) return 2;
          st[2 * (sp - 1) + 1] = (uint64_t)-a;
        }
        break;
      }
      case S_AND:
      case S_OR: {
        const uint32_t t = rd32(pc);
        pc += 4;
        if (type(sp - 1) != sv::BOOL) return 2;
        const bool a = st[2 * (sp - 1) + 1] != 0;
        if (a == (op == S_OR)) pc = t;  // short circuit: the result is the left side
        else --sp;
        break;
      }
      case S_COAL: {
        const uint32_t t = rd32(pc);
        pc += 4;
        if (type(sp - 1) != sv::UNIT) pc = t;
        else --sp;
        break;
      }
      case S_CHKB:
        if (type(sp - 1) != sv::BOOL) return 2;
        break;
      case S_IF: {
        const uint32_t t = rd32(pc);
        pc += 4;
        --sp;
        if (type(sp) != sv::BOOL) return 2;
        if (!st[2 * sp + 1]) pc = t;
        break;
      }
      case S_JMP: pc = rd32(pc); break;
      case S_POP: --sp; break;
      case S_DROP: sp -= rd16(pc); pc += 2; break;
      case S_DROPKEEP: {
        const uint32_t n = rd16(pc);
        pc += 2;
        st[2 * (sp - 1 - n)] = st[2 * (sp - 1)];
        st[2 * (sp - 1 - n) + 1] = st[2 * (sp - 1) + 1];
        sp -= n;
        break;
      }
      case S_END:
        if (sp == 0 || type(sp - 1) != sv::BOOL) return 2;
        return st[2 * (sp - 1) + 1] ? 1 : 0;
      case S_TICK:
        if (++ops > kMaxScriptOps) return 2;
        break;
      case S_ARR: {
        const uint32_t n = rd16(pc);
        pc += 2;
        if (!charge(16u * n)) return 2;
        uint64_t* c = n ? new_cells(n) : nullptr;
        if (n && !c) return 2;
        sp -= n;
        for (uint32_t k = 0; k < 2 * n; ++k) c[k] = st[2 * sp + k];
        st[2 * sp] = sv::ARR | sv::ARENA | ((uint64_t)n << 32);
        st[2 * sp + 1] = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
        ++sp;
        break;
      }
      case S_INDEX: {
        const uint32_t ia = sp - 2, ii = sp - 1;
        if (type(ia) != sv::ARR || type(ii) != sv::INT) return 2;
        const int64_t n = (int64_t)len_of(st[2 * ia]);
        int64_t i = (int64_t)st[2 * ii + 1];
        if (i < 0) i += n;  // (i64::MIN + n stays negative)
        if (i < 0 || i >= n) return 2;
        const uint64_t* c = cells_of(st[2 * ia + 1]) + 2 * i;
        st[2 * ia] = c[0];
        st[2 * ia + 1] = c[1];
        --sp;
        break;
      }
      case S_SETIDX: {
        const uint32_t v = fp + rd16(pc);
        pc += 2;
        const uint32_t ii = sp - 2, iv = sp - 1;
        if ((vars[2 * v] & 0xffu) != sv::ARR || type(ii) != sv::INT) return 2;
        const uint32_t n = len_of(vars[2 * v]);
        int64_t i = (int64_t)st[2 * ii + 1];
        if (i < 0) i += (int64_t)n;
        if (i < 0 || i >= (int64_t)n) return 2;
        if (!charge(16u * n)) return 2;
        uint64_t* c = new_cells(n);
        if (!c) return 2;
        const uint64_t* o = cells_of(vars[2 * v + 1]);
        for (uint32_t k = 0; k < 2 * n; ++k) c[k] = o[k];
        c[2 * i] = st[2 * iv];
        c[2 * i + 1] = st[2 * iv + 1];
        vars[2 * v + 1] = (uint64_t)((uint8_t*)c - arena);
        sp -= 2;
        break;
      }
      case S_INRANGE: {
        const uint32_t incl = code[pc++];
        const uint32_t ix = sp - 3, il = sp - 2, ih = sp - 1;
        if (type(il) != sv::INT || type(ih) != sv::INT || type(ix) != sv::INT) return 2;
        const int64_t x = (int64_t)st[2 * ix + 1], lo = (int64_t)st[2 * il + 1], hi = (int64_t)st[2 * ih + 1];
        set(ix, sv::BOOL, (x >= lo && (incl ? x <= hi : x < hi)) ? 1u : 0u);
        sp -= 2;
        break;
      }
      case S_RCASE: {
        const int64_t lo = (int64_t)rd64(pc), hi = (int64_t)rd64(pc + 8);
        const uint32_t incl = code[pc + 16];
        pc += 17;
        const int64_t x = (int64_t)st[2 * (sp - 1) + 1];
        const bool in = type(sp - 1) == sv::INT && x >= lo && (incl ? x <= hi : x < hi);
        set(sp - 1, sv::BOOL, in ? 1u : 0u);
        break;
      }
      case S_RANGECHK:
        if (type(sp - 1) != sv::INT || type(sp - 2) != sv::INT) return 2;
        break;
      case S_FORR: {
        const uint32_t si = fp + rd16(pc), se = fp + rd16(pc + 2), incl = code[pc + 4], ex = rd32(pc + 5);
        pc += 9;
        const int64_t i = (int64_t)vars[2 * si + 1], e = (int64_t)vars[2 * se + 1];
        if (incl ? i > e : i >= e) {
          pc = ex;
          break;
        }
        set(sp++, sv::INT, (uint64_t)i);
        if (i == INT64_MAX) vars[2 * se + 1] = (uint64_t)(INT64_MAX - 1);  // (inclusive, last value)
        else vars[2 * si + 1] = (uint64_t)(i + 1);
        break;
      }
      case S_FORA: {
        const uint32_t sa = fp + rd16(pc), si = fp + rd16(pc + 2), withi = code[pc + 4], ex = rd32(pc + 5);
        pc += 9;
        if ((vars[2 * sa] & 0xffu) != sv::ARR) return 2;
        const uint64_t i = vars[2 * si + 1];
        if (i >= len_of(vars[2 * sa])) {
          pc = ex;
          break;
        }
        const uint64_t* c = cells_of(vars[2 * sa + 1]) + 2 * i;
        st[2 * sp] = c[0];
        st[2 * sp + 1] = c[1];
        ++sp;
        if (withi) set(sp++, sv::INT, i);
        vars[2 * si + 1] = i + 1;
        break;
      }
      case S_CALLF: {
        const uint32_t at = rd32(pc), nargs = code[pc + 4], cslots = rd16(pc + 5);
        pc += 7;
        if (nf >= nframes) return 2;               // "Stack overflow"
        if (++ops > kMaxScriptOps) return 2;
        sp -= nargs;
        const uint32_t nfp = fp + cslots;
        for (uint32_t k = 0; k < nargs; ++k) {
          vars[2 * (nfp + k)] = st[2 * (sp + k)];
          vars[2 * (nfp + k) + 1] = st[2 * (sp + k) + 1];
        }
        frames[2 * nf] = (uint64_t)pc | ((uint64_t)fp << 32);
        frames[2 * nf + 1] = sp;
        ++nf;
        fp = nfp;
        pc = at;
        break;
      }
      case S_RET: {
        const uint64_t r0 = st[2 * (sp - 1)], r1 = st[2 * (sp - 1) + 1];
        --nf;
        pc = (uint32_t)frames[2 * nf];
        fp = (uint32_t)(frames[2 * nf] >> 32);
        sp = (uint32_t)frames[2 * nf + 1];
        st[2 * sp] = r0;
        st[2 * sp + 1] = r1;
        ++sp;
        break;
      }
      case S_FN: {
        const uint32_t fid = code[pc++];
        if (fid == F_LEN || fid == F_IS_EMPTY || fid == F_TO_STRING || fid == F_TYPE_OF) {
          const uint32_t i = sp - 1, t = type(i);
          const uint64_t w0 = st[2 * i], w1 = st[2 * i + 1];
          if (fid == F_TYPE_OF) {
            const uint32_t o = t == sv::UNIT ? 0u : t == sv::BOOL ? 2u : t == sv::INT ? 6u : t == sv::STR ? 9u : 15u;
            const uint32_t n = t == sv::UNIT ? 2u : t == sv::BOOL ? 4u : t == sv::INT ? 3u : t == sv::STR ? 6u : 5u;
            st[2 * i] = sv::STR | ((uint64_t)n << 32);
            st[2 * i + 1] = tnames + o;
          } else if (fid == F_TO_STRING) {
            if (t == sv::STR) break;
            uint8_t tmp[24];
            const uint8_t* p;
            uint32_t n;
            if (!text_of(w0, w1, tmp, &p, &n)) return 2;
            if (!charge(n)) return 2;
            uint8_t* d = new_str(n);
            if (!d && n) return 2;
            for (uint32_t k = 0; k < n; ++k) d[k] = p[k];
            st[2 * i] = sv::STR | sv::ARENA | ((uint64_t)n << 32);
            st[2 * i + 1] = d ? (uint64_t)(d - arena) : 0u;
          } else {
            uint64_t n;
            if (t == sv::ARR) {
              n = len_of(w0);
            } else if (t == sv::STR) {  // characters: UTF-8 lead bytes
              const uint8_t* p = bytes_of(w0, w1);
              n = 0;
              for (uint32_t k = 0; k < len_of(w0); ++k) n += (p[k] & 0xC0u) != 0x80u;
            } else {
              return 2;
            }
            if (fid == F_LEN) set(i, sv::INT, n);
            else set(i, sv::BOOL, n == 0 ? 1u : 0u);
          }
          break;
        }
        // two arguments: (a, b) on the stack; F_IN is contains(b, a)
        uint32_t ic = sp - 2, ix = sp - 1;
        if (fid == F_IN) {
          ic = sp - 1;
          ix = sp - 2;
        }
        const uint32_t tc = type(ic), tx = type(ix);
        const uint64_t c0 = st[2 * ic], c1 = st[2 * ic + 1], x0 = st[2 * ix], x1 = st[2 * ix + 1];
        uint64_t r = 0;
        if (fid == F_PUSH) {
          if (tc != sv::ARR) return 2;
          const uint32_t n = len_of(c0);
          if (!charge(16u * (n + 1))) return 2;
          uint64_t* c = new_cells(n + 1);
          if (!c) return 2;
          const uint64_t* o = cells_of(c1);
          for (uint32_t k = 0; k < 2 * n; ++k) c[k] = o[k];
          c[2 * n] = x0;
          c[2 * n + 1] = x1;
          st[2 * (sp - 2)] = sv::ARR | sv::ARENA | ((uint64_t)(n + 1) << 32);
          st[2 * (sp - 2) + 1] = (uint64_t)((uint8_t*)c - arena);
          --sp;
          break;
        }
        if (fid == F_CONTAINS || fid == F_IN) {
          if (tc == sv::ARR) {
            const uint64_t* c = cells_of(c1);
            for (uint32_t k = 0; k < len_of(c0) && !r; ++k) {
              const int e = veq(c[2 * k], c[2 * k + 1], x0, x1);
              if (e < 0) return 2;
              r = (uint64_t)e;
            }
          } else if (tc == sv::STR && tx == sv::STR) {
            const uint8_t *hs = bytes_of(c0, c1), *nd = bytes_of(x0, x1);
            const uint32_t hn = len_of(c0), nn = len_of(x0);
            for (uint32_t k = 0; k + nn <= hn && !r; ++k) {
              bool m = true;
              for (uint32_t j = 0; m && j < nn; ++j) m = hs[k + j] == nd[j];
              r = m;
            }
          } else {
            return 2;
          }
        } else {  // F_STARTS_WITH / F_ENDS_WITH
          if (tc != sv::STR || tx != sv::STR) return 2;
          const uint32_t hn = len_of(c0), nn = len_of(x0);
          const uint8_t *hs = bytes_of(c0, c1) + (fid == F_ENDS_WITH && nn <= hn ? hn - nn : 0u), *nd = bytes_of(x0, x1);
          r = nn <= hn;
          for (uint32_t j = 0; r && j < nn; ++j) r = hs[j] == nd[j];
        }
        set(sp - 2, sv::BOOL, r);
        --sp;
        break;
      }
      case S_BIN: {
        const uint32_t b_op = code[pc++];
        const uint32_t ib = sp - 1, ia = sp - 2;
        const uint32_t ta = type(ia), tb = type(ib);
        const uint64_t a0 = st[2 * ia], va = st[2 * ia + 1], b0 = st[2 * ib], vb = st[2 * ib + 1];
        --sp;
        if (b_op == SB_EQ || b_op == SB_NE) {  // different types: not equal (rhai's built-in comparison)
          const int e = veq(a0, va, b0, vb);
          if (e < 0) return 2;
          set(ia, sv::BOOL, (b_op == SB_EQ) == (e == 1) ? 1u : 0u);
          break;
        }
        if (b_op >= SB_LT && b_op <= SB_GE) {
          int c = 0;
          if (ta != tb) {
            set(ia, sv::BOOL, 0);
            break;
          }
          if (ta == sv::INT) {
            c = (int64_t)va < (int64_t)vb ? -1 : (int64_t)va > (int64_t)vb ? 1 : 0;
          } else if (ta == sv::STR) {
            const uint32_t la = len_of(a0), lb = len_of(b0);
            const uint8_t *pa = bytes_of(a0, va), *pb = bytes_of(b0, vb);
            uint32_t k = 0;
            while (k < la && k < lb && pa[k] == pb[k]) ++k;
            c = k < la && k < lb ? (pa[k] < pb[k] ? -1 : 1) : (la < lb ? -1 : la > lb ? 1 : 0);
          } else {
            return 2;
          }
          const bool r = b_op == SB_LT ? c < 0 : b_op == SB_LE ? c <= 0 : b_op == SB_GT ? c > 0 : c >= 0;
          set(ia, sv::BOOL, r ? 1u : 0u);
          break;
        }
        if (b_op <= SB_AND) {  // | ^ &
          if (ta == sv::BOOL && tb == sv::BOOL) {
            const bool a = va != 0, b = vb != 0;
            set(ia, sv::BOOL, (b_op == SB_OR ? (a || b) : b_op == SB_AND ? (a && b) : (a != b)) ? 1u : 0u);
            break;
          }
          if (ta == sv::INT && tb == sv::INT) {
            set(ia, sv::INT, b_op == SB_OR ? (va | vb) : b_op == SB_AND ? (va & vb) : (va ^ vb));
            break;
          }
          return 2;
        }
        if ((b_op == SB_ADD || b_op == SB_ADDA) && ta == sv::ARR) {
          // array + array concatenates; `+=` with anything else pushes it
          const bool app = tb == sv::ARR;
          if (!app && b_op == SB_ADD) return 2;
          const uint32_t na = len_of(a0), nb = app ? len_of(b0) : 1u;
          if (!charge(16u * (na + nb))) return 2;
          uint64_t* c = na + nb ? new_cells(na + nb) : nullptr;
          if (na + nb && !c) return 2;
          const uint64_t* pa = cells_of(va);
          for (uint32_t k = 0; k < 2 * na; ++k) c[k] = pa[k];
          if (app) {
            const uint64_t* pb = cells_of(vb);
            for (uint32_t k = 0; k < 2 * nb; ++k) c[2 * na + k] = pb[k];
          } else {
            c[2 * na] = b0;
            c[2 * na + 1] = vb;
          }
          st[2 * ia] = sv::ARR | sv::ARENA | ((uint64_t)(na + nb) << 32);
          st[2 * ia + 1] = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
          break;
        }
        if ((b_op == SB_ADD || b_op == SB_ADDA) && (ta == sv::STR || tb == sv::STR)) {
          // string + any (the other side as to_string): one new string of the joined length
          uint8_t t1[24], t2[24];
          const uint8_t *pa, *pb;
          uint32_t la, lb;
          if (!text_of(a0, va, t1, &pa, &la) || !text_of(b0, vb, t2, &pb, &lb)) return 2;
          if (!charge(la + lb)) return 2;
          uint8_t* d = new_str(la + lb);
          if (!d && la + lb) return 2;
          for (uint32_t k = 0; k < la; ++k) d[k] = pa[k];
          for (uint32_t k = 0; k < lb; ++k) d[la + k] = pb[k];
          st[2 * ia] = sv::STR | sv::ARENA | ((uint64_t)(la + lb) << 32);
          st[2 * ia + 1] = d ? (uint64_t)(d - arena) : 0u;
          break;
        }
        if (ta != sv::INT || tb != sv::INT) return 2;
        const int64_t a = (int64_t)va, b = (int64_t)vb;
        long long r = 0;
        if (b_op == SB_ADD || b_op == SB_ADDA) {
          if (__builtin_add_overflow(a, b, &r)) return 2;
        } else if (b_op == SB_SUB) {
          if (__builtin_sub_overflow(a, b, &r)) return 2;
        } else if (b_op == SB_MUL) {
          if (__builtin_mul_overflow(a, b, &r)) return 2;
        } else {
          if (b == 0 || (a == INT64_MIN && b == -1)) return 2;
          r = b_op == SB_DIV ? a / b : a % b;
        }
        set(ia, sv::INT, (uint64_t)r);
        break;
      }
      default: return 2;
    }
  }
  return 2;
}

// Verdict word of one output column for one request. rej / mut: the request's rejected and mutated
// slots; vw: its violation words (valid where rej is set); prog: the record's programs (prog_off
// is record-relative); *wide gets the cause mask of a > 15-member group.
KW_HD inline uint32_t column_word(const ColInfo& ci, uint64_t rej, uint64_t mut, uint64_t init, const uint32_t* vw,
                                  const uint8_t* rec, uint64_t* wide) {
  if (ci.kind == CK_PLAIN) {
    if ((rej >> ci.slot) & 1ull) return ci.rejb | vw[ci.slot];
    return ((mut >> ci.slot) & 1ull) ? ci.mutw : ci.okw;
  }
  if (ci.kind == CK_GROUP) {
    const uint64_t mask = ci.nmem >= 64 ? ~0ull : (1ull << ci.nmem) - 1ull;
    const uint64_t ok = (~(rej | mut | init) >> ci.slot) & mask;
    uint64_t causes;
    if (run_group_prog(rec + ci.prog_off, ci.prog_len, ok, &causes)) return ci.okw;
    if (ci.nmem > 15) {  // 16 causes could read as the ARG sentinel
      *wide = causes;
      return ci.rejb | vword(KW_R_GROUP, kArgWide);
    }
    return ci.rejb | vword(KW_R_GROUP, (uint32_t)causes);
  }
  if (ci.kind == CK_TABLE) {
    const uint32_t ok = (uint32_t)((~(rej | mut | init) >> ci.slot) & ((1ull << ci.nmem) - 1ull));
    const uint32_t e = ((const uint32_t*)(rec + ci.prog_off))[ok];
    if (e & 2u) return ci.errw;  // kGtError
    if (e & 1u) return ci.okw;   // kGtValue
    const uint32_t causes = e >> 16;
    if (ci.nmem > 15) {
      *wide = causes;
      return ci.rejb | vword(KW_R_GROUP, kArgWide);
    }
    return ci.rejb | vword(KW_R_GROUP, causes);
  }
  return ci.okw;
}

}  // namespace kw
