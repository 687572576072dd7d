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
  // ---- helpers of the standard-package functions (r06; expr.cpp's interpreter states each rule)
  const uint32_t ctab = h[6], nch = h[7];  // the char table (kwdev.hpp): non-ASCII code points
  auto rd32p = [&](uint32_t off) {         // a u32 of the program (little-endian, any alignment)
    return (uint32_t)prog[off] | ((uint32_t)prog[off + 1] << 8) | ((uint32_t)prog[off + 2] << 16) |
           ((uint32_t)prog[off + 3] << 24);
  };
  auto ch_entry = [&](uint32_t c) -> int64_t {  // program offset of c's entry, or -1
    uint32_t lo = 0, hi = nch;
    while (lo < hi) {
      const uint32_t m = (lo + hi) / 2;
      if (rd32p(ctab + m * kChEntry) < c) lo = m + 1;
      else hi = m;
    }
    return lo < nch && rd32p(ctab + lo * kChEntry) == c ? (int64_t)(ctab + lo * kChEntry) : -1;
  };
  auto ch_flags = [&](uint32_t c) -> uint32_t {
    if (c < 0x80u) {
      const bool letter = (c | 0x20u) >= 'a' && (c | 0x20u) <= 'z';
      return ((c >= 9u && c <= 13u) || c == ' ' ? kChWs : 0u) | (letter ? kChCased : 0u) |
             (c == '\'' || c == '.' || c == ':' || c == '^' || c == '`' ? kChIgnorable : 0u);
    }
    const int64_t e = ch_entry(c);
    return e < 0 ? 0u : rd32p((uint32_t)e + 4u);
  };
  auto ch_map = [&](uint32_t c, bool up, uint32_t* m) -> uint32_t {  // full case mapping of c
    if (c < 0x80u) {
      m[0] = up && c >= 'a' && c <= 'z' ? c - 32u : !up && c >= 'A' && c <= 'Z' ? c + 32u : c;
      return 1;
    }
    const int64_t e = ch_entry(c);
    if (e < 0) {
      m[0] = c;
      return 1;
    }
    const uint32_t n = (rd32p((uint32_t)e + 4u) >> (up ? 10 : 8)) & 3u;
    for (uint32_t j = 0; j < n; ++j) m[j] = rd32p((uint32_t)e + (up ? 20u : 8u) + 4u * j);
    return n;
  };
  auto utf8_next = [](const uint8_t* p, uint32_t n, uint32_t k, uint32_t* c) -> uint32_t {
    const uint32_t b = p[k];
    const uint32_t len = b < 0x80u ? 1u : b < 0xE0u ? 2u : b < 0xF0u ? 3u : 4u;
    uint32_t v = len == 1 ? b : len == 2 ? (b & 0x1Fu) : len == 3 ? (b & 0x0Fu) : (b & 0x07u);
    for (uint32_t j = 1; j < len && k + j < n; ++j) v = (v << 6) | (p[k + j] & 0x3Fu);
    *c = v;
    return k + len;
  };
  auto put_utf8_at = [](uint32_t c, uint8_t* d) -> uint32_t {  // bytes of c (written when d)
    const uint32_t n = c < 0x80u ? 1u : c < 0x800u ? 2u : c < 0x10000u ? 3u : 4u;
    if (d) {
      if (n == 1) d[0] = (uint8_t)c;
      else {
        d[0] = (uint8_t)((n == 2 ? 0xC0u : n == 3 ? 0xE0u : 0xF0u) | (c >> (6 * (n - 1))));
        for (uint32_t j = 1; j < n; ++j) d[j] = (uint8_t)(0x80u | ((c >> (6 * (n - 1 - j))) & 0x3Fu));
      }
    }
    return n;
  };
  auto nchars = [](const uint8_t* p, uint32_t n) -> uint32_t {
    uint32_t c = 0;
    for (uint32_t k = 0; k < n; ++k) c += (p[k] & 0xC0u) != 0x80u;
    return c;
  };
  auto char_byte = [](const uint8_t* p, uint32_t n, uint32_t ch) -> uint32_t {  // byte offset of char ch
    uint32_t c = 0;
    for (uint32_t k = 0; k < n; ++k)
      if ((p[k] & 0xC0u) != 0x80u && c++ == ch) return k;
    return n;
  };
  // Σ at bytes [k, k1): preceded by a cased letter and not followed by one (Case_Ignorable skipped)
  auto final_sigma = [&](const uint8_t* p, uint32_t n, uint32_t k, uint32_t k1) -> bool {
    bool fin = false;
    for (uint32_t j = k; j > 0;) {
      uint32_t b = j - 1;
      while (b > 0 && (p[b] & 0xC0u) == 0x80u) --b;
      uint32_t c;
      utf8_next(p, n, b, &c);
      const uint32_t f = ch_flags(c);
      if (!(f & kChIgnorable)) {
        fin = (f & kChCased) != 0;
        break;
      }
      j = b;
    }
    if (!fin) return false;
    for (uint32_t j = k1; j < n;) {
      uint32_t c;
      const uint32_t j1 = utf8_next(p, n, j, &c);
      const uint32_t f = ch_flags(c);
      if (!(f & kChIgnorable)) return (f & kChCased) == 0;
      j = j1;
    }
    return true;
  };
  auto trim_ws = [&](const uint8_t* p, uint32_t* b, uint32_t* e) {  // White_Space off both ends
    while (*b < *e) {
      uint32_t c;
      const uint32_t k1 = utf8_next(p, *e, *b, &c);
      if (!(ch_flags(c) & kChWs)) break;
      *b = k1;
    }
    while (*e > *b) {
      uint32_t s = *e - 1;
      while (s > *b && (p[s] & 0xC0u) == 0x80u) --s;
      uint32_t c;
      utf8_next(p, *e, s, &c);
      if (!(ch_flags(c) & kChWs)) break;
      *e = s;
    }
  };
  // the first match of f at or after byte `from` (an empty f matches at every character boundary)
  auto next_match = [](const uint8_t* p, uint32_t n, const uint8_t* f, uint32_t fn, uint32_t from) -> int64_t {
    for (uint32_t k = from; k + fn <= n; ++k) {
      if (fn == 0) {
        if (k == n || (p[k] & 0xC0u) != 0x80u) return k;
        continue;
      }
      bool m = true;
      for (uint32_t j = 0; m && j < fn; ++j) m = p[k + j] == f[j];
      if (m) return k;
    }
    return -1;
  };
  // the last match of f ending at or before byte `end`
  auto prev_match = [](const uint8_t* p, uint32_t n, const uint8_t* f, uint32_t fn, uint32_t end) -> int64_t {
    if (end < fn) return -1;
    for (uint32_t k = end - fn + 1; k-- > 0;) {
      if (fn == 0) {
        if (k == n || (p[k] & 0xC0u) != 0x80u) return k;
        continue;
      }
      bool m = true;
      for (uint32_t j = 0; m && j < fn; ++j) m = p[k + j] == f[j];
      if (m) return k;
    }
    return -1;
  };
  auto find_bytes = [&](const uint8_t* p, uint32_t n, const uint8_t* f, uint32_t fn, uint32_t from) -> int64_t {
    return fn == 0 ? (from <= n ? (int64_t)from : -1) : next_match(p, n, f, fn, from);
  };
  auto str_slice = [](uint64_t w0, uint32_t b, uint32_t e) -> uint64_t {  // word 0 of bytes [b, e)
    return (w0 & 0xffffffffull) | ((uint64_t)(e - b) << 32);
  };
  auto arr_word = [](uint32_t n) -> uint64_t { return sv::ARR | sv::ARENA | ((uint64_t)n << 32); };
  // rhai's calc_offset_len and the element position of get / set / remove
  auto offset_len = [](uint32_t n, int64_t start, int64_t len, uint32_t* s0, uint32_t* ln) {
    uint32_t s;
    if (start < 0) {
      const uint64_t a = (uint64_t)0 - (uint64_t)start;
      s = a >= n ? 0u : n - (uint32_t)a;
    } else if ((uint64_t)start >= n) {
      *s0 = n;
      *ln = 0;
      return;
    } else {
      s = (uint32_t)start;
    }
    *s0 = s;
    *ln = len <= 0 ? 0u : (uint64_t)len > n - s ? n - s : (uint32_t)len;
  };
  auto elem_index = [](uint32_t n, int64_t i, uint32_t* at) -> bool {
    if (i < 0) {
      const uint64_t a = (uint64_t)0 - (uint64_t)i;
      if (a > n) return false;
      *at = n - (uint32_t)a;
      return true;
    }
    if ((uint64_t)i >= n) return false;
    *at = (uint32_t)i;
    return true;
  };
  auto vless = [&](uint64_t x0, uint64_t x1, uint64_t y0, uint64_t y1) -> bool {  // (one element type)
    const uint32_t t = (uint32_t)(x0 & 0xffu);
    if (t == sv::INT) return (int64_t)x1 < (int64_t)y1;
    if (t == sv::BOOL) return !x1 && y1;
    const uint32_t la = len_of(x0), lb = len_of(y0);
    const uint8_t *pa = bytes_of(x0, x1), *pb = bytes_of(y0, y1);
    uint32_t k = 0;
    while (k < la && k < lb && pa[k] == pb[k]) ++k;
    return k < la && k < lb ? pa[k] < pb[k] : la < lb;
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
      case S_XSTORE: {  // [.., changed receiver, result]: the receiver into a variable, keep the result
        const uint32_t v = fp + rd16(pc);
        pc += 2;
        vars[2 * v] = st[2 * (sp - 2)];
        vars[2 * v + 1] = st[2 * (sp - 2) + 1];
        st[2 * (sp - 2)] = st[2 * (sp - 1)];
        st[2 * (sp - 2) + 1] = st[2 * (sp - 1) + 1];
        --sp;
        break;
      }
      case S_FN: {
        const uint32_t fid = code[pc], na = code[pc + 1] & 0x7fu, mut = code[pc + 1] >> 7;
        pc += 2;
        const uint32_t A = sp - na;  // the arguments are st[A .. sp)
        // the result r (and for a `&mut` function the receiver as changed, rv) replace the arguments
        uint64_t r0 = sv::UNIT, r1 = 0, rv0 = st[2 * A], rv1 = st[2 * A + 1];
        const uint32_t t0 = type(A), t1 = na > 1 ? type(A + 1) : 0u, t2 = na > 2 ? type(A + 2) : 0u;
        const uint64_t a0 = st[2 * A], v0 = st[2 * A + 1];
        const int64_t i1 = na > 1 ? (int64_t)st[2 * (A + 1) + 1] : 0, i2 = na > 2 ? (int64_t)st[2 * (A + 2) + 1] : 0;
        const uint32_t n0 = len_of(a0);
        auto res_int = [&](int64_t x) {
          r0 = sv::INT;
          r1 = (uint64_t)x;
        };
        auto res_bool = [&](bool x) {
          r0 = sv::BOOL;
          r1 = x ? 1u : 0u;
        };
        switch (fid) {
          case F_LEN:
          case F_IS_EMPTY:
          case F_TYPE_OF:
          case F_TO_STRING: {
            if (fid == F_TYPE_OF) {
              const uint32_t o = t0 == sv::UNIT ? 0u : t0 == sv::BOOL ? 2u : t0 == sv::INT ? 6u : t0 == sv::STR ? 9u : 15u;
              const uint32_t n = t0 == sv::UNIT ? 2u : t0 == sv::BOOL ? 4u : t0 == sv::INT ? 3u : t0 == sv::STR ? 6u : 5u;
              r0 = sv::STR | ((uint64_t)n << 32);
              r1 = tnames + o;
            } else if (fid == F_TO_STRING) {
              if (t0 == sv::STR) {
                r0 = a0;
                r1 = v0;
                break;
              }
              uint8_t tmp[24];
              const uint8_t* p;
              uint32_t n;
              if (!text_of(a0, v0, tmp, &p, &n)) return 2;
              if (!charge(n)) return 2;
              uint8_t* d = new_str(n);
              if (!d && n) return 2;
              for (uint32_t k = 0; k < n; ++k) d[k] = p[k];
              r0 = sv::STR | sv::ARENA | ((uint64_t)n << 32);
              r1 = d ? (uint64_t)(d - arena) : 0u;
            } else {
              uint64_t n;
              if (t0 == sv::ARR) n = n0;
              else if (t0 == sv::STR) n = nchars(bytes_of(a0, v0), n0);
              else return 2;
              if (fid == F_LEN) res_int((int64_t)n);
              else res_bool(n == 0);
            }
            break;
          }
          case F_PUSH: {
            if (t0 != sv::ARR) return 2;
            if (!charge(16u * (n0 + 1))) return 2;
            uint64_t* c = new_cells(n0 + 1);
            if (!c) return 2;
            const uint64_t* o = cells_of(v0);
            for (uint32_t k = 0; k < 2 * n0; ++k) c[k] = o[k];
            c[2 * n0] = st[2 * (A + 1)];
            c[2 * n0 + 1] = st[2 * (A + 1) + 1];
            rv0 = arr_word(n0 + 1);
            rv1 = (uint64_t)((uint8_t*)c - arena);
            break;
          }
          case F_CONTAINS:
          case F_IN:
          case F_INDEX_OF:
          case F_INDEX_OF_FROM: {
            // F_IN is contains(b, a): the haystack is the second argument
            const uint32_t ic = fid == F_IN ? A + 1 : A, ix = fid == F_IN ? A : A + 1;
            const uint32_t tc = type(ic), tx = type(ix);
            const uint64_t c0 = st[2 * ic], c1 = st[2 * ic + 1], x0 = st[2 * ix], x1 = st[2 * ix + 1];
            const bool idx = fid == F_INDEX_OF || fid == F_INDEX_OF_FROM;
            if (fid == F_INDEX_OF_FROM && t2 != sv::INT) return 2;
            int64_t found = -1;
            if (tc == sv::ARR) {
              const uint32_t n = len_of(c0);
              uint32_t from = 0, ln;
              if (fid == F_INDEX_OF_FROM) offset_len(n, i2, 0, &from, &ln);
              const uint64_t* c = cells_of(c1);
              for (uint32_t k = from; k < n && found < 0; ++k) {
                const int e = veq(c[2 * k], c[2 * k + 1], x0, x1);
                if (e < 0) return 2;
                if (e) found = k;
              }
            } else if (tc == sv::STR && tx == sv::STR) {
              const uint8_t *hs = bytes_of(c0, c1), *nd = bytes_of(x0, x1);
              const uint32_t hn = len_of(c0), nn = len_of(x0);
              if (!idx) {
                found = find_bytes(hs, hn, nd, nn, 0) < 0 ? -1 : 0;
              } else if (hn) {
                uint32_t from = 0;
                bool none = false;
                if (fid == F_INDEX_OF_FROM) {
                  const uint32_t nc = nchars(hs, hn);
                  if (i2 < 0) {
                    const uint64_t m = (uint64_t)0 - (uint64_t)i2;
                    from = m > nc ? 0u : char_byte(hs, hn, nc - (uint32_t)m);
                  } else if ((uint64_t)i2 >= nc) {
                    none = i2 != 0;
                  } else {
                    from = char_byte(hs, hn, (uint32_t)i2);
                  }
                }
                const int64_t k = none ? -1 : find_bytes(hs, hn, nd, nn, from);
                found = k < 0 ? -1 : (int64_t)nchars(hs, (uint32_t)k);
              }
            } else {
              return 2;
            }
            if (idx) res_int(found);
            else res_bool(found >= 0);
            break;
          }
          case F_STARTS_WITH:
          case F_ENDS_WITH: {
            if (t0 != sv::STR || t1 != sv::STR) return 2;
            const uint32_t hn = n0, nn = len_of(st[2 * (A + 1)]);
            const uint8_t *hs = bytes_of(a0, v0) + (fid == F_ENDS_WITH && nn <= hn ? hn - nn : 0u),
                          *nd = bytes_of(st[2 * (A + 1)], st[2 * (A + 1) + 1]);
            bool m = nn <= hn;
            for (uint32_t j = 0; m && j < nn; ++j) m = hs[j] == nd[j];
            res_bool(m);
            break;
          }
          // ---- integers
          case F_ABS:
          case F_SIGN:
          case F_IS_ZERO:
          case F_IS_ODD:
          case F_IS_EVEN: {
            if (t0 != sv::INT) return 2;
            const int64_t x = (int64_t)v0;
            if (fid == F_ABS) {
              if (x == INT64_MIN) return 2;
              res_int(x < 0 ? -x : x);
            } else if (fid == F_SIGN) {
              res_int(x < 0 ? -1 : x > 0 ? 1 : 0);
            } else {
              res_bool(fid == F_IS_ZERO ? x == 0 : fid == F_IS_ODD ? (x & 1) != 0 : (x & 1) == 0);
            }
            break;
          }
          case F_MAX:
          case F_MIN: {
            if (t0 != sv::INT || t1 != sv::INT) return 2;
            const int64_t x = (int64_t)v0;
            res_int(fid == F_MAX ? (x >= i1 ? x : i1) : (x <= i1 ? x : i1));
            break;
          }
          case F_TO_HEX:
          case F_TO_OCTAL:
          case F_TO_BINARY: {
            if (t0 != sv::INT) return 2;
            const uint32_t bits = fid == F_TO_HEX ? 4u : fid == F_TO_OCTAL ? 3u : 1u;
            uint8_t tmp[64];
            uint32_t n = 0;
            uint64_t u = v0;
            do {
              tmp[n++] = (uint8_t)"0123456789abcdef"[u & ((1u << bits) - 1u)];
              u >>= bits;
            } while (u);
            if (!charge(n)) return 2;
            uint8_t* d = new_str(n);
            if (!d) return 2;
            for (uint32_t k = 0; k < n; ++k) d[k] = tmp[n - 1 - k];
            r0 = sv::STR | sv::ARENA | ((uint64_t)n << 32);
            r1 = (uint64_t)(d - arena);
            break;
          }
          case F_PARSE_INT:
          case F_PARSE_INT_R: {
            if (t0 != sv::STR || (fid == F_PARSE_INT_R && t1 != sv::INT)) return 2;
            const int64_t radix = fid == F_PARSE_INT_R ? i1 : 10;
            if (radix < 2 || radix > 36) return 2;
            const uint8_t* p = bytes_of(a0, v0);
            uint32_t b = 0, e = n0;
            trim_ws(p, &b, &e);
            if (b == e) return 2;
            bool neg = false;
            if (p[b] == '+' || p[b] == '-') {
              neg = p[b] == '-';
              if (++b == e) return 2;
            }
            long long acc = 0;
            for (uint32_t k = b; k < e; ++k) {
              const uint32_t c = p[k];
              const int64_t d = c >= '0' && c <= '9' ? (int64_t)c - '0' : c >= 'a' && c <= 'z' ? (int64_t)c - 'a' + 10
                                : c >= 'A' && c <= 'Z' ? (int64_t)c - 'A' + 10 : 99;
              if (d >= radix) return 2;
              if (__builtin_mul_overflow(acc, (long long)radix, &acc)) return 2;
              if (neg ? __builtin_sub_overflow(acc, (long long)d, &acc) : __builtin_add_overflow(acc, (long long)d, &acc))
                return 2;
            }
            res_int(acc);
            break;
          }
          // ---- strings
          case F_TO_UPPER:
          case F_TO_LOWER:
          case F_MAKE_UPPER:
          case F_MAKE_LOWER: {
            if (t0 != sv::STR) return 2;
            const bool up = fid == F_TO_UPPER || fid == F_MAKE_UPPER;
            const uint8_t* p = bytes_of(a0, v0);
            uint32_t n = 0;
            for (int pass = 0; pass < 2; ++pass) {
              uint8_t* d = nullptr;
              if (pass == 1) {
                if (!charge(n)) return 2;
                d = new_str(n);
                if (!d && n) return 2;
                r0 = sv::STR | sv::ARENA | ((uint64_t)n << 32);
                r1 = d ? (uint64_t)(d - arena) : 0u;
              }
              uint32_t w = 0;
              for (uint32_t k = 0; k < n0;) {
                uint32_t c;
                const uint32_t k1 = utf8_next(p, n0, k, &c);
                uint32_t m[3], nm;
                if (!up && c == 0x3A3u) {  // Σ: ς at the end of a word (Final_Sigma)
                  m[0] = final_sigma(p, n0, k, k1) ? 0x3C2u : 0x3C3u;
                  nm = 1;
                } else {
                  nm = ch_map(c, up, m);
                }
                for (uint32_t j = 0; j < nm; ++j) w += put_utf8_at(m[j], d ? d + w : nullptr);
                k = k1;
              }
              n = w;
            }
            if (fid == F_MAKE_UPPER || fid == F_MAKE_LOWER) {
              rv0 = r0;
              rv1 = r1;
              r0 = sv::UNIT;
              r1 = 0;
            }
            break;
          }
          case F_TRIM: {
            if (t0 != sv::STR) return 2;
            uint32_t b = 0, e = n0;
            trim_ws(bytes_of(a0, v0), &b, &e);
            rv0 = str_slice(a0, b, e);
            rv1 = v0 + b;
            break;
          }
          case F_SUB_STRING:
          case F_SUB_STRING_N:
          case F_CROP:
          case F_CROP_N: {
            const bool n3 = fid == F_SUB_STRING_N || fid == F_CROP_N;
            if (t0 != sv::STR || t1 != sv::INT || (n3 && t2 != sv::INT)) return 2;
            const uint8_t* p = bytes_of(a0, v0);
            const int64_t len = n3 ? i2 : (int64_t)n0;
            const uint32_t nc = nchars(p, n0);
            uint32_t b = 0, e = 0;
            if (nc && len > 0) {
              uint32_t off = 0;
              bool empty = false;
              if (i1 < 0) {
                const uint64_t m = (uint64_t)0 - (uint64_t)i1;
                off = m > nc ? 0u : nc - (uint32_t)m;
              } else if ((uint64_t)i1 >= nc) {
                empty = true;
              } else {
                off = (uint32_t)i1;
              }
              if (!empty) {
                const uint32_t take = (uint64_t)len > nc - off ? nc - off : (uint32_t)len;
                b = char_byte(p, n0, off);
                e = char_byte(p, n0, off + take);
              }
            }
            const uint64_t s0 = str_slice(a0, b, e), s1 = v0 + b;
            if (fid == F_SUB_STRING || fid == F_SUB_STRING_N) {
              r0 = s0;
              r1 = s1;
            } else {
              rv0 = s0;
              rv1 = s1;
            }
            break;
          }
          case F_REPLACE:
          case F_REMOVE: {
            if (fid == F_REMOVE && t0 == sv::ARR) {
              if (t1 != sv::INT) return 2;
              uint32_t at;
              if (!elem_index(n0, i1, &at)) break;
              if (!charge(16u * (n0 - 1))) return 2;
              uint64_t* c = n0 > 1 ? new_cells(n0 - 1) : nullptr;
              if (n0 > 1 && !c) return 2;
              const uint64_t* o = cells_of(v0);
              r0 = o[2 * at];
              r1 = o[2 * at + 1];
              for (uint32_t k = 0, j = 0; k < n0; ++k) {
                if (k == at) continue;
                c[2 * j] = o[2 * k];
                c[2 * j + 1] = o[2 * k + 1];
                ++j;
              }
              rv0 = arr_word(n0 - 1);
              rv1 = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
              break;
            }
            // replace(s, find, sub) / remove(s, sub) = replace(s, sub, "")
            if (t0 != sv::STR || t1 != sv::STR || (fid == F_REPLACE && t2 != sv::STR)) return 2;
            const uint32_t fn = len_of(st[2 * (A + 1)]);
            if (n0 == 0 || (fid == F_REMOVE && fn == 0)) break;
            const uint8_t *p = bytes_of(a0, v0), *f = bytes_of(st[2 * (A + 1)], st[2 * (A + 1) + 1]);
            const uint8_t* sub = fid == F_REPLACE ? bytes_of(st[2 * (A + 2)], st[2 * (A + 2) + 1]) : nullptr;
            const uint32_t sn = fid == F_REPLACE ? len_of(st[2 * (A + 2)]) : 0u;
            uint32_t nm = 0;
            for (int64_t k = next_match(p, n0, f, fn, 0); k >= 0; k = next_match(p, n0, f, fn, (uint32_t)k + (fn ? fn : 1u)))
              ++nm;
            const uint32_t n = n0 - nm * fn + nm * sn;
            if (!charge(n)) return 2;
            uint8_t* d = new_str(n);
            if (!d && n) return 2;
            uint32_t w = 0, from = 0;
            for (int64_t k = next_match(p, n0, f, fn, 0); k >= 0; k = next_match(p, n0, f, fn, (uint32_t)k + (fn ? fn : 1u))) {
              for (uint32_t j = from; j < (uint32_t)k; ++j) d[w++] = p[j];
              for (uint32_t j = 0; j < sn; ++j) d[w++] = sub[j];
              from = (uint32_t)k + fn;
            }
            for (uint32_t j = from; j < n0; ++j) d[w++] = p[j];
            rv0 = sv::STR | sv::ARENA | ((uint64_t)n << 32);
            rv1 = d ? (uint64_t)(d - arena) : 0u;
            break;
          }
          case F_SPLIT_WS:
          case F_SPLIT:
          case F_SPLIT_N:
          case F_SPLIT_REV:
          case F_SPLIT_REV_N: {
            if (fid == F_SPLIT && t0 == sv::ARR && t1 == sv::INT) {  // the array's tail from the index
              uint32_t s0, ln;
              offset_len(n0, i1, INT64_MAX, &s0, &ln);
              r0 = arr_word(n0 - s0);
              r1 = v0 + 16ull * s0;
              rv0 = arr_word(s0);
              break;
            }
            if (t0 != sv::STR) return 2;
            const uint8_t* p = bytes_of(a0, v0);
            if (fid == F_SPLIT && t1 == sv::INT) {  // at a character position
              const uint32_t nc = nchars(p, n0);
              uint32_t at;
              if (i1 <= 0) {
                const uint64_t m = (uint64_t)0 - (uint64_t)i1;
                at = m > nc ? 0u : nc - (uint32_t)m;
              } else {
                at = (uint64_t)i1 > nc ? nc : (uint32_t)i1;
              }
              const uint32_t bb = char_byte(p, n0, at);
              if (!charge(32u)) return 2;
              uint64_t* c = new_cells(2);
              if (!c) return 2;
              c[0] = str_slice(a0, 0, bb);
              c[1] = v0;
              c[2] = str_slice(a0, bb, n0);
              c[3] = v0 + bb;
              r0 = arr_word(2);
              r1 = (uint64_t)((uint8_t*)c - arena);
              break;
            }
            const bool rev = fid == F_SPLIT_REV || fid == F_SPLIT_REV_N, lim = fid == F_SPLIT_N || fid == F_SPLIT_REV_N;
            if (fid != F_SPLIT_WS && t1 != sv::STR) return 2;
            if (lim && t2 != sv::INT) return 2;
            const uint64_t maxp = lim ? (i2 < 1 ? 1ull : (uint64_t)i2) : ~0ull;
            const uint8_t* f = fid == F_SPLIT_WS ? nullptr : bytes_of(st[2 * (A + 1)], st[2 * (A + 1) + 1]);
            const uint32_t fn = fid == F_SPLIT_WS ? 0u : len_of(st[2 * (A + 1)]);
            uint64_t* c = nullptr;
            uint32_t np = 0;
            for (int pass = 0; pass < 2; ++pass) {
              if (pass == 1) {
                if (!charge(16u * np)) return 2;
                c = np ? new_cells(np) : nullptr;
                if (np && !c) return 2;
              }
              uint32_t w = 0;
              auto piece = [&](uint32_t b, uint32_t e) {
                if (c) {
                  c[2 * w] = str_slice(a0, b, e);
                  c[2 * w + 1] = v0 + b;
                }
                ++w;
              };
              if (fid == F_SPLIT_WS) {  // split_whitespace: the non-empty runs between White_Space
                for (uint32_t k = 0; k < n0;) {
                  uint32_t cp, k1 = utf8_next(p, n0, k, &cp);
                  if (ch_flags(cp) & kChWs) {
                    k = k1;
                    continue;
                  }
                  const uint32_t b = k;
                  while (k < n0) {
                    k1 = utf8_next(p, n0, k, &cp);
                    if (ch_flags(cp) & kChWs) break;
                    k = k1;
                  }
                  piece(b, k);
                }
              } else if (!rev) {
                uint32_t from = 0;
                for (int64_t k = next_match(p, n0, f, fn, 0); k >= 0;
                     k = next_match(p, n0, f, fn, (uint32_t)k + (fn ? fn : 1u))) {
                  if (w + 1 == maxp) break;
                  piece(from, (uint32_t)k);
                  from = (uint32_t)k + fn;
                }
                piece(from, n0);
              } else {
                uint32_t to = n0;
                for (int64_t k = prev_match(p, n0, f, fn, n0); k >= 0;
                     k = fn ? prev_match(p, n0, f, fn, (uint32_t)k) : (k == 0 ? -1 : prev_match(p, n0, f, fn, (uint32_t)k - 1))) {
                  if (w + 1 == maxp) break;
                  piece((uint32_t)k + fn, to);
                  to = (uint32_t)k;
                }
                piece(0, to);
              }
              np = w;
            }
            r0 = arr_word(np);
            r1 = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
            break;
          }
          case F_BYTES:
            if (t0 != sv::STR) return 2;
            res_int(n0);
            break;
          // ---- arrays, and the string forms of append / clear / truncate
          case F_APPEND: {
            if (t0 == sv::ARR && t1 == sv::ARR) {
              const uint32_t nb = len_of(st[2 * (A + 1)]);
              if (!charge(16u * (n0 + nb))) return 2;
              uint64_t* c = n0 + nb ? new_cells(n0 + nb) : nullptr;
              if (n0 + nb && !c) return 2;
              const uint64_t *pa = cells_of(v0), *pb = cells_of(st[2 * (A + 1) + 1]);
              for (uint32_t k = 0; k < 2 * n0; ++k) c[k] = pa[k];
              for (uint32_t k = 0; k < 2 * nb; ++k) c[2 * n0 + k] = pb[k];
              rv0 = arr_word(n0 + nb);
              rv1 = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
              break;
            }
            if (t0 != sv::STR) return 2;
            uint8_t tmp[24];
            const uint8_t* pb;
            uint32_t lb;
            if (!text_of(st[2 * (A + 1)], st[2 * (A + 1) + 1], tmp, &pb, &lb)) return 2;
            if (!charge(n0 + lb)) return 2;
            uint8_t* d = new_str(n0 + lb);
            if (!d && n0 + lb) return 2;
            const uint8_t* pa = bytes_of(a0, v0);
            for (uint32_t k = 0; k < n0; ++k) d[k] = pa[k];
            for (uint32_t k = 0; k < lb; ++k) d[n0 + k] = pb[k];
            rv0 = sv::STR | sv::ARENA | ((uint64_t)(n0 + lb) << 32);
            rv1 = d ? (uint64_t)(d - arena) : 0u;
            break;
          }
          case F_INSERT:
          case F_SET:
          case F_REVERSE:
          case F_SPLICE:
          case F_PAD: {
            // an array rebuilt into new cells: n cells from the old ones by the function's rule
            if (t0 != sv::ARR) return 2;
            if ((fid == F_INSERT || fid == F_SET || fid == F_PAD) && t1 != sv::INT) return 2;
            if (fid == F_SPLICE && (t1 != sv::INT || t2 != sv::INT || type(A + 3) != sv::ARR)) return 2;
            uint32_t at = 0, ln = 0, n = n0;
            if (fid == F_INSERT) {
              offset_len(n0, i1, 0, &at, &ln);
              n = n0 + 1;
            } else if (fid == F_SET) {
              if (!elem_index(n0, i1, &at)) break;
            } else if (fid == F_SPLICE) {
              if (n0) offset_len(n0, i1, i2, &at, &ln);
              n = n0 - ln + len_of(st[2 * (A + 3)]);
            } else if (fid == F_PAD) {
              if (i1 <= 0 || (uint64_t)i1 <= n0) break;
              if ((uint64_t)i1 > kMaxScriptAlloc) return 2;
              n = (uint32_t)i1;
            }
            if (!charge(16u * n)) return 2;
            uint64_t* c = n ? new_cells(n) : nullptr;
            if (n && !c) return 2;
            const uint64_t* o = cells_of(v0);
            auto put = [&](uint32_t k, const uint64_t* src) {
              c[2 * k] = src[0];
              c[2 * k + 1] = src[1];
            };
            if (fid == F_INSERT) {
              for (uint32_t k = 0, j = 0; k < n; ++k) put(k, k == at ? &st[2 * (A + 2)] : &o[2 * j++]);
            } else if (fid == F_SET) {
              for (uint32_t k = 0; k < n; ++k) put(k, k == at ? &st[2 * (A + 2)] : &o[2 * k]);
            } else if (fid == F_REVERSE) {
              for (uint32_t k = 0; k < n; ++k) put(k, &o[2 * (n - 1 - k)]);
            } else if (fid == F_SPLICE) {
              const uint32_t m = len_of(st[2 * (A + 3)]);
              const uint64_t* rp = cells_of(st[2 * (A + 3) + 1]);
              uint32_t w = 0;
              for (uint32_t k = 0; k < at; ++k) put(w++, &o[2 * k]);
              for (uint32_t k = 0; k < m; ++k) put(w++, &rp[2 * k]);
              for (uint32_t k = at + ln; k < n0; ++k) put(w++, &o[2 * k]);
            } else {  // pad
              for (uint32_t k = 0; k < n; ++k) put(k, k < n0 ? &o[2 * k] : &st[2 * (A + 2)]);
            }
            rv0 = arr_word(n);
            rv1 = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
            break;
          }
          case F_POP:
          case F_SHIFT:
            if (t0 != sv::ARR) return 2;  // (a string's pop returns a character: refused by name)
            if (n0) {
              const uint64_t* o = cells_of(v0);
              const uint32_t k = fid == F_POP ? n0 - 1 : 0u;
              r0 = o[2 * k];
              r1 = o[2 * k + 1];
              rv0 = arr_word(n0 - 1);
              rv1 = fid == F_POP ? v0 : v0 + 16u;
            }
            break;
          case F_SORT:
          case F_DEDUP: {
            if (t0 != sv::ARR) return 2;
            if (n0 <= 1) break;
            const uint64_t* o = cells_of(v0);
            if (fid == F_SORT) {
              const uint32_t te = (uint32_t)(o[0] & 0xffu);
              for (uint32_t k = 1; k < n0; ++k)
                if ((uint32_t)(o[2 * k] & 0xffu) != te) return 2;
              if (te == sv::ARR || te == sv::UNIT) break;
              if (!charge(16u * n0)) return 2;
              uint64_t* c = new_cells(n0);
              if (!c) return 2;
              for (uint32_t k = 0; k < 2 * n0; ++k) c[k] = o[k];
              for (uint32_t k = 1; k < n0; ++k) {  // insertion sort: stable, as Rust's sort_by
                const uint64_t x0 = c[2 * k], x1 = c[2 * k + 1];
                uint32_t j = k;
                while (j > 0 && vless(x0, x1, c[2 * (j - 1)], c[2 * (j - 1) + 1])) {
                  c[2 * j] = c[2 * (j - 1)];
                  c[2 * j + 1] = c[2 * (j - 1) + 1];
                  --j;
                }
                c[2 * j] = x0;
                c[2 * j + 1] = x1;
              }
              rv0 = arr_word(n0);
              rv1 = (uint64_t)((uint8_t*)c - arena);
              break;
            }
            // dedup: drop each element equal to the last one kept
            uint32_t n = 1, last = 0;
            for (uint32_t k = 1; k < n0; ++k) {
              const int e = veq(o[2 * k], o[2 * k + 1], o[2 * last], o[2 * last + 1]);
              if (e < 0) return 2;
              if (!e) {
                ++n;
                last = k;
              }
            }
            if (!charge(16u * n)) return 2;
            uint64_t* c = new_cells(n);
            if (!c) return 2;
            c[0] = o[0];
            c[1] = o[1];
            last = 0;
            for (uint32_t k = 1, w = 1; k < n0; ++k) {
              if (veq(o[2 * k], o[2 * k + 1], o[2 * last], o[2 * last + 1])) continue;
              c[2 * w] = o[2 * k];
              c[2 * w + 1] = o[2 * k + 1];
              ++w;
              last = k;
            }
            rv0 = arr_word(n);
            rv1 = (uint64_t)((uint8_t*)c - arena);
            break;
          }
          case F_CLEAR:
            if (t0 == sv::ARR) rv0 = arr_word(0);
            else if (t0 == sv::STR) rv0 = str_slice(a0, 0, 0);
            else return 2;
            break;
          case F_TRUNCATE:
          case F_CHOP: {
            if (t1 != sv::INT) return 2;
            if (t0 == sv::STR && fid == F_TRUNCATE) {
              const uint8_t* p = bytes_of(a0, v0);
              if (i1 <= 0) rv0 = str_slice(a0, 0, 0);
              else if ((uint64_t)i1 < nchars(p, n0)) rv0 = str_slice(a0, 0, char_byte(p, n0, (uint32_t)i1));
              break;
            }
            if (t0 != sv::ARR) return 2;
            if (i1 <= 0) {
              rv0 = arr_word(0);
            } else if ((uint64_t)i1 < n0) {
              rv0 = arr_word((uint32_t)i1);
              if (fid == F_CHOP) rv1 = v0 + 16ull * (n0 - (uint32_t)i1);
            }
            break;
          }
          case F_GET: {
            if (t0 != sv::ARR || t1 != sv::INT) return 2;
            uint32_t at;
            if (elem_index(n0, i1, &at)) {
              r0 = cells_of(v0)[2 * at];
              r1 = cells_of(v0)[2 * at + 1];
            }
            break;
          }
          case F_EXTRACT:
          case F_EXTRACT_N:
          case F_DRAIN:
          case F_RETAIN: {
            const bool n3 = fid != F_EXTRACT;
            if (t0 != sv::ARR || t1 != sv::INT || (n3 && t2 != sv::INT)) return 2;
            const int64_t len = n3 ? i2 : INT64_MAX;
            r0 = arr_word(0);
            r1 = 0;
            uint32_t s0 = 0, ln = 0;
            if (n0 && len > 0) offset_len(n0, i1, len, &s0, &ln);
            if (ln == 0) break;
            const uint64_t slice0 = arr_word(ln), slice1 = v0 + 16ull * s0;
            if (fid == F_EXTRACT || fid == F_EXTRACT_N) {
              r0 = slice0;
              r1 = slice1;
              break;
            }
            // drain: the range is the result, the rest a copy; retain: the other way round
            const uint32_t n = n0 - ln;
            if (!charge(16u * n)) return 2;
            uint64_t* c = n ? new_cells(n) : nullptr;
            if (n && !c) return 2;
            const uint64_t* o = cells_of(v0);
            for (uint32_t k = 0, w = 0; k < n0; ++k) {
              if (k >= s0 && k < s0 + ln) continue;
              c[2 * w] = o[2 * k];
              c[2 * w + 1] = o[2 * k + 1];
              ++w;
            }
            const uint64_t rest0 = arr_word(n), rest1 = c ? (uint64_t)((uint8_t*)c - arena) : 0u;
            if (fid == F_DRAIN) {
              r0 = slice0;
              r1 = slice1;
              rv0 = rest0;
              rv1 = rest1;
            } else {
              r0 = rest0;
              r1 = rest1;
              rv0 = slice0;
              rv1 = slice1;
            }
            break;
          }
          default: return 2;
        }
        sp = A;
        if (mut) {
          st[2 * sp] = rv0;
          st[2 * sp + 1] = rv1;
          ++sp;
        }
        st[2 * sp] = r0;
        st[2 * sp + 1] = r1;
        ++sp;
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
        if (b_op == SB_SUB && ta == sv::STR && tb == sv::STR) {  // every occurrence of b removed
          const uint32_t la = len_of(a0), lb = len_of(b0);
          if (la == 0 || lb == 0) break;
          const uint8_t *pa = bytes_of(a0, va), *pb = bytes_of(b0, vb);
          uint32_t nm = 0;
          for (int64_t k = next_match(pa, la, pb, lb, 0); k >= 0; k = next_match(pa, la, pb, lb, (uint32_t)k + lb)) ++nm;
          const uint32_t n = la - nm * lb;
          if (!charge(n)) return 2;
          uint8_t* d = new_str(n);
          if (!d && n) return 2;
          uint32_t w = 0, from = 0;
          for (int64_t k = next_match(pa, la, pb, lb, 0); k >= 0; k = next_match(pa, la, pb, lb, (uint32_t)k + lb)) {
            for (uint32_t j = from; j < (uint32_t)k; ++j) d[w++] = pa[j];
            from = (uint32_t)k + lb;
          }
          for (uint32_t j = from; j < la; ++j) d[w++] = pa[j];
          st[2 * ia] = sv::STR | sv::ARENA | ((uint64_t)n << 32);
          st[2 * ia + 1] = d ? (uint64_t)(d - arena) : 0u;
          break;
        }
        if (ta != sv::INT || tb != sv::INT) return 2;
        const int64_t a = (int64_t)va, b = (int64_t)vb;
        long long r = 0;
        if (b_op == SB_POW || b_op == SB_SHL || b_op == SB_SHR) {  // rhai's checked ** << >> (expr.cpp)
          int64_t y = b;
          uint32_t o = b_op;
          if (o != SB_POW && y < 0) {  // a negative shift shifts the other way
            if (y == INT64_MIN) return 2;
            y = -y;
            o = o == SB_SHL ? SB_SHR : SB_SHL;
          }
          if (o == SB_POW) {
            if (y < 0 || y > (int64_t)0xFFFFFFFFll) return 2;
            long long v = 1;
            for (int64_t k = 0; k < y; ++k) {
              if (__builtin_mul_overflow(v, (long long)a, &v)) return 2;
              if (v == 0 || ((v == 1 || v == -1) && (a == 1 || a == -1))) {
                if (v != 0 && a == -1) v = (y % 2 == 0) ? 1 : -1;
                break;
              }
            }
            r = v;
          } else {
            if (y >= 64) return 2;
            r = o == SB_SHL ? (long long)((uint64_t)a << y) : (long long)(a >> y);
          }
          set(ia, sv::INT, (uint64_t)r);
          break;
        }
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
