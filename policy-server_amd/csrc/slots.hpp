// slots.hpp — bit-parallel evaluation of a policy set against one request.
//
// A validate pass evaluates up to 64 "slots" per request: the selected plain policies, plus the
// members of the selected groups (evaluated eagerly, then combined by the group program like
// PolicyGroupEvaluator::validate [upstream], evaluation_environment.rs:587-651). A slot is one bit
// of a u64. For every pattern bit of a request column the host compiles the set of slots that an
// entity carrying that pattern violates (the SlotHdr tables below). A request is then evaluated by
// walking its entities once, in object order (containers, then labels): each entity ORs its table
// row into a "rejected" mask, and the slots that become rejected record the entity's (reason, arg).
// The first violation per slot wins, which is the families' own order (DESIGN.md §2,
// oracle/kworacle.c fam_*). The cost per request is O(entities + violations), not
// O(policies x entities).
//
// Shared by the device kernel (kernels.hip evaluate_slots_kernel: one lane per request, operands in
// LDS) and the host diagnostic kw_debug_host_walk (capi.cpp), which the CPU test suite uses to
// check the slot compiler against the oracle. The walks are templated on an entity accessor `S`
// (rf / coff / loff / cflags / cadd / cdrop, and m<MASK>(i): the pattern mask of string i).
#pragma once
#include <cstdint>

#include "../../include/kwgpu.h"
#include "kwdev.hpp"

namespace kw {

// Which mask array a classification writes (one u64 per string).
enum MaskArr : uint32_t { M_NS = 0, M_REG, M_TAG, M_IMG, M_CAPADD, M_CAPDROP, M_AA, M_LK, M_LV, NMASK };

constexpr uint32_t kSlots = 64;

// Per-pattern-bit slot tables, each u64[64] indexed by the column's pattern bit.
enum SlotTab : uint32_t {
  ST_NA_CAP = 0,  // COL_CAP: psp-capabilities slots (without "*") that do not allow the capability
  ST_REQD,        // COL_CAP: slots whose required_drop_capabilities lists the capability
  ST_DEFA,        // COL_CAP: slots whose default_add_capabilities lists the capability
  ST_NA_AA,       // COL_AA:  psp-apparmor slots that do not allow the profile
  ST_DENY,        // COL_LK:  safe-labels slots that deny the key
  ST_MAND,        // COL_LK:  safe-labels slots that make the key mandatory
  ST_NSOK,        // COL_NS:  namespace slots that accept the namespace
  ST_RA,          // COL_REG: trusted-repos slots whose registries.allow matches
  ST_RR,          // COL_REG: ... registries.reject
  ST_TR,          // COL_TAG: ... tags.reject
  ST_IA,          // COL_IMG: ... images.allow
  ST_IR,          // COL_IMG: ... images.reject
  NST
};

struct alignas(16) SlotHdr {
  uint64_t caps_strict;  // psp-capabilities slots without "*" in allowed_capabilities
  uint64_t caps;         // every psp-capabilities slot (mutation)
  uint64_t aa, lbl, ns, trs;
  uint64_t has_ra, has_ia;  // trusted-repos slots with a non-empty registries.allow / images.allow
  uint64_t priv[4];         // pod-privileged slots by (skip_init | skip_ephemeral << 1)
  uint64_t init;            // slots whose policy failed to initialise (group members: never ok)
  uint64_t reqd_union, defa_union, mand_union;  // pattern bits some slot lists (COL_CAP, COL_CAP, COL_LK)
  uint64_t cap_all;         // COL_CAP bit of "ALL" (0 = none)
  uint32_t ncols, nslots, nce, bytes;    // bytes: whole record (multiple of 16)
  uint32_t o_ce, o_mand, o_cols, o_cidx;  // byte offsets of the sections from the record start
  uint16_t tab_off[NST];        // byte offset of table k from the record start (0 = not emitted)
  uint16_t ce_off[kSlots + 1];  // constraint entries of label-key bit k: [ce_off[k], ce_off[k+1])
  uint16_t o_csoa;  // column arrays (kind | slot << 8, okw, mutw, rejb), each ncols rounded up to 4 u32
};
static_assert(sizeof(SlotHdr) == 336, "SlotHdr layout");

// safe-labels constrained_labels: the slots that constrain label-key bit k with value pattern
// `vbit` (the settings index of each slot's constraint on k is in the cidx section).
struct alignas(16) ConstrEnt {
  uint64_t slots;
  uint32_t vbit, pad;
};

enum ColKind : uint32_t { CK_CONST = 0, CK_PLAIN = 1, CK_GROUP = 2 };

// One output column (a selected policy). PLAIN: verdict of slot `slot`. GROUP: the postfix program
// at blob offset prog_off over the member slots [slot, slot + nmem). CONST: the word `okw` whatever
// the request (initialisation error, group expression that is not a bool). okw / mutw / rejb: the
// service-level verdict word of an accepted, an accepted-and-mutated and a rejected vanilla response
// (reason/arg bits clear in rejb).
struct alignas(16) ColInfo {
  uint32_t kind, slot, nmem, prog_off, prog_len, okw, mutw, rejb;
};
static_assert(sizeof(ColInfo) == 32, "ColInfo layout");

// Record: SlotHdr | emitted tables u64[64] | ConstrEnt ce[nce] | u32 column arrays[4][ncols↑4]
//         | ColInfo[ncols] | u8 mand[64][16] | u8 cidx[nslots][64]
// The device stages the record up to o_cols in LDS; the rest it reads from the global copy.
// mand[s]: the label-key bits of slot s's mandatory_labels in settings order, 0xff-terminated.
// cidx[s][k]: settings index of slot s's constraint on label-key bit k (read only to format a
// constraint violation).

KW_HD inline uint32_t kw_ctz64(uint64_t x) { return (uint32_t)__builtin_ctzll(x); }
KW_HD inline uint32_t pack2(uint32_t a, uint32_t b) { return ((a < 255u ? a : 255u) << 8) | (b < 255u ? b : 255u); }
KW_HD inline uint32_t pack1(uint32_t a) { return a < 65535u ? a : 65535u; }
KW_HD inline uint32_t vword(uint32_t reason, uint32_t arg) { return (reason << 8) | ((arg & 0xffffu) << 16); }

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

// Record the violation word of every slot in `nw` (the slots this entity rejects first).
KW_HD inline void put_viol(uint32_t* vw, uint64_t nw, uint32_t word) {
  while (nw) {
    vw[kw_ctz64(nw)] = word;
    nw &= nw - 1;
  }
}
// OR of table rows over the set bits of `bits`.
KW_HD inline uint64_t tab_or(const uint64_t* t, uint64_t bits) {
  uint64_t r = 0;
  while (bits) {
    r |= t[kw_ctz64(bits)];
    bits &= bits - 1;
  }
  return r;
}
// AND of table rows over the set bits of `bits`, starting from `all` (no bits: `all`).
KW_HD inline uint64_t tab_and(const uint64_t* t, uint64_t bits, uint64_t all) {
  uint64_t r = all;
  while (bits) {
    r &= t[kw_ctz64(bits)];
    bits &= bits - 1;
  }
  return r;
}

// The record's sections, resolved once (device: LDS pointers; host: the record bytes).
struct SlotView {
  const SlotHdr* h;
  const uint8_t* base;
  KW_HD const uint64_t* tab(uint32_t k) const { return (const uint64_t*)(base + h->tab_off[k]); }
  KW_HD const ConstrEnt* ce() const { return (const ConstrEnt*)(base + h->o_ce); }
  KW_HD const uint8_t* mand() const { return base + h->o_mand; }
  KW_HD const ColInfo* cols() const { return (const ColInfo*)(base + h->o_cols); }
};

// ---- per-entity violation sets, derived entity-parallel before the walks (the walks then only
// apply the first-violation order): an added capability violates the strict psp-capabilities slots
// that allow none of its pattern bits, an AppArmor profile the psp-apparmor slots that do not allow
// it, a label the safe-labels slots whose constraint on its key its value fails (vcon; the slots
// that deny the key are one table read in the walk).
KW_HD inline uint64_t derive_capadd(const SlotView& sv, uint64_t m) {
  return sv.h->caps_strict ? tab_and(sv.tab(ST_NA_CAP), m, sv.h->caps_strict) : 0ull;
}
KW_HD inline uint64_t derive_apparmor(const SlotView& sv, uint64_t m) {
  return sv.h->aa ? tab_and(sv.tab(ST_NA_AA), m, sv.h->aa) : 0ull;
}
KW_HD inline uint64_t derive_label(const SlotView& sv, uint64_t km, uint64_t vm) {
  uint64_t c = 0;
  if (km && sv.h->lbl) {
    const uint32_t kb = kw_ctz64(km);  // label keys are literal patterns: at most one bit
    const ConstrEnt* ce = sv.ce();
    for (uint32_t e = sv.h->ce_off[kb]; e < sv.h->ce_off[kb + 1]; ++e)
      if (!((vm >> ce[e].vbit) & 1ull)) c |= ce[e].slots;
  }
  return c;
}

// ---- walk A: pod-privileged + psp-capabilities (validation, then mutation), containers in order.
// Returns the rejected slots; *mut_out gets the mutated-and-not-rejected psp-capabilities slots.
template <class S>
KW_HD uint64_t walk_privileged_caps(const S& src, const SlotView& sv, uint64_t r, uint32_t* vw, uint64_t* mut_out) {
  const SlotHdr& h = *sv.h;
  uint64_t rej = 0, mut = 0;
  const uint64_t privany = h.priv[0] | h.priv[1] | h.priv[2] | h.priv[3];
  if ((src.rf(r) & KW_REQ_HAS_PODSPEC) && (privany | h.caps)) {
    const uint32_t cb = src.coff(r), ce = src.coff(r + 1);
    for (uint32_t c = cb; c < ce; ++c) {
      const uint32_t ci = c - cb;
      const uint32_t fl = src.cflags(c);
      if ((fl & KW_CTR_PRIVILEGED) && privany) {
        uint64_t cand = h.priv[0];
        if (!(fl & KW_CTR_INIT)) cand |= h.priv[1];
        if (!(fl & KW_CTR_EPHEMERAL)) cand |= h.priv[2];
        if (!(fl & (KW_CTR_INIT | KW_CTR_EPHEMERAL))) cand |= h.priv[3];
        const uint64_t nw = cand & ~rej;
        put_viol(vw, nw, vword(KW_R_PRIVILEGED, pack1(ci)));
        rej |= nw;
      }
      if (h.caps) {
        const uint32_t k0 = src.cadd(c), k1 = src.cadd(c + 1);
        uint64_t addm = 0, dropm = 0;
        for (uint32_t k = k0; k < k1; ++k) {
          addm |= src.template m<M_CAPADD>(k);
          const uint64_t nw = src.vadd(k) & ~rej;
          if (nw) {
            put_viol(vw, nw, vword(KW_R_CAP_NOT_ALLOWED, pack2(ci, k - k0)));
            rej |= nw;
          }
        }
        const uint32_t d0 = src.cdrop(c), d1 = src.cdrop(c + 1);
        for (uint32_t k = d0; k < d1; ++k) dropm |= src.template m<M_CAPDROP>(k);
        if (!(dropm & h.cap_all)) mut |= tab_or(sv.tab(ST_REQD), h.reqd_union & ~dropm);
        mut |= tab_or(sv.tab(ST_DEFA), h.defa_union & ~(addm | dropm));
      }
    }
  }
  *mut_out = mut & h.caps & ~rej;
  return rej;
}

// ---- walk B: psp-apparmor + trusted-repos, containers in order.
template <class S>
KW_HD uint64_t walk_apparmor_images(const S& src, const SlotView& sv, uint64_t r, uint32_t* vw) {
  const SlotHdr& h = *sv.h;
  uint64_t rej = 0;
  if ((src.rf(r) & KW_REQ_HAS_PODSPEC) && (h.aa | h.trs)) {
    const uint32_t cb = src.coff(r), ce = src.coff(r + 1);
    for (uint32_t c = cb; c < ce; ++c) {
      const uint32_t ci = c - cb;
      const uint32_t fl = src.cflags(c);
      if (h.aa && (fl & KW_CTR_HAS_APPARMOR)) {
        const uint64_t nw = src.vaa(c) & ~rej;
        put_viol(vw, nw, vword(KW_R_APPARMOR, pack1(ci)));
        rej |= nw;
      }
      if (h.trs && (fl & KW_CTR_HAS_IMAGE)) {
        const uint64_t reg = src.template m<M_REG>(c), tag = src.template m<M_TAG>(c), img = src.template m<M_IMG>(c);
        // reason precedence within a container (oracle fam_trusted): registry not allowed, registry
        // rejected, tag rejected, image not allowed, image rejected
        uint64_t why[5];
        why[0] = h.has_ra & ~tab_or(sv.tab(ST_RA), reg);
        why[1] = tab_or(sv.tab(ST_RR), reg);
        why[2] = tab_or(sv.tab(ST_TR), tag);
        why[3] = h.has_ia & ~tab_or(sv.tab(ST_IA), img);
        why[4] = tab_or(sv.tab(ST_IR), img);
        for (uint32_t k = 0; k < 5; ++k) {
          const uint64_t nw = why[k] & h.trs & ~rej;
          if (nw) {
            put_viol(vw, nw, vword(KW_R_REG_NOT_ALLOWED + k, pack1(ci)));
            rej |= nw;
          }
        }
      }
    }
  }
  return rej;
}

// ---- walk C: safe-labels (denied, then constrained, label by label in object order; then the
// first missing mandatory key). A constraint violation carries the label-key bit in its low byte
// until column_word resolves the slot's settings index (cidx).
template <class S>
KW_HD uint64_t walk_labels(const S& src, const SlotView& sv, uint64_t r, uint32_t* vw) {
  const SlotHdr& h = *sv.h;
  if (!h.lbl) return 0;
  uint64_t rej = 0;
  const uint32_t lb = src.loff(r), le = src.loff(r + 1);
  uint64_t present = 0;
  for (uint32_t l = lb; l < le; ++l) {
    const uint64_t km = src.template m<M_LK>(l);
    if (!km) continue;
    present |= km;
    const uint32_t li = l - lb;
    uint64_t nw = sv.tab(ST_DENY)[kw_ctz64(km)] & ~rej;
    if (nw) {
      put_viol(vw, nw, vword(KW_R_LABEL_DENIED, pack1(li)));
      rej |= nw;
    }
    nw = src.vcon(l) & ~rej;
    if (nw) {
      put_viol(vw, nw, vword(KW_R_LABEL_CONSTRAINT, pack2(li, 0)) | kw_ctz64(km));
      rej |= nw;
    }
  }
  uint64_t nw = tab_or(sv.tab(ST_MAND), h.mand_union & ~present) & ~rej;
  rej |= nw;
  const uint8_t* mand = sv.mand();
  while (nw) {  // the first missing mandatory key of each such slot, settings order
    const uint32_t s = kw_ctz64(nw);
    nw &= nw - 1;
    uint32_t i = 0;
    for (; i < 16; ++i) {
      const uint32_t kb = mand[s * 16 + i];
      if (kb == 0xffu || !((present >> kb) & 1ull)) break;
    }
    vw[s] = vword(KW_R_LABEL_MANDATORY, i);
  }
  return rej;
}

// ---- walk D: namespace allow-list.
template <class S>
KW_HD uint64_t walk_namespace(const S& src, const SlotView& sv, uint64_t r, uint32_t* vw) {
  const SlotHdr& h = *sv.h;
  if (!h.ns) return 0;
  uint64_t ok = 0;
  if (src.rf(r) & KW_REQ_HAS_NAMESPACE) ok = tab_or(sv.tab(ST_NSOK), src.template m<M_NS>(r));
  const uint64_t nw = h.ns & ~ok;
  put_viol(vw, nw, vword(KW_R_NAMESPACE, 0));
  return nw;
}

// Postfix group program over the member results. Each stack entry carries the set of members rhai
// would have called to produce it (short-circuit && / ||); causes = called members that rejected
// (evaluation_environment.rs:979-1042).
KW_HD inline bool run_group_prog(const uint8_t* prog, uint32_t len, uint32_t ok, uint16_t* gstk, uint32_t gstride,
                                 uint32_t* causes) {
  uint32_t vals = 0;
  int sp = 0;
  for (uint32_t pc = 0; pc < len; ++pc) {
    const uint32_t op = prog[pc];
    if (op <= G_CALL) {
      uint32_t v = op == G_CONST1 ? 1u : 0u, e = 0;
      if (op == G_CALL) {
        const uint32_t s = prog[++pc];
        v = (ok >> s) & 1u;
        e = 1u << s;
      }
      vals = (vals & ~(1u << sp)) | (v << sp);
      gstk[sp * gstride] = (uint16_t)e;
      ++sp;
    } else if (op == G_NOT) {
      vals ^= 1u << (sp - 1);
    } else {
      --sp;
      const uint32_t bv = (vals >> sp) & 1u, av = (vals >> (sp - 1)) & 1u;
      const uint32_t be = gstk[sp * gstride], ae = gstk[(sp - 1) * gstride];
      uint32_t v, e;
      if (op == G_AND) {
        v = av & bv;
        e = ae | (av ? be : 0u);
      } else if (op == G_OR) {
        v = av | bv;
        e = ae | (av ? 0u : be);
      } else if (op == G_EQ) {
        v = av == bv;
        e = ae | be;
      } else {
        v = av != bv;
        e = ae | be;
      }
      vals = (vals & ~(1u << (sp - 1))) | (v << (sp - 1));
      gstk[(sp - 1) * gstride] = (uint16_t)e;
    }
  }
  *causes = (uint32_t)gstk[0] & ~ok & 0xffffu;
  return vals & 1u;
}

// Verdict word of one output column for one request. rej / mut: the request's rejected and mutated
// slots; vw: its violation words (valid where rej is set); blob: the compiled tables (programs);
// cidx: the record's cidx section.
KW_HD inline uint32_t column_word(const ColInfo& ci, uint64_t rej, uint64_t mut, uint64_t init, const uint32_t* vw,
                                  const uint8_t* blob, const uint8_t* cidx, uint16_t* gstk, uint32_t gstride) {
  if (ci.kind == CK_PLAIN) {
    if ((rej >> ci.slot) & 1ull) {
      uint32_t w = vw[ci.slot];
      if (((w >> 8) & 0xffu) == KW_R_LABEL_CONSTRAINT)  // key bit -> the slot's settings index
        w = (w & ~0xffu) | ((uint32_t)cidx[ci.slot * 64u + (w & 63u)] << 16);
      return ci.rejb | w;
    }
    return ((mut >> ci.slot) & 1ull) ? ci.mutw : ci.okw;
  }
  if (ci.kind == CK_GROUP) {
    const uint32_t ok = (uint32_t)((~(rej | mut | init)) >> ci.slot) & ((1u << ci.nmem) - 1u);
    uint32_t causes;
    if (run_group_prog(blob + ci.prog_off, ci.prog_len, ok, gstk, gstride, &causes)) return ci.okw;
    return ci.rejb | vword(KW_R_GROUP, causes);
  }
  return ci.okw;
}

}  // namespace kw
