// slotplan.cpp — compile a selected policy list into slot-plan records (slotplan.hpp, slots.hpp).
#include "slotplan.hpp"

#include <cstring>
#include <map>

namespace kw {

namespace {

struct Builder {
  SlotHdr h;
  uint64_t tab[NST][kSlots];
  std::map<std::pair<uint32_t, uint32_t>, uint64_t> constr;  // (key bit, value bit) -> slots
  uint8_t cidx[kSlots][64];
  uint8_t mand[kSlots][16];
  std::vector<ColInfo> cols;
  uint32_t nslots = 0;
  bool groups = false;

  Builder() {
    memset(&h, 0, sizeof(h));
    memset(tab, 0, sizeof(tab));
    memset(mand, 0xff, sizeof(mand));
    memset(cidx, 0xff, sizeof(cidx));
  }

  static void each_bit(uint64_t m, uint64_t* t, uint64_t bit) {
    while (m) {
      t[__builtin_ctzll(m)] |= bit;
      m &= m - 1;
    }
  }

  // One evaluated policy (plain column or group member): its family's share of the tables.
  uint32_t add_slot(const DevPolicy& P) {
    const uint32_t s = nslots++;
    const uint64_t bit = 1ull << s;
    if (P.flags & PF_INIT_ERROR) {
      h.init |= bit;
      return s;
    }
    switch (P.family) {
      case FAM_PRIVILEGED: h.priv[P.flags & 3u] |= bit; break;
      case FAM_NAMESPACE:
        h.ns |= bit;
        if (P.nl[0]) each_bit(P.m[0], tab[ST_NSOK], bit);
        break;
      case FAM_TRUSTED_REPOS:
        h.trs |= bit;
        if (P.nl[0]) {
          h.has_ra |= bit;
          each_bit(P.m[0], tab[ST_RA], bit);
        }
        if (P.nl[1]) each_bit(P.m[1], tab[ST_RR], bit);
        if (P.nl[2]) each_bit(P.m[2], tab[ST_TR], bit);
        if (P.nl[3]) {
          h.has_ia |= bit;
          each_bit(P.m[3], tab[ST_IA], bit);
        }
        if (P.nl[4]) each_bit(P.m[4], tab[ST_IR], bit);
        break;
      case FAM_CAPABILITIES:
        h.caps |= bit;
        if (!(P.flags & PF_ALLOW_ALL)) {
          h.caps_strict |= bit;
          each_bit(~P.m[0], tab[ST_NA_CAP], bit);  // allowed U default_add
        }
        each_bit(P.m[1], tab[ST_REQD], bit);
        h.reqd_union |= P.m[1];
        each_bit(P.m[2], tab[ST_DEFA], bit);
        h.defa_union |= P.m[2];
        h.cap_all |= P.m[3];
        break;
      case FAM_APPARMOR:
        h.aa |= bit;
        each_bit(~P.m[0], tab[ST_NA_AA], bit);
        break;
      case FAM_LABELS:
        h.lbl |= bit;
        each_bit(P.m[0], tab[ST_DENY], bit);
        for (uint32_t k = 0; k < P.n_constr && k < 16; ++k) {
          const uint32_t kb = P.idx[16 + k] & 63u;
          constr[{kb, P.idx[32 + k] & 63u}] |= bit;
          cidx[s][kb] = (uint8_t)k;
        }
        for (uint32_t k = 0; k < P.n_mand && k < 16; ++k) {
          tab[ST_MAND][P.idx[k] & 63u] |= bit;
          h.mand_union |= 1ull << (P.idx[k] & 63u);
          mand[s][k] = P.idx[k];
        }
        break;
      default: break;  // FAM_NONE: no violation possible (eval_family default)
    }
    return s;
  }

  std::vector<uint8_t> emit() {
    bool emit_tab[NST] = {};
    emit_tab[ST_NA_CAP] = emit_tab[ST_REQD] = emit_tab[ST_DEFA] = h.caps != 0;
    emit_tab[ST_NA_AA] = h.aa != 0;
    emit_tab[ST_DENY] = emit_tab[ST_MAND] = h.lbl != 0;
    emit_tab[ST_NSOK] = h.ns != 0;
    emit_tab[ST_RA] = emit_tab[ST_RR] = emit_tab[ST_TR] = emit_tab[ST_IA] = emit_tab[ST_IR] = h.trs != 0;
    std::vector<ConstrEnt> ce;
    uint32_t k0 = 0;
    for (auto& [key, slots] : constr) {  // sorted by key bit
      const uint32_t kb = key.first;
      while (k0 <= kb) h.ce_off[k0++] = (uint16_t)ce.size();
      ConstrEnt e;
      memset(&e, 0, sizeof(e));
      e.slots = slots;
      e.vbit = key.second;
      ce.push_back(e);
    }
    while (k0 <= kSlots) h.ce_off[k0++] = (uint16_t)ce.size();
    uint32_t off = sizeof(SlotHdr);
    for (uint32_t k = 0; k < NST; ++k) {
      h.tab_off[k] = emit_tab[k] ? (uint16_t)off : 0;
      if (emit_tab[k]) off += sizeof(tab[k]);
    }
    h.o_ce = off;
    off += (uint32_t)(ce.size() * sizeof(ConstrEnt));
    // the device stages everything up to o_cols: the column arrays are the staged form of the
    // column records (P3 reads 4 columns per array with one 16-B LDS load) and the mandatory-key
    // lists (1 KB; P2 reads one per missing-mandatory slot of a request, a dependent chain that
    // global latency would serialise). ColInfo and cidx stay in global memory (group / constant
    // columns, the constraint index of a constraint violation)
    const uint32_t cs_n = ((uint32_t)cols.size() + 3u) & ~3u;
    off = (off + 15u) & ~15u;
    h.o_csoa = (uint16_t)off;
    off += 16u * cs_n;
    h.o_mand = h.lbl ? off : 0;
    if (h.lbl) off += sizeof(mand);
    h.o_cols = off;
    off += (uint32_t)(cols.size() * sizeof(ColInfo));
    off = (off + 15u) & ~15u;
    h.o_cidx = 0;
    if (h.lbl) {
      h.o_cidx = off;
      off += nslots * 64u;
      off = (off + 15u) & ~15u;
    }
    h.ncols = (uint32_t)cols.size();
    h.nslots = nslots;
    h.nce = (uint32_t)ce.size();
    h.bytes = off;
    std::vector<uint8_t> rec(off, 0);
    memcpy(rec.data(), &h, sizeof(h));
    for (uint32_t k = 0; k < NST; ++k)
      if (emit_tab[k]) memcpy(rec.data() + h.tab_off[k], tab[k], sizeof(tab[k]));
    if (!ce.empty()) memcpy(rec.data() + h.o_ce, ce.data(), ce.size() * sizeof(ConstrEnt));
    if (h.lbl) memcpy(rec.data() + h.o_mand, mand, sizeof(mand));
    if (!cols.empty()) memcpy(rec.data() + h.o_cols, cols.data(), cols.size() * sizeof(ColInfo));
    uint32_t* cs = (uint32_t*)(rec.data() + h.o_csoa);
    for (uint32_t j = 0; j < (uint32_t)cols.size(); ++j) {
      cs[j] = cols[j].kind | (cols[j].slot << 8);
      cs[cs_n + j] = cols[j].okw;
      cs[2 * cs_n + j] = cols[j].mutw;
      cs[3 * cs_n + j] = cols[j].rejb;
    }
    if (h.lbl) memcpy(rec.data() + h.o_cidx, cidx, (size_t)nslots * 64u);
    return rec;
  }
};

}  // namespace

Status build_slot_chunks(const Env& E, const int32_t* pols, uint32_t npol, int origin, std::vector<SlotChunk>* out) {
  out->clear();
  const DevHeader* H = (const DevHeader*)E.blob.data();
  const DevPolicy* dp = (const DevPolicy*)(E.blob.data() + H->policy_off);
  const int32_t* mem = (const int32_t*)(E.blob.data() + H->member_off);
  // slots a column needs: a plain policy 1, a group its members, a constant column none
  // Plain policies whose compiled settings are identical share one slot: the column words carry
  // mode and allowedToMutate, the slot only what the family computes. This is the compiled form of
  // the reference's module-digest sharing (evaluation_environment.rs:400-418), one level further:
  // equal settings, not only an equal module, evaluate once per request.
  auto slot_key = [&](const DevPolicy& P) {
    DevPolicy k = P;
    k.mode = k.a2m = 0;
    k.prog_off = k.prog_len = k.member_off = k.nmembers = k.pad0 = 0;
    memset(k.pad1, 0, sizeof(k.pad1));
    return std::string((const char*)&k, sizeof(k));
  };
  std::map<std::string, uint32_t> shared;  // slot key -> slot of the current chunk
  auto need = [&](int32_t p) -> uint32_t {
    const DevPolicy& P = dp[p];
    if (P.flags & PF_INIT_ERROR) return 0;
    if (P.family == FAM_GROUP) return (P.flags & PF_EXPR_ERROR) ? 0u : P.nmembers;
    return shared.count(slot_key(P)) ? 0u : 1u;
  };
  uint32_t j = 0;
  while (j < npol) {
    Builder b;
    shared.clear();
    SlotChunk ch;
    ch.col0 = j;
    while (j < npol && b.cols.size() < kSlots) {
      const int32_t p = pols[j];
      if (p < 0 || (size_t)p >= E.pol.size()) return {KW_E_ARG, "policy index out of range"};
      if (b.nslots + need(p) > kSlots) break;
      const DevPolicy& P = dp[p];
      ColInfo ci;
      memset(&ci, 0, sizeof(ci));
      if (P.flags & PF_INIT_ERROR) {  // PolicyInitialization -> reject 500 (service.rs:78-91)
        ci.kind = CK_CONST;
        ci.okw = ci.mutw = ci.rejb = kInitErrorWord;
      } else if (P.family == FAM_GROUP && (P.flags & PF_EXPR_ERROR)) {
        ci.kind = CK_CONST;
        ci.okw = ci.mutw = ci.rejb = finish_word(P.mode, P.a2m, origin, KW_R_GROUP_EXPR, 0, false);
      } else if (P.family == FAM_GROUP) {
        ci.kind = CK_GROUP;
        ci.slot = b.nslots;
        ci.nmem = P.nmembers;
        for (uint32_t s = 0; s < P.nmembers; ++s) b.add_slot(dp[mem[P.member_off + s]]);
        ci.prog_off = H->prog_off + P.prog_off;
        ci.prog_len = P.prog_len;
        ci.okw = finish_word(P.mode, P.a2m, origin, 0, 0, false);
        ci.mutw = ci.okw;
        ci.rejb = finish_word(P.mode, P.a2m, origin, KW_R_GROUP, 0, false) & ~0xff00u;
        b.groups = true;
      } else {
        ci.kind = CK_PLAIN;
        const std::string key = slot_key(P);
        auto it = shared.find(key);
        ci.slot = it != shared.end() ? it->second : (shared[key] = b.add_slot(P));
        ci.okw = finish_word(P.mode, P.a2m, origin, 0, 0, false);
        ci.mutw = finish_word(P.mode, P.a2m, origin, 0, 0, true);
        ci.rejb = finish_word(P.mode, P.a2m, origin, 1, 0, false) & ~0xff00u;
      }
      b.cols.push_back(ci);
      ++j;
    }
    if (j == ch.col0) return {KW_E_ARG, "a policy needs more than 64 evaluation slots"};
    ch.ncols = j - ch.col0;
    ch.nslots = b.nslots;
    ch.groups = b.groups;
    ch.rec = b.emit();
    const SlotHdr* sh = (const SlotHdr*)ch.rec.data();
    ch.staged = sh->o_cols;
    out->push_back(std::move(ch));
  }
  return {};
}

}  // namespace kw
