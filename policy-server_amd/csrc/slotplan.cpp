// slotplan.cpp — compile a selected policy list into slot-plan records (slotplan.hpp, slots.hpp).
#include "slotplan.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>

namespace kw {

namespace {

// Per-pattern slot masks of one column (pattern id -> slots), folded into per-class rows at emit.
using PMask = std::vector<uint64_t>;

struct Builder {
  const Env& E;
  SlotHdr h;
  uint32_t nslots = 0;
  std::vector<int32_t> slot_pol;
  std::vector<ColInfo> cols;
  std::vector<uint8_t> progs;
  std::vector<uint32_t> cap_local, mand_local;  // pattern ids holding a local bit
  PMask pm_ns, pm_ra, pm_rr, pm_tr, pm_ia, pm_ir, pm_cap_ok, pm_aa_ok, pm_deny;
  std::vector<uint64_t> fail;  // per COL_LV class
  uint64_t reqd_l[kSlots], defa_l[kSlots], mand_l[kSlots];
  std::vector<std::vector<uint8_t>> mlist;  // per slot
  bool groups = false;
  uint32_t nwide = 0;

  explicit Builder(const Env& e) : E(e) {
    memset(&h, 0, sizeof(h));
    memset(reqd_l, 0, sizeof(reqd_l));
    memset(defa_l, 0, sizeof(defa_l));
    memset(mand_l, 0, sizeof(mand_l));
    pm_ns.assign(E.cols[COL_NS].pats.size(), 0);
    pm_ra.assign(E.cols[COL_REG].pats.size(), 0);
    pm_rr = pm_ra;
    pm_tr.assign(E.cols[COL_TAG].pats.size(), 0);
    pm_ia.assign(E.cols[COL_IMG].pats.size(), 0);
    pm_ir = pm_ia;
    pm_cap_ok.assign(E.cols[COL_CAP].pats.size(), 0);
    pm_aa_ok.assign(E.cols[COL_AA].pats.size(), 0);
    pm_deny.assign(E.cols[COL_LK].pats.size(), 0);
    fail.assign(E.kv.size(), 0);
  }

  static uint32_t local(std::vector<uint32_t>* l, uint32_t pid) {
    for (size_t i = 0; i < l->size(); ++i)
      if ((*l)[i] == pid) return (uint32_t)i;
    l->push_back(pid);
    return (uint32_t)l->size() - 1;
  }
  // local bits a policy would add to this chunk
  uint32_t new_cap_bits(const PolicyRec& P) const {
    if (P.init_error || P.family != FAM_CAPABILITIES) return 0;
    std::vector<uint32_t> l = cap_local;
    for (int k : {1, 2, 3})
      for (uint32_t p : P.pid[k]) local(&l, p);
    return (uint32_t)(l.size() - cap_local.size());
  }
  uint32_t new_mand_bits(const PolicyRec& P) const {
    if (P.init_error || P.family != FAM_LABELS) return 0;
    std::vector<uint32_t> l = mand_local;
    for (uint32_t p : P.pid[1]) local(&l, p);
    return (uint32_t)(l.size() - mand_local.size());
  }

  // One evaluated policy (plain column or group member): its family's share of the tables.
  uint32_t add_slot(int32_t pi) {
    const PolicyRec& P = E.pol[(size_t)pi];
    const uint32_t s = nslots++;
    const uint64_t bit = 1ull << s;
    slot_pol.push_back(pi);
    mlist.emplace_back();
    if (P.init_error) {
      h.init |= bit;
      return s;
    }
    auto mark = [&](PMask& m, const std::vector<uint32_t>& ids) {
      for (uint32_t p : ids) m[p] |= bit;
    };
    switch (P.family) {
      case FAM_PRIVILEGED: h.priv[P.flags & 3u] |= bit; break;
      case FAM_NAMESPACE:
        h.ns |= bit;
        mark(pm_ns, P.pid[0]);
        break;
      case FAM_TRUSTED_REPOS:
        h.trs |= bit;
        if (!P.lists[0].empty()) h.has_ra |= bit;
        if (!P.lists[3].empty()) h.has_ia |= bit;
        mark(pm_ra, P.pid[0]);
        mark(pm_rr, P.pid[1]);
        mark(pm_tr, P.pid[2]);
        mark(pm_ia, P.pid[3]);
        mark(pm_ir, P.pid[4]);
        break;
      case FAM_CAPABILITIES: {
        h.caps |= bit;
        if (!(P.flags & PF_ALLOW_ALL)) {
          h.caps_strict |= bit;
          mark(pm_cap_ok, P.pid[0]);  // allowed_capabilities U default_add_capabilities
          mark(pm_cap_ok, P.pid[2]);
        }
        for (uint32_t p : P.pid[1]) {
          const uint32_t b = local(&cap_local, p);
          reqd_l[b] |= bit;
          h.reqd_union |= 1ull << b;
        }
        for (uint32_t p : P.pid[2]) {
          const uint32_t b = local(&cap_local, p);
          defa_l[b] |= bit;
          h.defa_union |= 1ull << b;
        }
        h.all_bit = 1ull << local(&cap_local, P.pid[3][0]);
        break;
      }
      case FAM_APPARMOR:
        h.aa |= bit;
        mark(pm_aa_ok, P.pid[0]);
        break;
      case FAM_LABELS: {
        h.lbl |= bit;
        mark(pm_deny, P.pid[0]);
        for (uint32_t p : P.pid[1]) {
          const uint32_t b = local(&mand_local, p);
          mand_l[b] |= bit;
          h.mand_union |= 1ull << b;
          mlist[s].push_back((uint8_t)b);
        }
        const ColumnInfo& lk = E.cols[COL_LK];
        for (size_t k = 0; k < P.pid[2].size(); ++k) {
          const uint32_t kc = lk.lit_cls[P.pid[2][k]], re = P.pid[3][k];
          if (kc >= E.kv_of_key.size()) continue;
          for (uint32_t c : E.kv_of_key[kc]) {
            const KvClass& kv = E.kv[c];
            const bool covered = std::find(kv.covered.begin(), kv.covered.end(), re) != kv.covered.end();
            const bool matched = std::find(kv.matched.begin(), kv.matched.end(), re) != kv.matched.end();
            if (covered && !matched) fail[c] |= bit;
          }
        }
        break;
      }
      default: break;  // FAM_NONE: no violation possible
    }
    return s;
  }

  std::vector<uint8_t> emit(uint32_t* staged) {
    const DevHeader* H = (const DevHeader*)E.blob.data();
    std::vector<uint8_t> rec(sizeof(SlotHdr), 0);
    auto align = [&]() {
      while (rec.size() % 16) rec.push_back(0);
    };
    auto table = [&](uint32_t k, Col c, auto row) {
      align();
      h.tab_off[k] = (uint32_t)rec.size();
      const uint32_t n = c == COL_LV ? (uint32_t)E.kv.size() : (uint32_t)E.cols[c].class_pats.size();
      for (uint32_t cls = 0; cls < n; ++cls) {
        const uint64_t v = row(cls);
        rec.insert(rec.end(), (const uint8_t*)&v, (const uint8_t*)&v + 8);
      }
      if (n == 0) rec.resize(rec.size() + 8, 0);
    };
    auto or_row = [&](Col c, const PMask& m) {
      return [&, c](uint32_t cls) {
        uint64_t v = 0;
        for (uint32_t p : E.cols[c].class_pats[cls]) v |= m[p];
        return v;
      };
    };
    if (h.ns) table(T_NSOK, COL_NS, or_row(COL_NS, pm_ns));
    if (h.trs) {
      table(T_RA, COL_REG, or_row(COL_REG, pm_ra));
      table(T_RR, COL_REG, or_row(COL_REG, pm_rr));
      table(T_TR, COL_TAG, or_row(COL_TAG, pm_tr));
      table(T_IA, COL_IMG, or_row(COL_IMG, pm_ia));
      table(T_IR, COL_IMG, or_row(COL_IMG, pm_ir));
    }
    if (h.caps) table(T_NACAP, COL_CAP, [&](uint32_t cls) { return h.caps_strict & ~or_row(COL_CAP, pm_cap_ok)(cls); });
    if (h.aa) table(T_NAAA, COL_AA, [&](uint32_t cls) { return h.aa & ~or_row(COL_AA, pm_aa_ok)(cls); });
    if (h.lbl) {
      table(T_DENY, COL_LK, or_row(COL_LK, pm_deny));
      table(T_FAIL, COL_LV, [&](uint32_t cls) { return fail[cls]; });
    }
    auto bytemap = [&](Col c, const std::vector<uint32_t>& locals) {
      const ColumnInfo& ci = E.cols[c];
      const uint32_t at = (uint32_t)rec.size();
      for (uint32_t cls = 0; cls < (uint32_t)ci.class_pats.size(); ++cls) {
        uint8_t b = 0xff;
        for (uint32_t p : ci.class_pats[cls])
          for (size_t i = 0; i < locals.size(); ++i)
            if (locals[i] == p) b = (uint8_t)i;
        rec.push_back(b);
      }
      align();
      return at;
    };
    // per-local-bit slot tables: only the bits the chunk uses (the record is staged per workgroup)
    if (h.caps) {
      align();
      h.o_capmb = bytemap(COL_CAP, cap_local);
      const size_t nb = std::max<size_t>(cap_local.size(), 1) * 8;
      h.o_reqd = (uint32_t)rec.size();
      rec.insert(rec.end(), (const uint8_t*)reqd_l, (const uint8_t*)reqd_l + nb);
      align();
      h.o_defa = (uint32_t)rec.size();
      rec.insert(rec.end(), (const uint8_t*)defa_l, (const uint8_t*)defa_l + nb);
    }
    if (h.lbl) {
      align();
      h.o_lkmb = bytemap(COL_LK, mand_local);
      h.o_mand = (uint32_t)rec.size();
      rec.insert(rec.end(), (const uint8_t*)mand_l, (const uint8_t*)mand_l + std::max<size_t>(mand_local.size(), 1) * 8);
      align();
      h.o_mlist = (uint32_t)rec.size();
      for (uint32_t s = 0; s < nslots; ++s)
        if (mlist[s].size() == 1) h.mand_one |= 1ull << s;
      rec.resize(rec.size() + 4u * std::max<uint32_t>(nslots, 1), 0);
      for (uint32_t s = 0; s < nslots; ++s) {
        const uint32_t at = (uint32_t)rec.size();
        memcpy(rec.data() + h.o_mlist + 4u * s, &at, 4);
        rec.insert(rec.end(), mlist[s].begin(), mlist[s].end());
        rec.push_back(0xff);
      }
      align();
      static const bool no_mpack = getenv("KW_NO_MPACK") != nullptr;  // A/B knob (kernels built without KW_MAND_BATCH)
      if (!no_mpack) {
        h.o_mpack = (uint32_t)rec.size();  // the first 8 keys of each list, packed (the kernel's fast path)
        rec.resize(rec.size() + 8u * std::max<uint32_t>(nslots, 1), 0xff);
        for (uint32_t s = 0; s < nslots; ++s)
          for (size_t i = 0; i < mlist[s].size() && i < 8; ++i) rec[h.o_mpack + 8u * s + i] = mlist[s][i];
        align();
      }
    }
    // column arrays: the staged form of the column records (P3 reads 4 columns per array with one
    // 16-B LDS load)
    const uint32_t cs_n = ((uint32_t)cols.size() + 3u) & ~3u;
    align();
    h.o_csoa = (uint32_t)rec.size();
    rec.resize(rec.size() + 16u * cs_n, 0);
    uint32_t* cs = (uint32_t*)(rec.data() + h.o_csoa);
    for (uint32_t j = 0; j < (uint32_t)cols.size(); ++j) {
      cs[j] = cols[j].kind | (cols[j].slot << 8);
      cs[cs_n + j] = cols[j].okw;
      cs[2 * cs_n + j] = cols[j].mutw;
      cs[3 * cs_n + j] = cols[j].rejb;
    }
    align();
    *staged = (uint32_t)rec.size();
    h.o_cols = (uint32_t)rec.size();
    h.o_prog = h.o_cols + (uint32_t)(cols.size() * sizeof(ColInfo));
    for (ColInfo& c : cols)
      if (c.kind == CK_GROUP || c.kind == CK_TABLE) c.prog_off += h.o_prog;
    rec.insert(rec.end(), (const uint8_t*)cols.data(), (const uint8_t*)(cols.data() + cols.size()));
    rec.insert(rec.end(), progs.begin(), progs.end());
    align();
    h.ncols = (uint32_t)cols.size();
    h.nslots = nslots;
    h.bytes = (uint32_t)rec.size();
    h.staged = *staged;
    h.nwide = nwide;
    (void)H;
    memcpy(rec.data(), &h, sizeof(h));
    return rec;
  }
};

// Slot-sharing key: what the family computes (mode and allowedToMutate live in the column words).
std::string slot_key(const PolicyRec& P) {
  std::string k;
  k.push_back((char)P.family);
  k.push_back((char)P.flags);
  k.push_back(P.init_error ? 1 : 0);
  for (int i = 0; i < 5; ++i) {
    k.push_back('|');
    for (uint32_t p : P.pid[i]) k.append((const char*)&p, 4);
    if (P.family == FAM_TRUSTED_REPOS || P.family == FAM_LABELS) k.push_back(P.lists[i].empty() ? 'e' : 'n');
  }
  return k;
}

}  // namespace

Status build_slot_chunks(const Env& E, const int32_t* pols, uint32_t npol, int origin, bool rows_mode,
                         std::vector<SlotChunk>* out) {
  out->clear();
  uint32_t wide_next = 0;
  uint32_t j = 0;
  while (j < npol) {
    Builder b(E);
    std::map<std::string, uint32_t> shared;  // slot key -> slot of the current chunk
    SlotChunk ch;
    ch.col0 = j;
    while (j < npol && b.cols.size() < kSlots) {
      const int32_t p = pols[j];
      if (p < 0 || (size_t)p >= E.pol.size()) return {KW_E_ARG, "policy index out of range"};
      const PolicyRec& P = E.pol[(size_t)p];
      // resources the column needs in this chunk: slots and local bits
      uint32_t need = 0, capb = 0, mandb = 0;
      const bool expr_err = P.is_group && (!P.prog.valid || P.prog.eval_error);
      // members (or a split policy's parts) run in their own pass, the combine kernel writes the column
      const bool wide_group = (P.is_group && !expr_err && P.prog.wide) || (!P.parts.empty() && !P.init_error);
      if (P.init_error || wide_group) {
      } else if (P.is_group) {
        if (!expr_err) {
          need = (uint32_t)P.members.size();
          std::vector<uint32_t> cl = b.cap_local, ml = b.mand_local;
          for (int32_t m : P.members) {
            const PolicyRec& M = E.pol[(size_t)m];
            if (M.init_error) continue;
            if (M.family == FAM_CAPABILITIES)
              for (int k : {1, 2, 3})
                for (uint32_t q : M.pid[k]) Builder::local(&cl, q);
            if (M.family == FAM_LABELS)
              for (uint32_t q : M.pid[1]) Builder::local(&ml, q);
          }
          capb = (uint32_t)(cl.size() - b.cap_local.size());
          mandb = (uint32_t)(ml.size() - b.mand_local.size());
        }
      } else if (!shared.count(slot_key(P))) {
        need = 1;
        capb = b.new_cap_bits(P);
        mandb = b.new_mand_bits(P);
      }
      if (b.nslots + need > kSlots || b.cap_local.size() + capb > (size_t)kMaxLocalBits ||
          b.mand_local.size() + mandb > (size_t)kMaxLocalBits)
        break;
      ColInfo ci;
      memset(&ci, 0, sizeof(ci));
      ci.policy = (uint32_t)p;
      ci.wide = ~0u;
      if (P.init_error) {  // PolicyInitialization -> reject 500 (service.rs:78-91)
        ci.kind = CK_CONST;
        ci.okw = ci.mutw = ci.rejb = kInitErrorWord;
      } else if (expr_err) {
        ci.kind = CK_CONST;
        ci.okw = ci.mutw = ci.rejb = finish_word(P.mode, 0, origin, KW_R_GROUP_EXPR, 0, false);
      } else if (wide_group) {  // placeholder: the wide-group combine kernel writes the column
        ci.kind = CK_WIDE;
        ci.okw = ci.mutw = ci.rejb = 0;
      } else if (P.is_group) {
        const bool table = !P.prog.table.empty();
        ci.kind = table ? CK_TABLE : CK_GROUP;
        ci.slot = b.nslots;
        ci.nmem = (uint32_t)P.members.size();
        for (int32_t m : P.members) b.add_slot(m);
        while (table && b.progs.size() % 4) b.progs.push_back(0);  // u32 entries
        ci.prog_off = (uint32_t)b.progs.size();  // rebased to the record at emit
        if (table) {
          ci.prog_len = (uint32_t)(P.prog.table.size() * 4);
          b.progs.insert(b.progs.end(), (const uint8_t*)P.prog.table.data(),
                         (const uint8_t*)(P.prog.table.data() + P.prog.table.size()));
        } else {
          ci.prog_len = (uint32_t)P.prog.code.size();
          b.progs.insert(b.progs.end(), P.prog.code.begin(), P.prog.code.end());
        }
        ci.errw = finish_word(P.mode, 0, origin, KW_R_GROUP_EXPR, 0, false);
        ci.okw = finish_word(P.mode, 0, origin, 0, 0, false);
        ci.mutw = ci.okw;
        ci.rejb = finish_word(P.mode, 0, origin, KW_R_GROUP, 0, false) & ~0xff00u;
        if (ci.nmem > 15) {
          ci.wide = rows_mode ? 0u : wide_next++;
          ++b.nwide;
        }
        b.groups = true;
      } else {
        ci.kind = CK_PLAIN;
        const std::string key = slot_key(P);
        auto it = shared.find(key);
        ci.slot = it != shared.end() ? it->second : (shared[key] = b.add_slot(p));
        ci.okw = finish_word(P.mode, P.allowed_to_mutate, origin, 0, 0, false);
        ci.mutw = finish_word(P.mode, P.allowed_to_mutate, origin, 0, 0, true);
        ci.rejb = finish_word(P.mode, P.allowed_to_mutate, origin, 1, 0, false) & ~0xff00u;
      }
      b.cols.push_back(ci);
      ++j;
    }
    if (j == ch.col0) return {KW_E_ARG, "a policy needs more than 64 evaluation slots"};
    ch.ncols = j - ch.col0;
    ch.nslots = b.nslots;
    ch.groups = b.groups;
    ch.nwide = b.nwide;
    ch.rec = b.emit(&ch.staged);
    out->push_back(std::move(ch));
  }
  return {};
}

}  // namespace kw
