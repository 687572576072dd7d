// capi.cpp — extern "C" implementation of include/kwgpu.h: environment and batch lifetime, HBM
// residency, launch of the hot path (kernels.hip) and the host epilogue (service.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kwgpu.h"
#include "automaton.hpp"
#include "batch.hpp"
#include "env.hpp"
#include "kernels.hpp"
#include "metrics.hpp"
#include "service.hpp"
#include "slotplan.hpp"

using namespace kw;

struct kw_env {
  Env e;
};

namespace kw {

// Requests per tile of the slot kernel: kSlotRows, or KW_SLOT_ROWS (8..64, A/B knob) when set.
uint32_t slot_rows() {
  static const uint32_t r = [] {
    const char* e = getenv("KW_SLOT_ROWS");
    const int v = e ? atoi(e) : 0;
    return (v >= 8 && v <= (int)kSlotRows) ? (uint32_t)v : kSlotRows;
  }();
  return r;
}

// Per-tile entity counts and staged byte ranges of a batch, reduced to a high quantile (tile_stats).
struct TileStats {
  uint32_t ctr = 0, lbl = 0, kadd = 0, kdrop = 0;
  uint32_t bytes[NMASK] = {};
};

// Device copy of a batch: one allocation for the input columns, lazily sized mask / verdict /
// policy-list buffers, a private stream and timing events.
struct DeviceBatch {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* cols = nullptr;
  size_t cols_bytes = 0;
  // device views of the columns
  const uint8_t* req_flags = nullptr;
  const uint32_t *ctr_off = nullptr, *lbl_off = nullptr, *capadd_off = nullptr, *capdrop_off = nullptr;
  const uint8_t* ctr_flags = nullptr;
  struct DCol {
    const uint32_t* off = nullptr;
    const uint8_t* bytes = nullptr;
    uint64_t n = 0;
    uint64_t nbytes = 0;
  } ns, ctr_image, ctr_aa, cap_add, cap_drop, lbl_key, lbl_val;
  uint64_t* masks[NMASK] = {};
  size_t mask_cap[NMASK] = {};
  uint32_t* verdicts = nullptr;
  size_t verdict_cap = 0;
  uint32_t* sched = nullptr;  // slot-kernel tile counters (zeroed once; each launch leaves them zero)
  int32_t* pols = nullptr;
  size_t pols_cap = 0;
  size_t last_verdicts = 0;
  std::vector<int32_t> host_pols;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  // device copies of the last all-pairs pass's per-chunk TileArgs and slot records (read by the
  // kernel from memory, not kernargs); host copies detect a changed plan
  TileArgs* d_tiles = nullptr;
  size_t d_tiles_cap = 0;
  std::vector<TileArgs> h_tiles;
  uint8_t* d_slots = nullptr;
  size_t d_slots_cap = 0;
  std::vector<uint8_t> h_slots;
  // host-built tile descriptors + overflow list, cached for one plan geometry (desc_key)
  TileDesc* desc = nullptr;
  size_t desc_cap = 0;
  uint32_t* overflow = nullptr;  // [count, tile indices...]
  size_t overflow_cap = 0;
  uint32_t n_overflow = 0;
  uint64_t ndesc = 0;  // tile descriptors (halved runs included)
  uint64_t desc_key = 0;
  // slot-kernel tile capacities of this batch (plan_pass)
  bool stats_valid = false;
  std::vector<TileStats> tile_need;  // per-tile entity counts and staged string bytes
  std::vector<TileStats> tile_q;     // their quantiles at kTileQuantiles
  uint64_t cap_key = 0;              // layout inputs of the last capacity choice, and the choice
  int cap_choice = -1;
  ~DeviceBatch() {
    if (device >= 0) (void)hipSetDevice(device);
    (void)hipFree(d_tiles);
    (void)hipFree(d_slots);
    (void)hipFree(desc);
    (void)hipFree(overflow);
    (void)hipFree(cols);
    for (auto* m : masks) (void)hipFree(m);
    (void)hipFree(verdicts);
    (void)hipFree(sched);
    (void)hipFree(pols);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

}  // namespace kw

struct kw_batch {
  Batch b;
  std::unique_ptr<DeviceBatch> dev;
};

namespace {

void put_err(char* buf, size_t cap, const std::string& s) {
  if (!buf || cap == 0) return;
  size_t n = std::min(cap - 1, s.size());
  memcpy(buf, s.data(), n);
  buf[n] = 0;
}

int put_out(const std::string& s, char* buf, size_t cap, size_t* need) {
  if (need) *need = s.size() + 1;
  if (!buf || cap < s.size() + 1) return KW_E_NOSPACE;
  memcpy(buf, s.data(), s.size());
  buf[s.size()] = 0;
  return KW_OK;
}

#define HIPCHK(x)                       \
  do {                                  \
    hipError_t _e = (x);                \
    if (_e != hipSuccess) return KW_E_DEVICE; \
  } while (0)

template <typename T>
int ensure(T** p, size_t* cap, size_t n) {
  if (*cap >= n && *p) return KW_OK;
  (void)hipFree(*p);
  *p = nullptr;
  size_t want = std::max<size_t>(n, 1);
  HIPCHK(hipMalloc((void**)p, want * sizeof(T)));
  *cap = want;
  return KW_OK;
}

int upload_env(kw_env* env, int device) {
  if (device < 0) return KW_OK;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(&env->e.d_blob, env->e.blob.size()));
  HIPCHK(hipMemcpy(env->e.d_blob, env->e.blob.data(), env->e.blob.size(), hipMemcpyHostToDevice));
  env->e.device = device;
  return KW_OK;
}

// Columns a launch needs: which mask arrays the selected policies read.
struct Needs {
  bool m[NMASK] = {};
};

void add_needs(const Env& E, int32_t p, Needs* n) {
  const PolicyRec& r = E.pol[(size_t)p];
  if (E.always_ns) n->m[M_NS] = true;
  switch (r.family) {
    case FAM_NAMESPACE: n->m[M_NS] = true; break;
    case FAM_TRUSTED_REPOS: n->m[M_REG] = n->m[M_TAG] = n->m[M_IMG] = true; break;
    case FAM_CAPABILITIES: n->m[M_CAPADD] = n->m[M_CAPDROP] = true; break;
    case FAM_APPARMOR: n->m[M_AA] = true; break;
    case FAM_LABELS: n->m[M_LK] = n->m[M_LV] = true; break;
    case FAM_GROUP:
      for (int32_t m : r.members) add_needs(E, m, n);
      break;
    default: break;
  }
}

struct PassPlan {
  bool rows_mode = false;
  bool fused = false;
  ClassifyJobs jobs;
  EvalArgs args;
  TileArgs tile;                   // geometry shared by every chunk
  std::vector<SlotChunk> chunks;   // all-pairs mode: column chunks
  std::vector<TileArgs> tiles;     // one per chunk
  std::vector<uint8_t> slot_blob;  // the chunks' slot records, concatenated
  std::vector<uint32_t> slot_at;   // offset of each chunk's record in slot_blob
  uint32_t grid = 0;
  double classify_bytes = 0, evaluate_bytes = 0;
};

Col mask_col(int m) {
  switch (m) {
    case M_NS: return COL_NS;
    case M_REG: return COL_REG;
    case M_TAG: return COL_TAG;
    case M_IMG: return COL_IMG;
    case M_CAPADD:
    case M_CAPDROP: return COL_CAP;
    case M_AA: return COL_AA;
    case M_LK: return COL_LK;
    default: return COL_LV;
  }
}

const DeviceBatch::DCol& mask_strings(const DeviceBatch& D, int m) {
  switch (m) {
    case M_NS: return D.ns;
    case M_REG:
    case M_TAG:
    case M_IMG: return D.ctr_image;
    case M_CAPADD: return D.cap_add;
    case M_CAPDROP: return D.cap_drop;
    case M_AA: return D.ctr_aa;
    case M_LK: return D.lbl_key;
    default: return D.lbl_val;
  }
}

constexpr uint32_t kFusedTableBudget = 48 * 1024;  // DFA chains staged per workgroup
constexpr uint32_t kTileLdsBudget = 160 * 1024;  // slot-kernel LDS per workgroup (gfx950: 160 KB per CU)
constexpr double kTileQuantiles[] = {1.0, 0.99995, 0.9999, 0.9995, 0.999, 0.998};  // capacity candidates

// Per-tile entity counts and staged byte ranges of a batch (kSlotRows-request tiles), reduced to a
// high quantile: the LDS capacities of the slot kernel. Tiles above them (the tail) take the
// overflow path. Computed once per resident batch.

const StrCol& host_strings(const Batch& B, int m);

// What each tile of `rows` requests stages: entity counts and the 16-B aligned byte span of each
// staged string column.
std::vector<TileStats> tile_needs(const Batch& B, uint32_t rows) {
  const uint64_t ntiles = (B.n + rows - 1) / rows;
  std::vector<TileStats> v(ntiles);
  for (uint64_t t = 0; t < ntiles; ++t) {
    const uint64_t r0 = t * rows, r1 = std::min<uint64_t>(B.n, (t + 1) * rows);
    TileStats& st = v[t];
    st.ctr = B.ctr_off[r1] - B.ctr_off[r0];
    st.lbl = B.lbl_off[r1] - B.lbl_off[r0];
    st.kadd = B.capadd_off[B.ctr_off[r1]] - B.capadd_off[B.ctr_off[r0]];
    st.kdrop = B.capdrop_off[B.ctr_off[r1]] - B.capdrop_off[B.ctr_off[r0]];
    for (int m : {M_NS, M_IMG, M_AA, M_CAPADD, M_CAPDROP, M_LK, M_LV}) {
      const StrCol& c = host_strings(B, m);
      uint64_t g0, g1;
      switch (m) {
        case M_NS: g0 = r0; g1 = r1; break;
        case M_CAPADD: g0 = B.capadd_off[B.ctr_off[r0]]; g1 = B.capadd_off[B.ctr_off[r1]]; break;
        case M_CAPDROP: g0 = B.capdrop_off[B.ctr_off[r0]]; g1 = B.capdrop_off[B.ctr_off[r1]]; break;
        case M_LK: case M_LV: g0 = B.lbl_off[r0]; g1 = B.lbl_off[r1]; break;
        default: g0 = B.ctr_off[r0]; g1 = B.ctr_off[r1]; break;
      }
      st.bytes[m] = ((c.off[g1] + 15u) & ~15u) - (c.off[g0] & ~15u);
    }
  }
  return v;
}

// Per-dimension quantile of the tile needs (quantile 1 = the batch maximum).
TileStats tile_quantile(const std::vector<TileStats>& need, double quantile) {
  TileStats st;
  if (need.empty()) return st;
  const uint64_t n = need.size();
  const uint64_t q = quantile >= 1.0 ? n - 1 : (uint64_t)(quantile * (double)(n - 1));
  std::vector<uint32_t> v(n);
  auto quant = [&](auto f) {
    for (uint64_t t = 0; t < n; ++t) v[t] = f(need[t]);
    std::nth_element(v.begin(), v.begin() + (long)q, v.end());
    return v[q];
  };
  st.ctr = quant([](const TileStats& x) { return x.ctr; });
  st.lbl = quant([](const TileStats& x) { return x.lbl; });
  st.kadd = quant([](const TileStats& x) { return x.kadd; });
  st.kdrop = quant([](const TileStats& x) { return x.kdrop; });
  for (int m : {M_NS, M_IMG, M_AA, M_CAPADD, M_CAPDROP, M_LK, M_LV})
    st.bytes[m] = quant([m](const TileStats& x) { return x.bytes[m]; });
  return st;
}

// Build the classification jobs (two-kernel mode) and the evaluation arguments of one pass.
int plan_pass(const kw_env* env, kw_batch* kb, const Needs& need, uint64_t npairs, uint32_t npol, int origin,
              const int32_t* d_pols, const int32_t* d_row_policy, PassPlan* plan) {
  const Env& E = env->e;
  DeviceBatch& D = *kb->dev;
  const Batch& B = kb->b;
  const DevHeader* H = (const DevHeader*)E.blob.data();
  memset(&plan->jobs, 0, sizeof(plan->jobs));
  memset(&plan->args, 0, sizeof(plan->args));
  memset(&plan->tile, 0, sizeof(plan->tile));
  plan->chunks.clear();
  plan->rows_mode = d_row_policy != nullptr;
  auto chain_bytes = [&](uint32_t off) -> uint32_t {
    return off ? ((const DevDfa*)(E.blob.data() + off))->chain_bytes : 0u;
  };
  // literal-eligible masks classify with the column's perfect-hash table in the fused kernel
  auto lit_of = [&](int m) -> uint32_t {
    if (m != M_NS && m != M_AA && m != M_CAPADD && m != M_CAPDROP && m != M_LK) return 0u;
    return H->lit_off[mask_col(m)];
  };
  // what the fused kernel stages for a column: its literal table, else its DFA chain
  // label values classified per key (one small DFA per constrained key) inside the label-key item
  const bool kv = H->kv_off && lit_of(M_LK) && need.m[M_LK] && H->dfa_off[COL_LK];
  auto stage_rec = [&](int m, uint32_t* blob_off) -> uint32_t {
    if (m == M_LV && kv) {
      *blob_off = H->kv_off;
      return H->kv_bytes;
    }
    if (uint32_t lo = lit_of(m)) {
      *blob_off = lo;
      return ((const DevLit*)(E.blob.data() + lo))->bytes;
    }
    *blob_off = H->dfa_off[mask_col(m)];
    return chain_bytes(*blob_off);
  };
  // masks this pass reads, restricted to columns that have patterns
  bool use[NMASK] = {};
  for (int m = 0; m < (int)NMASK; ++m) use[m] = need.m[m] && H->dfa_off[mask_col(m)] != 0;
  for (int m = 0; m < (int)NMASK; ++m)
    if (use[m])
      if (int rc = ensure(&D.masks[m], &D.mask_cap[m], mask_strings(D, m).n)) return rc;

  // fused when every needed chain fits the per-workgroup table budget
  uint32_t table_bytes = 0;
  bool col_staged[NCOL] = {};
  for (int m = 0; m < (int)NMASK; ++m)
    if (use[m] && !col_staged[mask_col(m)]) {
      col_staged[mask_col(m)] = true;
      uint32_t o;
      table_bytes += stage_rec(m, &o);
    }
  plan->fused = !plan->rows_mode && table_bytes <= kFusedTableBudget;
  for (int m : {M_NS, M_AA, M_CAPADD, M_CAPDROP, M_LK})  // the fused classifier is the literal hash
    if (use[m] && !lit_of(m)) plan->fused = false;

  // ---- classify jobs (two-kernel mode and the micro-batch mode)
  ClassifyJobs& J = plan->jobs;
  uint32_t blocks = 0, lds_max = 0;
  double cbytes = 0;
  auto add_job = [&](const DeviceBatch::DCol& c, int mode, std::initializer_list<MaskArr> outs) -> int {
    ClassifyJob job;
    memset(&job, 0, sizeof(job));
    job.off = c.off;
    job.bytes = c.bytes;
    job.n = (uint32_t)c.n;
    job.mode = (uint32_t)mode;
    int k = 0;
    uint32_t pos = 0;
    bool any = false;
    for (MaskArr o : outs) {
      if (use[o]) {
        uint32_t off = H->dfa_off[mask_col(o)];
        job.out[k] = D.masks[o];
        job.dfa[k] = off;
        job.lds_pos[k] = pos;
        pos += chain_bytes(off);
        any = true;
        cbytes += 8.0 * (double)c.n;
      }
      ++k;
    }
    if (!any || c.n == 0) return KW_OK;
    if (J.n >= kMaxJobs) return KW_E_ARG;
    job.lds_bytes = pos;
    uint32_t nb = (uint32_t)std::min<uint64_t>((c.n + kClassifyThreads - 1) / kClassifyThreads, 1024);
    job.block_begin = blocks;
    job.nblocks = nb;
    blocks += nb;
    lds_max = std::max(lds_max, pos);
    cbytes += (double)c.nbytes + 4.0 * (double)(c.n + 1);
    J.j[J.n++] = job;
    return KW_OK;
  };
  if (!plan->fused) {
    int rc;
    if ((rc = add_job(D.ns, 0, {M_NS}))) return rc;
    if ((rc = add_job(D.ctr_image, 1, {M_REG, M_TAG, M_IMG}))) return rc;
    if ((rc = add_job(D.cap_add, 0, {M_CAPADD}))) return rc;
    if ((rc = add_job(D.cap_drop, 0, {M_CAPDROP}))) return rc;
    if ((rc = add_job(D.ctr_aa, 0, {M_AA}))) return rc;
    if ((rc = add_job(D.lbl_key, 0, {M_LK}))) return rc;
    if ((rc = add_job(D.lbl_val, 0, {M_LV}))) return rc;
    J.total_blocks = blocks;
    J.lds_bytes = lds_max <= 96 * 1024 ? lds_max : 0;  // very large automata are read through L1/L2
  }
  plan->classify_bytes = plan->fused ? 0.0 : cbytes;

  // ---- evaluation arguments
  EvalArgs& A = plan->args;
  A.sched = nullptr;  // run_pass sets the slot kernel's tile counters
  A.blob = (const uint8_t*)E.d_blob;
  A.nrows = B.n;
  A.npairs = npairs;
  A.npol = npol;
  A.origin = origin;
  A.pols = d_pols;
  A.row_policy = d_row_policy;
  A.req_flags = D.req_flags;
  A.ctr_off = D.ctr_off;
  A.lbl_off = D.lbl_off;
  A.ctr_flags = D.ctr_flags;
  A.capadd_off = D.capadd_off;
  A.capdrop_off = D.capdrop_off;
  for (int m = 0; m < (int)NMASK; ++m) A.m[m] = use[m] ? D.masks[m] : nullptr;
  A.out = D.verdicts;

  // algorithmic bytes: request headers once, the entity columns and strings the selected
  // policies read, masks (two-kernel mode only) and the verdict words written
  double nc = (double)B.containers(), nl = (double)B.labels(), n = (double)B.n;
  double eb = n * (1 + 4 + 4) + 4.0 * (double)npairs;
  bool ctr = use[M_REG] || use[M_TAG] || use[M_IMG] || use[M_AA] || use[M_CAPADD] || use[M_CAPDROP];
  for (uint32_t j = 0; j < npol && !ctr; ++j) ctr = true;  // every pod-spec family reads ctr_flags
  if (ctr) eb += nc * 1.0;
  if (use[M_CAPADD] || use[M_CAPDROP]) eb += nc * 8.0;
  double strings = 0;
  for (int m = 0; m < (int)NMASK; ++m) {
    if (!use[m]) continue;
    if ((m == M_TAG || m == M_IMG) && use[M_REG]) continue;  // one image column feeds three masks
    if (m == M_IMG && use[M_TAG]) continue;
    const DeviceBatch::DCol& c = mask_strings(D, m);
    strings += (double)c.nbytes + 4.0 * (double)c.n;
  }
  double masks = 0;
  for (int m = 0; m < (int)NMASK; ++m)
    if (use[m]) masks += 8.0 * (double)mask_strings(D, m).n;
  (void)nl;
  plan->evaluate_bytes = plan->fused ? eb + strings : eb + masks;
  if (plan->rows_mode) return KW_OK;

  // ---- slot chunks (all-pairs mode): one slot-kernel launch per chunk of <= 64 slots / columns
  if (!plan->rows_mode) {
    Status st = build_slot_chunks(E, kb->dev->host_pols.data(), npol, origin, &plan->chunks);
    if (!st.ok()) return st.code;
  }

  // ---- tile geometry and LDS layout (slot kernel: kSlotRows requests per tile)
  TileArgs& T = plan->tile;
  auto align = [](uint32_t x) { return (x + 15u) & ~15u; };
  const uint32_t rows = slot_rows();
  if (!D.stats_valid) {
    D.tile_need = tile_needs(B, rows);
    D.tile_q.clear();
    for (double q : kTileQuantiles) D.tile_q.push_back(tile_quantile(D.tile_need, q));
    D.cap_choice = -1;
    D.stats_valid = true;
  }
  uint32_t chain_len[NMASK];  // per-string masks are whole-chain results (image chains walk in one item)
  for (int m = 0; m < (int)NMASK; ++m) chain_len[m] = 1;
  uint32_t slot_bytes = 16, nslots = 1;
  bool groups = false;
  for (const SlotChunk& c : plan->chunks) {
    slot_bytes = std::max<uint32_t>(slot_bytes, c.staged);
    nslots = std::max(nslots, c.nslots);
    groups = groups || c.groups;
  }
  const uint32_t vw_stride = nslots | 1u;  // odd stride: lanes (requests) spread over the banks
  // LDS layout for capacities `ts` (shrunk by `scale` only when over the budget); returns the bytes
  auto layout = [&](const TileStats& ts) -> uint32_t {
    memset(&T, 0, sizeof(T));
    double scale = 1.0;
    for (;;) {
      uint32_t cmax = (uint32_t)std::max(1.0, scale * ts.ctr);
      uint32_t kmax = (uint32_t)std::max(1.0, scale * std::max(ts.kadd, ts.kdrop));
      uint32_t lmax = (uint32_t)std::max(1.0, scale * ts.lbl);
      uint32_t off = 16;
      const uint32_t stage_at = off;
      if (plan->fused) off = align(off + table_bytes);
      T.o_slot = off;
      off = align(off + slot_bytes);
      T.o_rf = off;
      off = align(off + rows);
      T.o_coff = off;
      off = align(off + (rows + 1) * 4);
      T.o_loff = off;
      off = align(off + (rows + 1) * 4);
      T.o_cflags = off;
      off = align(off + cmax + 8);  // staged from the dword holding the first flag
      T.o_cadd = off;
      off = align(off + (cmax + 1) * 4);
      T.o_cdrop = off;
      off = align(off + (cmax + 1) * 4);
      T.use_mask = 0;
      for (int m = 0; m < (int)NMASK; ++m) {
        T.o_m[m] = 0;
        if (use[m]) T.use_mask |= 1u << m;
        if (!use[m] || m == M_LV || m == M_AA) continue;  // AppArmor profiles / label values: into V_c / V_l
        const uint32_t cnt = m == M_NS ? rows : (m == M_CAPADD || m == M_CAPDROP) ? kmax : m == M_LK ? lmax : cmax;
        const bool lit = m == M_NS || m == M_CAPADD || m == M_CAPDROP || m == M_LK;
        T.o_m[m] = off;
        T.mask_cap[m] = cnt;
        off = align(off + cnt * (lit ? 1u : 8u));
      }
      T.o_vadd = T.o_vl = 0;
      if (use[M_CAPADD]) {
        T.o_vadd = off;
        off = align(off + kmax * 8);
      }
      if (use[M_LK]) {
        T.o_vl = off;
        off = align(off + lmax * 8);
      }
      T.o_vc = off;  // V_c per container
      off = align(off + cmax * 8);
      T.o_own_c = off;
      off = align(off + cmax);
      T.o_own_l = off;
      off = align(off + lmax);
      T.o_rej = off;
      off = align(off + rows * 8);
      T.o_mut = off;
      off = align(off + rows * 8);
      T.o_byp = off;
      off = align(off + rows);
      T.o_sa = off;
      off = align(off + NMASK * 4);
      T.o_nx = off;
      off = align(off + 8);
      T.o_gstk = 0;
      if (groups) {
        T.o_gstk = off;
        off = align(off + kMaxGroupStack * kSlotThreads * 2);
      }
      // union: the staged strings (P0-P1) and the violation words (P2-P3)
      const uint32_t u0 = off;
      uint32_t su = u0;
      for (int m = 0; m < (int)NMASK; ++m) T.o_so[m] = T.o_sb[m] = T.sb_cap[m] = 0;
      if (plan->fused)
        for (int m : {M_NS, M_IMG, M_AA, M_CAPADD, M_CAPDROP, M_LK, M_LV}) {
          const bool needm = m == M_IMG ? (use[M_REG] || use[M_TAG] || use[M_IMG]) : use[m];
          if (!needm) continue;
          const DeviceBatch::DCol& sc = mask_strings(D, m);
          const uint32_t cnt = m == M_NS ? rows : (m == M_CAPADD || m == M_CAPDROP) ? kmax : (m == M_LK || m == M_LV) ? lmax : cmax;
          T.o_so[m] = su;
          su = align(su + (cnt + 1) * 4);
          (void)sc;
          T.sb_cap[m] = align((uint32_t)std::min(16384.0, scale * ts.bytes[m]));  // longer tiles take the overflow path
          T.o_sb[m] = su;
          su = align(su + T.sb_cap[m] + 16);  // slack: dword reads may run <= 7 bytes past a string
        }
      T.o_vw = u0;
      T.vw_stride = vw_stride;
      off = std::max(su, align(u0 + rows * vw_stride * 4));
      if (off > kTileLdsBudget && scale > 0.1) {
        scale *= 0.8;
        continue;
      }
      T.rows = rows;
      T.cmax = cmax;
      T.kmax = kmax;
      T.lmax = lmax;
      T.lds_bytes = off;
      // column chains and strings (the overflow kernel reads them in both modes)
      for (int m = 0; m < (int)NMASK; ++m) {
        if (!use[m]) continue;
        T.dfa_head[m] = H->dfa_off[mask_col(m)];
        const DeviceBatch::DCol& sc = mask_strings(D, m);
        T.s_off[m] = sc.off;
        T.s_bytes[m] = sc.bytes;
      }
      // column tables staged once per workgroup (fused)
      if (plan->fused) {
        uint32_t at = stage_at;
        uint32_t col_at[NCOL] = {};
        bool staged[NCOL] = {};
        for (int m = 0; m < (int)NMASK; ++m) {
          if (!use[m]) continue;
          Col c = mask_col(m);
          if (!staged[c]) {
            staged[c] = true;
            col_at[c] = at;
            uint32_t bo;
            const uint32_t nb = stage_rec(m, &bo);
            T.stage_blob[T.nstage] = bo;
            T.stage_lds[T.nstage] = at;
            T.stage_bytes[T.nstage] = nb;
            at += nb;
            ++T.nstage;
          }
          if (lit_of(m)) {
            T.lit_lds[m] = col_at[c];
          } else if (m == M_LV && kv) {
            T.kv_lds = col_at[c];
            T.kv_blob = H->kv_off;
          } else {
            T.dfa_lds[m] = col_at[c];
          }
        }
      }
      break;
    }
    return T.lds_bytes;
  };
  // the batch maximum when it costs no occupancy over the high quantile (no overflow tiles at all)
  auto per_cu = [](uint32_t b) { return std::min<uint32_t>(2048 / kSlotThreads, (160 * 1024) / std::max<uint32_t>(b, 1)); };
  // Capacities: the highest occupancy (workgroups per CU, LDS-bound) whose layout splits at most
  // 2 % of the tiles (a tile beyond the capacities runs as halves, upload_tile_descs), over
  // per-dimension quantiles of the tile needs; at a given occupancy the largest capacities (fewest
  // split tiles). Chosen once per batch and layout signature.
  uint64_t key = ((uint64_t)table_bytes << 40) ^ ((uint64_t)slot_bytes << 20) ^ ((uint64_t)nslots << 8) ^
                 (groups ? 1u : 0u) ^ (plan->fused ? 2u : 0u);
  for (int m = 0; m < (int)NMASK; ++m) key = key * 3 + (use[m] ? 1 : 0);
  if (D.cap_choice < 0 || D.cap_key != key) {
    const uint64_t ntl = D.tile_need.size();
    int best = 0;
    uint32_t best_cu = 0;
    for (int k = 0; k < (int)D.tile_q.size(); ++k) {
      const uint32_t cu = per_cu(layout(D.tile_q[k]));
      if (T.lds_bytes > kTileLdsBudget) continue;
      uint64_t over = 0;  // tiles beyond these capacities (split by the descriptors' fit test)
      for (const TileStats& x : D.tile_need) {
        bool o = x.ctr > T.cmax || x.lbl > T.lmax || x.kadd > T.kmax || x.kdrop > T.kmax;
        for (int m = 0; m < (int)NMASK && !o; ++m) o = T.sb_cap[m] && x.bytes[m] > T.sb_cap[m];
        over += o;
      }
      if (getenv("KW_TILE_DEBUG") && (atoi(getenv("KW_TILE_DEBUG")) & 256))
        fprintf(stderr, "[kw tile] candidate q=%g lds=%u wg/cu=%u split=%llu/%llu\n", kTileQuantiles[k], T.lds_bytes, cu,
                (unsigned long long)over, (unsigned long long)ntl);
      const double max_split = getenv("KW_TILE_SPLIT") ? atof(getenv("KW_TILE_SPLIT")) : 0.02;  // A/B knob
      if (k > 0 && (double)over > max_split * (double)ntl) continue;
      if (cu > best_cu) {
        best = k;
        best_cu = cu;
      }
    }
    D.cap_key = key;
    D.cap_choice = best;
  }
  if (const char* fq = getenv("KW_TILE_QUANTILE"))  // tests / diagnostics: force the capacity quantile
    layout(tile_quantile(D.tile_need, atof(fq)));
  else
    layout(D.tile_q[D.cap_choice]);
  if (T.lds_bytes > kTileLdsBudget) return KW_E_ARG;  // policy set too large for one tile
  if (const char* dbg = getenv("KW_TILE_DEBUG")) T.debug = (uint32_t)atoi(dbg);  // phase ablation (diagnostics)
  if (T.debug & 256u)
    fprintf(stderr, "[kw tile] fused=%d rows=%u cmax=%u kmax=%u lmax=%u lds=%u slot=%u chunks=%zu sb=%u/%u/%u/%u/%u/%u/%u\n",
            (int)plan->fused, T.rows, T.cmax, T.kmax, T.lmax, T.lds_bytes, slot_bytes, plan->chunks.size(), T.sb_cap[M_NS],
            T.sb_cap[M_IMG], T.sb_cap[M_AA], T.sb_cap[M_CAPADD], T.sb_cap[M_CAPDROP], T.sb_cap[M_LK], T.sb_cap[M_LV]);
  for (int m = 0; m < (int)NMASK; ++m) T.chain_len[m] = chain_len[m];
  if (use[M_REG] || use[M_TAG] || use[M_IMG]) {  // one parse of the image column feeds all three
    T.s_off[M_IMG] = D.ctr_image.off;
    T.s_bytes[M_IMG] = D.ctr_image.bytes;
  }
  // every column the kernel dereferences must be present (a null column is a device fault)
  if (!A.req_flags || !A.ctr_off || !A.lbl_off || !A.ctr_flags || !A.capadd_off || !A.capdrop_off || !A.out || !A.pols)
    return KW_E_ARG;
  for (int m = 0; m < (int)NMASK; ++m) {
    if (use[m] && !A.m[m]) return KW_E_ARG;
    if (use[m]) {
      int sm = (m == M_REG || m == M_TAG) ? (int)M_IMG : m;
      if (!T.s_off[sm] || !T.s_bytes[sm]) return KW_E_ARG;
    }
  }
  // per-chunk TileArgs (slot_plan pointers are filled in at upload, run_pass)
  const char* p3env = getenv("KW_P3");  // A/B of the verdict-store form (default: items)
  const uint32_t p3_item = (p3env && std::string(p3env) == "lane") ? 0u : 1u;
  plan->tiles.clear();
  plan->slot_at.clear();
  plan->slot_blob.clear();
  for (const SlotChunk& c : plan->chunks) {
    TileArgs t = T;
    plan->slot_at.push_back((uint32_t)plan->slot_blob.size());
    plan->slot_blob.insert(plan->slot_blob.end(), c.rec.begin(), c.rec.end());
    t.slot_bytes = c.staged;
    t.col0 = c.col0;
    t.ncols = c.ncols;
    t.vec4 = (npol % 4u == 0 && c.col0 % 4u == 0 && c.ncols % 4u == 0) ? 1u : 0u;
    t.o_gstk = c.groups ? T.o_gstk : 0u;
    const SlotHdr* sh = (const SlotHdr*)c.rec.data();
    t.o_cols_rec = sh->o_cols;
    t.o_cidx_rec = sh->o_cidx;
    t.slot_init = sh->init;
    t.p3_item = p3_item;
    plan->tiles.push_back(t);
  }
  uint64_t ntiles = (B.n + T.rows - 1) / T.rows;
  uint32_t wg_per_cu = std::max<uint32_t>(1, std::min<uint32_t>(2048 / kSlotThreads, (160 * 1024) / std::max<uint32_t>(T.lds_bytes, 1)));
  plan->grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ntiles, 256ull * wg_per_cu));
  return KW_OK;
}

const StrCol& host_strings(const Batch& B, int m) {
  switch (m) {
    case M_NS: return B.ns;
    case M_REG:
    case M_TAG:
    case M_IMG: return B.ctr_image;
    case M_CAPADD: return B.cap_add;
    case M_CAPDROP: return B.cap_drop;
    case M_AA: return B.ctr_aa;
    case M_LK: return B.lbl_key;
    default: return B.lbl_val;
  }
}

// Tile descriptors (kernels.hpp TileDesc) and the overflow list of one plan geometry, built from the
// host copy of the batch and uploaded once; reused while the geometry stays the same.
int upload_tile_descs(const Batch& B, DeviceBatch* D, const TileArgs& T) {
  uint64_t key = 1469598103934665603ull;
  auto mix = [&](uint64_t v) { key = (key ^ v) * 1099511628211ull; };
  mix(T.rows);
  mix(T.cmax);
  mix(T.kmax);
  mix(T.lmax);
  for (int m = 0; m < (int)NMASK; ++m) {
    mix(T.o_sb[m] != 0);
    mix(T.sb_cap[m]);
  }
  if (D->desc && key == D->desc_key) return KW_OK;
  const uint64_t ntiles = (B.n + T.rows - 1) / T.rows;
  std::vector<TileDesc> desc;
  desc.reserve(ntiles + ntiles / 64 + 1);
  std::vector<uint32_t> ovf{0};
  // descriptor of requests [r0, r1); false when it exceeds the capacities
  auto make = [&](uint64_t r0, uint64_t r1, TileDesc* dp) {
    TileDesc& d = *dp;
    memset(&d, 0, sizeof(d));
    d.r0lo = (uint32_t)r0;
    d.r0hi = (uint32_t)(r0 >> 32);
    d.nr = (uint32_t)(r1 - r0);
    d.cb = B.ctr_off[r0];
    d.ce = B.ctr_off[r1];
    d.lb = B.lbl_off[r0];
    d.le = B.lbl_off[r1];
    d.kab = B.capadd_off[d.cb];
    d.kae = B.capadd_off[d.ce];
    d.kdb = B.capdrop_off[d.cb];
    d.kde = B.capdrop_off[d.ce];
    bool fits = d.ce - d.cb <= T.cmax && d.kae - d.kab <= T.kmax && d.kde - d.kdb <= T.kmax && d.le - d.lb <= T.lmax;
    for (int m = 0; m < (int)NMASK; ++m) {
      if (!T.o_sb[m]) continue;
      const uint64_t g0 = m == M_NS ? r0 : m == M_CAPADD ? d.kab : m == M_CAPDROP ? d.kdb : (m == M_LK || m == M_LV) ? d.lb : d.cb;
      const uint64_t g1 = m == M_NS ? r1 : m == M_CAPADD ? d.kae : m == M_CAPDROP ? d.kde : (m == M_LK || m == M_LV) ? d.le : d.ce;
      const StrCol& c = host_strings(B, m);
      d.sa[m] = c.off[g0] & ~15u;
      d.nv[m] = (((c.off[g1] + 15u) & ~15u) - d.sa[m]) / 16u;
      fits = fits && d.nv[m] * 16u <= T.sb_cap[m];
    }
    d.fits = fits ? 1u : 0u;
    return fits;
  };
  // a run that does not fit is halved until its parts do; a single request that does not fit
  // goes to the overflow kernels
  std::vector<std::pair<uint64_t, uint64_t>> todo;
  for (uint64_t tile = 0; tile < ntiles; ++tile) {
    todo.assign(1, {tile * T.rows, std::min<uint64_t>(B.n, (tile + 1) * T.rows)});
    while (!todo.empty()) {
      const auto [r0, r1] = todo.back();
      todo.pop_back();
      TileDesc d;
      if (make(r0, r1, &d)) {
        desc.push_back(d);
      } else if (r1 - r0 > 1) {
        const uint64_t mid = r0 + (r1 - r0) / 2;
        todo.push_back({mid, r1});
        todo.push_back({r0, mid});
      } else {
        if (r0 > 0xffffffffull) return KW_E_ARG;  // overflow list holds u32 request indices
        ovf.push_back((uint32_t)r0);
      }
    }
  }
  ovf[0] = (uint32_t)(ovf.size() - 1);
  HIPCHK(hipStreamSynchronize(D->stream));  // a running pass may still read the previous descriptors
  if (int rc = ensure(&D->desc, &D->desc_cap, std::max<size_t>(desc.size(), 1))) return rc;
  if (int rc = ensure(&D->overflow, &D->overflow_cap, ovf.size())) return rc;
  if (!desc.empty()) HIPCHK(hipMemcpy(D->desc, desc.data(), desc.size() * sizeof(TileDesc), hipMemcpyHostToDevice));
  D->ndesc = desc.size();
  HIPCHK(hipMemcpy(D->overflow, ovf.data(), ovf.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  D->n_overflow = ovf[0];
  D->desc_key = key;
  return KW_OK;
}

int run_pass(const kw_env* env, kw_batch* kb, const PassPlan& plan, bool timed) {
  DeviceBatch& D = *kb->dev;
  if (timed) HIPCHK(hipEventRecord(D.ev[0], D.stream));
  if (!plan.fused) HIPCHK(launch_classify((const uint8_t*)env->e.d_blob, plan.jobs, D.stream));
  if (timed) HIPCHK(hipEventRecord(D.ev[1], D.stream));
  if (plan.rows_mode) {
    HIPCHK(launch_evaluate_rows(plan.args, D.stream));
  } else {
    // per-chunk TileArgs + slot records, uploaded when the plan changes
    if (int rc = ensure(&D.d_slots, &D.d_slots_cap, plan.slot_blob.size())) return rc;
    if (int rc = ensure(&D.d_tiles, &D.d_tiles_cap, plan.tiles.size())) return rc;
    std::vector<TileArgs> tiles = plan.tiles;
    for (size_t k = 0; k < tiles.size(); ++k) tiles[k].slot_plan = D.d_slots + plan.slot_at[k];
    if (D.h_slots != plan.slot_blob || D.h_tiles.size() != tiles.size() ||
        (!tiles.empty() && std::memcmp(D.h_tiles.data(), tiles.data(), tiles.size() * sizeof(TileArgs)) != 0)) {
      HIPCHK(hipStreamSynchronize(D.stream));  // a running pass may still read the previous plan
      D.h_slots = plan.slot_blob;
      D.h_tiles = tiles;
      HIPCHK(hipMemcpy(D.d_slots, D.h_slots.data(), D.h_slots.size(), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(D.d_tiles, D.h_tiles.data(), D.h_tiles.size() * sizeof(TileArgs), hipMemcpyHostToDevice));
    }
    if (int rc = upload_tile_descs(kb->b, &D, plan.tile)) return rc;
    EvalArgs sa = plan.args;
    sa.ndesc = D.ndesc;
    // dynamic tile schedule (per-XCD counters); KW_SCHED=static selects the strided schedule (A/B)
    static const bool dyn = !(getenv("KW_SCHED") && std::string(getenv("KW_SCHED")) == "static");
    if (dyn && !D.sched) {
      HIPCHK(hipMalloc((void**)&D.sched, 512 * sizeof(uint32_t)));
      HIPCHK(hipMemsetAsync(D.sched, 0, 512 * sizeof(uint32_t), D.stream));
    }
    sa.sched = dyn ? D.sched : nullptr;
    for (size_t k = 0; k < tiles.size(); ++k)
      HIPCHK(launch_evaluate_slots(sa, tiles[k], D.d_tiles + k, D.desc, plan.fused, plan.grid, D.stream));
    if (!tiles.empty()) HIPCHK(launch_overflow(sa, D.d_tiles, D.overflow, D.n_overflow, D.stream));
  }
  if (timed) HIPCHK(hipEventRecord(D.ev[2], D.stream));
  return KW_OK;
}

int validate_common(const kw_env* env, kw_batch* kb, const int32_t* policies, uint32_t npol, const int32_t* row_policy,
                    int origin, PassPlan* plan) {
  if (!env || !kb) return KW_E_ARG;
  const Env& E = env->e;
  if (E.device < 0 || !E.d_blob) return KW_E_DEVICE;  // no silent host fallback: the hot path is the GPU
  if (!kb->dev) return KW_E_ARG;                        // batch not resident
  if (kb->dev->device != E.device) return KW_E_ARG;
  if (origin != KW_ORIGIN_VALIDATE && origin != KW_ORIGIN_AUDIT) return KW_E_ARG;
  DeviceBatch& D = *kb->dev;
  HIPCHK(hipSetDevice(D.device));
  Needs need;
  uint64_t npairs;
  const int32_t* d_pols = nullptr;
  const int32_t* d_rows = nullptr;
  const int32_t np = (int32_t)E.pol.size();
  if (row_policy) {
    for (uint64_t r = 0; r < kb->b.n; ++r) {
      if (row_policy[r] < 0 || row_policy[r] >= np) return KW_E_ARG;
      add_needs(E, row_policy[r], &need);
    }
    npairs = kb->b.n;
    if (int rc = ensure(&D.pols, &D.pols_cap, kb->b.n)) return rc;
    HIPCHK(hipMemcpyAsync(D.pols, row_policy, kb->b.n * sizeof(int32_t), hipMemcpyHostToDevice, D.stream));
    d_rows = D.pols;
    npol = 1;
    D.host_pols.clear();
  } else {
    if (npol == 0 || !policies) return KW_E_ARG;
    for (uint32_t j = 0; j < npol; ++j) {
      if (policies[j] < 0 || policies[j] >= np) return KW_E_ARG;
      add_needs(E, policies[j], &need);
    }
    npairs = kb->b.n * (uint64_t)npol;
    if (int rc = ensure(&D.pols, &D.pols_cap, npol)) return rc;
    HIPCHK(hipMemcpyAsync(D.pols, policies, npol * sizeof(int32_t), hipMemcpyHostToDevice, D.stream));
    d_pols = D.pols;
    D.host_pols.assign(policies, policies + npol);
  }
  if (int rc = ensure(&D.verdicts, &D.verdict_cap, npairs)) return rc;
  D.last_verdicts = npairs;
  return plan_pass(env, kb, need, npairs, npol, origin, d_pols, d_rows, plan);
}

}  // namespace

extern "C" {

const char* kw_version(void) { return "kwgpu 0.1 (gfx950)"; }

int kw_env_build(const char* json, size_t len, const kw_env_options* opts, kw_env** out, char* err, size_t errlen) {
  if (!json || !out) return KW_E_ARG;
  auto env = std::make_unique<kw_env>();
  Status st = build_env(json, len, opts ? opts->continue_on_errors != 0 : false,
                        opts ? opts->always_accept_namespace : nullptr, &env->e);
  if (!st.ok()) {
    put_err(err, errlen, st.message);
    return st.code;
  }
  int dev = opts ? opts->device : -1;
  if (int rc = upload_env(env.get(), dev)) {
    put_err(err, errlen, "cannot upload compiled tables to the device");
    return rc;
  }
  *out = env.release();
  return KW_OK;
}

int kw_env_serialize(const kw_env* env, void* buf, size_t cap, size_t* need) {
  if (!env) return KW_E_ARG;
  std::vector<uint8_t> s = env_serialize(env->e);
  if (need) *need = s.size();
  if (!buf || cap < s.size()) return KW_E_NOSPACE;
  memcpy(buf, s.data(), s.size());
  return KW_OK;
}

int kw_env_deserialize(const void* blob, size_t len, int device, kw_env** out, char* err, size_t errlen) {
  if (!blob || !out) return KW_E_ARG;
  auto env = std::make_unique<kw_env>();
  Status st = env_from_blob(blob, len, &env->e);
  if (!st.ok()) {
    put_err(err, errlen, st.message);
    return st.code;
  }
  if (int rc = upload_env(env.get(), device)) return rc;
  *out = env.release();
  return KW_OK;
}

void kw_env_destroy(kw_env* env) {
  if (!env) return;
  if (env->e.d_blob) {
    (void)hipSetDevice(env->e.device);
    (void)hipFree(env->e.d_blob);
  }
  delete env;
}

int kw_env_lookup(const kw_env* env, const char* id, size_t len, int32_t* idx) {
  if (!env || !id || !idx) return KW_E_ARG;
  return env_lookup(env->e, std::string(id, len), idx).code;
}

int kw_env_policy_count(const kw_env* env) { return env ? (int)env->e.pol.size() : -1; }

int kw_env_policy_id(const kw_env* env, int32_t idx, char* buf, size_t cap) {
  if (!env || idx < 0 || (size_t)idx >= env->e.pol.size()) return KW_E_ARG;
  return put_out(env->e.pol[(size_t)idx].id, buf, cap, nullptr);
}

int kw_env_is_group(const kw_env* env, int32_t idx) {
  if (!env || idx < 0 || (size_t)idx >= env->e.pol.size()) return -1;
  return env->e.pol[(size_t)idx].is_group ? 1 : 0;
}

int kw_env_get_policy_mode(const kw_env* env, int32_t idx, int* mode) {
  if (!env || !mode || idx < 0 || (size_t)idx >= env->e.pol.size()) return KW_E_ARG;
  const PolicyRec& r = env->e.pol[(size_t)idx];
  if (!r.registered) return KW_E_NOT_FOUND;
  *mode = r.mode;
  return KW_OK;
}

int kw_env_get_policy_allowed_to_mutate(const kw_env* env, int32_t idx, int* allowed) {
  if (!env || !allowed || idx < 0 || (size_t)idx >= env->e.pol.size()) return KW_E_ARG;
  const PolicyRec& r = env->e.pol[(size_t)idx];
  if (!r.registered) return KW_E_NOT_FOUND;
  *allowed = r.allowed_to_mutate ? 1 : 0;
  return KW_OK;
}

int kw_env_should_always_accept_requests_made_inside_of_namespace(const kw_env* env, const char* ns, size_t len) {
  if (!env || !ns) return 0;
  return env->e.always_ns && *env->e.always_ns == std::string(ns, len) ? 1 : 0;
}

int kw_env_policy_initialization_error(const kw_env* env, int32_t idx, char* buf, size_t cap) {
  if (!env || idx < 0 || (size_t)idx >= env->e.pol.size()) return -1;
  const PolicyRec& r = env->e.pol[(size_t)idx];
  if (!r.init_error) return 0;
  put_err(buf, cap, r.init_message);
  return 1;
}

int kw_env_validate_settings(const kw_env* env, int32_t idx, char* buf, size_t cap) {
  if (!env || idx < 0 || (size_t)idx >= env->e.pol.size()) return KW_E_ARG;
  Status st = env_validate_settings(env->e, idx);
  if (!st.ok()) put_err(buf, cap, st.message);
  return st.code;
}

int kw_env_group_members(const kw_env* env, int32_t group, int32_t* out, int cap) {
  if (!env || group < 0 || (size_t)group >= env->e.pol.size()) return -1;
  const PolicyRec& r = env->e.pol[(size_t)group];
  int n = (int)r.members.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = r.members[(size_t)i];
  return n;
}

int kw_pattern_match(int kind, const char* pat, const char* s, size_t len) {
  if (!pat || (!s && len)) return -1;
  std::vector<Pattern> ps{{(Pattern::Kind)kind, pat}};
  Dfa d;
  std::string err;
  if (!compile_dfa(ps, &d, &err)) return -1;
  return (d.run((const uint8_t*)s, len) & 1ull) ? 1 : 0;
}

namespace {
// Host walks of the compiled blob, mirroring the kernels (diagnostics / tests only).
uint64_t blob_dfa_run(const uint8_t* blob, uint32_t off, const uint8_t* s, size_t n) {
  const DevDfa* d = (const DevDfa*)(blob + off);
  const uint16_t* trans = (const uint16_t*)(blob + d->trans_off);
  const uint64_t* acc = (const uint64_t*)(blob + d->acc_off);
  uint32_t st = d->start;
  for (size_t i = 0; i < n && st != 0; ++i) st = trans[(size_t)st * d->ncls + d->cls[s[i]]];
  return acc[st];
}
uint64_t blob_chain_run(const uint8_t* blob, uint32_t head, const uint8_t* s, size_t n) {
  uint64_t m = 0;
  for (uint32_t o = head; o; o = ((const DevDfa*)(blob + o))->next) m |= blob_dfa_run(blob, o, s, n);
  return m;
}
uint64_t blob_lit_lookup(const uint8_t* blob, uint32_t off, const uint8_t* s, size_t n) {
  const DevLit* L = (const DevLit*)(blob + off);
  const uint8_t* rec = blob + off;
  std::vector<uint32_t> w((n + 3) / 4, 0u);
  if (n) memcpy(w.data(), s, n);
  uint32_t h = lit_init(L->seed, (uint32_t)n);
  for (uint32_t x : w) h = lit_mix(h, x);
  h = lit_final(h);
  const uint32_t slot = ((const uint32_t*)(rec + L->slot_off))[h & (L->nslots - 1)];
  if (!slot || lit_slot_len(slot) != n) return 0;
  const uint32_t* pw = (const uint32_t*)(rec + L->word_off) + lit_slot_word(slot);
  for (size_t i = 0; i < w.size(); ++i)
    if (w[i] != pw[i]) return 0;
  return 1ull << (lit_slot_pat(slot) - 1);
}
}  // namespace

int kw_env_classify_check(const kw_env* env, int col, const char* key, size_t klen, const char* s, size_t len,
                          uint64_t* dfa_mask, uint64_t* fast_mask) {
  if (!env || col < 0 || col >= (int)NCOL || (!s && len) || !dfa_mask || !fast_mask) return KW_E_ARG;
  const uint8_t* blob = env->e.blob.data();
  const DevHeader* H = (const DevHeader*)blob;
  const uint8_t* u = (const uint8_t*)s;
  *dfa_mask = H->dfa_off[col] ? blob_chain_run(blob, H->dfa_off[col], u, len) : 0ull;
  *fast_mask = 0;
  if (col == COL_LV) {
    if (!H->kv_off || !H->lit_off[COL_LK] || (!key && klen)) return 0;
    const uint64_t km = blob_lit_lookup(blob, H->lit_off[COL_LK], (const uint8_t*)key, klen);
    const uint8_t* R = blob + H->kv_off;
    uint64_t keybits = 0;  // value patterns constrained on this key: every bit its DFA can accept
    for (uint32_t rel = km ? ((const uint16_t*)R)[__builtin_ctzll(km)] : 0u; rel;) {  // the key's chain
      const KvDfa& d = *(const KvDfa*)(R + rel);
      const uint64_t* accv = (const uint64_t*)(R + d.accv_off);
      for (uint32_t q = 0; q < d.nstates; ++q) keybits |= accv[R[d.acc_off + q]];
      uint32_t st = d.start;
      for (size_t i = 0; i < len && st != 0; ++i) st = kv_step(R, d, st, u[i]);
      *fast_mask |= accv[R[d.acc_off + st]];
      rel = d.next;
    }
    *dfa_mask &= keybits;
    return 1;
  }
  if (!H->lit_off[col]) return 0;
  *fast_mask = blob_lit_lookup(blob, H->lit_off[col], u, len);
  return 1;
}

}  // extern "C"

namespace {
// Host restatement of the kernel's image-reference classification (kernels.hip parse_image /
// image_part), for the diagnostic walk below.
uint64_t host_image_part(const uint8_t* blob, uint32_t head, int k, const uint8_t* s, size_t n) {
  const size_t NONE = (size_t)-1;
  size_t at = NONE, slash0 = NONE, slash1 = NONE, last_colon = NONE;
  bool dotcolon = false;
  for (size_t q = 0; q < n; ++q) {
    const uint8_t c = s[q];
    if (c == '@') {
      at = q;
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
  auto eq = [&](size_t e, const char* lit) { return e == strlen(lit) && memcmp(s, lit, e) == 0; };
  const size_t name_end = at != NONE ? at : n;
  const bool is_reg = slash0 != NONE && (dotcolon || eq(slash0, "localhost"));
  const size_t rest_b = is_reg ? slash0 + 1 : 0;
  const size_t colon = (last_colon != NONE && last_colon >= rest_b) ? last_colon : NONE;
  const size_t path_end = colon != NONE ? colon : name_end;
  const size_t fsr = is_reg ? slash1 : slash0;
  const bool path_slash = fsr != NONE && fsr < path_end;
  const bool is_docker = !is_reg || eq(slash0, "docker.io");
  const bool eff_tag = colon != NONE || at == NONE;
  std::string t;
  auto app = [&](size_t b, size_t e) { t.append((const char*)s + b, e - b); };
  if (k == 0) {
    if (is_reg) app(0, slash0);
    else t = "docker.io";
  } else if (k == 1) {
    if (colon != NONE) app(colon + 1, name_end);
    else if (at == NONE) t = "latest";
    else return 0;
  } else {
    if (is_reg) app(0, slash0);
    else t = "docker.io";
    t += '/';
    if (is_docker && !path_slash) t += "library/";
    app(rest_b, path_end);
    if (eff_tag) {
      t += ':';
      if (colon != NONE) app(colon + 1, name_end);
      else t += "latest";
    }
    if (at != NONE) app(at, n);
  }
  return blob_chain_run(blob, head, (const uint8_t*)t.data(), t.size());
}

struct HostSrc {
  const Batch* b;
  const SlotView* sv;
  const std::vector<uint64_t>* mk[NMASK];
  uint8_t rf(uint64_t r) const { return b->req_flags[r]; }
  uint32_t coff(uint64_t r) const { return b->ctr_off[r]; }
  uint32_t loff(uint64_t r) const { return b->lbl_off[r]; }
  uint8_t cflags(uint32_t c) const { return b->ctr_flags[c]; }
  uint32_t cadd(uint32_t c) const { return b->capadd_off[c]; }
  uint32_t cdrop(uint32_t c) const { return b->capdrop_off[c]; }
  template <int K>
  uint64_t m(uint64_t i) const {
    return mk[K] ? (*mk[K])[i] : 0ull;
  }
  uint64_t vadd(uint32_t k) const { return derive_capadd(*sv, m<M_CAPADD>(k)); }
  uint64_t vaa(uint32_t c) const { return derive_apparmor(*sv, m<M_AA>(c)); }
  uint64_t vcon(uint32_t l) const { return derive_label(*sv, m<M_LK>(l), m<M_LV>(l)); }
};
}  // namespace

extern "C" {

int kw_debug_host_walk(const kw_env* env, const kw_batch* kb, const int32_t* policies, uint32_t npol, int origin,
                       uint32_t* out) {
  if (!env || !kb || (!policies && npol) || (!out && npol && kb->b.n)) return KW_E_ARG;
  const Env& E = env->e;
  const Batch& B = kb->b;
  const uint8_t* blob = E.blob.data();
  const DevHeader* H = (const DevHeader*)blob;
  std::vector<SlotChunk> chunks;
  Status st = build_slot_chunks(E, policies, npol, origin, &chunks);
  if (!st.ok()) return st.code;
  // classification of every string, with the column automata of the blob
  std::vector<uint64_t> mv[NMASK];
  auto chain = [&](Col c, const StrCol& sc, std::vector<uint64_t>* o) {
    if (!H->dfa_off[c]) return false;
    o->resize(sc.n());
    for (size_t i = 0; i < sc.n(); ++i)
      (*o)[i] = blob_chain_run(blob, H->dfa_off[c], sc.bytes.data() + sc.off[i], sc.off[i + 1] - sc.off[i]);
    return true;
  };
  HostSrc src;
  src.b = &B;
  for (auto& p : src.mk) p = nullptr;
  if (chain(COL_NS, B.ns, &mv[M_NS])) src.mk[M_NS] = &mv[M_NS];
  if (chain(COL_CAP, B.cap_add, &mv[M_CAPADD])) src.mk[M_CAPADD] = &mv[M_CAPADD];
  if (chain(COL_CAP, B.cap_drop, &mv[M_CAPDROP])) src.mk[M_CAPDROP] = &mv[M_CAPDROP];
  if (chain(COL_AA, B.ctr_aa, &mv[M_AA])) src.mk[M_AA] = &mv[M_AA];
  if (chain(COL_LK, B.lbl_key, &mv[M_LK])) src.mk[M_LK] = &mv[M_LK];
  if (chain(COL_LV, B.lbl_val, &mv[M_LV])) src.mk[M_LV] = &mv[M_LV];
  const Col icol[3] = {COL_REG, COL_TAG, COL_IMG};
  const int imask[3] = {M_REG, M_TAG, M_IMG};
  for (int k = 0; k < 3; ++k) {
    if (!H->dfa_off[icol[k]]) continue;
    std::vector<uint64_t>& o = mv[imask[k]];
    o.assign(B.ctr_image.n(), 0);
    for (size_t c = 0; c < B.ctr_image.n(); ++c)
      if (B.ctr_flags[c] & KW_CTR_HAS_IMAGE)
        o[c] = host_image_part(blob, H->dfa_off[icol[k]], k, B.ctr_image.bytes.data() + B.ctr_image.off[c],
                               B.ctr_image.off[c + 1] - B.ctr_image.off[c]);
    src.mk[imask[k]] = &o;
  }
  std::vector<uint32_t> vw(kSlots);
  uint16_t gstk[kMaxGroupStack];
  for (const SlotChunk& ch : chunks) {
    SlotView sv;
    sv.h = (const SlotHdr*)ch.rec.data();
    sv.base = ch.rec.data();
    src.sv = &sv;
    const ColInfo* cols = sv.cols();
    const uint8_t* cidx = ch.rec.data() + sv.h->o_cidx;
    for (uint64_t r = 0; r < B.n; ++r) {
      const uint32_t rf = B.req_flags[r];
      const bool byp = H->bypass_bit >= 0 && !(rf & KW_REQ_RAW) && (rf & KW_REQ_HAS_NAMESPACE) && src.mk[M_NS] &&
                       (((*src.mk[M_NS])[r] >> H->bypass_bit) & 1ull);
      uint64_t mut = 0;
      uint64_t rej = walk_privileged_caps(src, sv, r, vw.data(), &mut);
      rej |= walk_apparmor_images(src, sv, r, vw.data());
      rej |= walk_labels(src, sv, r, vw.data());
      rej |= walk_namespace(src, sv, r, vw.data());
      for (uint32_t j = 0; j < ch.ncols; ++j)
        out[r * npol + ch.col0 + j] =
            byp ? kBypassWord : column_word(cols[j], rej, mut, sv.h->init, vw.data(), blob, cidx, gstk, 1);
    }
  }
  return KW_OK;
}

int kw_batch_from_json(const char* const* docs, const size_t* lens, size_t n, int doc_kind, kw_batch** out,
                       int64_t* bad_row, char* err, size_t errlen) {
  if (!out || (n && (!docs || !lens))) return KW_E_ARG;
  auto kb = std::make_unique<kw_batch>();
  // contiguous document ranges flattened by up to KW_FLATTEN_THREADS threads (default: the
  // hardware threads, at most 16), then concatenated in order; the first bad row wins
  uint32_t nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (const char* t = getenv("KW_FLATTEN_THREADS")) nt = (uint32_t)std::max(1, atoi(t));
  nt = (uint32_t)std::min<uint64_t>(nt, std::max<size_t>(1, n / 2048));
  std::vector<Batch> part(nt);
  std::vector<int64_t> bad(nt, -1);
  std::vector<std::string> perr(nt);
  auto work = [&](uint32_t t) {
    const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
    for (size_t i = i0; i < i1; ++i)
      if (!flatten_document(docs[i], lens[i], doc_kind, &part[t], &perr[t])) {
        bad[t] = (int64_t)i;
        return;
      }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  for (uint32_t t = 0; t < nt; ++t)
    if (bad[t] >= 0) {
      if (bad_row) *bad_row = bad[t];
      put_err(err, errlen, perr[t]);
      return KW_E_PAYLOAD;
    }
  if (nt == 1) {
    kb->b = std::move(part[0]);
  } else {
    for (uint32_t t = 0; t < nt; ++t) {
      kb->b.append(part[t]);
      part[t] = Batch();  // release as we go
    }
  }
  kb->b.finalize();
  *out = kb.release();
  return KW_OK;
}

int kw_batch_from_soa(const kw_soa* soa, kw_batch** out) {
  if (!soa || !out) return KW_E_ARG;
  auto kb = std::make_unique<kw_batch>();
  std::string e;
  if (!batch_from_soa(*soa, &kb->b, &e)) return KW_E_ARG;
  kb->b.finalize();
  *out = kb.release();
  return KW_OK;
}

int kw_batch_view(const kw_batch* b, kw_soa* view) {
  if (!b || !view) return KW_E_ARG;
  b->b.view(view);
  return KW_OK;
}

int kw_batch_to_device(kw_batch* kb, int device) {
  if (!kb || device < 0) return KW_E_ARG;
  HIPCHK(hipSetDevice(device));
  auto D = std::make_unique<DeviceBatch>();
  D->device = device;
  HIPCHK(hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking));
  for (auto& e : D->ev) HIPCHK(hipEventCreate(&e));
  Batch& B = kb->b;
  B.finalize();
  // one allocation, 256-B aligned sub-arrays
  struct Piece {
    const void* src;
    size_t bytes;
    size_t at;
  };
  std::vector<Piece> pieces;
  size_t total = 0;
  auto add = [&](const void* src, size_t bytes) {
    size_t at = total;
    pieces.push_back({src, bytes, at});
    total += (bytes + 255) & ~(size_t)255;
    return at;
  };
  size_t o_rf = add(B.req_flags.data(), B.req_flags.size());
  size_t o_co = add(B.ctr_off.data(), B.ctr_off.size() * 4);
  size_t o_lo = add(B.lbl_off.data(), B.lbl_off.size() * 4);
  size_t o_cf = add(B.ctr_flags.data(), B.ctr_flags.size());
  size_t o_ca = add(B.capadd_off.data(), B.capadd_off.size() * 4);
  size_t o_cd = add(B.capdrop_off.data(), B.capdrop_off.size() * 4);
  struct ColAt {
    size_t off, bytes;
  };
  auto addcol = [&](const StrCol& c) { return ColAt{add(c.off.data(), c.off.size() * 4), add(c.bytes.data(), c.bytes.size())}; };
  ColAt c_ns = addcol(B.ns), c_img = addcol(B.ctr_image), c_aa = addcol(B.ctr_aa), c_add = addcol(B.cap_add),
        c_drop = addcol(B.cap_drop), c_lk = addcol(B.lbl_key), c_lv = addcol(B.lbl_val);
  D->cols_bytes = total;
  HIPCHK(hipMalloc((void**)&D->cols, std::max<size_t>(total, 256)));
  for (auto& p : pieces)
    if (p.bytes) HIPCHK(hipMemcpy(D->cols + p.at, p.src, p.bytes, hipMemcpyHostToDevice));
  D->req_flags = D->cols + o_rf;
  D->ctr_off = (const uint32_t*)(D->cols + o_co);
  D->lbl_off = (const uint32_t*)(D->cols + o_lo);
  D->ctr_flags = D->cols + o_cf;
  D->capadd_off = (const uint32_t*)(D->cols + o_ca);
  D->capdrop_off = (const uint32_t*)(D->cols + o_cd);
  auto dcol = [&](const StrCol& c, ColAt at) {
    DeviceBatch::DCol d;
    d.off = (const uint32_t*)(D->cols + at.off);
    d.bytes = D->cols + at.bytes;
    d.n = c.n();
    d.nbytes = c.off.back();
    return d;
  };
  D->ns = dcol(B.ns, c_ns);
  D->ctr_image = dcol(B.ctr_image, c_img);
  D->ctr_aa = dcol(B.ctr_aa, c_aa);
  D->cap_add = dcol(B.cap_add, c_add);
  D->cap_drop = dcol(B.cap_drop, c_drop);
  D->lbl_key = dcol(B.lbl_key, c_lk);
  D->lbl_val = dcol(B.lbl_val, c_lv);
  kb->dev = std::move(D);
  return KW_OK;
}

void kw_batch_destroy(kw_batch* b) { delete b; }

int kw_validate_batch(const kw_env* env, kw_batch* b, const int32_t* policies, uint32_t npol, int origin, void* stream) {
  (void)stream;
  PassPlan plan;
  if (int rc = validate_common(env, b, policies, npol, nullptr, origin, &plan)) return rc;
  return run_pass(env, b, plan, false);
}

int kw_validate_rows(const kw_env* env, kw_batch* b, const int32_t* row_policy, int origin, void* stream) {
  (void)stream;
  if (!row_policy) return KW_E_ARG;
  PassPlan plan;
  if (int rc = validate_common(env, b, nullptr, 0, row_policy, origin, &plan)) return rc;
  return run_pass(env, b, plan, false);
}

int kw_batch_verdicts(kw_batch* b, uint32_t* host_out, size_t count) {
  if (!b || !b->dev || !host_out) return KW_E_ARG;
  DeviceBatch& D = *b->dev;
  if (count > D.last_verdicts) return KW_E_ARG;
  HIPCHK(hipSetDevice(D.device));
  HIPCHK(hipMemcpyAsync(host_out, D.verdicts, count * sizeof(uint32_t), hipMemcpyDeviceToHost, D.stream));
  HIPCHK(hipStreamSynchronize(D.stream));
  return KW_OK;
}

int kw_validate_timed(const kw_env* env, kw_batch* b, const int32_t* policies, uint32_t npol, int origin, int warmup,
                      int reps, kw_timing* out) {
  if (!out || reps <= 0) return KW_E_ARG;
  PassPlan plan;
  if (int rc = validate_common(env, b, policies, npol, nullptr, origin, &plan)) return rc;
  DeviceBatch& D = *b->dev;
  for (int i = 0; i < warmup; ++i)
    if (int rc = run_pass(env, b, plan, false)) return rc;
  HIPCHK(hipStreamSynchronize(D.stream));
  double cl = 0, ev = 0;
  for (int i = 0; i < reps; ++i) {
    if (int rc = run_pass(env, b, plan, true)) return rc;
    HIPCHK(hipEventSynchronize(D.ev[2]));
    float a = 0, c = 0;
    HIPCHK(hipEventElapsedTime(&a, D.ev[0], D.ev[1]));
    HIPCHK(hipEventElapsedTime(&c, D.ev[1], D.ev[2]));
    cl += a;
    ev += c;
  }
  out->classify_ms = cl / reps;
  out->evaluate_ms = ev / reps;
  out->total_ms = (cl + ev) / reps;
  out->classify_bytes = plan.classify_bytes;
  out->evaluate_bytes = plan.evaluate_bytes;
  return KW_OK;
}

int kw_format_response(const kw_env* env, const kw_batch* b, uint64_t row, int32_t policy, uint32_t verdict,
                       const uint32_t* member_verdicts, char* buf, size_t cap, size_t* need) {
  if (!env || !b || row >= b->b.n || policy < 0 || (size_t)policy >= env->e.pol.size()) return KW_E_ARG;
  std::string out;
  Status st = format_response(env->e, b->b, row, policy, verdict, member_verdicts, &out);
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  return put_out(out, buf, cap, need);
}

int kw_format_response_doc(const kw_env* env, const kw_batch* b, uint64_t row, int32_t policy, uint32_t verdict,
                           const uint32_t* member_verdicts, const char* doc, size_t doc_len, int doc_kind, char* buf,
                           size_t cap, size_t* need) {
  if (!env || !b || row >= b->b.n || policy < 0 || (size_t)policy >= env->e.pol.size() || (!doc && doc_len))
    return KW_E_ARG;
  std::string out;
  Status st = format_response(env->e, b->b, row, policy, verdict, member_verdicts, &out, doc, doc_len, doc_kind);
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  return put_out(out, buf, cap, need);
}

int kw_evaluate(const kw_env* env, const char* policy_id, const char* doc, size_t doc_len, int doc_kind, int origin,
                char* buf, size_t cap, size_t* need) {
  if (!env || !policy_id || !doc) return KW_E_ARG;
  const Env& E = env->e;
  int32_t idx;
  Status st = env_lookup(E, policy_id, &idx);  // service.rs:37 + PolicyNotFound
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  kw_batch* kb = nullptr;
  char err[512];
  int rc = kw_batch_from_json(&doc, &doc_len, 1, doc_kind, &kb, nullptr, err, sizeof(err));
  if (rc) {
    put_out(err, buf, cap, need);
    return rc;
  }
  std::unique_ptr<kw_batch> hold(kb);
  if (E.device < 0) {
    put_out("engine has no device: the hot path runs only on the GPU", buf, cap, need);
    return KW_E_DEVICE;
  }
  if ((rc = kw_batch_to_device(kb, E.device))) return rc;
  std::vector<int32_t> pols{idx};
  const PolicyRec& P = E.pol[(size_t)idx];
  for (int32_t m : P.members) pols.push_back(m);
  if ((rc = kw_validate_batch(env, kb, pols.data(), (uint32_t)pols.size(), origin, nullptr))) return rc;
  std::vector<uint32_t> v(pols.size());
  if ((rc = kw_batch_verdicts(kb, v.data(), v.size()))) return rc;
  std::string out;
  st = format_response(E, kb->b, 0, idx, v[0], v.size() > 1 ? v.data() + 1 : nullptr, &out, doc, doc_len, doc_kind);
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  return put_out(out, buf, cap, need);
}

int kw_service_constraints(uint32_t in, int mode, int allowed_to_mutate, uint32_t* out_flags) {
  // validation_response_with_constraints (service.rs:160-208); bit0 allowed, bit1 patch, bit2 status
  uint32_t o = in;
  int fst;
  if (mode == KW_MODE_MONITOR) {
    o = 1u;
    fst = KW_FST_NONE;
  } else if ((in & 2u) && !allowed_to_mutate) {
    o = 4u;
    fst = KW_FST_MUTATION_REFUSED;
  } else {
    fst = (in & 4u) ? KW_FST_VANILLA : KW_FST_NONE;
  }
  if (out_flags) *out_flags = o;
  return fst;
}

}  // extern "C"

// ---- metrics (metrics.hpp)
struct kw_metrics {
  kw::Metrics m;
};

kw_metrics* kw_metrics_create(void) { return new (std::nothrow) kw_metrics(); }
void kw_metrics_destroy(kw_metrics* m) { delete m; }

int kw_metrics_record(kw_metrics* m, const kw_env* env, const kw_batch* b, const uint64_t* rows,
                      const int32_t* policies, const uint32_t* verdicts, const uint64_t* latency_ms, size_t n,
                      int origin) {
  if (!m || !env || !b || (n && (!rows || !policies || !verdicts || !latency_ms))) return KW_E_ARG;
  if (origin != KW_ORIGIN_VALIDATE && origin != KW_ORIGIN_AUDIT) return KW_E_ARG;
  for (size_t i = 0; i < n; ++i)
    if (rows[i] >= b->b.n || policies[i] < 0 || (size_t)policies[i] >= env->e.pol.size()) return KW_E_ARG;
  for (size_t i = 0; i < n; ++i) m->m.record(env->e, b->b, rows[i], policies[i], verdicts[i], origin, latency_ms[i]);
  return KW_OK;
}

int kw_metrics_render(const kw_metrics* m, char* buf, size_t cap, size_t* need) {
  if (!m) return KW_E_ARG;
  return put_out(m->m.render(), buf, cap, need);
}

void kw_metrics_reset(kw_metrics* m) {
  if (m) m->m.reset();
}
