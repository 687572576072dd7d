// kernels.hpp — launch interface of the device hot path (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kwdev.hpp"
#include "slots.hpp"

namespace kw {

struct ClassifyJob {
  const uint32_t* off;   // string offsets (n+1)
  const uint8_t* bytes;  // pool (16 B zero tail)
  uint64_t* out[3];      // plain: out[0]; image: registry, tag, image masks
  uint32_t dfa[3];       // blob offsets of DevDfa (0 = column has no patterns)
  uint32_t lds_pos[3];   // LDS byte position of each staged DFA
  uint32_t lds_bytes;    // bytes staged for this job
  uint32_t n;            // strings
  uint32_t mode;         // 0 plain, 1 image reference
  uint32_t block_begin;  // first block of this job
  uint32_t nblocks;      // blocks of this job
};

constexpr int kMaxJobs = 8;
constexpr int kClassifyThreads = 256;
constexpr int kEvalThreads = 256;

struct ClassifyJobs {
  ClassifyJob j[kMaxJobs];
  int n;
  uint32_t total_blocks;
  uint32_t lds_bytes;  // dynamic LDS per block (max over jobs); 0 = tables read from global
};

struct EvalArgs {
  const uint8_t* blob;
  uint64_t nrows;
  uint64_t ndesc;             // slot kernel: tile descriptors (TileDesc) to walk
  uint64_t npairs;
  uint32_t npol;              // policies per row (all-pairs mode)
  int32_t origin;
  const int32_t* pols;        // all-pairs mode: npol policy indices
  const int32_t* row_policy;  // micro-batch mode: one policy per row (pols unused)
  const uint8_t* req_flags;
  const uint32_t* ctr_off;
  const uint32_t* lbl_off;
  const uint8_t* ctr_flags;
  const uint32_t* capadd_off;
  const uint32_t* capdrop_off;
  const uint64_t* m[NMASK];   // nullptr = column carries no patterns (all-zero masks)
  uint32_t* out;
  uint32_t* sched;  // slot kernel: per-XCD tile counters (256 u32 + 256 u32 done counts), nullptr = static
};

// Slot kernel geometry: one tile = 64 requests (one lane per request in the walk), 256 threads.
constexpr uint32_t kSlotRows = 64;
constexpr uint32_t kSlotThreads = 256;

// All-pairs evaluation (kernels.hip evaluate_slots_kernel): LDS layout, capacities and the
// column chunk one launch writes. Lives in device memory (one per chunk); read with scalar loads.
struct TileArgs {
  uint32_t rows;                  // requests per tile (kSlotRows)
  uint32_t cmax, kmax, lmax;      // container / capability / label capacity of a staged tile
  uint32_t o_rf, o_coff, o_loff, o_cflags, o_cadd, o_cdrop, o_gstk;  // LDS byte offsets
  uint32_t o_m[NMASK];            // LDS byte offset of each per-string array P1 fills, 0 = none: u8 pattern
                                  // index (0xff none) for NS / CAPADD / CAPDROP / LK, u64 masks for
                                  // REG / TAG / IMG; AA and LV only feed the violation sets
  uint32_t use_mask;              // bit m: mask m has patterns (its strings are classified)
  uint32_t o_vadd, o_vl, o_vc;    // u64 violation sets: per added capability, per label (V_l), per container (V_c)
  uint32_t o_own_c, o_own_l;      // u8 tile-local request of each staged container / label
  uint32_t o_rej, o_mut, o_byp;   // per-request walk results: rejected / mutated slots, bypass flag
  uint32_t o_nx;                  // u32[2]: next tile index (dynamic schedule), double-buffered
  uint32_t o_sa;                  // u32[NMASK]: the tile's staged byte start per string column (TileDesc.sa)
  uint32_t o_vw, vw_stride;       // violation words [rows][vw_stride] (aliases the staged strings)
  uint32_t o_slot, slot_bytes;    // staged SlotHdr record of this chunk
  uint32_t col0, ncols, vec4;     // output columns [col0, col0 + ncols); vec4: 16-B verdict stores
  const uint8_t* slot_plan;       // device copy of this chunk's SlotHdr record
  uint32_t o_cols_rec, o_cidx_rec;  // ColInfo / cidx sections of the record (global reads in P3)
  uint32_t p3_item, pad_p3;       // P3 form: 0 = one lane per request, 1 = (request, 4 columns) items
  uint64_t slot_init;             // SlotHdr.init of this chunk
  uint32_t chain_len[NMASK];      // DFAs in the chain of each mask's column (1 when absent)
  uint32_t mask_cap[NMASK];       // entries of each staged mask array
  uint32_t debug;                 // diagnostics: bit0 skip classification, bit1 skip walk, bit2 skip output
  uint32_t lds_bytes;
  // FUSED: column tables (literal hash, DFA chains) staged once per workgroup
  uint32_t nstage;
  uint32_t stage_blob[NCOL], stage_lds[NCOL], stage_bytes[NCOL];
  uint32_t dfa_head[NMASK];       // blob offset of the chain used for mask k (0 = none)
  uint32_t dfa_lds[NMASK];        // LDS offset of that chain's head
  uint32_t lit_lds[NMASK];        // LDS offset of the column's literal table (replaces the DFA), 0 = none
  uint32_t kv_lds, kv_blob;       // per-key label-value DFA region: LDS and blob offsets (0 = LV chain)
  const uint32_t* s_off[NMASK];   // string offsets feeding mask k (M_REG/TAG use M_IMG's column)
  const uint8_t* s_bytes[NMASK];
  // FUSED: each tile's strings staged in LDS (M_NS, M_IMG, M_AA, M_CAPADD, M_CAPDROP, M_LK, M_LV):
  // absolute offsets (rebased by the tile's staged start, o_sa), bytes copied from the 16-B aligned start;
  // 0 = not staged
  uint32_t o_so[NMASK], o_sb[NMASK], sb_cap[NMASK];
};

hipError_t launch_classify(const uint8_t* d_blob, const ClassifyJobs& jobs, hipStream_t s);
hipError_t launch_evaluate_rows(const EvalArgs& a, hipStream_t s);

// Per-tile geometry, precomputed on the host from the batch's offsets (one s_load burst per tile
// instead of a chain of dependent global loads): entity ranges, the 16-B aligned byte range of each
// staged string column, and whether the tile fits the LDS capacities.
// A tile is a run of at most kSlotRows requests; runs that exceed the LDS capacities are halved
// until they fit, and single requests that still do not fit go to the overflow kernels.
struct alignas(16) TileDesc {
  uint32_t cb, ce, lb, le, kab, kae, kdb, kde;
  uint32_t sa[NMASK];  // staged column m: first byte (16-B aligned) of the tile's strings in the pool
  uint32_t nv[NMASK];  //                  16-B vectors to copy
  uint32_t fits;
  uint32_t r0lo, r0hi, nr;  // first request (64-bit) and request count
  uint32_t pad[2];
};
static_assert(sizeof(TileDesc) == 128, "TileDesc layout");

// One launch of the slot kernel for one column chunk. t: host copy (launch geometry); d_t: the
// same TileArgs resident in device memory (read by the kernel).
hipError_t launch_evaluate_slots(const EvalArgs& a, const TileArgs& t, const TileArgs* d_t, const TileDesc* d_desc,
                                 bool fused, uint32_t grid, hipStream_t s);
// Requests that do not fit the LDS capacities even alone (d_overflow: [count, request indices...],
// host-built with the descriptors), evaluated from global memory for every column.
hipError_t launch_overflow(const EvalArgs& a, const TileArgs* d_t, const uint32_t* d_overflow, uint32_t n_overflow,
                           hipStream_t s);

}  // namespace kw
