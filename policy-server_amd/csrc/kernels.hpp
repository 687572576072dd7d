// kernels.hpp — launch interface of the device hot path (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kwdev.hpp"

namespace kw {

// Which mask array a classification job writes (one u64 per string).
enum MaskArr : uint32_t { M_NS = 0, M_REG, M_TAG, M_IMG, M_CAPADD, M_CAPDROP, M_AA, M_LK, M_LV, NMASK };

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
};

#ifndef KW_TILE_THREADS
#define KW_TILE_THREADS 1024
#endif
// 1024: one workgroup per CU (16 waves share one LDS copy of the tables, 160 KB);
// 512: two workgroups per CU (80 KB each) whose barriers interleave
constexpr int kTileThreads = KW_TILE_THREADS;

// Tiled all-pairs evaluation (kernels.hip evaluate_tiled_kernel): LDS layout and capacities.
struct TileArgs {
  uint32_t rows;                  // requests per tile
  uint32_t cmax, kmax, lmax;      // container / capability / label capacity of a staged tile
  uint32_t o_rf, o_coff, o_loff, o_cflags, o_cadd, o_cdrop, o_gstk;  // LDS byte offsets
  uint32_t o_m[NMASK];            // LDS byte offset of each staged mask array, 0 = not read
  uint32_t o_feat, o_pos;         // per-row features (RowFeat) and first-occurrence tables
  uint32_t ncap_bits, naa_bits, nkey_bits;  // pattern counts of the literal columns
  uint64_t cap_all_mask;          // COL_CAP bit of the "ALL" capability (0 if none)
  uint32_t chain_len[NMASK];      // DFAs in the chain of each mask's column (1 when absent)
  uint32_t mask_cap[NMASK];       // entries of each staged mask array
  uint32_t debug;                 // diagnostics: bit0 skip DFA, bit1 skip row features, bit2 skip evaluation
  uint32_t lds_bytes;
  // FUSED: DFA chains staged once per workgroup, and the string columns they classify
  uint32_t nstage;
  uint32_t stage_blob[NCOL], stage_lds[NCOL], stage_bytes[NCOL];
  uint32_t dfa_head[NMASK];       // blob offset of the chain used for mask k (0 = none)
  uint32_t dfa_lds[NMASK];        // LDS offset of that chain's head
  uint32_t lit_lds[NMASK];        // LDS offset of the column's literal table (replaces the DFA), 0 = none
  uint32_t kv_lds, kv_blob;       // per-key label-value DFA region: LDS and blob offsets (0 = LV chain)
  const uint32_t* s_off[NMASK];   // string offsets feeding mask k (M_REG/TAG use M_IMG's column)
  const uint8_t* s_bytes[NMASK];
  // FUSED: each tile's strings staged in LDS (M_NS, M_IMG, M_AA, M_CAPADD, M_CAPDROP, M_LK, M_LV):
  // offsets rebased to the staged bytes, bytes copied from the 16-B aligned start; 0 = not staged
  uint32_t o_so[NMASK], o_sb[NMASK], sb_cap[NMASK];
};

hipError_t launch_classify(const uint8_t* d_blob, const ClassifyJobs& jobs, hipStream_t s);
hipError_t launch_evaluate_rows(const EvalArgs& a, hipStream_t s);
// t: host copy (launch geometry); d_t: the same TileArgs resident in device memory (read by the kernel)
// Per-tile geometry, precomputed on the host from the batch's offsets (one s_load burst per tile
// instead of a chain of dependent global loads): entity ranges, the 16-B aligned byte range of each
// staged string column, and whether the tile fits the LDS capacities.
struct alignas(16) TileDesc {
  uint32_t cb, ce, lb, le, kab, kae, kdb, kde;
  uint32_t sa[NMASK];  // staged column m: first byte (16-B aligned) of the tile's strings in the pool
  uint32_t nv[NMASK];  //                  16-B vectors to copy
  uint32_t fits;
  uint32_t pad[5];
};
static_assert(sizeof(TileDesc) == 128, "TileDesc layout");

// d_overflow: [count, tile indices...] of the tiles that do not fit (host-built with the
// descriptors); a second launch evaluates them when n_overflow > 0
hipError_t launch_evaluate_tiled(const EvalArgs& a, const TileArgs& t, const TileArgs* d_t, const TileDesc* d_desc,
                                 bool fused, uint32_t grid, const uint32_t* d_overflow, uint32_t n_overflow,
                                 hipStream_t s);

}  // namespace kw
