// kernels.hpp — launch interface of the device hot path (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kwdev.hpp"
#include "slots.hpp"

namespace kw {

// String columns a tile stages (each feeds the classification of one or more request columns).
enum Str : uint32_t { S_NS = 0, S_IMG, S_AA, S_CAPADD, S_CAPDROP, S_LK, S_LV, NSTR };

// Pass-side data of arguments that do not fit a verdict word's 16-bit ARG (kArgWide): an entity
// index >= 65535 (only requests beyond the tile capacities have one: the overflow kernel appends a
// record) and the cause mask of a > 15-member group (dense [row][nwide] array).
struct WideRec {
  uint32_t row_lo, row_hi, policy, value;
};

struct EvalArgs {
  const uint8_t* blob;
  uint64_t nrows;
  uint64_t ndesc;  // tile descriptors (TileDesc) to walk
  uint32_t npol;   // verdict words per row (all-pairs: the policy list; rows mode: 1)
  int32_t origin;
  const uint8_t* req_flags;
  const uint32_t* ctr_off;
  const uint32_t* lbl_off;
  const uint8_t* ctr_flags;
  const uint32_t* capadd_off;
  const uint32_t* capdrop_off;
  uint32_t* out;
  uint32_t* sched;  // per-XCD tile counters (256 u32 + 256 u32 done counts), nullptr = static schedule
  // overflow path: per-string classes in HBM (absolute entity indices), the wide-argument list
  uint16_t *g_ns, *g_aa, *g_img, *g_capadd, *g_capdrop, *g_lk, *g_lv;
  // NFA elements (kwdev.hpp DevNfa): their classes, computed by nfa_classify_kernel before the tile
  // kernel, [label][nlv] and [container][il.n()] at the element's chain position (nullptr = none)
  const uint16_t *nfa_lv, *nfa_img;
  uint32_t* wide_count;
  WideRec* wide_rec;
  uint32_t wide_cap;
  uint64_t* wide_groups;  // dense [row][nwide] cause masks
  uint32_t nwide;
  const uint32_t* rowcol;  // rows mode: per row (chunk << 16) | column, all-pairs: nullptr
  // diagnostics (KW_TILE_DEBUG & 512): per workgroup kPhaseWords u64: shader-clock cycles of thread
  // 0 summed over its tiles [staging P0, classify P1, derive D, walk P2, verdicts P3 + next tile,
  // tiles, whole workgroup, table staging], then the kSegWords segment clocks (Seg) summed over the
  // workgroup's waves; nullptr = off
  uint64_t* phase;
};
// Per-wave segment clocks of the timing instantiation: P1 / P2 item segments (wave-uniform per
// loop iteration), each phase's busy time and its barrier wait.
enum Seg : uint32_t {
  SG_P1_LABEL = 0, SG_P1_CAPSTR, SG_P1_CTR, SG_P1_IMAGE, SG_P1_REQ, SG_P2_CTR, SG_P2_LABEL, SG_P2_REQ,
  SG_P1_BUSY, SG_P1_WAIT, SG_P2_BUSY, SG_P2_WAIT, SG_P0_WAIT, SG_P3_BUSY, SG_P3_WAIT,
  SG_START,  // the workgroup's start (s_memrealtime, 100 MHz): residency of the grid
  SG_P0_TOP, SG_P0_REQ, SG_P0_STR,  // P0 issue: tile loop top to the descriptor fields, request-array copies, string copies
  kSegWords = 19
};
constexpr uint32_t kPhaseWords = 8 + kSegWords;

// Slot kernel geometry: one tile = up to 64 requests (one lane per request where a lane walks a
// request), 256 threads.
constexpr uint32_t kSlotRows = 64;
#ifndef KW_THREADS  // threads per tile workgroup (build-time A/B)
#define KW_THREADS 256
#endif
constexpr uint32_t kSlotThreads = KW_THREADS;
// Workgroups of `bytes` dynamic LDS one gfx950 CU holds at once (256 threads, LDS-bound): the CU's
// 160 KiB are allocated in 1280-byte granules, 128 of them — measured (scripts/lds_occ.hip,
// profiles/r05_lds_residency.txt): 53760 B holds 3, 53768 B holds 2, 32000 B 5, 32004 B 4. The HIP
// occupancy API's floor(160 KiB / bytes) overstates it between granule boundaries (r05: a C5 heavy
// layout of 53664 B planned at 3 ran at 2, a third of its grid waiting for the first two-thirds).
constexpr uint32_t kLdsGranule = 1280, kLdsGranules = 128;
constexpr uint32_t lds_workgroups_per_cu(uint32_t bytes) {
  const uint32_t g = (bytes + kLdsGranule - 1) / kLdsGranule;
  return g ? kLdsGranules / g : kLdsGranules;
}
// Families a tile-kernel instantiation carries (TileArgs::feat).
constexpr uint32_t kFeatImg = 1, kFeatLbl = 2, kFeatCtr = 4, kFeatGrp = 8, kFeatAll = 15;
// A pass whose classifiers hold NFA elements runs the one instantiation that reads their classes
// (kFeatAll | kFeatNfa): no other instantiation carries that code.
constexpr uint32_t kFeatNfa = 16;
// Tiles with many containers per request (TileArgs::ctr_ranges) in the label / container family set
// with LDS tables (C5's heavy region): P2 takes a container's predecessor sets from a segmented
// wave OR-scan. Its own instantiation, so the others (C4's) keep their code and registers.
constexpr uint32_t kFeatRng = 32;
#ifndef KW_PREFETCH  // tile kernel: the code of the next-tile L2 prefetch (run only when the plan asks:
#define KW_PREFETCH 1   // capi.cpp l2_prefetch, off by default; r02 s60: running it cost C4 0.3442 vs 0.3294 ms)
#endif
#ifndef KW_PF_LANES  // lanes per wave issuing the next tile's L2 prefetch (its LDS landing line: 4 B each)
#define KW_PF_LANES 64
#endif
constexpr uint32_t kPfLanes = KW_PF_LANES;
constexpr uint32_t kMaxChunks = 8;  // chunks of one launch (<= 512 slots); longer lists take several launches

struct ChunkArgs {
  const uint8_t* rec;  // device copy of the SlotHdr record (ColInfo and programs are read here)
  uint32_t o_lds;      // LDS offset of the record's staged prefix (tables in LDS), else 0
  uint32_t col0, ncols, vec4;
  uint64_t init;
};

// Per-launch geometry and LDS layout. Lives in device memory; the kernel reads it with scalar loads.
struct TileArgs {
  uint32_t rows;                  // requests per tile
  uint32_t cmax, kmax, lmax;      // container / capability / label capacity of a staged tile
  uint32_t o_rf, o_coff, o_loff, o_cflags, o_cadd, o_cdrop;  // staged headers (LDS byte offsets)
  // per-entity classes (u16): namespace [rows], AppArmor [cmax], image [cmax][il.n()], added /
  // dropped capabilities [kmax], label keys [lmax], label values [lmax][nlv]. In a single-chunk
  // pass whose value classes fold into the walk, o_lv's region doubles as the label-pair helper
  // lanes' per-wave 128-B mailboxes (kernels.hip label_pairs: needs lmax * nlv * 2 >= 4 x 128)
  uint32_t o_ns, o_aa, o_img, o_capadd, o_capdrop, o_lk, o_lv;
  ImgLayout il;
  uint32_t nlv;
  uint32_t need;  // bit per Str: the pass classifies that string column
  uint32_t o_vadd, o_vl, o_vc, o_vtr;  // u64 violation sets: per added capability, per label, per container (2)
  uint32_t o_own_c, o_own_l;           // u8 tile-local request of each staged container / label
  uint32_t o_rej, o_mut, o_byp;        // per-request results: rejected / mutated slots, bypass flag
  uint32_t o_nx;                       // u32[4]: the tile after next (dynamic schedule), double-buffered; P1 / P2 block counters
  uint32_t o_desc;                     // TileDesc[2]: this tile's and the next tile's descriptor
  uint32_t o_pf;                       // 4 x kPfLanes B: LDS-DMA landing of the L2 prefetch (never read)
  uint32_t prefetch;                   // warm L2 with the next tile (small tiles at >= 3 workgroups per CU)
  uint32_t feat;                       // kFeat* families of the launch (selects the kernel instantiation)
  uint32_t ctr_ranges;                 // many containers per request: P2 ORs predecessor ranges four a round
  uint32_t o_sa;                       // u32[NSTR]: the tile's staged byte start per string column
  uint32_t o_vw, vw_stride;            // violation words [rows][vw_stride] (aliases the staged strings)
  uint32_t o_so[NSTR], o_sb[NSTR], sb_cap[NSTR];  // staged string offsets / bytes (0 = not staged)
  const uint32_t* s_off[NSTR];
  const uint8_t* s_bytes[NSTR];
  // column classifiers: LDS offsets when staged (lds_tables), blob offsets always
  uint32_t lds_tables;
  uint32_t lit_lds[NCOL], dfa_lds[NCOL], kv_lds;
  uint32_t lit_blob[NCOL], dfa_blob[NCOL], kv_blob, nlk;
  uint32_t nstage;
  uint32_t stage_blob[NCOL + kMaxChunks], stage_lds[NCOL + kMaxChunks], stage_bytes[NCOL + kMaxChunks];
  uint32_t bypass_cls, docker_io_cls, latest_cls;
  uint32_t nchunk;
  ChunkArgs chunk[kMaxChunks];
  uint32_t rows_mode;
  uint32_t debug;  // diagnostics: bit0 skip classification, bit1 skip walk, bit2 skip output; 512 phase
                  // clocks; 1024 skip mandatory labels, 2048 skip label-value DFAs, 4096 skip predecessor ORs,
                  // 8192 skip capability mutations (P2), 16384 skip container / label violation words (P2),
                  // 32768 / 65536 skip the image DFA chains / literal lookups (P1)
  uint32_t lds_bytes;
};

// Per-tile geometry, precomputed on the host from the batch's offsets (one s_load burst per tile
// instead of a chain of dependent global loads): entity ranges, the 16-B aligned byte range of each
// staged string column, and whether the tile fits the LDS capacities.
// A tile is a run of at most kSlotRows requests; runs that exceed the LDS capacities are halved
// until they fit, and single requests that still do not fit go to the overflow kernels.
struct alignas(16) TileDesc {
  uint32_t cb, ce, lb, le, kab, kae, kdb, kde;
  uint32_t sa[NSTR];  // staged column: first byte (16-B aligned) of the tile's strings in the pool
  uint32_t pad0;
  uint32_t nv[NSTR];  //                16-B vectors to copy
  uint32_t fits;
  uint32_t r0lo, r0hi, nr;  // first request (64-bit) and request count
  uint32_t pad[4];
};
static_assert(sizeof(TileDesc) == 128, "TileDesc layout");

// One launch of the tile kernel over chunks t.chunk[0..nchunk). t: host copy (launch geometry);
// d_t: the same TileArgs resident in device memory (read by the kernel).
hipError_t launch_evaluate_tiles(const EvalArgs& a, const TileArgs& t, const TileArgs* d_t, const TileDesc* d_desc,
                                 uint32_t grid, hipStream_t s);
// Requests that do not fit the LDS capacities even alone (d_overflow: [count, request indices...],
// host-built with the descriptors): classified into HBM, then walked sequentially per request.
// Wide policy groups (expr.hpp: more than 64 members, or a value stack deeper than 64): the
// members ran as a separate all-pairs pass into `member_words` [row][nmw]; the combine kernel runs
// each group's jump code per row over their results. One record per wide group column of the pass.
struct WideGroupArgs {
  uint32_t prog_off, prog_len;  // jump code in `progs`
  uint32_t col;                 // all-pairs: the group's output column; rows mode: its column id
  uint32_t nmem, midx_off;      // member slot s -> member_words column midx[midx_off + s]
  uint32_t okw, rejb;           // the group's accepted / rejected verdict words (reason GROUP, ARG wide)
  uint32_t cause_off, cause_words;  // its cause bitset in the per-row side data
  uint32_t errw;                // script programs: the evaluation-error verdict word (reason GROUP_EXPR)
  uint32_t kind;                // 0 jump code (run_wide_prog), 1 script bytecode (run_script_prog),
                                // 2 / 3 a split safe-labels / psp-capabilities policy (combine_parts)
  uint32_t mutw;                // split psp-capabilities: the mutated verdict word
};

constexpr uint32_t kSplitMember = 0x80000000u;  // a group's midx entry naming a split member's record

// A split policy's word from its parts' words (env.cpp split_policy): the first part that rejects
// (safe-labels: a mandatory index offset by the part's start), else — psp-capabilities, whose later
// parts validate nothing — mutated when any part mutated, else accepted. part(s): part s's word.
template <class Part>
KW_HD inline uint32_t combine_parts(const WideGroupArgs& g, const uint32_t* part_off, Part part) {
  bool mutated = false;
  for (uint32_t s = 0; s < g.nmem; ++s) {
    const uint32_t x = part(s);
    if (!(x & KW_V_ALLOWED)) {
      uint32_t reason = KW_REASON(x), arg = KW_ARG(x);
      if (reason == KW_R_LABEL_MANDATORY && arg != kArgWide) arg += part_off[s];
      return g.rejb | vword(reason, arg);
    }
    if (x & KW_V_MUTATED) mutated = true;
  }
  return mutated ? g.mutw : g.okw;
}
struct WideGroupPass {
  const WideGroupArgs* groups;
  uint32_t ngroups;
  const uint8_t* progs;
  const uint32_t* midx;
  const uint32_t* member_words;  // [row][nmw]
  uint32_t nmw;
  uint32_t* out;                 // the pass's verdict words
  uint32_t npol;                 // all-pairs stride; rows mode: 1
  const uint32_t* rowcol;        // rows mode: the row's column id (== WideGroupArgs::col), nullptr = all pairs
  uint64_t* causes;              // [row][cause_stride] u64
  uint32_t cause_stride;
  uint64_t* stack;               // scratch: stack_words u64 per thread of the grid
  uint32_t stack_words;
  uint64_t nrows;
};
hipError_t launch_wide_groups(const WideGroupPass& w, uint32_t grid, hipStream_t s);

hipError_t launch_overflow(const EvalArgs& a, const TileArgs* d_t, const uint32_t* d_overflow, uint32_t n_overflow,
                           hipStream_t s);

// The NFA elements of a pass (kwdev.hpp DevNfa): every label value under its key's chain and every
// image reference under the registry / tag / image chains, one thread per entity, a Pike VM per
// element with its lists in `scratch` (words_per_thread u32 per thread of the grid: the largest
// program's nfa_scratch_words, then room for a normalised image reference of subj_bytes).
struct NfaPass {
  uint16_t* lv;   // [nlabels][nlv]
  uint16_t* img;  // [nctrs][nim]
  uint32_t* scratch;
  uint64_t words_per_thread;
  uint32_t nfa_words, subj_bytes;
  uint32_t nlv, nim;
  uint64_t nlabels, nctrs;
  uint32_t do_lv, do_img;
};
// Bulk path (kw_validate_host): a chunk's column ranges arrive in one H2D copy, packed, and this
// kernel moves each range to its place in the batch's device image (one copy per chunk instead of
// one per column: a pinned H2D copy costs ~9.6 us on its own, profiles/r05_bulk_copies.txt).
// src_off == dst_off (mod 16), so the body moves 16-byte words.
constexpr uint32_t kMaxScatterSegs = 24;
struct ScatterSeg {
  uint64_t dst_off, src_off, bytes;
};
struct ScatterArgs {
  uint8_t* dst;
  const uint8_t* src;
  uint32_t nseg;
  ScatterSeg seg[kMaxScatterSegs];
};
hipError_t launch_scatter(const ScatterArgs& a, hipStream_t s);

hipError_t launch_nfa_classify(const EvalArgs& a, const TileArgs* d_t, const NfaPass& np, uint32_t threads, hipStream_t s);
// threads of the NFA pass's grid for `items` entities within a scratch budget
uint32_t nfa_threads(uint64_t items, uint64_t words_per_thread);

}  // namespace kw
