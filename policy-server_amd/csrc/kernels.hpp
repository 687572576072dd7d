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

hipError_t launch_classify(const uint8_t* d_blob, const ClassifyJobs& jobs, hipStream_t s);
hipError_t launch_evaluate(const EvalArgs& a, hipStream_t s);

}  // namespace kw
