// slotplan.hpp — host compiler of a selected policy list into slot-plan records (slots.hpp).
//
// The list is what EvaluationEnvironment::validate is asked to answer for every request of a batch
// (one output column per policy id). Plain policies take one slot each (policies with identical
// compiled settings share one); a group takes one slot per member (evaluation_environment.rs:596-651
// builds the member table per request; here it is built once per policy list). Columns are cut into
// chunks of at most 64 slots, 64 columns and 64 local bits of each kind; one launch of the device
// evaluates every chunk of a list over each staged tile of requests.
#pragma once
#include <cstdint>
#include <vector>

#include "env.hpp"
#include "slots.hpp"

namespace kw {

struct SlotChunk {
  uint32_t col0 = 0, ncols = 0, nslots = 0;
  bool groups = false;
  uint32_t nwide = 0;         // > 15-member group columns (their cause masks go to the dense side array)
  std::vector<uint8_t> rec;   // SlotHdr record, 16-B multiple
  uint32_t staged = 0;        // leading bytes the device stages in LDS (all but ColInfo and programs)
};

// wide_base: first dense-array index of this list's wide groups (all-pairs: running over chunks;
// rows mode passes rows_mode = true and every wide group uses index 0 of its row).
Status build_slot_chunks(const Env& E, const int32_t* pols, uint32_t npol, int origin, bool rows_mode,
                         std::vector<SlotChunk>* out);

}  // namespace kw
