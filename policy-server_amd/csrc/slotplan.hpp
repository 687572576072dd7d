// slotplan.hpp — host compiler of a selected policy list into slot-plan records (slots.hpp).
//
// The list is what EvaluationEnvironment::validate is asked to answer for every request of a batch
// (one output column per policy id). Plain policies take one slot each; a group takes one slot per
// member (evaluation_environment.rs:596-651 builds the member table per request; here it is built
// once per policy list). Columns are cut into chunks of at most 64 slots and 64 columns; the
// device runs one slot-kernel launch per chunk.
#pragma once
#include <cstdint>
#include <vector>

#include "env.hpp"
#include "slots.hpp"

namespace kw {

struct SlotChunk {
  uint32_t col0 = 0, ncols = 0, nslots = 0;
  bool groups = false;        // the chunk evaluates a group program (needs the LDS group stack)
  std::vector<uint8_t> rec;   // SlotHdr record, 16-B multiple
  uint32_t staged = 0;        // leading bytes the device stages in LDS (all but the ColInfo and cidx sections)
};

Status build_slot_chunks(const Env& E, const int32_t* pols, uint32_t npol, int origin, std::vector<SlotChunk>* out);

}  // namespace kw
