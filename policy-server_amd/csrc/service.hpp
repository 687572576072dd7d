// service.hpp — the service::evaluate epilogue on the host: verdict word -> AdmissionResponse JSON.
//
// Mirrors src/api/service.rs:30-152 (namespace bypass response, PolicyInitialization -> reject 500,
// validate vs audit) and validation_response_with_constraints (service.rs:160-208), plus the
// group response shape of PolicyGroupEvaluator [upstream] (message + details.causes with
// field "spec.policies.<member>", evaluation_environment.rs:979-995, integration_test.rs:118-131).
#pragma once
#include <cstdint>
#include <string>

#include "batch.hpp"
#include "env.hpp"

namespace kw {

// Rejection message of a policy for a row (DESIGN.md §Policy families, message templates), from
// the reason and its full argument (an entity index within the request, a settings index or a group
// cause mask). An argument out of range for the row is an engine error, never another entity's text.
Status policy_message(const Env& env, const Batch& b, uint64_t row, int32_t pidx, uint32_t reason, uint64_t arg,
                      std::string* msg);

// Full AdmissionResponse JSON for (row, policy, verdict). member_v: member verdict words for a
// group (settings order). Returns a non-ok Status for EvaluationError outcomes.
// doc / doc_len / doc_kind: the row's original document; required only to build the JSONPatch of
// an accepted mutation (F_PATCH), which is not recoverable from the flattened columns.
Status format_response(const Env& env, const Batch& b, uint64_t row, int32_t pidx, uint32_t v, const uint32_t* member_v,
                       std::string* out, const char* doc = nullptr, size_t doc_len = 0, int doc_kind = 0);

// psp-capabilities mutation of one document: the JSONPatch (RFC 6902) ops that add
// the policy's missing required drops and default adds to every container, as compact JSON.
Status capabilities_patch(const PolicyRec& P, const char* doc, size_t len, int doc_kind, std::string* ops);

// Host restatement of the image split used only for message text (registry / tag names).
void image_parts(std::string_view image, std::string* registry, std::string* tag, bool* has_tag);

}  // namespace kw
