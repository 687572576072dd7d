// expr.hpp — policy-group expressions: the rhai subset used by policies.yml groups
// (policies.yml.example:32, README.md:97-123) compiled to a postfix program for the device.
//
// Reference behaviour (PolicyGroupEvaluator [upstream policy-evaluator v0.24.0, rhai 1.21.0]), as
// pinned by src/evaluation/evaluation_environment.rs:1075-1112:
//   valid:   "true || happy_policy_1()", "2 > 1", and "1 + 1" (the int is accepted at validation)
//   invalid: "unknown_policy() || happy_policy_1()" (function not found),
//            "something that doesn't make sense" (syntax), "happy_policy_1() + 1" (bool + int)
// and evaluated with rhai's short-circuit || and && (evaluation_environment.rs:979-1042): a member
// contributes a cause only if it was actually called. The device evaluates every member eagerly
// (one slot each), then runs the expression as short-circuit jump code over the member results: a
// member counts as called exactly when rhai would have called it, which gives the same causes.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace kw {

struct GroupProgram {
  bool valid = false;          // validate_settings() result
  std::string error;           // message when !valid
  bool eval_error = false;     // valid, but the result is not a bool (e.g. "1 + 1")
  std::string eval_message;
  std::vector<uint8_t> code;   // G_* jump code (kwdev.hpp): G_CALL + slot byte, G_JT / G_JF + u16 target
};

// members: member names in settings order (the slot of a call is its index here).
GroupProgram compile_group_expression(const std::string& expr, const std::vector<std::string>& members);

}  // namespace kw
