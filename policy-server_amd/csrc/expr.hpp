// expr.hpp — policy-group expressions: the rhai script subset used by policies.yml groups
// (policies.yml.example:32, README.md:97-123), interpreted on the host and compiled for the device.
//
// Reference behaviour (PolicyGroupEvaluator [upstream policy-evaluator v0.24.0, rhai 1.21.0], absent
// from the reference tree), as pinned by src/evaluation/evaluation_environment.rs:1075-1112:
//   valid:   "true || happy_policy_1()", "2 > 1", and "1 + 1" (the int is accepted at validation)
//   invalid: "unknown_policy() || happy_policy_1()" (function not found),
//            "something that doesn't make sense" (syntax), "happy_policy_1() + 1" (bool + int)
// and evaluated with rhai's short-circuit || and && (evaluation_environment.rs:979-1042): a member
// contributes a cause only if it was actually called. Validation therefore runs the script with
// every member returning true and refuses it on any error; evaluation runs it with the members'
// real results and needs a bool.
//
// Language (rhai semantics, parity unpinned beyond the vectors above): statements separated by `;`
// (`let name = expr;`, expression statements), blocks `{ ... }` whose value is their last
// expression without a `;`, `if c { } else if c { } else { }` expressions, literals (true / false,
// integers with `_` separators, "strings" with \n \t \r \0 \\ \" \' escapes), variables, member
// calls `name()`, unary ! - +, and the binary operators || | ^ && & == != < <= > >= + - * / % with
// rhai's precedence. Values are (), bool, i64 or string; == / != / < ... between different types
// are false (!= true), as rhai's built-in comparisons; other mismatches are "Function not found"
// errors; i64 arithmetic is checked (overflow and division by zero are errors).
//
// Device forms (slotplan.cpp), chosen at load:
//   jump code  bool-only programs (member calls, ! && || == != over bools, constants folded) with at
//              most 64 members and a value stack of at most 64: run per request (slots.hpp);
//   table      anything else with at most 16 members: the interpreter's outcome for every vector
//              of member results (2^n entries: value, error, causes);
//   wide       bool-only programs with more than 64 members or a deeper stack: the members run as a
//              separate pass and a combine kernel runs the jump code (u16 member operands, stack in
//              global scratch) over their verdict words;
//   script     anything else with more than 16 members: the same separate member pass, and the
//              combine kernel runs typed bytecode (slots.hpp run_script_prog: (), bool, i64 and
//              string values, `let` slots, rhai's checked arithmetic; the host interpreter words the
//              messages). No member count is refused.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace kw {

struct ExprAst;  // expr.cpp

// Outcome of one run of the script over member results.
struct ExprOutcome {
  bool error = false;      // evaluation error (message), or a non-bool result (the "Output type" error)
  bool value = false;      // the bool result when !error
  std::string message;     // error text (rhai-shaped)
  std::vector<uint32_t> called;  // members called, in call order (each once)
};

struct GroupProgram {
  bool valid = false;          // validate_settings() result
  std::string error;           // message when !valid
  bool eval_error = false;     // valid, but every run fails the same way (e.g. "1 + 1": not a bool)
  std::string eval_message;
  // device forms (exactly one is set when valid && !eval_error)
  std::vector<uint8_t> code;   // G_* jump code (kwdev.hpp); G_CALL16 operands when wide
  uint32_t depth = 0;          // value-stack depth of `code`
  bool wide = false;           // jump code for the wide path (> 64 members or depth > 64), or a script
  bool script = false;         // `code` is typed script bytecode (kwdev.hpp SOp), run on the wide path
  std::vector<uint32_t> table; // 2^nmem entries: bit 0 value, bit 1 error, bits 16..31 causes
  std::shared_ptr<const ExprAst> ast;
  uint32_t nmem = 0;
  // host interpreter (kw_format_response's messages, the host diagnostics)
  ExprOutcome run(const std::function<bool(uint32_t)>& member_ok) const;
};

// Table entry layout
constexpr uint32_t kGtValue = 1u, kGtError = 2u;
constexpr uint32_t kMaxTableMembers = 16;
constexpr uint32_t kMaxWideStack = 1u << 16;  // value-stack bound of the wide path (scratch words)

// The response message of a run that failed (ExprOutcome::message): a non-bool result or an error.
std::string group_eval_message(const std::string& outcome_message);

// members: member names in settings order (the slot of a call is its index here).
// force_wide: a form the wide path runs (wide jump code or script bytecode), for groups whose
// members' words are combined in the wide path (a split member).
GroupProgram compile_group_expression(const std::string& expr, const std::vector<std::string>& members,
                                      bool force_wide = false);

}  // namespace kw
