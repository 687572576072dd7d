// automaton.hpp — pattern sets -> one multi-pattern DFA per request column.
//
// This is the load-time "compile" step that replaces precompile_policies / PrecompiledPolicy
// (src/lib.rs:287-307, src/evaluation/precompiled_policy.rs:46-64) for the declarative class:
// instead of AOT-compiling a Wasm module per policy, every string pattern that any policy's
// settings name for a column (registries, tags, images, capability names, AppArmor profiles,
// label keys, label-value regexes, namespaces) becomes one bit of a single DFA for that column.
// Running the DFA over a string yields the bitmask of all patterns the string matches; policies
// are then bit tests on those masks (kernels.hip).
//
// Pattern semantics:
//   Literal: whole-string byte equality.
//   Glob:    whole-string fnmatch(3) with flags 0: '*' any bytes (including '/'), '?' one byte,
//            '[...]' / '[!...]' / '[^...]' sets with ranges and [:class:], '\' escapes.
//   Regex:   POSIX ERE subset with search semantics (Rust Regex::is_match): alternation, groups,
//            * + ? {m} {m,} {m,n}, '.', sets, '^' '$' assertions, \d \D \w \W \s \S escapes.
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <vector>

namespace kw {

struct Pattern {
  enum Kind : uint8_t { Literal = 0, Glob = 1, Regex = 2 };
  Kind kind = Literal;
  std::string text;
  bool operator==(const Pattern& o) const { return kind == o.kind && text == o.text; }
};

// A compiled column automaton. State 0 is the dead state; `start` is the initial state.
struct Dfa {
  uint32_t nstates = 0;
  uint32_t ncls = 0;
  uint32_t start = 0;
  std::array<uint8_t, 256> cls{};  // byte -> class
  std::vector<uint16_t> trans;      // [state][class]
  std::vector<uint64_t> accept;     // [state] bitmask of patterns matched if input ends here
  uint64_t run(const uint8_t* s, size_t n) const;
};

constexpr uint32_t kMaxDfaStates = 8192;
constexpr size_t kMaxPatternsPerColumn = 64;
// per-DFA table budget of a column chain (LDS-resident in the classify kernel)
constexpr size_t kMaxDfaTableBytes = 24 * 1024;

// Compiles up to 64 patterns into one minimised DFA. Returns false with a message on a
// syntax error or when the automaton exceeds kMaxDfaStates.
bool compile_dfa(const std::vector<Pattern>& pats, Dfa* out, std::string* err);
// Compiles a column's patterns into a chain of DFAs, each within `max_table_bytes` of tables
// (greedy packing in pattern order); accept masks keep the global pattern bit of each pattern.
bool compile_column(const std::vector<Pattern>& pats, size_t max_table_bytes, std::vector<Dfa>* out,
                    std::string* err);
// Syntax check of one regex (used by settings validation).
bool regex_ok(const std::string& re, std::string* err);

}  // namespace kw
