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
//   Regex:   the Rust `regex` crate dialect of DESIGN.md §2 with search semantics
//            (Regex::is_match), matched over UTF-8 (automaton.cpp RParser).
// A pattern whose DFA exceeds the state budget becomes an NFA element of its chain (Dfa::nfa, the
// program of kwdev.hpp DevNfa), so no valid pattern fails a column.
#pragma once
#include <array>
#include <cstddef>
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
// Accepting is by *class*: every state carries the id of the set of patterns matched if the input
// ends there (acc[state]; class 0 = the empty set), and classes[c] lists that set (pattern indices,
// ascending). There is no bound on the number of patterns: a string's classification is one small
// integer, and the policy tables are indexed by it (slots.hpp), not by pattern bits.
struct Dfa {
  uint32_t nstates = 0;
  uint32_t ncls = 0;
  uint32_t start = 0;
  // States [abs_lo, nstates) are absorbing (every byte keeps them), as is the dead state 0: a walk
  // may stop as soon as it reaches one (kernels.hip), the accept class cannot change any more.
  uint32_t abs_lo = 0;
  std::array<uint8_t, 256> cls{};              // byte -> byte class
  std::vector<uint16_t> trans;                  // [state][byte class]
  std::vector<uint32_t> acc;                    // [state] accept class
  std::vector<std::vector<uint32_t>> classes;   // accept class -> pattern indices (classes[0] empty)
  // an NFA element: one pattern, classes {{}, {0}}, no tables; `prog` is its DevNfa record
  bool nfa = false;
  std::vector<uint8_t> prog;
  uint32_t run(const uint8_t* s, size_t n) const;  // accept class of the whole string
  size_t table_bytes() const { return nfa ? 0 : trans.size() * 2 + (size_t)nstates * 2 + 256; }
};

constexpr uint32_t kMaxDfaStates = 8192;

// Compiles patterns into one minimised DFA. Returns false with a message on a syntax error or
// when the automaton exceeds `max_states` (<= kMaxDfaStates).
bool compile_dfa(const std::vector<Pattern>& pats, Dfa* out, std::string* err, uint32_t max_states = kMaxDfaStates);
// Compiles a column's patterns into a chain of DFAs (greedy packing in pattern order), each within
// `max_table_bytes` of tables and `max_states` states; a string's pattern set is the union of its
// classes in every DFA of the chain. Class sets hold the column's pattern indices.
// firsts (optional): the index of the first pattern of each DFA (DFA k covers [firsts[k], firsts[k+1])).
bool compile_column(const std::vector<Pattern>& pats, size_t max_table_bytes, uint32_t max_states, std::vector<Dfa>* out,
                    std::string* err, std::vector<uint32_t>* firsts = nullptr);
// Syntax check of one regex (used by settings validation).
bool regex_ok(const std::string& re, std::string* err);
// Syntax check of any pattern (no automaton is built, so no size limit applies).
bool pattern_ok(const Pattern& p, std::string* err);
// One pattern as an NFA element (Dfa::nfa); false only on a syntax error or an NFA beyond
// kMaxNfaStates (Rust's compiled-size limit has the same role).
bool compile_nfa(const Pattern& p, Dfa* out, std::string* err);
// Runs a DevNfa record on the host (the kernels' nfa_run over host scratch).
bool run_nfa_record(const uint8_t* rec, const uint8_t* s, size_t n);

}  // namespace kw
