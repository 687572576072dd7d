// env.hpp — EvaluationEnvironment for the declarative policy class.
//
// Mirrors src/evaluation/evaluation_environment.rs: the builder (EvaluationEnvironmentBuilder,
// :130-366) turns the policies document into an immutable registry of policies and groups; the
// accessors (:373-469) answer mode / allowed-to-mutate / namespace-bypass / settings questions.
// Where the reference registers a PolicyEvaluatorPre per Wasm digest (:391-431), this builder
// collects every string pattern the policies' settings name per request column and compiles each
// column into a classifier (literal perfect hash, DFA chain, per-key label-value DFAs; kwdev.hpp),
// emitted as one position-independent blob that every GPU receives. What each class means for each
// policy is compiled per policy list (slotplan.cpp).
#pragma once
#include <cstdint>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "automaton.hpp"
#include "expr.hpp"
#include "kwdev.hpp"

namespace kw {

struct PolicyRec {
  std::string id;           // PolicyID Display (policy_id.rs:20-27): "name" or "group/name"
  std::string name, group;  // group empty unless a member
  std::string module;
  bool is_group = false;
  bool is_member = false;
  int32_t parent = -1;
  uint8_t family = FAM_NONE;
  uint8_t mode = 0;         // KW_MODE_*
  bool allowed_to_mutate = false;
  bool registered = false;  // present in policy_id_to_settings (mode/mutate lookups succeed)
  bool init_error = false;
  std::string init_message;
  uint8_t flags = 0;        // PF_SKIP_INIT | PF_SKIP_EPHEMERAL | PF_ALLOW_ALL
  // settings lists, same meaning as the oracle (DESIGN.md §Policy families)
  std::vector<std::string> lists[5];
  // the lists as pattern ids of their request column (env.cpp compile): namespace [0] COL_NS;
  // trusted-repos [0,1] COL_REG, [2] COL_TAG, [3,4] COL_IMG; capabilities [0] allowed (without "*"),
  // [1] required drops, [2] default adds, [3] {"ALL"} COL_CAP; apparmor [0] COL_AA; labels [0] denied,
  // [1] mandatory (settings order), [2] constrained keys COL_LK, [3] their regexes COL_LV
  std::vector<uint32_t> pid[5];
  // group
  std::string expression, message;
  std::vector<std::string> member_names;  // settings order
  std::vector<int32_t> members;
  GroupProgram prog;
  std::string broken_member;  // member id that failed to initialise (validate -> PolicyNotFound)
  // a policy beyond the 64 local bits of one slot-plan chunk (more than 64 distinct mandatory labels,
  // more than 63 required-drop / default-add capabilities) is evaluated as consecutive parts (hidden
  // records after the visible ones, each within the limit), combined on the wide path: the first
  // part that rejects (safe-labels: mandatory indices offset by part_off), or psp-capabilities' part
  // 0 validation then any part's mutation (env.cpp split_policy)
  std::vector<int32_t> parts;
  std::vector<uint32_t> part_off;
  bool is_part = false;
};

// Host description of one column's classifier (the blob holds its tables).
struct ColumnInfo {
  std::vector<Pattern> pats;                      // pattern id = index
  std::vector<std::vector<uint32_t>> class_pats;  // global class -> pattern ids it matches (class 0: none)
  std::vector<uint32_t> lit_cls;                  // pattern id -> literal class (0 = not in the literal table)
  uint64_t nfa_words = 0;                         // largest NFA element's scratch (nfa_scratch_words), 0 = none
};

// COL_LV class: label-key class `key`, the value regexes of the key's DFA that produced it
// (`covered`) and those it matched.
struct KvClass {
  uint32_t key = 0;
  std::vector<uint32_t> covered, matched;
};

struct Env {
  std::string source;  // the policies document (re-sent with the blob to other ranks)
  std::vector<PolicyRec> pol;  // the visible policies [0, nvisible), then the parts of split ones
  size_t nvisible = 0;
  std::unordered_map<std::string, int32_t> ids;
  std::optional<std::string> always_ns;
  bool continue_on_errors = false;
  ColumnInfo cols[NCOL];
  std::vector<KvClass> kv;                    // per COL_LV class
  std::vector<std::vector<uint32_t>> kv_of_key;  // label-key class -> its COL_LV classes
  std::vector<uint8_t> blob;  // compiled tables (host copy)
  // device copy
  int device = -1;
  void* d_blob = nullptr;
  ~Env();
};

// EvaluationError-coded result: code is a KW_* status, message its Display string.
struct Status {
  int code = 0;
  std::string message;
  bool ok() const { return code == 0; }
};

Status build_env(const char* json, size_t len, bool continue_on_errors, const char* always_ns, Env* env);
Status env_from_blob(const void* blob, size_t len, Env* env);
std::vector<uint8_t> env_serialize(const Env& env);
// PolicyID::from_str + lookup
Status env_lookup(const Env& env, const std::string& id, int32_t* idx);
// EvaluationEnvironment::validate_settings (evaluation_environment.rs:472-510)
Status env_validate_settings(const Env& env, int32_t idx);

const char* family_name(uint8_t fam);

// Host classification with the blob's tables (diagnostics and the host walk; the kernels run the
// same tables). Classes of string s in column c: the literal class when the column has a literal
// table, then one per DFA of the chain (COL_NS / COL_REG / COL_TAG / COL_IMG / COL_CAP / COL_AA / COL_LK).
std::vector<uint32_t> host_classes(const Env& env, Col c, const uint8_t* s, size_t n);
// COL_LV classes of value s under label-key class `key` (one per DFA of the key's chain).
std::vector<uint32_t> host_value_classes(const Env& env, uint32_t key, const uint8_t* s, size_t n);

}  // namespace kw
