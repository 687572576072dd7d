// env.hpp — EvaluationEnvironment for the declarative policy class.
//
// Mirrors src/evaluation/evaluation_environment.rs: the builder (EvaluationEnvironmentBuilder,
// :130-366) turns the policies document into an immutable registry of policies and groups; the
// accessors (:373-469) answer mode / allowed-to-mutate / namespace-bypass / settings questions.
// Where the reference registers a PolicyEvaluatorPre per Wasm digest (:391-431), this builder
// compiles each policy's settings into column DFAs + bitmask parameters (kwdev.hpp) and emits one
// position-independent blob that every GPU receives.
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
  // group
  std::string expression, message;
  std::vector<std::string> member_names;  // settings order
  std::vector<int32_t> members;
  GroupProgram prog;
  std::string broken_member;  // member id that failed to initialise (validate -> PolicyNotFound)
};

struct Env {
  std::string source;  // the policies document (re-sent with the blob to other ranks)
  std::vector<PolicyRec> pol;
  std::unordered_map<std::string, int32_t> ids;
  std::optional<std::string> always_ns;
  bool continue_on_errors = false;
  std::vector<Pattern> cols[NCOL];
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

}  // namespace kw
