// env.cpp — policies document -> EvaluationEnvironment (env.hpp).
//
// Schema (src/config.rs):
//   PolicyOrPolicyGroup is an untagged enum (config.rs:360-394): an entry is a Policy when it has
//   a string `module` and valid optional fields (policyMode "monitor"|"protect" default protect,
//   allowedToMutate bool, settings map|null, contextAwareResources list); otherwise a PolicyGroup
//   (policyMode, policies: map name -> PolicyGroupMember with deny_unknown_fields (config.rs:342),
//   expression string, message string); otherwise "data did not match any variant".
//   validate_policies (config.rs:237-258) rejects '/' in policy and member names.
// Builder (evaluation_environment.rs:198-365): PolicyID parse; per policy bootstrap + settings
// validation; under continue_on_errors failures are recorded in policy_initialization_errors
// instead of aborting; group members are Protect / not allowed to mutate (:297-301); groups are
// not allowed to mutate (:270-274).
#include "env.hpp"

#include <algorithm>
#include <map>
#include <cstring>

#include "../../include/kwgpu.h"
#include "json.hpp"

namespace kw {

const char* family_name(uint8_t f) {
  switch (f) {
    case FAM_PRIVILEGED: return "pod-privileged";
    case FAM_NAMESPACE: return "namespace-validate";
    case FAM_TRUSTED_REPOS: return "trusted-repos";
    case FAM_CAPABILITIES: return "psp-capabilities";
    case FAM_APPARMOR: return "psp-apparmor";
    case FAM_LABELS: return "safe-labels";
    case FAM_GROUP: return "policy-group";
    default: return "unknown";
  }
}

// Module URL -> declarative family (DESIGN.md §Policy families). Anything else is outside the
// class this engine serves and fails bootstrap like an unfetchable module would.
static uint8_t detect_family(const std::string& module) {
  auto has = [&](const char* s) { return module.find(s) != std::string::npos; };
  if (has("pod-privileged")) return FAM_PRIVILEGED;
  if (has("namespace-validate")) return FAM_NAMESPACE;
  if (has("trusted-repos")) return FAM_TRUSTED_REPOS;
  if (has("psp-capabilities")) return FAM_CAPABILITIES;
  if (has("psp-apparmor")) return FAM_APPARMOR;
  if (has("safe-labels")) return FAM_LABELS;
  return FAM_NONE;
}

namespace {

struct Entry {
  std::string name;
  bool is_group = false;
  std::string module;
  uint8_t mode = 0;
  bool a2m = false;
  int64_t settings = -1;  // node index or -1 (None / null)
  std::string expression, message;
  struct Member {
    std::string name, module;
    int64_t settings = -1;
  };
  std::vector<Member> members;
};

bool parse_mode(const JDoc& d, int64_t n, uint8_t* mode, std::string* err) {
  if (n < 0 || d.is((uint32_t)n, JType::Null)) {
    *mode = KW_MODE_PROTECT;
    return true;
  }
  if (!d.is((uint32_t)n, JType::Str)) {
    *err = "invalid type for policyMode";
    return false;
  }
  std::string_view s = d.str((uint32_t)n);
  if (s == "protect") *mode = KW_MODE_PROTECT;
  else if (s == "monitor") *mode = KW_MODE_MONITOR;
  else {
    *err = "unknown variant `" + std::string(s) + "`, expected `monitor` or `protect`";
    return false;
  }
  return true;
}

bool check_settings_node(const JDoc& d, int64_t n) {
  return n < 0 || d.is((uint32_t)n, JType::Null) || d.is((uint32_t)n, JType::Obj);
}

bool check_ctx_resources(const JDoc& d, int64_t n) {
  if (n < 0 || d.is((uint32_t)n, JType::Null)) return true;
  if (!d.is((uint32_t)n, JType::Arr)) return false;
  for (uint32_t k = 0; k < d.count((uint32_t)n); ++k) {
    uint32_t it = d.kids((uint32_t)n)[k].node;
    if (!d.is(it, JType::Obj)) return false;
    int64_t av = d.get(it, "apiVersion"), kd = d.get(it, "kind");
    if (av < 0 || kd < 0 || !d.is((uint32_t)av, JType::Str) || !d.is((uint32_t)kd, JType::Str)) return false;
  }
  return true;
}

// untagged PolicyOrPolicyGroup
bool parse_entry(const JDoc& d, const std::string& name, uint32_t node, Entry* e, std::string* err) {
  e->name = name;
  if (!d.is(node, JType::Obj)) {
    *err = "data did not match any variant of untagged enum PolicyOrPolicyGroup";
    return false;
  }
  // variant 1: Policy
  {
    int64_t mod = d.get(node, "module");
    std::string merr;
    bool ok = mod >= 0 && d.is((uint32_t)mod, JType::Str);
    uint8_t mode = 0;
    if (ok) ok = parse_mode(d, d.get(node, "policyMode"), &mode, &merr);
    int64_t a2m = d.get(node, "allowedToMutate");
    if (ok && a2m >= 0 && !d.is((uint32_t)a2m, JType::Null) && !d.is((uint32_t)a2m, JType::Bool)) ok = false;
    int64_t st = d.get(node, "settings");
    if (ok && !check_settings_node(d, st)) ok = false;
    if (ok && !check_ctx_resources(d, d.get(node, "contextAwareResources"))) ok = false;
    if (ok) {
      e->is_group = false;
      e->module = std::string(d.str((uint32_t)mod));
      e->mode = mode;
      e->a2m = a2m >= 0 && d.is((uint32_t)a2m, JType::Bool) && d.n((uint32_t)a2m).b;
      e->settings = (st >= 0 && d.is((uint32_t)st, JType::Obj)) ? st : -1;
      return true;
    }
  }
  // variant 2: PolicyGroup
  {
    std::string merr;
    uint8_t mode = 0;
    bool ok = parse_mode(d, d.get(node, "policyMode"), &mode, &merr);
    int64_t pols = d.get(node, "policies"), ex = d.get(node, "expression"), msg = d.get(node, "message");
    ok = ok && pols >= 0 && d.is((uint32_t)pols, JType::Obj) && ex >= 0 && d.is((uint32_t)ex, JType::Str) &&
         msg >= 0 && d.is((uint32_t)msg, JType::Str);
    if (ok) {
      for (uint32_t k = 0; k < d.count((uint32_t)pols) && ok; ++k) {
        const JKid& kid = d.kids((uint32_t)pols)[k];
        uint32_t m = kid.node;
        if (!d.is(m, JType::Obj)) {
          ok = false;
          break;
        }
        Entry::Member mem;
        mem.name = std::string(d.key(kid));
        for (uint32_t j = 0; j < d.count(m); ++j) {
          std::string_view key = d.key(d.kids(m)[j]);
          if (key != "module" && key != "settings" && key != "contextAwareResources") {
            ok = false;  // deny_unknown_fields (config.rs:342)
            break;
          }
        }
        int64_t mm = d.get(m, "module");
        if (!ok || mm < 0 || !d.is((uint32_t)mm, JType::Str)) {
          ok = false;
          break;
        }
        int64_t st = d.get(m, "settings");
        if (!check_settings_node(d, st) || !check_ctx_resources(d, d.get(m, "contextAwareResources"))) {
          ok = false;
          break;
        }
        mem.module = std::string(d.str((uint32_t)mm));
        mem.settings = (st >= 0 && d.is((uint32_t)st, JType::Obj)) ? st : -1;
        e->members.push_back(mem);
      }
    }
    if (ok) {
      e->is_group = true;
      e->mode = mode;
      e->expression = std::string(d.str((uint32_t)ex));
      e->message = std::string(d.str((uint32_t)msg));
      return true;
    }
  }
  *err = "data did not match any variant of untagged enum PolicyOrPolicyGroup";
  return false;
}

// ---- settings helpers: errors become "Policy settings are invalid: <msg>" (evaluation_environment.rs:487-492)
bool get_list(const JDoc& d, int64_t obj, const char* key, const std::string& path, std::vector<std::string>* out,
              std::string* err) {
  if (obj < 0) return true;
  int64_t n = d.get((uint32_t)obj, key);
  if (n < 0 || d.is((uint32_t)n, JType::Null)) return true;
  if (!d.is((uint32_t)n, JType::Arr)) {
    *err = path + " must be a list of strings";
    return false;
  }
  for (uint32_t k = 0; k < d.count((uint32_t)n); ++k) {
    uint32_t it = d.kids((uint32_t)n)[k].node;
    if (!d.is(it, JType::Str)) {
      *err = path + " must be a list of strings";
      return false;
    }
    out->push_back(std::string(d.str(it)));
  }
  return true;
}

bool get_obj(const JDoc& d, int64_t obj, const char* key, const std::string& path, int64_t* out, std::string* err) {
  *out = -1;
  if (obj < 0) return true;
  int64_t n = d.get((uint32_t)obj, key);
  if (n < 0 || d.is((uint32_t)n, JType::Null)) return true;
  if (!d.is((uint32_t)n, JType::Obj)) {
    *err = path + " must be a mapping";
    return false;
  }
  *out = n;
  return true;
}

bool get_bool(const JDoc& d, int64_t obj, const char* key, bool* out, std::string* err) {
  *out = false;
  if (obj < 0) return true;
  int64_t n = d.get((uint32_t)obj, key);
  if (n < 0 || d.is((uint32_t)n, JType::Null)) return true;
  if (!d.is((uint32_t)n, JType::Bool)) {
    *err = std::string(key) + " must be a boolean";
    return false;
  }
  *out = d.n((uint32_t)n).b;
  return true;
}

// Settings validation per family (DESIGN.md §Policy families). Fills rec lists/flags.
bool compile_settings(const JDoc& d, int64_t s, PolicyRec* rec, std::string* err) {
  switch (rec->family) {
    case FAM_PRIVILEGED: {
      bool a, b;
      if (!get_bool(d, s, "skip_init_containers", &a, err)) return false;
      if (!get_bool(d, s, "skip_ephemeral_containers", &b, err)) return false;
      rec->flags |= (a ? PF_SKIP_INIT : 0) | (b ? PF_SKIP_EPHEMERAL : 0);
      return true;
    }
    case FAM_NAMESPACE: {
      int64_t n = s < 0 ? -1 : d.get((uint32_t)s, "valid_namespace");
      if (n < 0 || !d.is((uint32_t)n, JType::Str) || d.str((uint32_t)n).empty()) {
        *err = "valid_namespace must be a non-empty string";
        return false;
      }
      rec->lists[0].push_back(std::string(d.str((uint32_t)n)));
      return true;
    }
    case FAM_TRUSTED_REPOS: {
      int64_t reg, tags, imgs;
      if (!get_obj(d, s, "registries", "registries", &reg, err)) return false;
      if (!get_obj(d, s, "tags", "tags", &tags, err)) return false;
      if (!get_obj(d, s, "images", "images", &imgs, err)) return false;
      if (!get_list(d, reg, "allow", "registries.allow", &rec->lists[0], err)) return false;
      if (!get_list(d, reg, "reject", "registries.reject", &rec->lists[1], err)) return false;
      if (!get_list(d, tags, "reject", "tags.reject", &rec->lists[2], err)) return false;
      if (!get_list(d, imgs, "allow", "images.allow", &rec->lists[3], err)) return false;
      if (!get_list(d, imgs, "reject", "images.reject", &rec->lists[4], err)) return false;
      if (!rec->lists[0].empty() && !rec->lists[1].empty()) {
        *err = "registries: allow and reject lists are mutually exclusive";
        return false;
      }
      if (!rec->lists[3].empty() && !rec->lists[4].empty()) {
        *err = "images: allow and reject lists are mutually exclusive";
        return false;
      }
      for (int k = 0; k < 5; ++k)
        for (auto& g : rec->lists[k]) {
          std::vector<Pattern> one{{Pattern::Glob, g}};
          Dfa tmp;
          std::string e2;
          if (!compile_dfa(one, &tmp, &e2)) {
            *err = "invalid pattern '" + g + "': " + e2;
            return false;
          }
        }
      return true;
    }
    case FAM_CAPABILITIES: {
      if (!get_list(d, s, "allowed_capabilities", "allowed_capabilities", &rec->lists[0], err)) return false;
      if (!get_list(d, s, "required_drop_capabilities", "required_drop_capabilities", &rec->lists[1], err))
        return false;
      if (!get_list(d, s, "default_add_capabilities", "default_add_capabilities", &rec->lists[2], err))
        return false;
      for (auto& c : rec->lists[0])
        if (c == "*") rec->flags |= PF_ALLOW_ALL;
      std::string overlap;
      for (auto& c : rec->lists[2])
        if (std::find(rec->lists[1].begin(), rec->lists[1].end(), c) != rec->lists[1].end())
          overlap += (overlap.empty() ? "" : ", ") + c;
      if (!overlap.empty()) {
        *err = "these capabilities cannot be both added by default and required to be dropped: " + overlap;
        return false;
      }
      return true;
    }
    case FAM_APPARMOR:
      return get_list(d, s, "allowed_profiles", "allowed_profiles", &rec->lists[0], err);
    case FAM_LABELS: {
      if (!get_list(d, s, "denied_labels", "denied_labels", &rec->lists[0], err)) return false;
      if (!get_list(d, s, "mandatory_labels", "mandatory_labels", &rec->lists[1], err)) return false;
      int64_t c;
      if (!get_obj(d, s, "constrained_labels", "constrained_labels", &c, err)) return false;
      if (c >= 0) {
        for (uint32_t k = 0; k < d.count((uint32_t)c); ++k) {
          const JKid& kid = d.kids((uint32_t)c)[k];
          if (!d.is(kid.node, JType::Str)) {
            *err = "constrained_labels values must be strings";
            return false;
          }
          std::string key(d.key(kid)), re(d.str(kid.node));
          std::string rerr;
          if (!regex_ok(re, &rerr)) {
            *err = "constrained label '" + key + "' has an invalid regular expression: " + rerr;
            return false;
          }
          rec->lists[2].push_back(key);
          rec->lists[3].push_back(re);
        }
      }
      for (auto& k : rec->lists[0]) {
        bool both = std::find(rec->lists[1].begin(), rec->lists[1].end(), k) != rec->lists[1].end() ||
                    std::find(rec->lists[2].begin(), rec->lists[2].end(), k) != rec->lists[2].end();
        if (both) {
          *err = "label '" + k + "' cannot be both denied and mandatory or constrained";
          return false;
        }
      }
      if (rec->lists[1].size() > (size_t)kMaxListIdx || rec->lists[2].size() > (size_t)kMaxListIdx) {
        *err = "at most 16 mandatory and 16 constrained labels are supported";
        return false;
      }
      return true;
    }
  }
  return true;
}

int32_t pattern_bit(std::vector<Pattern>* col, Pattern::Kind k, const std::string& s) {
  Pattern p{k, s};
  for (size_t i = 0; i < col->size(); ++i)
    if ((*col)[i] == p) return (int32_t)i;
  col->push_back(p);
  return (int32_t)col->size() - 1;
}

template <typename T>
void put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* p = (const uint8_t*)&v;
  b->insert(b->end(), p, p + sizeof(T));
}
void align16(std::vector<uint8_t>* b) {
  while (b->size() % 16) b->push_back(0);
}

// Appends one DevDfa record (header, accept masks, transitions; 16-B aligned) and returns its
// blob offset. trans_off / acc_off are blob offsets.
size_t emit_dfa(const Dfa& dfa, std::vector<uint8_t>* b) {
  align16(b);
  const size_t hdr_at = b->size();
  DevDfa dd;
  memset(&dd, 0, sizeof(dd));
  dd.nstates = dfa.nstates;
  dd.ncls = dfa.ncls;
  dd.start = dfa.start;
  memcpy(dd.cls, dfa.cls.data(), 256);
  put(b, dd);
  align16(b);
  const uint32_t acc_off = (uint32_t)b->size();
  for (uint64_t a : dfa.accept) put(b, a);
  align16(b);
  const uint32_t trans_off = (uint32_t)b->size();
  for (uint16_t t : dfa.trans) put(b, t);
  align16(b);
  DevDfa* w = (DevDfa*)(b->data() + hdr_at);
  w->acc_off = acc_off;
  w->trans_off = trans_off;
  w->bytes = (uint32_t)(b->size() - hdr_at);
  w->chain_bytes = w->bytes;
  return hdr_at;
}

// Canonical dwords of a string: little-endian, the last one zero-padded (what the kernels build
// from the staged bytes with v_alignbyte).
std::vector<uint32_t> lit_words(const std::string& s) {
  std::vector<uint32_t> w((s.size() + 3) / 4, 0u);
  if (!s.empty()) memcpy(w.data(), s.data(), s.size());
  return w;
}
uint32_t lit_hash(const std::vector<uint32_t>& w, uint32_t len, uint32_t seed) {
  uint32_t h = lit_init(seed, len);
  for (uint32_t x : w) h = lit_mix(h, x);
  return lit_final(h);
}

// Appends a DevLit record (kwdev.hpp) for an all-literal column: the smallest power-of-two table
// (>= 2x the patterns) and seed for which the hash is collision-free over the patterns.
bool build_literal_table(const std::vector<Pattern>& pats, std::vector<uint8_t>* b) {
  const uint32_t npat = (uint32_t)pats.size();
  std::vector<std::vector<uint32_t>> words;
  std::vector<uint32_t> wi;  // word index of each pattern
  uint32_t nwords = 0;
  for (const Pattern& p : pats) {
    if (p.text.size() > 4095) return false;  // packed slot fields (kwdev.hpp DevLit)
    words.push_back(lit_words(p.text));
    wi.push_back(nwords);
    nwords += (uint32_t)words.back().size();
  }
  if (nwords >= 8192 || npat > 126) return false;
  for (uint32_t nslots = 16; nslots <= 4096; nslots *= 2) {
    if (nslots < 2 * npat) continue;
    for (uint32_t seed = 1; seed <= 4096; ++seed) {
      std::vector<uint32_t> slot(nslots, 0);
      bool ok = true;
      for (uint32_t i = 0; i < npat && ok; ++i) {
        const uint32_t len = (uint32_t)pats[i].text.size();
        uint32_t h = lit_hash(words[i], len, seed) & (nslots - 1);
        if (slot[h]) ok = false;
        else slot[h] = (i + 1) | (len << 7) | (wi[i] << 19);
      }
      if (!ok) continue;
      const size_t at = b->size();
      DevLit L;
      memset(&L, 0, sizeof(L));
      L.nslots = nslots;
      L.seed = seed;
      L.npat = npat;
      put(b, L);
      L.slot_off = (uint32_t)(b->size() - at);
      for (uint32_t x : slot) put(b, x);
      align16(b);
      L.word_off = (uint32_t)(b->size() - at);
      for (const auto& w : words)
        for (uint32_t x : w) put(b, x);
      for (int k = 0; k < 8; ++k) put(b, 0u);
      align16(b);
      L.bytes = (uint32_t)(b->size() - at);
      memcpy(b->data() + at, &L, sizeof(L));
      return true;
    }
  }
  return false;
}

}  // namespace

Env::~Env() = default;  // device memory released by capi (needs HIP)

// Register a (non-group) policy: family detection = our bootstrap; settings compilation = our
// validate_settings. Returns a non-ok Status when the reference would fail there.
static Status bootstrap(const JDoc& d, int64_t settings, PolicyRec* rec) {
  rec->family = detect_family(rec->module);
  if (rec->family == FAM_NONE) {
    // bootstrap_policy fails before register (evaluation_environment.rs:344-351): not registered
    return {KW_E_BOOTSTRAP, "bootstrap failure: " + rec->id + ": policy module '" + rec->module +
                                "' is not in the declarative policy class served by kwgpu"};
  }
  rec->registered = true;  // register() (:391-431) succeeded
  std::string err;
  if (!compile_settings(d, settings, rec, &err))
    return {KW_E_INIT, "Policy settings are invalid: " + err};
  return {};
}

Status build_env(const char* json, size_t len, bool continue_on_errors, const char* always_ns, Env* env) {
  JDoc d;
  std::string perr;
  if (!d.parse(json, len, &perr)) return {KW_E_BOOTSTRAP, "bootstrap failure: cannot parse policies: " + perr};
  if (!d.is(0, JType::Obj)) return {KW_E_BOOTSTRAP, "bootstrap failure: policies must be a mapping"};
  env->continue_on_errors = continue_on_errors;
  env->source.assign(json, len);
  if (always_ns) env->always_ns = std::string(always_ns);

  std::vector<Entry> entries;
  for (uint32_t k = 0; k < d.count(0); ++k) {
    const JKid& kid = d.kids(0)[k];
    Entry e;
    std::string err;
    if (!parse_entry(d, std::string(d.key(kid)), kid.node, &e, &err))
      return {KW_E_BOOTSTRAP, "bootstrap failure: " + err};
    entries.push_back(std::move(e));
  }
  // validate_policies (config.rs:237-258)
  for (auto& e : entries) {
    if (e.name.find('/') != std::string::npos)
      return {KW_E_BOOTSTRAP, "bootstrap failure: policy name '" + e.name + "' contains a '/' character"};
    if (e.is_group) {
      std::string bad;
      for (auto& m : e.members)
        if (m.name.find('/') != std::string::npos) bad += (bad.empty() ? "\"" : ", \"") + m.name + "\"";
      if (!bad.empty())
        return {KW_E_BOOTSTRAP, "bootstrap failure: policy group '" + e.name +
                                    "' contains policies with invalid names: [" + bad + "]"};
    }
  }

  // build_evaluation_environment (evaluation_environment.rs:198-332). Indices: top-level entries
  // in document order, then group members (group order, settings order).
  std::vector<std::pair<size_t, size_t>> member_slots;  // (entry, member)
  for (size_t i = 0; i < entries.size(); ++i) {
    PolicyRec rec;
    rec.name = rec.id = entries[i].name;
    if (rec.id.empty()) return {KW_E_INVALID_ID, "Not a valid Policy ID: "};
    rec.mode = entries[i].mode;
    if (entries[i].is_group) {
      rec.is_group = true;
      rec.family = FAM_GROUP;
      rec.registered = true;  // register_policy_group (:434-442)
      rec.expression = entries[i].expression;
      rec.message = entries[i].message;
      for (auto& m : entries[i].members) rec.member_names.push_back(m.name);
    } else {
      rec.module = entries[i].module;
      rec.allowed_to_mutate = entries[i].a2m;
    }
    env->ids[rec.id] = (int32_t)env->pol.size();
    env->pol.push_back(std::move(rec));
  }
  for (size_t i = 0; i < entries.size(); ++i) {
    if (!entries[i].is_group) continue;
    int32_t g = env->ids[entries[i].name];
    for (auto& m : entries[i].members) {
      PolicyRec rec;
      rec.name = m.name;
      rec.group = entries[i].name;
      rec.id = entries[i].name + "/" + m.name;
      rec.module = m.module;
      rec.is_member = true;
      rec.parent = g;
      rec.mode = KW_MODE_PROTECT;       // members always Protect (:297-301)
      rec.allowed_to_mutate = false;
      int32_t idx = (int32_t)env->pol.size();
      env->ids[rec.id] = idx;
      env->pol[(size_t)g].members.push_back(idx);
      env->pol.push_back(std::move(rec));
      member_slots.push_back({i, (size_t)(&m - &entries[i].members[0])});
    }
  }
  // bootstrap + settings for every policy and member, in build order
  size_t mslot = 0;
  for (size_t i = 0; i < env->pol.size(); ++i) {
    PolicyRec& rec = env->pol[i];
    if (rec.is_group) continue;
    int64_t settings;
    if (rec.is_member) {
      auto& ms = member_slots[mslot++];
      settings = entries[ms.first].members[ms.second].settings;
    } else {
      settings = entries[i].settings;
    }
    Status st = bootstrap(d, settings, &rec);
    if (!st.ok()) {
      if (!continue_on_errors) return st;
      rec.init_error = true;
      rec.init_message = st.message;
      if (rec.is_member) {
        PolicyRec& g = env->pol[(size_t)rec.parent];
        if (g.broken_member.empty()) g.broken_member = rec.id;
      }
    }
  }
  // group expressions (validated here; the reference evaluates them per request)
  for (auto& rec : env->pol) {
    if (!rec.is_group) continue;
    if (rec.member_names.size() > (size_t)kMaxGroupMembers) {
      rec.prog.valid = false;
      rec.prog.error = "policy groups with more than 16 members are not supported by the engine";
      continue;
    }
    rec.prog = compile_group_expression(rec.expression, rec.member_names);
  }

  // ---- column pattern tables and device parameters
  std::vector<DevPolicy> dp(env->pol.size());
  std::vector<uint8_t> progs;
  std::vector<int32_t> mems;
  int32_t bypass_bit = -1;
  if (env->always_ns) bypass_bit = pattern_bit(&env->cols[COL_NS], Pattern::Literal, *env->always_ns);
  for (size_t i = 0; i < env->pol.size(); ++i) {
    PolicyRec& r = env->pol[i];
    DevPolicy& P = dp[i];
    memset(&P, 0, sizeof(P));
    P.family = r.family;
    P.mode = r.mode;
    P.a2m = r.allowed_to_mutate;
    P.flags = r.flags | (r.registered ? PF_REGISTERED : 0) | (r.init_error ? PF_INIT_ERROR : 0);
    if (r.init_error) continue;
    auto bits = [&](Col c, Pattern::Kind k, const std::vector<std::string>& l) {
      uint64_t m = 0;
      for (auto& s : l) m |= 1ull << (pattern_bit(&env->cols[c], k, s) & 63);
      return m;
    };
    for (int k = 0; k < 5; ++k) P.nl[k] = (uint8_t)std::min<size_t>(255, r.lists[k].size());
    switch (r.family) {
      case FAM_NAMESPACE: P.m[0] = bits(COL_NS, Pattern::Literal, r.lists[0]); break;
      case FAM_TRUSTED_REPOS:
        P.m[0] = bits(COL_REG, Pattern::Glob, r.lists[0]);
        P.m[1] = bits(COL_REG, Pattern::Glob, r.lists[1]);
        P.m[2] = bits(COL_TAG, Pattern::Glob, r.lists[2]);
        P.m[3] = bits(COL_IMG, Pattern::Glob, r.lists[3]);
        P.m[4] = bits(COL_IMG, Pattern::Glob, r.lists[4]);
        break;
      case FAM_CAPABILITIES: {
        std::vector<std::string> allowed;
        for (auto& c : r.lists[0])
          if (c != "*") allowed.push_back(c);
        P.m[0] = bits(COL_CAP, Pattern::Literal, allowed) | bits(COL_CAP, Pattern::Literal, r.lists[2]);
        P.m[1] = bits(COL_CAP, Pattern::Literal, r.lists[1]);
        P.m[2] = bits(COL_CAP, Pattern::Literal, r.lists[2]);
        P.m[3] = bits(COL_CAP, Pattern::Literal, {"ALL"});
        break;
      }
      case FAM_APPARMOR: P.m[0] = bits(COL_AA, Pattern::Literal, r.lists[0]); break;
      case FAM_LABELS: {
        P.m[0] = bits(COL_LK, Pattern::Literal, r.lists[0]);
        P.m[1] = bits(COL_LK, Pattern::Literal, r.lists[1]);
        P.n_mand = (uint8_t)r.lists[1].size();
        P.n_constr = (uint8_t)r.lists[2].size();
        for (size_t k = 0; k < r.lists[1].size(); ++k)
          P.idx[k] = (uint8_t)pattern_bit(&env->cols[COL_LK], Pattern::Literal, r.lists[1][k]);
        for (size_t k = 0; k < r.lists[2].size(); ++k) {
          P.idx[16 + k] = (uint8_t)pattern_bit(&env->cols[COL_LK], Pattern::Literal, r.lists[2][k]);
          P.idx[32 + k] = (uint8_t)pattern_bit(&env->cols[COL_LV], Pattern::Regex, r.lists[3][k]);
        }
        break;
      }
      case FAM_GROUP: {
        if (!r.prog.valid || r.prog.eval_error) {
          P.flags |= PF_EXPR_ERROR;
          break;
        }
        P.prog_off = (uint32_t)progs.size();
        P.prog_len = (uint32_t)r.prog.code.size();
        progs.insert(progs.end(), r.prog.code.begin(), r.prog.code.end());
        P.member_off = (uint32_t)mems.size();
        P.nmembers = (uint32_t)r.members.size();
        mems.insert(mems.end(), r.members.begin(), r.members.end());
        break;
      }
      default: break;
    }
  }
  for (int c = 0; c < (int)NCOL; ++c)
    if (env->cols[c].size() > kMaxPatternsPerColumn)
      return {KW_E_BOOTSTRAP, std::string("bootstrap failure: the policy set needs more than 64 distinct patterns "
                                          "for one request column (column ") + std::to_string(c) + ")"};

  // ---- DFAs and blob
  std::vector<uint8_t>& b = env->blob;
  b.clear();
  DevHeader hdr;
  memset(&hdr, 0, sizeof(hdr));
  put(&b, hdr);
  align16(&b);
  for (int c = 0; c < (int)NCOL; ++c) {
    if (env->cols[c].empty()) continue;
    std::vector<Dfa> chain;
    std::string err;
    if (!compile_column(env->cols[c], kMaxDfaTableBytes, &chain, &err))
      return {KW_E_BOOTSTRAP, "bootstrap failure: cannot compile column automaton: " + err};
    std::vector<size_t> at;
    for (const Dfa& dfa : chain) at.push_back(emit_dfa(dfa, &b));
    uint32_t tail = 0;
    for (size_t k = chain.size(); k-- > 0;) {
      DevDfa* w = (DevDfa*)(b.data() + at[k]);
      w->next = k + 1 < chain.size() ? (uint32_t)at[k + 1] : 0;
      tail += w->bytes;
      w->chain_bytes = tail;
    }
    hdr.dfa_off[c] = (uint32_t)at[0];
  }
  // literal columns: perfect-hash tables (the fused kernel's fast path; DFAs stay for the others)
  for (int c = 0; c < (int)NCOL; ++c) {
    if (env->cols[c].empty()) continue;
    bool lit = true;
    for (const Pattern& p : env->cols[c]) lit = lit && p.kind == Pattern::Literal;
    if (!lit) continue;
    align16(&b);
    const size_t at = b.size();
    if (build_literal_table(env->cols[c], &b)) hdr.lit_off[c] = (uint32_t)at;
    else b.resize(at);  // no table (oversized literals): the column keeps its DFA chain
  }
  // per-key label-value DFAs: a label's value is only ever tested against the regexes constrained
  // on its own key, so one small DFA per constrained key replaces the chain over all value regexes
  if (hdr.lit_off[COL_LK] && !env->cols[COL_LV].empty()) {
    std::vector<std::vector<uint32_t>> vals(kMaxPatternsPerColumn);
    for (const DevPolicy& P : dp) {
      if (P.family != FAM_LABELS) continue;
      for (uint32_t k = 0; k < P.n_constr; ++k) {
        auto& v = vals[P.idx[16 + k]];
        if (std::find(v.begin(), v.end(), (uint32_t)P.idx[32 + k]) == v.end()) v.push_back(P.idx[32 + k]);
      }
    }
    // one DFA per key while the union of its regexes stays small, else a short chain of DFAs
    // (compile_column's greedy groups) instead of one large product automaton
    std::vector<std::vector<Dfa>> kd(kMaxPatternsPerColumn);
    bool ok = true;
    for (size_t k = 0; k < vals.size() && ok; ++k) {
      if (vals[k].empty()) continue;
      std::vector<Pattern> pats;
      for (uint32_t v : vals[k]) pats.push_back(env->cols[COL_LV][v]);
      std::string err;
      ok = compile_column(pats, kKvDfaBytes, &kd[k], &err);
      for (Dfa& d : kd[k]) {
        ok = ok && d.trans.size() * 2 <= kMaxDfaTableBytes;
        for (uint64_t& a : d.accept) {  // local pattern bits -> the column's global bits
          uint64_t g = 0;
          for (size_t i = 0; i < vals[k].size(); ++i)
            if ((a >> i) & 1ull) g |= 1ull << vals[k][i];
          a = g;
        }
      }
    }
    for (size_t k = 0; k < kd.size() && ok; ++k)
      for (const Dfa& d : kd[k]) ok = ok && d.nstates <= 256 && d.ncls <= 255;  // u8 transitions and classes
    if (ok) {
      std::vector<uint8_t> r;  // the region, region-relative offsets
      r.resize(2 * kMaxPatternsPerColumn, 0);
      std::map<std::vector<uint8_t>, uint16_t> cls_pool;
      auto at16 = [&](size_t n) {  // reserve n bytes at a 16-B boundary
        while (r.size() % 16) r.push_back(0);
        const size_t o = r.size();
        r.resize(o + n, 0);
        return o;
      };
      std::vector<size_t> recs;  // KvDfa record positions, linked per key below
      std::map<std::vector<uint8_t>, uint16_t> chains;  // keys constrained by the same regexes share one chain
      for (size_t k = 0; k < kd.size(); ++k) {
        if (kd[k].empty()) continue;
        std::vector<uint8_t> sig;
        for (const Dfa& d : kd[k]) {
          const uint32_t hd[3] = {d.nstates, d.ncls, d.start};
          sig.insert(sig.end(), (const uint8_t*)hd, (const uint8_t*)(hd + 3));
          sig.insert(sig.end(), d.cls.begin(), d.cls.end());
          sig.insert(sig.end(), (const uint8_t*)d.trans.data(), (const uint8_t*)(d.trans.data() + d.trans.size()));
          sig.insert(sig.end(), (const uint8_t*)d.accept.data(), (const uint8_t*)(d.accept.data() + d.accept.size()));
        }
        auto hit = chains.find(sig);
        if (hit != chains.end()) {
          ((uint16_t*)r.data())[k] = hit->second;
          continue;
        }
        size_t prev = 0;
        for (const Dfa& d : kd[k]) {
          KvDfa kv;
          memset(&kv, 0, sizeof(kv));
          bool uniform_hi = true;
          for (int c = 128; c < 256; ++c) uniform_hi = uniform_hi && d.cls[c] == d.cls[128];
          kv.wide = uniform_hi ? 0 : 1;
          kv.hi = d.cls[128];
          std::vector<uint8_t> cm(d.cls.begin(), d.cls.begin() + (kv.wide ? 256 : 128));
          auto it = cls_pool.find(cm);
          if (it == cls_pool.end()) {
            const size_t o = at16(cm.size());
            memcpy(r.data() + o, cm.data(), cm.size());
            it = cls_pool.emplace(cm, (uint16_t)o).first;
          }
          kv.cls_off = it->second;
          std::vector<uint64_t> accv;
          std::vector<uint8_t> acc(d.nstates);
          for (uint32_t q = 0; q < d.nstates; ++q) {
            size_t x = std::find(accv.begin(), accv.end(), d.accept[q]) - accv.begin();
            if (x == accv.size()) accv.push_back(d.accept[q]);
            acc[q] = (uint8_t)x;  // nstates <= 256: at most 256 distinct masks
          }
          kv.ncls = (uint8_t)d.ncls;
          kv.start = (uint8_t)d.start;
          kv.nstates = (uint16_t)d.nstates;
          const size_t rec = at16(sizeof(KvDfa));
          kv.accv_off = (uint16_t)at16(accv.size() * 8);
          memcpy(r.data() + kv.accv_off, accv.data(), accv.size() * 8);
          kv.acc_off = (uint16_t)r.size();
          r.insert(r.end(), acc.begin(), acc.end());
          kv.trans_off = (uint16_t)r.size();
          for (uint16_t tq : d.trans) r.push_back((uint8_t)tq);
          memcpy(r.data() + rec, &kv, sizeof(kv));
          if (prev) ((KvDfa*)(r.data() + prev))->next = (uint16_t)rec;
          else ((uint16_t*)r.data())[k] = (uint16_t)rec;
          prev = rec;
          recs.push_back(rec);
        }
        chains.emplace(std::move(sig), ((uint16_t*)r.data())[k]);
      }
      while (r.size() % 16) r.push_back(0);
      r.resize(r.size() + 16, 0);  // slack: dword-granular readers may run past the last table
      ok = r.size() < 65536;        // u16 offsets
      if (ok) {
        align16(&b);
        hdr.kv_off = (uint32_t)b.size();
        hdr.kv_bytes = (uint32_t)r.size();
        b.insert(b.end(), r.begin(), r.end());
      }
    }
  }
  align16(&b);
  hdr.policy_off = (uint32_t)b.size();
  for (auto& P : dp) put(&b, P);
  align16(&b);
  hdr.prog_off = (uint32_t)b.size();
  b.insert(b.end(), progs.begin(), progs.end());
  align16(&b);
  hdr.member_off = (uint32_t)b.size();
  for (int32_t m : mems) put(&b, m);
  align16(&b);
  hdr.magic = kBlobMagic;
  hdr.version = kBlobVersion;
  hdr.npolicies = (uint32_t)env->pol.size();
  hdr.blob_bytes = (uint32_t)b.size();
  hdr.bypass_bit = bypass_bit;
  memcpy(b.data(), &hdr, sizeof(hdr));
  return {};
}

Status env_lookup(const Env& env, const std::string& id, int32_t* idx) {
  // PolicyID::from_str (policy_id.rs:29-47): "" or more than one '/' is invalid
  if (id.empty()) return {KW_E_INVALID_ID, "Not a valid Policy ID: "};
  size_t slashes = (size_t)std::count(id.begin(), id.end(), '/');
  if (slashes > 1) return {KW_E_INVALID_ID, "Not a valid Policy ID: " + id};
  auto it = env.ids.find(id);
  if (it == env.ids.end()) return {KW_E_NOT_FOUND, "unknown policy: " + id};
  *idx = it->second;
  return {};
}

Status env_validate_settings(const Env& env, int32_t idx) {
  const PolicyRec& r = env.pol[(size_t)idx];
  if (r.is_group) {
    if (!r.broken_member.empty()) return {KW_E_NOT_FOUND, "unknown policy: " + r.broken_member};
    if (!r.prog.valid) return {KW_E_INIT, r.prog.error.empty() ? r.id + " settings are not valid" : r.prog.error};
    return {};
  }
  if (!r.registered) return {KW_E_NOT_FOUND, "unknown policy: " + r.id};
  if (r.init_error) return {KW_E_INIT, r.init_message};
  return {};
}

// Serialised environment (what rank 0 broadcasts): header, the policies document, the
// always-accept namespace and the compiled device tables. A receiving rank rebuilds the host-side
// records from the document and checks that its own compilation is byte-identical to the tables
// it received (the tables themselves are what the device uses).
struct SerHdr {
  uint32_t magic, flags;
  uint64_t json_len, ns_len, blob_len;
};
std::vector<uint8_t> env_serialize(const Env& env) {
  std::vector<uint8_t> out;
  SerHdr h{0x4b575331u, (env.continue_on_errors ? 1u : 0u) | (env.always_ns ? 2u : 0u), env.source.size(),
           env.always_ns ? env.always_ns->size() : 0, env.blob.size()};
  put(&out, h);
  out.insert(out.end(), env.source.begin(), env.source.end());
  if (env.always_ns) out.insert(out.end(), env.always_ns->begin(), env.always_ns->end());
  out.insert(out.end(), env.blob.begin(), env.blob.end());
  return out;
}

Status env_from_blob(const void* data, size_t len, Env* env) {
  if (len < sizeof(SerHdr)) return {KW_E_ARG, "serialized environment too short"};
  SerHdr h;
  memcpy(&h, data, sizeof(h));
  if (h.magic != 0x4b575331u || sizeof(SerHdr) + h.json_len + h.ns_len + h.blob_len != len)
    return {KW_E_ARG, "malformed serialized environment"};
  const char* p = (const char*)data + sizeof(SerHdr);
  std::string json(p, h.json_len);
  std::string ns(p + h.json_len, h.ns_len);
  const uint8_t* blob = (const uint8_t*)p + h.json_len + h.ns_len;
  Status st = build_env(json.data(), json.size(), h.flags & 1, (h.flags & 2) ? ns.c_str() : nullptr, env);
  if (!st.ok()) return st;
  if (env->blob.size() != h.blob_len || memcmp(env->blob.data(), blob, h.blob_len) != 0)
    return {KW_E_BOOTSTRAP, "bootstrap failure: received compiled tables differ from the local compilation"};
  return {};
}

}  // namespace kw
