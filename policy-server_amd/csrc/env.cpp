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

// `#[serde(default)] policy_mode: PolicyMode` inside an untagged enum (config.rs:369-371,
// :384-385): an absent key is the default (Protect); a present key goes through serde's buffered
// enum deserializer, which takes a variant name as a string, or a single-key map whose value is
// unit ({protect: null}). An explicit null is neither, so it fails the variant.
bool parse_mode(const JDoc& d, int64_t n, uint8_t* mode, std::string* err) {
  if (n < 0) {
    *mode = KW_MODE_PROTECT;
    return true;
  }
  if (d.is((uint32_t)n, JType::Obj)) {
    auto ms = d.members((uint32_t)n);
    uint32_t cnt = 0, only = 0;
    for (uint32_t m : ms) {
      only = m;
      ++cnt;
    }
    if (cnt != 1 || !d.is(only, JType::Null)) {
      *err = "invalid value: map, expected map with a single key";
      return false;
    }
    std::string_view k = d.key(only);
    if (k == "protect") *mode = KW_MODE_PROTECT;
    else if (k == "monitor") *mode = KW_MODE_MONITOR;
    else {
      *err = "unknown variant `" + std::string(k) + "`, expected `monitor` or `protect`";
      return false;
    }
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

// `#[serde(default)] context_aware_resources: BTreeSet<..>` (config.rs:349-350, :376-378): absent
// is the empty set; an explicit null is not a sequence and fails the variant.
bool check_ctx_resources(const JDoc& d, int64_t n) {
  if (n < 0) return true;
  if (!d.is((uint32_t)n, JType::Arr)) return false;
  for (uint32_t it : d.members((uint32_t)n)) {
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
      for (uint32_t m : d.members((uint32_t)pols)) {
        if (!ok) break;
        if (!d.is(m, JType::Obj)) {
          ok = false;
          break;
        }
        Entry::Member mem;
        mem.name = std::string(d.key(m));
        for (uint32_t f : d.members(m)) {
          std::string_view key = d.key(f);
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
  for (uint32_t it : d.members((uint32_t)n)) {
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
          std::string e2;
          if (!pattern_ok({Pattern::Glob, g}, &e2)) {  // syntax only: a large automaton runs as an NFA
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
        for (uint32_t kid : d.members((uint32_t)c)) {
          if (!d.is(kid, JType::Str)) {
            *err = "constrained_labels values must be strings";
            return false;
          }
          std::string key(d.key(kid)), re(d.str(kid));
          std::string rerr;
          if (!regex_ok(re, &rerr)) {  // (the parser's detail stays out: the oracle words it its own way)
            *err = "constrained label '" + key + "' has an invalid regular expression";
            return false;
          }
          // a repeated key keeps its first position and its last regex (a JSON map, as serde reads it)
          auto dup = std::find(rec->lists[2].begin(), rec->lists[2].end(), key);
          if (dup != rec->lists[2].end()) {
            rec->lists[3][(size_t)(dup - rec->lists[2].begin())] = re;
          } else {
            rec->lists[2].push_back(key);
            rec->lists[3].push_back(re);
          }
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
      return true;
    }
  }
  return true;
}


// Pattern id of (kind, text) in a column, added when new.
uint32_t pattern_id(ColumnInfo* col, Pattern::Kind k, const std::string& s) {
  Pattern p{k, s};
  for (size_t i = 0; i < col->pats.size(); ++i)
    if (col->pats[i] == p) return (uint32_t)i;
  col->pats.push_back(p);
  return (uint32_t)col->pats.size() - 1;
}

// A glob without metacharacters is a literal under fnmatch(3) flags 0.
bool glob_is_literal(const std::string& g) { return g.find_first_of("*?[\\") == std::string::npos; }

template <typename T>
void put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* p = (const uint8_t*)&v;
  b->insert(b->end(), p, p + sizeof(T));
}
void align16(std::vector<uint8_t>* b) {
  while (b->size() % 16) b->push_back(0);
}

// Canonical dwords of a string: little-endian, the last one zero-padded (what the kernels build
// from the staged bytes).
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

// Appends a DevLit record (kwdev.hpp) over literal strings `lits` (class of lits[i] = i + 1).
// Up to 48 strings: one bucket, the smallest power-of-two table (>= 2x) and seed for which the hash
// alone is collision-free. Larger sets: hash-and-displace with ~2 strings per bucket and a load
// factor of at most 1/2 (buckets placed largest first, each with the first displacement whose slots
// are all free).
bool build_literal_table(const std::vector<std::string>& lits, std::vector<uint8_t>* b, std::string* err) {
  const uint32_t npat = (uint32_t)lits.size();
  std::vector<std::vector<uint32_t>> words;
  std::vector<uint32_t> wi;
  uint32_t nwords = 0;
  for (const std::string& s : lits) {
    if (s.size() > 65535) {
      *err = "literal pattern longer than 65535 bytes";
      return false;
    }
    words.push_back(lit_words(s));
    wi.push_back(nwords);
    nwords += (uint32_t)words.back().size();
  }
  if (npat >= 65535) {
    *err = "more than 65534 literal patterns in one column";
    return false;
  }
  auto emit = [&](uint32_t nslots, uint32_t seed, uint32_t nb_log2, const std::vector<uint32_t>& slot_of,
                  const std::vector<uint16_t>& disp) {
    const size_t at = b->size();
    DevLit L;
    memset(&L, 0, sizeof(L));
    L.nslots = nslots;
    L.seed = seed;
    L.npat = npat;
    L.nb_log2 = nb_log2;
    put(b, L);
    L.slot_off = (uint32_t)(b->size() - at);
    std::vector<uint32_t> sx(nslots, 0), sy(nslots, 0);
    for (uint32_t i = 0; i < npat; ++i) {
      sx[slot_of[i]] = (i + 1) | ((uint32_t)lits[i].size() << 16);
      sy[slot_of[i]] = wi[i];
    }
    for (uint32_t k = 0; k < nslots; ++k) {
      put(b, sx[k]);
      put(b, sy[k]);
    }
    align16(b);
    L.disp_off = 0;
    if (nb_log2) {
      L.disp_off = (uint32_t)(b->size() - at);
      for (uint16_t d : disp) put(b, d);
      align16(b);
    }
    L.word_off = (uint32_t)(b->size() - at);
    for (const auto& w : words)
      for (uint32_t x : w) put(b, x);
    for (int k = 0; k < 8; ++k) put(b, 0u);
    align16(b);
    L.bytes = (uint32_t)(b->size() - at);
    memcpy(b->data() + at, &L, sizeof(L));
  };
  if (npat <= 48) {
    for (uint32_t nslots = 16; nslots <= 8192; nslots *= 2) {
      if (nslots < 2 * npat) continue;
      for (uint32_t seed = 1; seed <= 4096; ++seed) {
        std::vector<uint32_t> slot_of(npat);
        std::vector<uint8_t> used(nslots, 0);
        bool ok = true;
        for (uint32_t i = 0; i < npat && ok; ++i) {
          const uint32_t h = lit_slot_index(lit_hash(words[i], (uint32_t)lits[i].size(), seed), 0, nslots);
          if (used[h]) ok = false;
          used[h] = 1;
          slot_of[i] = h;
        }
        if (!ok) continue;
        emit(nslots, seed, 0, slot_of, {});
        return true;
      }
    }
  }
  uint32_t nslots = 16, nb_log2 = 1;
  while (nslots < 2 * npat) nslots *= 2;
  while ((1u << nb_log2) < (npat + 1) / 2) ++nb_log2;
  const uint32_t nb = 1u << nb_log2;
  for (uint32_t seed = 1; seed <= 64; ++seed) {
    std::vector<uint32_t> g(npat);
    std::vector<std::vector<uint32_t>> bucket(nb);
    for (uint32_t i = 0; i < npat; ++i) {
      g[i] = lit_hash(words[i], (uint32_t)lits[i].size(), seed);
      bucket[g[i] >> (32 - nb_log2)].push_back(i);
    }
    std::vector<uint32_t> order(nb);
    for (uint32_t k = 0; k < nb; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return bucket[x].size() > bucket[y].size(); });
    std::vector<uint8_t> used(nslots, 0);
    std::vector<uint16_t> disp(nb, 0);
    std::vector<uint32_t> slot_of(npat);
    bool ok = true;
    for (uint32_t bk : order) {
      if (bucket[bk].empty()) break;
      bool placed = false;
      for (uint32_t d = 0; d < std::min<uint32_t>(65536u, nslots) && !placed; ++d) {  // lit_disp(d) = d: every mask once
        std::vector<uint32_t> sl;
        bool fit = true;
        for (uint32_t i : bucket[bk]) {
          const uint32_t s = lit_slot_index(g[i], d, nslots);
          if (used[s] || std::find(sl.begin(), sl.end(), s) != sl.end()) {
            fit = false;
            break;
          }
          sl.push_back(s);
        }
        if (!fit) continue;
        for (size_t q = 0; q < sl.size(); ++q) {
          used[sl[q]] = 1;
          slot_of[bucket[bk][q]] = sl[q];
        }
        disp[bk] = (uint16_t)d;
        placed = true;
      }
      if (!placed) {
        ok = false;
        break;
      }
    }
    if (!ok) continue;
    emit(nslots, seed, nb_log2, slot_of, disp);
    return true;
  }
  *err = "cannot build the literal hash table";
  return false;
}

// Appends one DevDfa record (header, accept classes, transitions; 16-B aligned) and returns its
// blob offset. `cls_map`: the DFA's local accept class -> the column's global class.
// Appends an NFA element's program (DevNfa) and returns its blob offset.
size_t emit_nfa_prog(const Dfa& dfa, std::vector<uint8_t>* b) {
  align16(b);
  const size_t at = b->size();
  b->insert(b->end(), dfa.prog.begin(), dfa.prog.end());
  align16(b);
  return at;
}

size_t emit_dfa(const Dfa& dfa, const std::vector<uint32_t>& cls_map, std::vector<uint8_t>* b, size_t nfa_prog = 0) {
  align16(b);
  const size_t hdr_at = b->size();
  DevDfa dd;
  memset(&dd, 0, sizeof(dd));
  if (dfa.nfa) {  // an NFA element: no tables; acc = its two global classes (no match, match)
    dd.kind = 1;
    dd.trans_off = (uint32_t)nfa_prog;
    put(b, dd);
    align16(b);
    const uint32_t acc_off = (uint32_t)b->size();
    put(b, (uint16_t)cls_map[0]);
    put(b, (uint16_t)cls_map[1]);
    align16(b);
    DevDfa* w = (DevDfa*)(b->data() + hdr_at);
    w->acc_off = acc_off;
    w->bytes = (uint32_t)(b->size() - hdr_at);
    w->chain_bytes = w->bytes;
    return hdr_at;
  }
  dd.nstates = dfa.nstates;
  dd.ncls = dfa.ncls;
  dd.start = dfa.start;
  dd.abs_lo = dfa.abs_lo;
  auto feed = [&](uint32_t st, const char* s) {
    for (; *s; ++s) st = dfa.trans[(size_t)st * dfa.ncls + dfa.cls[(uint8_t)*s]];
    return st;
  };
  const uint32_t dk = feed(dfa.start, "docker.io"), dks = feed(dk, "/"), dkl = feed(dks, "library/");
  dd.pre0 = dk | (dks << 16);
  dd.pre1 = dkl | (feed(dfa.start, "latest") << 16);
  memcpy(dd.cls, dfa.cls.data(), 256);
  put(b, dd);
  align16(b);
  const uint32_t acc_off = (uint32_t)b->size();
  for (uint32_t a : dfa.acc) put(b, (uint16_t)cls_map[a]);
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

constexpr size_t kDfaTableBudget = 64 * 1024;  // per DFA of a column chain
constexpr size_t kKvDfaBudget = 3072;  // per DFA of a label key's value chain (its region is staged per workgroup: occupancy)

// Compiles one column (ColumnInfo.pats) into its blob records: the literal table over the literal
// patterns (COL_IMG: none, its strings are constructed), then the DFA chain over the rest.
Status compile_col(Col c, ColumnInfo* ci, DevCol* dc, std::vector<uint8_t>* b) {
  memset(dc, 0, sizeof(*dc));
  ci->class_pats.assign(1, {});
  ci->lit_cls.assign(ci->pats.size(), 0);
  std::vector<std::string> lits;
  std::vector<uint32_t> lit_pid, rest_pid;
  for (uint32_t p = 0; p < (uint32_t)ci->pats.size(); ++p) {
    if (ci->pats[p].kind == Pattern::Literal && c != COL_IMG) {
      lits.push_back(ci->pats[p].text);
      lit_pid.push_back(p);
    } else {
      rest_pid.push_back(p);
    }
  }
  if (!lits.empty()) {
    align16(b);
    const size_t at = b->size();
    std::string err;
    if (!build_literal_table(lits, b, &err)) return {KW_E_BOOTSTRAP, "bootstrap failure: " + err};
    dc->lit_off = (uint32_t)at;
    dc->lit_bytes = (uint32_t)(b->size() - at);
    dc->nlit = (uint32_t)lits.size();
    for (size_t i = 0; i < lit_pid.size(); ++i) {
      ci->lit_cls[lit_pid[i]] = (uint32_t)i + 1;
      ci->class_pats.push_back({lit_pid[i]});
    }
  }
  if (!rest_pid.empty()) {
    std::vector<Pattern> pats;
    for (uint32_t p : rest_pid) pats.push_back(ci->pats[p]);
    std::vector<Dfa> chain;
    std::string err;
    if (!compile_column(pats, kDfaTableBudget, kMaxDfaStates, &chain, &err))
      return {KW_E_BOOTSTRAP, "bootstrap failure: cannot compile column automaton: " + err};
    // NFA elements' programs first (read from HBM by nfa_classify_kernel, never staged), so the
    // chain itself stays contiguous (the tile kernel stages it whole)
    std::vector<size_t> prog_at(chain.size(), 0);
    for (size_t k = 0; k < chain.size(); ++k)
      if (chain[k].nfa) {
        prog_at[k] = emit_nfa_prog(chain[k], b);
        ci->nfa_words = std::max<uint64_t>(ci->nfa_words, nfa_scratch_words(*(const DevNfa*)chain[k].prog.data()));
      }
    std::vector<size_t> at;
    for (size_t k = 0; k < chain.size(); ++k) {
      const Dfa& dfa = chain[k];
      std::vector<uint32_t> cls_map(dfa.classes.size(), 0);
      for (size_t a = 1; a < dfa.classes.size(); ++a) {
        cls_map[a] = (uint32_t)ci->class_pats.size();
        std::vector<uint32_t> pids;
        for (uint32_t q : dfa.classes[a]) pids.push_back(rest_pid[q]);
        ci->class_pats.push_back(pids);
      }
      at.push_back(emit_dfa(dfa, cls_map, b, prog_at[k]));
    }
    for (const Dfa& dfa : chain)
      if (dfa.nfa) dc->flags |= 1u;  // the column has NFA elements
    uint32_t tail = 0;
    for (size_t k = chain.size(); k-- > 0;) {
      DevDfa* w = (DevDfa*)(b->data() + at[k]);
      w->next = k + 1 < chain.size() ? (uint32_t)at[k + 1] : 0;
      tail += w->bytes;
      w->chain_bytes = tail;
    }
    dc->dfa_off = (uint32_t)at[0];
    dc->ndfa = (uint32_t)chain.size();
    dc->dfa_bytes = tail;
  }
  dc->nclass = (uint32_t)ci->class_pats.size();
  if (dc->nclass > 65535) return {KW_E_BOOTSTRAP, "bootstrap failure: a request column needs more than 65535 classes"};
  return {};
}

// The per-key label-value region (kwdev.hpp DevHeader kv_*): for each label-key class, a chain of
// small DFAs over the regexes constrained on that key (keys with the same regexes share one chain).
Status compile_kv(Env* env, DevHeader* hdr, std::vector<uint8_t>* b) {
  const uint32_t nlk = hdr->col[COL_LK].nclass;
  const ColumnInfo& lk = env->cols[COL_LK];
  std::vector<std::vector<uint32_t>> vals(nlk);  // key class -> LV pattern ids
  for (const PolicyRec& r : env->pol) {
    if (r.family != FAM_LABELS || r.init_error) continue;
    for (size_t k = 0; k < r.pid[2].size(); ++k) {
      auto& v = vals[lk.lit_cls[r.pid[2][k]]];
      if (std::find(v.begin(), v.end(), r.pid[3][k]) == v.end()) v.push_back(r.pid[3][k]);
    }
  }
  std::vector<uint8_t> R(8u * nlk, 0);  // kidx[nlk] | kbase[nlk]
  auto at16 = [&](size_t n) {
    while (R.size() % 16) R.push_back(0);
    const size_t o = R.size();
    R.resize(o + n, 0);
    return o;
  };
  std::map<std::vector<uint8_t>, uint32_t> cls_pool;
  struct Shared {
    uint32_t head;
    std::vector<std::pair<std::vector<uint32_t>, std::vector<std::vector<uint32_t>>>> dfas;  // (covered, class sets)
  };
  std::map<std::vector<uint32_t>, Shared> chains;  // regex list -> compiled chain
  env->kv.clear();
  env->kv_of_key.assign(nlk, {});
  uint32_t longest = 0;
  for (uint32_t k = 1; k < nlk; ++k) {
    if (vals[k].empty()) continue;
    auto hit = chains.find(vals[k]);
    if (hit == chains.end()) {
      std::vector<Pattern> pats;
      for (uint32_t v : vals[k]) pats.push_back(env->cols[COL_LV].pats[v]);
      std::vector<Dfa> kd;
      std::vector<uint32_t> firsts;
      std::string err;
      if (!compile_column(pats, kKvDfaBudget, kMaxDfaStates, &kd, &err, &firsts))
        return {KW_E_BOOTSTRAP, "bootstrap failure: cannot compile label value automaton: " + err};
      Shared sh;
      sh.head = 0;
      size_t prev = 0;
      uint32_t cbase = 0;
      for (const Dfa& d : kd) {
        if (d.ncls > 65535 || d.nstates > 65535) return {KW_E_BOOTSTRAP, "bootstrap failure: label value automaton too large"};
        KvDfa kv;
        memset(&kv, 0, sizeof(kv));
        if (d.nfa) {  // an NFA element: its program in the blob (before the region), classes {0, 1}
          kv.nfa = 1;
          kv.trans_off = (uint32_t)emit_nfa_prog(d, b);
          env->cols[COL_LV].nfa_words =
              std::max<uint64_t>(env->cols[COL_LV].nfa_words, nfa_scratch_words(*(const DevNfa*)d.prog.data()));
          kv.cbase = (uint16_t)cbase;
          const size_t rec = at16(sizeof(KvDfa));
          kv.acc_off = (uint32_t)at16(4);
          ((uint16_t*)(R.data() + kv.acc_off))[0] = 0;
          ((uint16_t*)(R.data() + kv.acc_off))[1] = 1;
          memcpy(R.data() + rec, &kv, sizeof(kv));
          if (prev) ((KvDfa*)(R.data() + prev))->next = (uint32_t)rec;
          else sh.head = (uint32_t)rec;
          prev = rec;
          const size_t q = sh.dfas.size();
          const uint32_t f0 = firsts[q], f1 = q + 1 < firsts.size() ? firsts[q + 1] : (uint32_t)vals[k].size();
          std::vector<uint32_t> covered(vals[k].begin() + f0, vals[k].begin() + f1);
          std::vector<std::vector<uint32_t>> sets;
          for (const auto& cs : d.classes) {
            std::vector<uint32_t> m;
            for (uint32_t i : cs) m.push_back(vals[k][i]);
            sets.push_back(m);
          }
          sh.dfas.push_back({covered, sets});
          cbase += 2;
          hdr->col[COL_LV].flags |= 1u;
          continue;
        }
        bool uniform_hi = true;
        for (int c = 128; c < 256; ++c) uniform_hi = uniform_hi && d.cls[c] == d.cls[128];
        kv.wide = uniform_hi ? 0 : 1;
        kv.hi = d.cls[128];
        // narrow maps carry the class of every byte >= 128 as entry 128, so a class load indexes
        // min(byte, 128) (kernels.hip classify_value_as) instead of selecting `hi` per byte
        std::vector<uint8_t> cm(d.cls.begin(), d.cls.begin() + (kv.wide ? 256 : 129));
        auto it = cls_pool.find(cm);
        if (it == cls_pool.end()) {
          const size_t o = at16(cm.size());
          memcpy(R.data() + o, cm.data(), cm.size());
          it = cls_pool.emplace(cm, (uint32_t)o).first;
        }
        kv.cls_off = it->second;
        kv.ncls = (uint16_t)d.ncls;
        kv.start = d.start;
        kv.nstates = (uint16_t)d.nstates;
        kv.abs_lo = (uint16_t)d.abs_lo;
        kv.t16 = d.nstates > 256 ? 1 : 0;
        kv.cbase = (uint16_t)cbase;
        const size_t rec = at16(sizeof(KvDfa));
        kv.acc_off = (uint32_t)at16(d.nstates * 2u);
        for (uint32_t q = 0; q < d.nstates; ++q) ((uint16_t*)(R.data() + kv.acc_off))[q] = (uint16_t)d.acc[q];
        kv.trans_off = (uint32_t)at16(d.trans.size() * (kv.t16 ? 2u : 1u));
        for (size_t q = 0; q < d.trans.size(); ++q) {
          if (kv.t16) ((uint16_t*)(R.data() + kv.trans_off))[q] = d.trans[q];
          else R[kv.trans_off + q] = (uint8_t)d.trans[q];
        }
        memcpy(R.data() + rec, &kv, sizeof(kv));
        if (prev) ((KvDfa*)(R.data() + prev))->next = (uint32_t)rec;
        else sh.head = (uint32_t)rec;
        prev = rec;
        // covered regexes: the DFA's group of the key's list (compile_column packs in order)
        const size_t q = sh.dfas.size();
        const uint32_t f0 = firsts[q], f1 = q + 1 < firsts.size() ? firsts[q + 1] : (uint32_t)vals[k].size();
        std::vector<uint32_t> covered(vals[k].begin() + f0, vals[k].begin() + f1);
        std::vector<std::vector<uint32_t>> sets;
        for (const auto& cs : d.classes) {
          std::vector<uint32_t> m;
          for (uint32_t i : cs) m.push_back(vals[k][i]);
          sets.push_back(m);
        }
        sh.dfas.push_back({covered, sets});
        cbase += (uint32_t)d.classes.size();
        if (cbase > 65535) return {KW_E_BOOTSTRAP, "bootstrap failure: label value automaton too large"};
      }
      hit = chains.emplace(vals[k], std::move(sh)).first;
    }
    ((uint32_t*)R.data())[k] = hit->second.head;
    ((uint32_t*)R.data())[nlk + k] = (uint32_t)env->kv.size();
    longest = std::max(longest, (uint32_t)hit->second.dfas.size());
    for (const auto& d : hit->second.dfas)
      for (const auto& set : d.second) {
        KvClass kc;
        kc.key = k;
        kc.covered = d.first;
        kc.matched = set;
        env->kv_of_key[k].push_back((uint32_t)env->kv.size());
        env->kv.push_back(std::move(kc));
      }
  }
  if (env->kv.size() > 65535) return {KW_E_BOOTSTRAP, "bootstrap failure: more than 65535 label value classes"};
  while (R.size() % 16) R.push_back(0);
  R.resize(R.size() + 16, 0);  // slack: dword-granular readers may run past the last table
  if (env->kv.empty()) return {};
  align16(b);
  hdr->kv_off = (uint32_t)b->size();
  hdr->kv_bytes = (uint32_t)R.size();
  b->insert(b->end(), R.begin(), R.end());
  hdr->col[COL_LV].nclass = (uint32_t)env->kv.size();
  hdr->col[COL_LV].ndfa = longest;
  hdr->col[COL_LV].dfa_bytes = (uint32_t)R.size();
  return {};
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

// A policy whose local bits exceed one chunk's 64 becomes consecutive parts (PolicyRec::parts),
// each within the limit, appended as hidden records:
//  safe-labels: the mandatory list cut into runs of <= 64 distinct keys (settings order); part 0
//   also holds the denied and constrained labels. The first part that rejects decides: label
//   violations come first (part 0), then the first missing mandatory key in settings order, its
//   index offset by the run's start (part_off).
//  psp-capabilities: the required drops and default adds cut into parts of <= 63 distinct names
//   (+ "ALL"); part 0 validates the added capabilities against allowed + every default add (the
//   allowance rule of the whole policy), the other parts allow everything; the policy rejects when
//   part 0 rejects, else is mutated when any part is.
static void split_policy(Env* env, size_t idx) {
  auto distinct_runs = [](const std::vector<std::string>& l, size_t cap) {
    std::vector<std::pair<size_t, size_t>> runs;  // [begin, end) positions
    size_t b = 0;
    std::vector<std::string> seen;
    for (size_t i = 0; i < l.size(); ++i) {
      if (std::find(seen.begin(), seen.end(), l[i]) == seen.end()) {
        if (seen.size() == cap) {
          runs.push_back({b, i});
          b = i;
          seen.clear();
        }
        seen.push_back(l[i]);
      }
    }
    runs.push_back({b, l.size()});
    return runs;
  };
  PolicyRec& P0 = env->pol[idx];
  std::vector<PolicyRec> parts;
  std::vector<uint32_t> offs;
  if (P0.family == FAM_LABELS) {
    std::vector<std::string> keys = P0.lists[1];
    std::sort(keys.begin(), keys.end());
    if ((size_t)(std::unique(keys.begin(), keys.end()) - keys.begin()) <= (size_t)kMaxLocalBits) return;
    const auto runs = distinct_runs(P0.lists[1], kMaxLocalBits);
    for (size_t k = 0; k < runs.size(); ++k) {
      PolicyRec q;
      q.family = FAM_LABELS;
      if (k == 0) {
        q.lists[0] = P0.lists[0];
        q.lists[2] = P0.lists[2];
        q.lists[3] = P0.lists[3];
      }
      q.lists[1].assign(P0.lists[1].begin() + (long)runs[k].first, P0.lists[1].begin() + (long)runs[k].second);
      parts.push_back(std::move(q));
      offs.push_back((uint32_t)runs[k].first);
    }
  } else if (P0.family == FAM_CAPABILITIES) {
    std::vector<std::string> all = P0.lists[1];
    all.insert(all.end(), P0.lists[2].begin(), P0.lists[2].end());
    all.push_back("ALL");
    std::sort(all.begin(), all.end());
    if ((size_t)(std::unique(all.begin(), all.end()) - all.begin()) <= (size_t)kMaxLocalBits) return;
    // drops then adds as one list of (kind, name), cut into runs of <= 63 distinct names
    std::vector<std::string> names;
    for (auto& c : P0.lists[1]) names.push_back("d" + c);
    for (auto& c : P0.lists[2]) names.push_back("a" + c);
    std::vector<std::string> bare;
    for (auto& n : names) bare.push_back(n.substr(1));
    const auto runs = distinct_runs(bare, kMaxLocalBits - 1);
    for (size_t k = 0; k < runs.size(); ++k) {
      PolicyRec q;
      q.family = FAM_CAPABILITIES;
      if (k == 0) {
        q.lists[0] = P0.lists[0];
        q.lists[0].insert(q.lists[0].end(), P0.lists[2].begin(), P0.lists[2].end());
        q.flags = P0.flags & PF_ALLOW_ALL;
      } else {
        q.flags = PF_ALLOW_ALL;
      }
      for (size_t i = runs[k].first; i < runs[k].second; ++i)
        q.lists[names[i][0] == 'd' ? 1 : 2].push_back(names[i].substr(1));
      parts.push_back(std::move(q));
      offs.push_back(0);
    }
  } else {
    return;
  }
  const std::string id = P0.id;
  const int32_t parent = (int32_t)idx;
  std::vector<int32_t> at;
  for (size_t k = 0; k < parts.size(); ++k) {
    PolicyRec& q = parts[k];
    q.id = id + "#part" + std::to_string(k);
    q.name = q.id;
    q.module = env->pol[idx].module;
    q.mode = KW_MODE_PROTECT;
    q.registered = true;
    q.is_part = true;
    q.parent = parent;
    at.push_back((int32_t)env->pol.size());
    env->pol.push_back(std::move(q));
  }
  env->pol[idx].parts = at;
  env->pol[idx].part_off = offs;
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
  for (uint32_t kid : d.members(0)) {
    Entry e;
    std::string err;
    if (!parse_entry(d, std::string(d.key(kid)), kid, &e, &err))
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
    rec.prog = compile_group_expression(rec.expression, rec.member_names);
  }
  // policies beyond one chunk's local bits: hidden parts after the visible records
  env->nvisible = env->pol.size();
  for (size_t i = 0; i < env->nvisible; ++i)
    if (!env->pol[i].is_group && !env->pol[i].init_error) split_policy(env, i);
  // a group with a split member reads that member's word combined from its parts: only the wide
  // path's combine kernel does, so the group takes a wide form (wide jump code or script bytecode)
  for (size_t i = 0; i < env->nvisible; ++i) {
    PolicyRec& g = env->pol[i];
    if (!g.is_group || !g.prog.valid || g.prog.eval_error || g.prog.wide) continue;
    bool split_member = false;
    for (int32_t m : g.members) split_member = split_member || (!env->pol[(size_t)m].parts.empty() && !env->pol[(size_t)m].init_error);
    if (split_member) g.prog = compile_group_expression(g.expression, g.member_names, /*force_wide=*/true);
  }

  // ---- the request columns' patterns: every list of every initialised policy as pattern ids
  if (env->always_ns) pattern_id(&env->cols[COL_NS], Pattern::Literal, *env->always_ns);
  for (PolicyRec& r : env->pol) {
    if (r.is_group || r.init_error) continue;
    auto ids = [&](Col c, Pattern::Kind k, const std::vector<std::string>& l) {
      std::vector<uint32_t> v;
      for (const auto& s : l) {
        const Pattern::Kind kk = (k == Pattern::Glob && c != COL_IMG && glob_is_literal(s)) ? Pattern::Literal : k;
        v.push_back(pattern_id(&env->cols[c], kk, s));
      }
      return v;
    };
    switch (r.family) {
      case FAM_NAMESPACE: r.pid[0] = ids(COL_NS, Pattern::Literal, r.lists[0]); break;
      case FAM_TRUSTED_REPOS:
        r.pid[0] = ids(COL_REG, Pattern::Glob, r.lists[0]);
        r.pid[1] = ids(COL_REG, Pattern::Glob, r.lists[1]);
        r.pid[2] = ids(COL_TAG, Pattern::Glob, r.lists[2]);
        r.pid[3] = ids(COL_IMG, Pattern::Glob, r.lists[3]);
        r.pid[4] = ids(COL_IMG, Pattern::Glob, r.lists[4]);
        break;
      case FAM_CAPABILITIES: {
        std::vector<std::string> allowed;
        for (auto& c : r.lists[0])
          if (c != "*") allowed.push_back(c);
        r.pid[0] = ids(COL_CAP, Pattern::Literal, allowed);
        r.pid[1] = ids(COL_CAP, Pattern::Literal, r.lists[1]);
        r.pid[2] = ids(COL_CAP, Pattern::Literal, r.lists[2]);
        r.pid[3] = ids(COL_CAP, Pattern::Literal, {"ALL"});
        break;
      }
      case FAM_APPARMOR: r.pid[0] = ids(COL_AA, Pattern::Literal, r.lists[0]); break;
      case FAM_LABELS:
        r.pid[0] = ids(COL_LK, Pattern::Literal, r.lists[0]);
        r.pid[1] = ids(COL_LK, Pattern::Literal, r.lists[1]);
        r.pid[2] = ids(COL_LK, Pattern::Literal, r.lists[2]);
        r.pid[3] = ids(COL_LV, Pattern::Regex, r.lists[3]);
        break;
      default: break;
    }
  }

  // ---- blob: header, the column classifiers, the per-key label-value region
  std::vector<uint8_t>& b = env->blob;
  b.clear();
  DevHeader hdr;
  memset(&hdr, 0, sizeof(hdr));
  put(&b, hdr);
  align16(&b);
  for (int c = 0; c < (int)NCOL; ++c) {
    if (c == COL_LV) continue;
    Status st = compile_col((Col)c, &env->cols[c], &hdr.col[c], &b);
    if (!st.ok()) return st;
  }
  env->cols[COL_LV].class_pats.clear();
  env->cols[COL_LV].lit_cls.assign(env->cols[COL_LV].pats.size(), 0);
  if (Status st = compile_kv(env, &hdr, &b); !st.ok()) return st;
  auto lit_class = [&](Col c, const char* s) -> uint32_t {
    const ColumnInfo& ci = env->cols[c];
    for (size_t p = 0; p < ci.pats.size(); ++p)
      if (ci.pats[p].kind == Pattern::Literal && ci.pats[p].text == s) return ci.lit_cls[p];
    return 0;
  };
  if (env->always_ns) hdr.bypass_cls = lit_class(COL_NS, env->always_ns->c_str());
  hdr.docker_io_cls = lit_class(COL_REG, "docker.io");
  hdr.latest_cls = lit_class(COL_TAG, "latest");
  uint64_t nfa_words = 0;
  for (int c = 0; c < (int)NCOL; ++c) nfa_words = std::max(nfa_words, env->cols[c].nfa_words);
  if (nfa_words > 0xffffffffull) return {KW_E_BOOTSTRAP, "bootstrap failure: pattern automaton too large"};
  hdr.nfa_words = (uint32_t)nfa_words;
  align16(&b);
  hdr.magic = kBlobMagic;
  hdr.version = kBlobVersion;
  hdr.blob_bytes = (uint32_t)b.size();
  for (int c = 0; c < (int)NCOL; ++c) hdr.npatterns += (uint32_t)env->cols[c].pats.size();
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

// ---- host classification with the blob's tables (mirrors kernels.hip)
namespace {
uint32_t blob_lit(const uint8_t* blob, uint32_t off, const uint8_t* s, size_t n) {
  const DevLit* L = (const DevLit*)(blob + off);
  const uint8_t* rec = blob + off;
  std::vector<uint32_t> w((n + 3) / 4, 0u);
  if (n) memcpy(w.data(), s, n);
  uint32_t h = lit_init(L->seed, (uint32_t)n);
  for (uint32_t x : w) h = lit_mix(h, x);
  const uint32_t g = lit_final(h);
  const uint32_t d = L->nb_log2 ? ((const uint16_t*)(rec + L->disp_off))[g >> (32 - L->nb_log2)] : 0u;
  const uint32_t* slot = (const uint32_t*)(rec + L->slot_off) + 2u * lit_slot_index(g, d, L->nslots);
  if (!slot[0] || lit_slot_len(slot[0]) != n) return 0;
  const uint32_t* pw = (const uint32_t*)(rec + L->word_off) + slot[1];
  for (size_t i = 0; i < w.size(); ++i)
    if (w[i] != pw[i]) return 0;
  return lit_slot_cls(slot[0]);
}
uint32_t blob_dfa(const uint8_t* blob, uint32_t off, const uint8_t* s, size_t n) {
  const DevDfa* d = (const DevDfa*)(blob + off);
  if (d->kind == 1) return ((const uint16_t*)(blob + d->acc_off))[run_nfa_record(blob + d->trans_off, s, n) ? 1 : 0];
  const uint16_t* trans = (const uint16_t*)(blob + d->trans_off);
  const uint16_t* acc = (const uint16_t*)(blob + d->acc_off);
  uint32_t st = d->start;
  for (size_t i = 0; i < n && st != 0; ++i) st = trans[(size_t)st * d->ncls + d->cls[s[i]]];
  return acc[st];
}
}  // namespace

std::vector<uint32_t> host_classes(const Env& env, Col c, const uint8_t* s, size_t n) {
  const DevHeader* H = (const DevHeader*)env.blob.data();
  const DevCol& dc = H->col[c];
  std::vector<uint32_t> out;
  if (dc.lit_off) out.push_back(blob_lit(env.blob.data(), dc.lit_off, s, n));
  for (uint32_t o = dc.dfa_off; o; o = ((const DevDfa*)(env.blob.data() + o))->next)
    out.push_back(blob_dfa(env.blob.data(), o, s, n));
  return out;
}

std::vector<uint32_t> host_value_classes(const Env& env, uint32_t key, const uint8_t* s, size_t n) {
  const DevHeader* H = (const DevHeader*)env.blob.data();
  std::vector<uint32_t> out;
  if (!H->kv_off || key == 0 || key >= H->col[COL_LK].nclass) return out;
  const uint8_t* R = env.blob.data() + H->kv_off;
  const uint32_t nlk = H->col[COL_LK].nclass;
  const uint32_t kbase = ((const uint32_t*)R)[nlk + key];
  for (uint32_t rel = ((const uint32_t*)R)[key]; rel;) {
    const KvDfa& d = *(const KvDfa*)(R + rel);
    uint32_t st = d.start;
    if (d.nfa) {
      out.push_back(kbase + d.cbase + (run_nfa_record(env.blob.data() + d.trans_off, s, n) ? 1u : 0u));
      rel = d.next;
      continue;
    }
    for (size_t i = 0; i < n && st != 0; ++i) st = kv_step(R, d, st, s[i]);
    out.push_back(kbase + d.cbase + ((const uint16_t*)(R + d.acc_off))[st]);
    rel = d.next;
  }
  return out;
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
