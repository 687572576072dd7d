// service.cpp — see service.hpp.
#include "service.hpp"

#include <algorithm>

#include "json.hpp"

namespace kw {

void image_parts(std::string_view s, std::string* registry, std::string* tag, bool* has_tag) {
  size_t at = s.find('@');
  std::string_view name = at == std::string_view::npos ? s : s.substr(0, at);
  size_t slash = name.find('/');
  size_t rest_b = 0;
  bool is_reg = false;
  if (slash != std::string_view::npos) {
    std::string_view c0 = name.substr(0, slash);
    is_reg = c0.find('.') != std::string_view::npos || c0.find(':') != std::string_view::npos || c0 == "localhost";
  }
  if (is_reg) {
    *registry = std::string(name.substr(0, slash));
    rest_b = slash + 1;
  } else {
    *registry = "docker.io";
  }
  std::string_view rest = name.substr(rest_b);
  size_t colon = rest.rfind(':');
  if (colon != std::string_view::npos) {
    *tag = std::string(rest.substr(colon + 1));
    *has_tag = true;
  } else if (at == std::string_view::npos) {
    *tag = "latest";
    *has_tag = true;
  } else {
    tag->clear();
    *has_tag = false;
  }
}

bool WideData::lookup(uint64_t row, int32_t policy, uint64_t* v) const {
  if (nwide) {
    if (rows_mode) {
      if (row < groups.size()) {
        // rows mode: the row's own column is the only wide one it can have
        for (int32_t p : wide_policy)
          if (p == policy) {
            *v = groups[row];
            return true;
          }
      }
    } else {
      for (uint32_t k = 0; k < nwide && k < wide_policy.size(); ++k)
        if (wide_policy[k] == policy && row * nwide + k < groups.size()) {
          *v = groups[row * nwide + k];
          return true;
        }
    }
  }
  auto it = std::lower_bound(recs.begin(), recs.end(), std::make_pair(row, policy), [](const Rec& r, const std::pair<uint64_t, int32_t>& k) {
    return r.row < k.first || (r.row == k.first && r.policy < k.second);
  });
  if (it != recs.end() && it->row == row && it->policy == policy) {
    *v = it->value;
    return true;
  }
  return false;
}

// The full argument of a verdict word: its ARG, or the pass's side value when ARG is kArgWide.
static Status full_arg(const Batch& b, uint64_t row, int32_t pidx, uint32_t arg, uint64_t* out) {
  if (arg != 0xffffu) {
    *out = arg;
    return {};
  }
  if (!b.wide.lookup(row, pidx, out)) return {KW_E_ENGINE, "verdict argument not found in the pass's side data"};
  return {};
}

Status policy_message(const Env& env, const Batch& b, uint64_t row, int32_t pidx, uint32_t reason, uint64_t arg,
                      std::string* msg) {
  const PolicyRec& P = env.pol[(size_t)pidx];
  const uint32_t cb = b.ctr_off[row], ce = b.ctr_off[row + 1], lb = b.lbl_off[row], le = b.lbl_off[row + 1];
  auto q = [](std::string_view s) { return "'" + std::string(s) + "'"; };
  const Status bad{KW_E_ENGINE, "verdict argument out of range for the request"};
  std::string_view name, image, s1, s2;
  switch (reason) {
    case KW_R_PRIVILEGED: *msg = "Privileged container is not allowed"; return {};  // integration_test.rs:64
    case KW_R_NAMESPACE:
      *msg = "namespace " + q(b.ns.at(row)) + " is not accepted: only " + q(P.lists[0].empty() ? "" : P.lists[0][0]) +
             " is allowed";
      return {};
    case KW_R_REG_NOT_ALLOWED:
    case KW_R_REG_REJECTED:
    case KW_R_TAG_REJECTED:
    case KW_R_IMG_NOT_ALLOWED:
    case KW_R_IMG_REJECTED: {  // arg: container index within the request
      if (arg >= ce - cb || !b.ctr_name.get(cb + arg, &name) || !b.ctr_image.get(cb + arg, &image)) return bad;
      std::string reg, tag;
      bool has_tag;
      image_parts(image, &reg, &tag, &has_tag);
      const std::string head = "container " + q(name) + " uses image " + q(image);
      if (reason == KW_R_REG_NOT_ALLOWED) *msg = head + ": registry " + q(reg) + " is not in the allowed registries";
      else if (reason == KW_R_REG_REJECTED) *msg = head + ": registry " + q(reg) + " is rejected";
      else if (reason == KW_R_TAG_REJECTED) *msg = head + ": tag " + q(tag) + " is rejected";
      else if (reason == KW_R_IMG_NOT_ALLOWED) *msg = head + ", which is not in the allowed images";
      else *msg = head + ", which is rejected";
      return {};
    }
    case KW_R_CAP_NOT_ALLOWED: {  // arg: index in the request's capabilities.add lists, flattened
      const uint64_t k0 = b.capadd_off[cb], k = k0 + arg;
      if (k >= b.capadd_off[ce]) return bad;
      // the container whose add list holds entry k
      const uint32_t c = (uint32_t)(std::upper_bound(b.capadd_off.begin() + cb, b.capadd_off.begin() + ce + 1, (uint32_t)k) -
                                    b.capadd_off.begin()) - 1;
      if (c < cb || c >= ce || !b.ctr_name.get(c, &name) || !b.cap_add.get(k, &s1)) return bad;
      *msg = "container " + q(name) + " adds capability " + q(s1) + ", which is not allowed";
      return {};
    }
    case KW_R_APPARMOR:
      if (arg >= ce - cb || !b.ctr_name.get(cb + arg, &name) || !b.ctr_aa.get(cb + arg, &s1)) return bad;
      *msg = "container " + q(name) + " uses AppArmor profile " + q(s1) + ", which is not allowed";
      return {};
    case KW_R_LABEL_DENIED:
      if (arg >= le - lb || !b.lbl_key.get(lb + arg, &s1)) return bad;
      *msg = "label " + q(s1) + " is denied";
      return {};
    case KW_R_LABEL_CONSTRAINT: {  // arg: label index; the constraint is the policy's on that key
      if (arg >= le - lb || !b.lbl_key.get(lb + arg, &s1) || !b.lbl_val.get(lb + arg, &s2)) return bad;
      for (size_t i = 0; i < P.lists[2].size(); ++i)
        if (P.lists[2][i] == s1) {
          *msg = "label " + q(s1) + " value " + q(s2) + " does not match the constraint " + q(P.lists[3][i]);
          return {};
        }
      return bad;
    }
    case KW_R_LABEL_MANDATORY:
      if (arg >= P.lists[1].size()) return bad;
      *msg = "mandatory label " + q(P.lists[1][arg]) + " is missing";
      return {};
    case KW_R_GROUP: *msg = P.message; return {};
    case KW_R_GROUP_EXPR: *msg = P.prog.valid ? P.prog.eval_message : P.prog.error; return {};
    case KW_R_INIT_ERROR: *msg = P.init_message; return {};
  }
  msg->clear();
  return {};
}

static void put_kv(std::string* o, const char* k, std::string_view v) {
  o->push_back('"');
  o->append(k);
  o->append("\":");
  json_escape(o, v);
}

namespace {

std::string base64(const std::string& in) {
  static const char* T = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  o.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    const uint32_t x = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    o += T[x >> 18];
    o += T[(x >> 12) & 63];
    o += T[(x >> 6) & 63];
    o += T[x & 63];
  }
  if (i + 1 == in.size()) {
    const uint32_t x = (uint8_t)in[i] << 16;
    o += T[x >> 18];
    o += T[(x >> 12) & 63];
    o += "==";
  } else if (i + 2 == in.size()) {
    const uint32_t x = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    o += T[x >> 18];
    o += T[(x >> 12) & 63];
    o += T[(x >> 6) & 63];
    o += '=';
  }
  return o;
}

void json_list(std::string* o, const std::vector<std::string>& l) {
  o->append("[");
  for (size_t i = 0; i < l.size(); ++i) {
    if (i) o->append(",");
    json_escape(o, l[i]);  // quoted
  }
  o->append("]");
}

}  // namespace

Status capabilities_patch(const PolicyRec& P, const char* doc, size_t len, int doc_kind, std::string* ops) {
  thread_local JDoc d;
  std::string perr;
  if (!d.parse(doc, len, &perr) || !d.is(0, JType::Obj)) return {KW_E_ARG, "document does not parse"};
  (void)doc_kind;  // AdmissionReview and RawReview both carry the object under request.object
  const int64_t req = d.get(0, "request");
  const PodSpecRef ps = find_podspec(d, req);
  ops->assign("[");
  bool first_op = true;
  auto op = [&](const std::string& path, const std::string& value) {
    if (!first_op) ops->append(",");
    first_op = false;
    ops->append("{\"op\":\"add\",\"path\":");
    json_escape(ops, path);
    ops->append(",\"value\":");
    ops->append(value);
    ops->append("}");
  };
  auto uniq = [](const std::vector<std::string>& l) {
    std::vector<std::string> o;
    for (const auto& x : l)
      if (std::find(o.begin(), o.end(), x) == o.end()) o.push_back(x);
    return o;
  };
  const std::vector<std::string> reqd = uniq(P.lists[1]), defa = uniq(P.lists[2]);
  if (ps.spec >= 0) {
    const char* lists[3] = {"containers", "initContainers", "ephemeralContainers"};
    for (const char* ln : lists) {
      const int64_t arr = d.get((uint32_t)ps.spec, ln);
      if (arr < 0 || !d.is((uint32_t)arr, JType::Arr)) continue;
      uint32_t k = 0;  // item index (the JSON Pointer's)
      for (uint32_t c : d.members((uint32_t)arr)) {
        const uint32_t ki = k++;
        if (!d.is(c, JType::Obj)) continue;
        const int64_t sc = d.get(c, "securityContext");
        const bool sc_obj = sc >= 0 && d.is((uint32_t)sc, JType::Obj);
        const int64_t caps = sc_obj ? d.get((uint32_t)sc, "capabilities") : -1;
        const bool caps_obj = caps >= 0 && d.is((uint32_t)caps, JType::Obj);
        const int64_t add = caps_obj ? d.get((uint32_t)caps, "add") : -1, drop = caps_obj ? d.get((uint32_t)caps, "drop") : -1;
        const bool add_arr = add >= 0 && d.is((uint32_t)add, JType::Arr), drop_arr = drop >= 0 && d.is((uint32_t)drop, JType::Arr);
        auto has = [&](int64_t a, bool is_arr, const std::string& x) {
          if (!is_arr) return false;
          for (uint32_t it : d.members((uint32_t)a)) {
            if (d.is(it, JType::Str) && d.str(it) == x) return true;
          }
          return false;
        };
        std::vector<std::string> mdrop, madd;
        if (!has(drop, drop_arr, "ALL"))
          for (const auto& x : reqd)
            if (!has(drop, drop_arr, x)) mdrop.push_back(x);
        for (const auto& x : defa)
          if (!has(add, add_arr, x) && !has(drop, drop_arr, x)) madd.push_back(x);
        if (mdrop.empty() && madd.empty()) continue;
        const std::string base = std::string(ps.pointer) + "/" + ln + "/" + std::to_string(ki) + "/securityContext";
        std::string cap_obj = "{";
        if (!madd.empty()) {
          cap_obj += "\"add\":";
          json_list(&cap_obj, madd);
        }
        if (!mdrop.empty()) {
          if (!madd.empty()) cap_obj += ",";
          cap_obj += "\"drop\":";
          json_list(&cap_obj, mdrop);
        }
        cap_obj += "}";
        if (!sc_obj) {
          op(base, "{\"capabilities\":" + cap_obj + "}");
        } else if (!caps_obj) {
          op(base + "/capabilities", cap_obj);
        } else {
          for (const auto* pr : {&madd, &mdrop}) {
            if (pr->empty()) continue;
            const bool is_add = pr == &madd;
            const std::string lp = base + "/capabilities/" + (is_add ? "add" : "drop");
            if (!(is_add ? add_arr : drop_arr)) {
              std::string v;
              json_list(&v, *pr);
              op(lp, v);
            } else {
              for (const auto& x : *pr) {
                std::string v;
                json_escape(&v, x);
                op(lp + "/-", v);
              }
            }
          }
        }
      }
    }
  }
  ops->append("]");
  return {};
}

Status format_response(const Env& env, const Batch& b, uint64_t row, int32_t pidx, uint32_t v, const uint32_t* member_v,
                       std::string* out, const char* doc, size_t doc_len, int doc_kind) {
  const PolicyRec& P = env.pol[(size_t)pidx];
  out->clear();
  std::string_view uid = b.uid.at(row);
  const uint32_t fst = (v & KW_F_STATUS_MASK) >> KW_F_STATUS_SHIFT;
  const uint32_t reason = KW_REASON(v), arg = KW_ARG(v);
  if (v & KW_BYPASS) {
    // service.rs:42-48: the bypass path still resolves the policy mode -> PolicyNotFound
    if (!P.registered) return {KW_E_NOT_FOUND, "unknown policy: " + P.id};
    out->append("{");
    put_kv(out, "uid", uid);
    out->append(",\"allowed\":true}");
    return {};
  }
  if (P.is_group && !P.broken_member.empty()) return {KW_E_NOT_FOUND, "unknown policy: " + P.broken_member};
  if ((v & KW_F_PATCH) != 0) {  // accepted mutation: the response carries the JSONPatch
    if (!doc) return {KW_E_ARG, "the original document is required to format a mutation (kw_format_response_doc)"};
    if (P.family != FAM_CAPABILITIES) return {KW_E_ENGINE, "mutation by a non-mutating policy family"};
    std::string ops;
    Status st = capabilities_patch(P, doc, doc_len, doc_kind, &ops);
    if (!st.ok()) return st;
    out->append("{");
    put_kv(out, "uid", uid);
    out->append(",\"allowed\":true,\"patchType\":\"JSONPatch\",");
    put_kv(out, "patch", base64(ops));
    out->append("}");
    return {};
  }
  out->append("{");
  put_kv(out, "uid", uid);
  out->append((v & KW_F_ALLOWED) ? ",\"allowed\":true" : ",\"allowed\":false");
  if (fst == KW_FST_NONE) {
    out->append("}");
    return {};
  }
  out->append(",\"status\":{");
  if (fst == KW_FST_INIT_ERROR) {
    put_kv(out, "message", P.init_message);
    out->append(",\"code\":500}}");  // AdmissionResponse::reject(uid, msg, 500), service.rs:86-90
    return {};
  }
  if (fst == KW_FST_MUTATION_REFUSED) {
    put_kv(out, "message", "Request rejected by policy " + P.id +
                               ". The policy attempted to mutate the request, but it is currently configured to not "
                               "allow mutations.");
    out->append("}}");
    return {};
  }
  // vanilla status
  uint64_t full = 0;
  // causes: multi-word side data (a wide group of more than 15 members; smaller ones carry them in ARG)
  const bool big_group = reason == KW_R_GROUP && P.is_group && P.prog.wide && arg == KW_ARG_WIDE;
  if (reason != KW_R_GROUP_EXPR && reason != KW_R_INIT_ERROR && !big_group) {
    Status st = full_arg(b, row, pidx, arg, &full);
    if (!st.ok()) return st;
  }
  std::string msg;
  if (reason == KW_R_GROUP_EXPR && P.is_group && P.prog.valid && !P.prog.eval_error && member_v) {
    // a data-dependent evaluation error (truth-table groups): the host interpreter over the
    // members' results names it
    const ExprOutcome o = P.prog.run([&](uint32_t s) {
      const uint32_t mv = member_v[s];
      return (mv & KW_V_ALLOWED) && !(mv & KW_V_MUTATED);
    });
    msg = group_eval_message(o.error ? o.message : "no error");
  } else if (Status st = policy_message(env, b, row, pidx, reason, full, &msg); !st.ok()) {
    return st;
  }
  put_kv(out, "message", msg);
  if (reason == KW_R_GROUP_EXPR) {
    out->append(",\"code\":500}}");
    return {};
  }
  if (reason == KW_R_GROUP) {
    if (!member_v) return {KW_E_ARG, "member verdicts are required to format a policy-group rejection"};
    const uint64_t* big = nullptr;
    uint32_t big_words = 0;
    if (big_group && !(big = b.wide.lookup_big(row, pidx, &big_words)))
      return {KW_E_ENGINE, "group causes not found in the pass's side data"};
    out->append(",\"details\":{\"causes\":[");
    bool first = true;
    for (size_t s = 0; s < P.members.size(); ++s) {
      const bool cause = big ? (s / 64 < big_words && ((big[s / 64] >> (s % 64)) & 1ull)) : (s < 64 && ((full >> s) & 1ull));
      if (!cause) continue;
      int32_t m = P.members[s];
      uint32_t mv = member_v[s];
      std::string msg;
      if ((mv & KW_V_MUTATED) && (mv & KW_V_ALLOWED)) {
        msg = "mutation is not allowed inside of policy group";  // integration_test.rs:247-250
      } else {
        uint64_t marg = 0;
        if (Status st = full_arg(b, row, m, KW_ARG(mv), &marg); !st.ok()) return st;
        if (Status st = policy_message(env, b, row, m, KW_REASON(mv), marg, &msg); !st.ok()) return st;
      }
      if (!first) out->push_back(',');
      first = false;
      out->append("{");
      put_kv(out, "field", "spec.policies." + env.pol[(size_t)m].name);
      out->push_back(',');
      put_kv(out, "message", msg);
      out->append("}");
    }
    out->append("]}}}");
    return {};
  }
  out->append("}}");
  return {};
}

}  // namespace kw
