// service.cpp — see service.hpp.
#include "service.hpp"

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

std::string policy_message(const Env& env, const Batch& b, uint64_t row, int32_t pidx, uint32_t reason, uint32_t arg) {
  const PolicyRec& P = env.pol[(size_t)pidx];
  const uint32_t cb = b.ctr_off[row], lb = b.lbl_off[row];
  auto q = [](std::string_view s) { return "'" + std::string(s) + "'"; };
  auto cname = [&](uint32_t c) { return std::string(b.ctr_name.at(cb + c)); };
  auto cimage = [&](uint32_t c) { return std::string(b.ctr_image.at(cb + c)); };
  switch (reason) {
    case KW_R_PRIVILEGED: return "Privileged container is not allowed";  // integration_test.rs:64
    case KW_R_NAMESPACE:
      return "namespace " + q(b.ns.at(row)) + " is not accepted: only " + q(P.lists[0].empty() ? "" : P.lists[0][0]) +
             " is allowed";
    case KW_R_REG_NOT_ALLOWED:
    case KW_R_REG_REJECTED:
    case KW_R_TAG_REJECTED:
    case KW_R_IMG_NOT_ALLOWED:
    case KW_R_IMG_REJECTED: {
      std::string reg, tag;
      bool has_tag;
      image_parts(b.ctr_image.at(cb + arg), &reg, &tag, &has_tag);
      std::string head = "container " + q(cname(arg)) + " uses image " + q(cimage(arg));
      if (reason == KW_R_REG_NOT_ALLOWED) return head + ": registry " + q(reg) + " is not in the allowed registries";
      if (reason == KW_R_REG_REJECTED) return head + ": registry " + q(reg) + " is rejected";
      if (reason == KW_R_TAG_REJECTED) return head + ": tag " + q(tag) + " is rejected";
      if (reason == KW_R_IMG_NOT_ALLOWED) return head + ", which is not in the allowed images";
      return head + ", which is rejected";
    }
    case KW_R_CAP_NOT_ALLOWED: {
      uint32_t c = arg >> 8, k = arg & 0xff;
      uint32_t cap = b.capadd_off[cb + c] + k;
      return "container " + q(cname(c)) + " adds capability " + q(b.cap_add.at(cap)) + ", which is not allowed";
    }
    case KW_R_APPARMOR:
      return "container " + q(cname(arg)) + " uses AppArmor profile " + q(b.ctr_aa.at(cb + arg)) +
             ", which is not allowed";
    case KW_R_LABEL_DENIED: return "label " + q(b.lbl_key.at(lb + arg)) + " is denied";
    case KW_R_LABEL_CONSTRAINT: {
      uint32_t l = arg >> 8, i = arg & 0xff;
      return "label " + q(b.lbl_key.at(lb + l)) + " value " + q(b.lbl_val.at(lb + l)) + " does not match the constraint " +
             q(P.lists[3][i]);
    }
    case KW_R_LABEL_MANDATORY: return "mandatory label " + q(P.lists[1][arg]) + " is missing";
    case KW_R_GROUP: return P.message;
    case KW_R_GROUP_EXPR: return P.prog.valid ? P.prog.eval_message : P.prog.error;
    case KW_R_INIT_ERROR: return P.init_message;
  }
  return "";
}

static void put_kv(std::string* o, const char* k, std::string_view v) {
  o->push_back('"');
  o->append(k);
  o->append("\":");
  json_escape(o, v);
}

Status format_response(const Env& env, const Batch& b, uint64_t row, int32_t pidx, uint32_t v, const uint32_t* member_v,
                       std::string* out) {
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
  if ((v & KW_F_PATCH) != 0)
    return {KW_E_ENGINE, "JSONPatch generation for mutating policies is not implemented yet"};
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
  put_kv(out, "message", policy_message(env, b, row, pidx, reason, arg));
  if (reason == KW_R_GROUP_EXPR) {
    out->append(",\"code\":500}}");
    return {};
  }
  if (reason == KW_R_GROUP) {
    if (!member_v) return {KW_E_ARG, "member verdicts are required to format a policy-group rejection"};
    out->append(",\"details\":{\"causes\":[");
    bool first = true;
    for (size_t s = 0; s < P.members.size(); ++s) {
      if (!((arg >> s) & 1u)) continue;
      int32_t m = P.members[s];
      uint32_t mv = member_v[s];
      std::string msg = (mv & KW_V_MUTATED) && (mv & KW_V_ALLOWED)
                            ? std::string("mutation is not allowed inside of policy group")  // integration_test.rs:247-250
                            : policy_message(env, b, row, m, KW_REASON(mv), KW_ARG(mv));
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
