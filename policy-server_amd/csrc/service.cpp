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
      for (uint32_t k = 0; k < d.count((uint32_t)arr); ++k) {
        const uint32_t c = d.kids((uint32_t)arr)[k].node;
        if (!d.is(c, JType::Obj)) continue;
        const int64_t sc = d.get(c, "securityContext");
        const bool sc_obj = sc >= 0 && d.is((uint32_t)sc, JType::Obj);
        const int64_t caps = sc_obj ? d.get((uint32_t)sc, "capabilities") : -1;
        const bool caps_obj = caps >= 0 && d.is((uint32_t)caps, JType::Obj);
        const int64_t add = caps_obj ? d.get((uint32_t)caps, "add") : -1, drop = caps_obj ? d.get((uint32_t)caps, "drop") : -1;
        const bool add_arr = add >= 0 && d.is((uint32_t)add, JType::Arr), drop_arr = drop >= 0 && d.is((uint32_t)drop, JType::Arr);
        auto has = [&](int64_t a, bool is_arr, const std::string& x) {
          if (!is_arr) return false;
          for (uint32_t i = 0; i < d.count((uint32_t)a); ++i) {
            const uint32_t it = d.kids((uint32_t)a)[i].node;
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
        const std::string base = std::string(ps.pointer) + "/" + ln + "/" + std::to_string(k) + "/securityContext";
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
