// flatten.cpp — AdmissionReview / RawReview JSON -> SoA row (batch.hpp).
//
// Deserialization contract (what makes the reference answer 422 before evaluating):
//   AdmissionReviewRequest { kind?, apiVersion?, request: AdmissionRequest } (admission_review.rs:4-14)
//   AdmissionRequest [upstream policy-evaluator]: uid, kind{group,version,kind}, resource{group,
//   version,resource}, operation and userInfo are required; namespace/name are optional strings;
//   object/oldObject/options are arbitrary JSON.
//   RawReviewRequest { request: Value } (raw_review.rs:5-9).
// Extraction: namespace, operation, request kind, uid; the PodSpec of the
// object (Pod: spec; Deployment/ReplicaSet/StatefulSet/DaemonSet/Job/ReplicationController:
// spec.template.spec; CronJob: spec.jobTemplate.spec.template.spec), its containers,
// initContainers and ephemeralContainers (name, image, securityContext.privileged,
// securityContext.capabilities.add/drop, AppArmor profile from the pod-template annotation
// container.apparmor.security.beta.kubernetes.io/<name>), and object.metadata.labels.
#include <cstring>

#include "batch.hpp"
#include "json.hpp"

namespace kw {

void Batch::view(kw_soa* s) const {
  memset(s, 0, sizeof(*s));
  s->n_requests = n;
  s->req_flags = req_flags.data();
  s->ctr_off = ctr_off.data();
  s->lbl_off = lbl_off.data();
  s->uid = uid.view();
  s->ns = ns.view();
  s->op = op.view();
  s->kind = kind.view();
  s->ctr_flags = ctr_flags.data();
  s->capadd_off = capadd_off.data();
  s->capdrop_off = capdrop_off.data();
  s->ctr_name = ctr_name.view();
  s->ctr_image = ctr_image.view();
  s->ctr_apparmor = ctr_aa.view();
  s->cap_add = cap_add.view();
  s->cap_drop = cap_drop.view();
  s->lbl_key = lbl_key.view();
  s->lbl_val = lbl_val.view();
}

void Batch::append(const Batch& o) {
  auto shift = [](std::vector<uint32_t>* dst, const std::vector<uint32_t>& src) {
    const uint32_t base = dst->back();
    for (size_t i = 1; i < src.size(); ++i) dst->push_back(base + src[i]);
  };
  n += o.n;
  req_flags.insert(req_flags.end(), o.req_flags.begin(), o.req_flags.end());
  shift(&ctr_off, o.ctr_off);
  shift(&lbl_off, o.lbl_off);
  ctr_flags.insert(ctr_flags.end(), o.ctr_flags.begin(), o.ctr_flags.end());
  shift(&capadd_off, o.capadd_off);
  shift(&capdrop_off, o.capdrop_off);
  StrCol* mine[] = {&uid, &ns, &op, &kind, &rkind, &ctr_name, &ctr_image, &ctr_aa, &cap_add, &cap_drop, &lbl_key, &lbl_val};
  const StrCol* theirs[] = {&o.uid, &o.ns, &o.op, &o.kind, &o.rkind, &o.ctr_name, &o.ctr_image, &o.ctr_aa,
                            &o.cap_add, &o.cap_drop, &o.lbl_key, &o.lbl_val};
  for (size_t k = 0; k < sizeof(mine) / sizeof(mine[0]); ++k) mine[k]->append(*theirs[k]);
}

void Batch::finalize() {
  for (StrCol* c : {&uid, &ns, &op, &kind, &ctr_name, &ctr_image, &ctr_aa, &cap_add, &cap_drop, &lbl_key, &lbl_val})
    c->pad();
}

namespace {

constexpr std::string_view kAppArmorPrefix = "container.apparmor.security.beta.kubernetes.io/";

int64_t path(const JDoc& d, int64_t n, std::initializer_list<const char*> keys) {
  for (const char* k : keys) {
    if (n < 0) return -1;
    n = d.get((uint32_t)n, k);
  }
  return n;
}

bool is_str(const JDoc& d, int64_t n) { return n >= 0 && d.is((uint32_t)n, JType::Str); }
std::string_view sv(const JDoc& d, int64_t n) { return is_str(d, n) ? d.str((uint32_t)n) : std::string_view(); }

void push_caps(const JDoc& d, int64_t arr, StrCol* col, std::vector<uint32_t>* off) {
  if (arr >= 0 && d.is((uint32_t)arr, JType::Arr))
    for (uint32_t it : d.members((uint32_t)arr))
      if (d.is(it, JType::Str)) col->push(d.str(it));
  off->push_back((uint32_t)col->n());
}

int64_t obj_get(const JDoc& d, int64_t n, std::string_view k) { return n >= 0 ? d.get((uint32_t)n, k) : -1; }

}  // namespace

PodSpecRef find_podspec(const JDoc& d, int64_t req) {
  PodSpecRef r;
  const bool req_obj = req >= 0 && d.is((uint32_t)req, JType::Obj);
  const int64_t obj = req_obj ? d.get((uint32_t)req, "object") : -1;
  if (obj < 0 || !d.is((uint32_t)obj, JType::Obj)) return r;
  r.has_obj = true;
  const std::string_view rkind = sv(d, path(d, req, {"kind", "kind"}));
  const std::string_view k = is_str(d, d.get((uint32_t)obj, "kind")) ? d.str((uint32_t)d.get((uint32_t)obj, "kind")) : rkind;
  if (k == "Pod") {
    r.spec = d.get((uint32_t)obj, "spec");
    r.meta = d.get((uint32_t)obj, "metadata");
    r.pointer = "/spec";
  } else if (k == "Deployment" || k == "ReplicaSet" || k == "StatefulSet" || k == "DaemonSet" || k == "Job" ||
             k == "ReplicationController") {
    r.spec = path(d, obj, {"spec", "template", "spec"});
    r.meta = path(d, obj, {"spec", "template", "metadata"});
    r.pointer = "/spec/template/spec";
  } else if (k == "CronJob") {
    r.spec = path(d, obj, {"spec", "jobTemplate", "spec", "template", "spec"});
    r.meta = path(d, obj, {"spec", "jobTemplate", "spec", "template", "metadata"});
    r.pointer = "/spec/jobTemplate/spec/template/spec";
  }
  if (r.spec >= 0 && !d.is((uint32_t)r.spec, JType::Obj)) r.spec = -1;
  return r;
}

namespace {

// The request's members, picked in one pass (flatten_document's checks and the row's columns).
enum ReqKey { RK_UID, RK_KIND, RK_RESOURCE, RK_OPERATION, RK_USERINFO, RK_NAMESPACE, RK_NAME, RK_SUBRES, RK_REQSUBRES,
              RK_REQKIND, RK_OBJECT, RK_N };
constexpr std::string_view kReqKeys[RK_N] = {"uid",       "kind", "resource",    "operation",          "userInfo", "namespace",
                                             "name",      "subResource", "requestSubResource", "requestKind", "object"};

void flatten_request(const JDoc& d, int64_t req, const int64_t* rk, bool raw, Batch* b) {
  uint8_t rf = raw ? KW_REQ_RAW : 0;
  b->uid.push(sv(d, rk[RK_UID]));
  const int64_t nsn = rk[RK_NAMESPACE];
  if (is_str(d, nsn)) rf |= KW_REQ_HAS_NAMESPACE;
  b->ns.push(sv(d, nsn));
  b->op.push(sv(d, rk[RK_OPERATION]));
  b->kind.push(sv(d, obj_get(d, rk[RK_KIND], "kind")));
  b->rkind.push(sv(d, raw ? -1 : obj_get(d, rk[RK_REQKIND], "kind")));

  const PodSpecRef ps = find_podspec(d, req);
  if (ps.has_obj) rf |= KW_REQ_HAS_OBJECT;
  const int64_t spec = ps.spec, tmpl_meta = ps.meta;
  if (spec >= 0) rf |= KW_REQ_HAS_PODSPEC;
  b->req_flags.push_back(rf);

  // containers
  if (spec >= 0) {
    const int64_t annots = obj_get(d, tmpl_meta, "annotations");
    const bool have_annots = annots >= 0 && d.is((uint32_t)annots, JType::Obj);
    static constexpr std::string_view kLists[3] = {"containers", "initContainers", "ephemeralContainers"};
    static constexpr std::string_view kCtr[3] = {"name", "image", "securityContext"};
    static constexpr std::string_view kSc[2] = {"privileged", "capabilities"};
    static constexpr std::string_view kCaps[2] = {"add", "drop"};
    const uint8_t kinds[3] = {0, KW_CTR_INIT, KW_CTR_EPHEMERAL};
    int64_t arrs[3];
    d.pick((uint32_t)spec, kLists, 3, arrs);
    for (int li = 0; li < 3; ++li) {
      const int64_t arr = arrs[li];
      if (arr < 0 || !d.is((uint32_t)arr, JType::Arr)) continue;
      for (uint32_t c : d.members((uint32_t)arr)) {
        if (!d.is(c, JType::Obj)) continue;
        uint8_t cf = kinds[li];
        int64_t f[3], sc[2] = {-1, -1}, caps[2] = {-1, -1};
        d.pick(c, kCtr, 3, f);
        const std::string_view name = sv(d, f[0]);
        b->ctr_name.push(name);
        if (is_str(d, f[1])) cf |= KW_CTR_HAS_IMAGE;
        b->ctr_image.push(sv(d, f[1]));
        if (f[2] >= 0) d.pick((uint32_t)f[2], kSc, 2, sc);
        if (sc[0] >= 0 && d.is((uint32_t)sc[0], JType::Bool) && d.n((uint32_t)sc[0]).b) cf |= KW_CTR_PRIVILEGED;
        if (sc[1] >= 0) d.pick((uint32_t)sc[1], kCaps, 2, caps);
        push_caps(d, caps[0], &b->cap_add, &b->capadd_off);
        push_caps(d, caps[1], &b->cap_drop, &b->capdrop_off);
        std::string_view profile;
        if (have_annots) {
          for (uint32_t kid : d.members((uint32_t)annots)) {
            const std::string_view key = d.key(kid);
            if (key.size() == kAppArmorPrefix.size() + name.size() && key.substr(0, kAppArmorPrefix.size()) == kAppArmorPrefix &&
                key.substr(kAppArmorPrefix.size()) == name && d.is(kid, JType::Str)) {
              profile = d.str(kid);
              cf |= KW_CTR_HAS_APPARMOR;
            }
          }
        }
        b->ctr_aa.push(profile);
        b->ctr_flags.push_back(cf);
      }
    }
  }
  b->ctr_off.push_back((uint32_t)b->ctr_flags.size());

  // labels of the object itself
  const int64_t labels = ps.has_obj ? obj_get(d, obj_get(d, rk[RK_OBJECT], "metadata"), "labels") : -1;
  if (labels >= 0 && d.is((uint32_t)labels, JType::Obj)) {
    for (uint32_t kid : d.members((uint32_t)labels)) {
      if (!d.is(kid, JType::Str)) continue;
      b->lbl_key.push(d.key(kid));
      b->lbl_val.push(d.str(kid));
    }
  }
  b->lbl_off.push_back((uint32_t)b->lbl_key.n());
  b->n += 1;
}

std::string missing(const char* key) {
  return std::string("Failed to deserialize the JSON body into the target type: request: missing field `") + key + "`";
}
std::string bad_type(const char* key, const char* what) {
  return std::string("Failed to deserialize the JSON body into the target type: request.") + key + ": invalid type, expected " + what;
}

bool req_string(const JDoc& d, int64_t n, const char* key, std::string* err) {
  if (n < 0) {
    *err = missing(key);
    return false;
  }
  if (!d.is((uint32_t)n, JType::Str)) {
    *err = bad_type(key, "a string");
    return false;
  }
  return true;
}

bool req_object(const JDoc& d, int64_t n, const char* key, const std::string_view (&fields)[3], std::string* err) {
  if (n < 0) {
    *err = missing(key);
    return false;
  }
  if (!d.is((uint32_t)n, JType::Obj)) {
    *err = bad_type(key, "a struct");
    return false;
  }
  int64_t f[3];
  d.pick((uint32_t)n, fields, 3, f);
  for (int k = 0; k < 3; ++k)
    if (!req_string(d, f[k], fields[k].data(), err)) return false;
  return true;
}

// serde's derived structs (AdmissionReviewRequest, AdmissionRequest and its typed members, the
// raw review's envelope) refuse a repeated known field; `object` / `oldObject` / a raw request are
// serde_json::Value, where the last duplicate wins (JDoc::pick). `at`: the field path prefix.
bool no_dup(const JDoc& d, int64_t obj, const std::string_view* keys, int nkeys, const char* at, std::string* err) {
  if (obj < 0) return true;
  const int q = d.dup_field((uint32_t)obj, keys, nkeys);
  if (q < 0) return true;
  *err = std::string("Failed to deserialize the JSON body into the target type: ") + at + "duplicate field `" +
         std::string(keys[q]) + "`";
  return false;
}
// AdmissionRequest's fields (k8s admission/v1, policy-evaluator's AdmissionRequest) and those of its
// typed members
constexpr std::string_view kReqFields[] = {"uid",         "kind",        "resource", "subResource", "requestKind",
                                           "requestResource", "requestSubResource", "name", "namespace", "operation",
                                           "userInfo",    "object",      "oldObject", "dryRun",     "options"};
constexpr std::string_view kUserInfo[] = {"username", "uid", "groups", "extra"};
constexpr std::string_view kGvkF[] = {"group", "version", "kind"}, kGvrF[] = {"group", "version", "resource"};

bool opt_string(const JDoc& d, int64_t n, const char* key, std::string* err) {
  if (n < 0 || d.is((uint32_t)n, JType::Null) || d.is((uint32_t)n, JType::Str)) return true;
  *err = bad_type(key, "a string");
  return false;
}

}  // namespace

bool flatten_document(const char* doc, size_t len, int doc_kind, Batch* b, std::string* err) {
  thread_local JDoc d;
  std::string perr;
  if (!d.parse(doc, len, &perr)) {
    *err = "Failed to parse the request body as JSON: " + perr;
    return false;
  }
  if (!d.is(0, JType::Obj)) {
    *err = "Failed to deserialize the JSON body into the target type: invalid type, expected a struct";
    return false;
  }
  static constexpr std::string_view kTop[3] = {"request", "kind", "apiVersion"};
  int64_t top[3];
  d.pick(0, kTop, 3, top);
  const int64_t req = top[0];
  if (req < 0) {
    *err = "Failed to deserialize the JSON body into the target type: missing field `request`";
    return false;
  }
  if (!no_dup(d, 0, kTop, doc_kind == KW_DOC_RAW_REVIEW ? 1 : 3, "", err)) return false;
  int64_t rk[RK_N];
  if (d.is((uint32_t)req, JType::Obj)) {
    d.pick((uint32_t)req, kReqKeys, RK_N, rk);
  } else {
    for (int64_t& x : rk) x = -1;
  }
  if (doc_kind == KW_DOC_RAW_REVIEW) {
    flatten_request(d, req, rk, true, b);
    return true;
  }
  if (!no_dup(d, req, kReqFields, 15, "request: ", err)) return false;
  {
    static constexpr std::string_view kSub[4] = {"kind", "requestKind", "resource", "requestResource"};
    int64_t sub[4];
    d.pick((uint32_t)req, kSub, 4, sub);
    if (!no_dup(d, sub[0], kGvkF, 3, "request.kind: ", err) || !no_dup(d, sub[1], kGvkF, 3, "request.requestKind: ", err) ||
        !no_dup(d, sub[2], kGvrF, 3, "request.resource: ", err) ||
        !no_dup(d, sub[3], kGvrF, 3, "request.requestResource: ", err) ||
        !no_dup(d, rk[RK_USERINFO], kUserInfo, 4, "request.userInfo: ", err))
      return false;
  }
  if (!opt_string(d, top[1], "kind", err) || !opt_string(d, top[2], "apiVersion", err)) {
    err->replace(err->find("request."), 8, "");  // top-level fields
    return false;
  }
  if (!d.is((uint32_t)req, JType::Obj)) {
    *err = "Failed to deserialize the JSON body into the target type: request: invalid type, expected struct AdmissionRequest";
    return false;
  }
  static constexpr std::string_view kGvk[3] = {"group", "version", "kind"}, kGvr[3] = {"group", "version", "resource"};
  if (!req_string(d, rk[RK_UID], "uid", err)) return false;
  if (!req_object(d, rk[RK_KIND], "kind", kGvk, err)) return false;
  if (!req_object(d, rk[RK_RESOURCE], "resource", kGvr, err)) return false;
  if (!req_string(d, rk[RK_OPERATION], "operation", err)) return false;
  const int64_t ui = rk[RK_USERINFO];
  if (ui < 0 || !d.is((uint32_t)ui, JType::Obj)) {
    *err = missing("userInfo");
    return false;
  }
  if (!opt_string(d, rk[RK_NAMESPACE], "namespace", err) || !opt_string(d, rk[RK_NAME], "name", err) ||
      !opt_string(d, rk[RK_SUBRES], "subResource", err) || !opt_string(d, rk[RK_REQSUBRES], "requestSubResource", err))
    return false;
  flatten_request(d, req, rk, false, b);
  return true;
}

bool batch_from_soa(const kw_soa& s, Batch* b, std::string* err) {
  auto copy = [](const kw_strcol& c, StrCol* o) {
    o->off.assign(c.off, c.off + c.n + 1);
    uint32_t base = c.off[0];
    if (base != 0)
      for (auto& x : o->off) x -= base;
    o->bytes.reserve((size_t)(c.off[c.n] - base) + 32);  // room for the device padding (finalize)
    o->bytes.assign(c.bytes + base, c.bytes + c.off[c.n]);
  };
  uint64_t n = s.n_requests;
  if (!s.req_flags || !s.ctr_off || !s.lbl_off) {
    *err = "incomplete SoA";
    return false;
  }
  b->n = n;
  b->req_flags.assign(s.req_flags, s.req_flags + n);
  b->ctr_off.assign(s.ctr_off, s.ctr_off + n + 1);
  b->lbl_off.assign(s.lbl_off, s.lbl_off + n + 1);
  uint64_t nc = s.ctr_off[n] - s.ctr_off[0];
  b->ctr_flags.assign(s.ctr_flags + s.ctr_off[0], s.ctr_flags + s.ctr_off[n]);
  b->capadd_off.assign(s.capadd_off, s.capadd_off + nc + 1);
  b->capdrop_off.assign(s.capdrop_off, s.capdrop_off + nc + 1);
  if (s.ctr_off[0] != 0 || s.lbl_off[0] != 0 || s.capadd_off[0] != 0 || s.capdrop_off[0] != 0) {
    *err = "SoA offsets must start at 0";
    return false;
  }
  copy(s.uid, &b->uid);
  copy(s.ns, &b->ns);
  copy(s.op, &b->op);
  copy(s.kind, &b->kind);
  b->rkind.clear();
  for (uint64_t i = 0; i < n; ++i) b->rkind.push("");  // not part of kw_soa
  copy(s.ctr_name, &b->ctr_name);
  copy(s.ctr_image, &b->ctr_image);
  copy(s.ctr_apparmor, &b->ctr_aa);
  copy(s.cap_add, &b->cap_add);
  copy(s.cap_drop, &b->cap_drop);
  copy(s.lbl_key, &b->lbl_key);
  copy(s.lbl_val, &b->lbl_val);
  // consistency: every per-entity column must match its table size
  if (b->uid.n() != n || b->ns.n() != n || b->op.n() != n || b->kind.n() != n || b->ctr_name.n() != nc ||
      b->ctr_image.n() != nc || b->ctr_aa.n() != nc || b->cap_add.n() != b->capadd_off.back() ||
      b->cap_drop.n() != b->capdrop_off.back() || b->lbl_key.n() != b->lbl_off.back() ||
      b->lbl_val.n() != b->lbl_off.back()) {
    *err = "SoA column sizes are inconsistent";
    return false;
  }
  return true;
}

}  // namespace kw
