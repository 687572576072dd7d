// metrics.cpp — batched policy-evaluation metrics (metrics.hpp).
#include "metrics.hpp"

#include <algorithm>

namespace kw {

constexpr uint64_t Metrics::kBounds[];

namespace {

// Prometheus label value escaping: backslash, double quote, newline.
void put_label(std::string* o, bool first, const char* key, std::string_view v) {
  if (!first) o->push_back(',');
  o->append(key);
  o->append("=\"");
  for (char c : v) {
    if (c == '\\') o->append("\\\\");
    else if (c == '"') o->append("\\\"");
    else if (c == '\n') o->append("\\n");
    else o->push_back(c);
  }
  o->push_back('"');
}

}  // namespace

void Metrics::record(const Env& env, const Batch& b, uint64_t row, int32_t policy, uint32_t v, int origin,
                     uint64_t latency_ms) {
  if (policy < 0 || (size_t)policy >= env.nvisible || row >= b.n) return;
  const PolicyRec& P = env.pol[(size_t)policy];
  const bool raw = (b.req_flags[row] & KW_REQ_RAW) != 0;
  const uint32_t fst = (v & KW_F_STATUS_MASK) >> KW_F_STATUS_SHIFT;
  std::string key;
  if (fst == KW_FST_INIT_ERROR) {
    // PolicyInitializationError (metrics.rs:125-140; service.rs:78-84): the counter only
    put_label(&key, true, "policy_name", P.id);
    put_label(&key, false, "initialization_error", P.init_message);
    std::lock_guard<std::mutex> g(mu_);
    ++total_[key];
    return;
  }
  const char* mode = P.mode == KW_MODE_MONITOR ? "monitor" : "protect";  // config.rs:296-302
  bool accepted, mutated;
  int error_code = -1;
  if (v & KW_BYPASS) {  // service.rs:45-58: accepted, not mutated, no error code
    accepted = true;
    mutated = false;
  } else {  // the vanilla response (service.rs:97-105)
    accepted = (v & KW_V_ALLOWED) != 0;
    mutated = (v & KW_V_MUTATED) != 0;
    if (KW_REASON(v) == KW_R_GROUP_EXPR) error_code = 500;  // reject(uid, rhai error, 500)
  }
  put_label(&key, true, "policy_name", P.id);
  put_label(&key, false, "policy_mode", mode);
  if (raw) {  // RawPolicyEvaluation (metrics.rs:96-123)
    put_label(&key, false, "accepted", accepted ? "true" : "false");
    put_label(&key, false, "mutated", mutated ? "true" : "false");
  } else {  // PolicyEvaluation (metrics.rs:49-94)
    put_label(&key, false, "resource_kind", row < b.rkind.n() ? b.rkind.at(row) : std::string_view());
    put_label(&key, false, "resource_request_operation", b.op.at(row));
    put_label(&key, false, "accepted", accepted ? "true" : "false");
    put_label(&key, false, "mutated", mutated ? "true" : "false");
    put_label(&key, false, "request_origin", origin == KW_ORIGIN_AUDIT ? "audit" : "validate");
    if (b.req_flags[row] & KW_REQ_HAS_NAMESPACE) put_label(&key, false, "resource_namespace", b.ns.at(row));
  }
  if (error_code >= 0) put_label(&key, false, "error_code", std::to_string(error_code));
  std::lock_guard<std::mutex> g(mu_);
  ++total_[key];
  Hist& h = latency_[key];
  const size_t k = std::lower_bound(kBounds, kBounds + kNB, latency_ms) - kBounds;  // first bound >= latency
  ++h.bucket[k];
  h.sum += latency_ms;
  ++h.count;
}

std::string Metrics::render() const {
  std::lock_guard<std::mutex> g(mu_);
  std::string o;
  o.append("# TYPE kubewarden_policy_evaluations_total counter\n");
  for (const auto& [k, n] : total_) {
    o.append("kubewarden_policy_evaluations_total{").append(k).append("} ").append(std::to_string(n)).push_back('\n');
  }
  o.append("# TYPE kubewarden_policy_evaluation_latency_milliseconds histogram\n");
  for (const auto& [k, h] : latency_) {
    uint64_t cum = 0;
    for (size_t i = 0; i <= kNB; ++i) {
      cum += h.bucket[i];
      o.append("kubewarden_policy_evaluation_latency_milliseconds_bucket{").append(k).append(",le=\"");
      o.append(i < kNB ? std::to_string(kBounds[i]) : std::string("+Inf")).append("\"} ");
      o.append(std::to_string(cum)).push_back('\n');
    }
    o.append("kubewarden_policy_evaluation_latency_milliseconds_sum{").append(k).append("} ");
    o.append(std::to_string(h.sum)).push_back('\n');
    o.append("kubewarden_policy_evaluation_latency_milliseconds_count{").append(k).append("} ");
    o.append(std::to_string(h.count)).push_back('\n');
  }
  return o;
}

void Metrics::reset() {
  std::lock_guard<std::mutex> g(mu_);
  total_.clear();
  latency_.clear();
}

}  // namespace kw
