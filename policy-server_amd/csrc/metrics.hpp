// metrics.hpp — batched policy-evaluation metrics, kept off the device path.
//
// Reference: src/metrics.rs:49-140 (the attribute sets PolicyEvaluation, RawPolicyEvaluation,
// PolicyInitializationError), src/metrics/policy_evaluations_total.rs (counter
// kubewarden_policy_evaluations_total), src/metrics/policy_evaluations_latency.rs (u64 histogram
// kubewarden_policy_evaluation_latency_milliseconds) and the recording sites in service::evaluate
// (src/api/service.rs:40-71 namespace bypass, :78-91 initialization error, :118-150 evaluated).
// The reference records one data point per (request, policy) call through OpenTelemetry; here a
// validate pass records all its rows under one lock, from the verdict words the host already holds.
// Export is Prometheus text (kwhost GET /metrics) instead of OTLP/gRPC: the attribute keys, their
// order and the metric names are the reference's.
#pragma once
#include <cstdint>
#include <map>
#include <mutex>
#include <string>

#include "batch.hpp"
#include "env.hpp"

namespace kw {

class Metrics {
 public:
  // One evaluated (row, policy) of a pass: `verdict` is the final verdict word of kw_validate_*,
  // `latency_ms` the time from the request's arrival to its verdict (service.rs:37, :97).
  void record(const Env& env, const Batch& b, uint64_t row, int32_t policy, uint32_t verdict, int origin,
              uint64_t latency_ms);
  std::string render() const;  // Prometheus text exposition format 0.0.4
  void reset();

  // OpenTelemetry SDK default explicit bucket boundaries (milliseconds)
  static constexpr uint64_t kBounds[] = {0, 5, 10, 25, 50, 75, 100, 250, 500, 750, 1000, 2500, 5000, 7500, 10000};
  static constexpr size_t kNB = sizeof(kBounds) / sizeof(kBounds[0]);

 private:
  struct Hist {
    uint64_t bucket[kNB + 1] = {};  // per-bucket counts; the last is (10000, +inf)
    uint64_t sum = 0, count = 0;
  };
  mutable std::mutex mu_;
  std::map<std::string, uint64_t> total_;  // label set -> kubewarden_policy_evaluations_total
  std::map<std::string, Hist> latency_;    // label set -> latency histogram
};

}  // namespace kw
