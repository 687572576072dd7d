// kwhost — HTTP front of the admission engine: /validate, /audit and /validate_raw/{policy_id}
// served from micro-batches on the GPU.
//
// Reference: the axum router (src/lib.rs:206-225), validate_handler / audit_handler /
// validate_raw_handler (src/api/handlers.rs:69-174), the JsonExtractor rejection (handlers.rs:29-39,
// api_error.rs:7-30), handle_evaluation_error (handlers.rs:321-342) and the per-request
// semaphore + spawn_blocking (acquire_semaphore_and_evaluate, handlers.rs:256-286), which this
// server replaces with a micro-batcher: connection threads park their request in a queue; one
// batcher thread takes up to --max-batch requests (waiting at most --max-wait-us after the first)
// whenever one of --workers pipeline workers is idle, and hands the batch to it. A worker flattens
// the batch with kw_batch_from_json, uploads it on its own HIP stream (pooled device memory, pinned
// staging: no allocation per batch), evaluates it with one kw_validate_rows call per (document kind,
// origin) and hands each connection its formatted AdmissionReview; with two or more workers the
// flattening and formatting of one batch overlap the GPU work of the next.
//
// Status mapping (reference behaviour):
//   body not JSON                        400  "Failed to parse the request body as JSON: ..."
//   JSON not an AdmissionReview / Raw    422  "Failed to deserialize the JSON body into the target type: ..."
//   body over --max-body-bytes (2 MiB)   413  "Failed to buffer the request body: length limit exceeded"
//                                             (axum's DefaultBodyLimit; the connection is then closed)
//   Content-Type not application/json    415  "Expected request with `Content-Type: application/json`"
//   /validate rejections are {"message", "status"} JSON (JsonExtractor); /audit and /validate_raw
//   use axum's plain-text rejection body.
//   unknown policy                       404  {"message":"unknown policy: <id>","status":404}
//   any other evaluation error           500  {"message":"Something went wrong","status":500}
//   GET /readiness                       200  (empty)
//   GET /metrics                         200  Prometheus text: kubewarden_policy_evaluations_total and
//                                             kubewarden_policy_evaluation_latency_milliseconds
//                                             (src/metrics.rs; the reference exports them over OTLP)
//   unknown route                        404  (empty)
//
// Usage: kwhost --policies policies.yml [--addr 127.0.0.1] [--port 3000] [--device 0 | --devices 0,1,..]
//   [--max-batch 512] [--max-wait-us 200] [--workers 4] [--max-body-bytes 2097152]
//   [--always-accept-admission-reviews-on-namespace NS] [--continue-on-errors] [--no-device]
// --devices (r06) shards the serving front over several GPUs: the environment is compiled once, on
// the first device, and its blob deserialized onto every other one (the same path as the batch
// shards' RCCL broadcast, kw_env_serialize / kw_env_deserialize: each copy re-derives its host
// records and byte-compares the tables); pipeline worker k runs on devices[k % n] with that device's
// environment, so the batcher's idle-worker hand-off balances the devices. A device may be listed
// twice (two environments, one GPU: the multi-device path on a one-GPU box).
// --policies is the reference's policies.yml (read with the native YAML reader, config.rs:449-453;
// a file whose first character is '{' is read as JSON). --no-device serves the HTTP layer without
// device tables: every evaluation then fails with 500 (used by the CPU test suite for routing and
// error mapping; never a CPU fallback).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <deque>
#include <fstream>
#include <mutex>
#include <string_view>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kwgpu.h"

namespace {

struct Opts {
  std::string policies, addr = "127.0.0.1", always_ns;
  int port = 3000, device = 0, max_batch = 512, max_wait_us = 200, workers = 4;
  size_t max_body = 2u << 20;  // axum DefaultBodyLimit (2 MiB)
  bool continue_on_errors = false, no_device = false;
  std::vector<int> devices;  // --devices (default: {device})
  int stats_ms = 0;  // --stats-ms N: a JSON line of cumulative stage times on stderr every N ms
};

// Where a worker's time goes (--stats-ms): cumulative nanoseconds per stage over all batches.
struct StageStats {
  static constexpr size_t kMaxDev = 16;
  std::atomic<uint64_t> batches{0}, rows{0}, wait_ns{0}, flatten_ns{0}, gpu_ns{0}, format_ns{0}, handoff_ns{0};
  std::atomic<uint64_t> device_batches[kMaxDev] = {};  // batches per entry of --devices
};
static uint64_t ns_since(std::chrono::steady_clock::time_point t) {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count();
}

enum Route { R_VALIDATE, R_AUDIT, R_RAW };

struct Reply {
  int status = 500;
  std::string body, ctype = "application/json";
};

// One parked request: filled by its connection thread, answered by the batcher.
struct Job {
  Route route;
  std::string policy, body;
  Reply reply;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();  // arrival (service.rs:37)
  bool done = false;
  std::mutex m;
  std::condition_variable cv;
  void finish(Reply r) {
    std::lock_guard<std::mutex> g(m);
    reply = std::move(r);
    done = true;
    cv.notify_one();
  }
};

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof(b), "\\u%04x", c);
          o += b;
        } else {
          o += (char)c;
        }
    }
  }
  return o;
}

Reply api_error(int status, const std::string& msg) {  // ApiError::into_response (api_error.rs:22-30)
  Reply r;
  r.status = status;
  r.body = "{\"message\":\"" + json_escape(msg) + "\",\"status\":" + std::to_string(status) + "}";
  return r;
}

// Extractor rejection: JsonExtractor (validate) answers ApiError JSON, axum::Json (audit, raw) the
// rejection's plain body text.
Reply rejection(Route route, int status, const std::string& msg) {
  if (route == R_VALIDATE) return api_error(status, msg);
  Reply r;
  r.status = status;
  r.body = msg;
  r.ctype = "text/plain; charset=utf-8";
  return r;
}

Reply evaluation_error(int code, const std::string& msg) {  // handle_evaluation_error (handlers.rs:321-342)
  if (code == KW_E_NOT_FOUND) return api_error(404, msg);
  return api_error(500, "Something went wrong");
}

class Server {
 public:
  Server(const Opts& o, std::vector<kw_env*> envs) : o_(o), envs_(std::move(envs)) {}
  size_t max_body() const { return o_.max_body; }

  void submit(Job* j) {
    {
      std::lock_guard<std::mutex> g(qm_);
      q_.push_back(j);
    }
    qcv_.notify_one();
  }

  // The batcher: once a worker is idle, take up to max_batch jobs (waiting max_wait_us after the
  // first) and hand them to it.
  void batcher() {
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(wm_);
        wcv_.wait(lk, [&] { return idle_ > 0; });
        --idle_;
      }
      std::vector<Job*> jobs;
      {
        std::unique_lock<std::mutex> lk(qm_);
        qcv_.wait(lk, [&] { return !q_.empty(); });
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(o_.max_wait_us);
        qcv_.wait_until(lk, deadline, [&] { return (int)q_.size() >= o_.max_batch; });
        while (!q_.empty() && (int)jobs.size() < o_.max_batch) {
          jobs.push_back(q_.front());
          q_.pop_front();
        }
      }
      {
        std::lock_guard<std::mutex> g(wm_);
        work_.push_back(std::move(jobs));
      }
      wcv_.notify_all();
    }
  }

  // A pipeline worker: its own device (o_.devices[k % n]) and stream; one batch at a time.
  void worker(int k) {
    const size_t d = (size_t)k % o_.devices.size();
    const int device = o_.devices[d];
    kw_env* env = envs_[d];
    void* stream = nullptr;
    if (!o_.no_device && kw_stream_create(device, &stream) != KW_OK) stream = nullptr;
    for (;;) {
      std::vector<Job*> jobs;
      {
        std::unique_lock<std::mutex> lk(wm_);
        wcv_.wait(lk, [&] { return !work_.empty(); });
        jobs = std::move(work_.front());
        work_.pop_front();
      }
      {
        uint64_t w = 0;
        for (Job* j : jobs) w += ns_since(j->t0);
        stats_.wait_ns += w;  // arrival -> a worker holds the batch (summed over requests)
        stats_.batches += 1;
        stats_.rows += jobs.size();
        stats_.device_batches[d % StageStats::kMaxDev] += 1;
      }
      // partition first: a job belongs to its connection thread again once it is answered
      std::vector<Job*> part[3];
      for (Job* j : jobs) part[j->route].push_back(j);
      for (Route r : {R_VALIDATE, R_AUDIT, R_RAW})
        if (!part[r].empty()) run(r, part[r], env, device, stream);
      {
        std::lock_guard<std::mutex> g(wm_);
        ++idle_;
      }
      wcv_.notify_all();
    }
  }

  void start() {
    idle_ = std::max(1, o_.workers);
    for (int k = 0; k < std::max(1, o_.workers); ++k) std::thread(&Server::worker, this, k).detach();
    std::thread(&Server::batcher, this).detach();
  }

 private:
  // One kw_validate_rows pass over the jobs of one route. A group's members run as extra rows of
  // the same document (their verdicts give the causes of a rejected group).
  void run(Route route, std::vector<Job*> jobs, kw_env* env_, int device, void* stream) {
    const int kind = route == R_RAW ? KW_DOC_RAW_REVIEW : KW_DOC_ADMISSION_REVIEW;
    const int origin = route == R_AUDIT ? KW_ORIGIN_AUDIT : KW_ORIGIN_VALIDATE;
    // 1. the extractor: bodies that are not a request of this route's type are answered first
    //    (the handler's extractor runs before the policy lookup)
    kw_batch* b = nullptr;
    char err[1024] = {0};
    const auto t_flat = std::chrono::steady_clock::now();
    for (;;) {
      if (jobs.empty()) return;
      std::vector<const char*> docs;
      std::vector<size_t> lens;
      for (Job* j : jobs) {
        docs.push_back(j->body.data());
        lens.push_back(j->body.size());
      }
      int64_t bad = -1;
      const int rc = kw_batch_from_json(docs.data(), lens.data(), docs.size(), kind, &b, &bad, err, sizeof(err));
      if (rc == KW_OK) break;
      if (rc != KW_E_PAYLOAD || bad < 0 || bad >= (int64_t)jobs.size()) {
        for (Job* j : jobs) j->finish(evaluation_error(rc, err));
        return;
      }
      const std::string msg(err);
      const int status = msg.rfind("Failed to parse", 0) == 0 ? 400 : 422;  // JsonSyntaxError vs JsonDataError
      jobs[(size_t)bad]->finish(rejection(route, status, msg));
      jobs.erase(jobs.begin() + bad);
    }
    // 2. policy lookup (service.rs:37 PolicyID parse, PolicyNotFound -> 404)
    struct Row {
      Job* job;
      int32_t policy;
      uint32_t first, nmem;
    };
    std::vector<Row> rows;
    std::vector<const char*> docs;
    std::vector<size_t> lens;
    std::vector<int32_t> row_policy;
    bool regroup = false;  // some job failed its lookup or is a group: the batch is rebuilt from `docs`
    for (Job* j : jobs) {
      int32_t idx = -1;
      const int rc = kw_env_lookup(env_, j->policy.data(), j->policy.size(), &idx);
      if (rc != KW_OK) {
        j->finish(evaluation_error(rc, rc == KW_E_NOT_FOUND ? "unknown policy: " + j->policy : ""));
        regroup = true;
        continue;
      }
      int32_t mem[256];
      const int nm = kw_env_is_group(env_, idx) ? kw_env_group_members(env_, idx, mem, 256) : 0;
      regroup = regroup || nm > 0;
      rows.push_back({j, idx, (uint32_t)row_policy.size(), (uint32_t)(nm > 0 ? nm : 0)});
      docs.push_back(j->body.data());
      lens.push_back(j->body.size());
      row_policy.push_back(idx);
      for (int k = 0; k < nm; ++k) {  // a group's members run as extra rows of the same document
        docs.push_back(j->body.data());
        lens.push_back(j->body.size());
        row_policy.push_back(mem[k]);
      }
    }
    int rc = KW_OK;
    if (regroup) {
      kw_batch_destroy(b);
      b = nullptr;
      if (rows.empty()) return;
      int64_t bad = -1;
      rc = kw_batch_from_json(docs.data(), lens.data(), docs.size(), kind, &b, &bad, err, sizeof(err));
    }
    // 3. upload, evaluate, read back
    stats_.flatten_ns += ns_since(t_flat);
    const auto t_gpu = std::chrono::steady_clock::now();
    if (rc == KW_OK && o_.no_device) rc = KW_E_DEVICE;
    if (rc == KW_OK) rc = stream ? kw_batch_to_device_async(b, device, stream) : kw_batch_to_device(b, device);
    if (rc == KW_OK) rc = kw_validate_rows(env_, b, row_policy.data(), origin, stream);
    std::vector<uint32_t> v(row_policy.size());
    if (rc == KW_OK) rc = kw_batch_verdicts(b, v.data(), v.size());
    if (rc != KW_OK) {
      for (Row& r : rows) r.job->finish(evaluation_error(rc, err));
      if (b) kw_batch_destroy(b);
      return;
    }
    // metrics of the addressed policies (service.rs:40-150), latency = arrival -> verdict
    if (metrics_) {
      const auto now = std::chrono::steady_clock::now();
      std::vector<uint64_t> mrow, mlat;
      std::vector<int32_t> mpol;
      std::vector<uint32_t> mv;
      for (Row& r : rows) {
        mrow.push_back(r.first);
        mpol.push_back(r.policy);
        mv.push_back(v[r.first]);
        mlat.push_back((uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(now - r.job->t0).count());
      }
      kw_metrics_record(metrics_, envs_[0], b, mrow.data(), mpol.data(), mv.data(), mlat.data(), mrow.size(), origin);
    }
    // 4. service epilogue + response envelope (AdmissionReviewResponse / RawReviewResponse)
    stats_.gpu_ns += ns_since(t_gpu);
    const auto t_fmt = std::chrono::steady_clock::now();
    std::vector<char> buf(4096);
    uint64_t handoff = 0;
    for (Row& r : rows) {
      size_t need = 0;
      const uint32_t* mv = r.nmem ? v.data() + r.first + 1 : nullptr;
      const std::string& body = r.job->body;  // an accepted mutation's patch is built from the document
      auto fmt = [&] {
        return kw_format_response_doc(env_, b, r.first, r.policy, v[r.first], mv, body.data(), body.size(), kind,
                                      buf.data(), buf.size(), &need);
      };
      int frc = fmt();
      if (frc == KW_E_NOSPACE) {
        buf.resize(need + 1);
        frc = fmt();
      }
      if (frc != KW_OK) {
        r.job->finish(evaluation_error(frc, buf.data()));
        continue;
      }
      Reply rep;
      rep.status = 200;
      const std::string resp(buf.data(), strnlen(buf.data(), buf.size()));  // need counts the NUL
      rep.body = route == R_RAW ? "{\"response\":" + resp + "}"
                                : "{\"kind\":\"AdmissionReview\",\"apiVersion\":\"admission.k8s.io/v1\",\"response\":" + resp + "}";
      const auto t_h = std::chrono::steady_clock::now();
      r.job->finish(std::move(rep));  // wakes the connection thread (a futex wake per request)
      handoff += ns_since(t_h);
    }
    kw_batch_destroy(b);
    stats_.format_ns += ns_since(t_fmt) - handoff;
    stats_.handoff_ns += handoff;
  }

 public:
  StageStats stats_;
  void stats_loop() {
    for (;;) {
      std::this_thread::sleep_for(std::chrono::milliseconds(o_.stats_ms));
      const uint64_t rows = stats_.rows, batches = stats_.batches;
      std::string per_dev;
      for (size_t d = 0; d < o_.devices.size() && d < StageStats::kMaxDev; ++d)
        per_dev += (d ? ", " : "") + std::to_string((unsigned long long)stats_.device_batches[d]);
      fprintf(stderr,
              "{\"kwhost_stats\": {\"batches\": %llu, \"rows\": %llu, \"mean_batch\": %.1f, \"wait_s_per_request\": %.3g, "
              "\"worker_s\": {\"flatten\": %.4f, \"gpu_upload_validate_readback\": %.4f, \"format\": %.4f, \"handoff\": %.4f}, "
              "\"device_batches\": [%s]}}\n",
              (unsigned long long)batches, (unsigned long long)rows, batches ? (double)rows / batches : 0.0,
              rows ? stats_.wait_ns / 1e9 / rows : 0.0, stats_.flatten_ns / 1e9, stats_.gpu_ns / 1e9, stats_.format_ns / 1e9,
              stats_.handoff_ns / 1e9, per_dev.c_str());
      fflush(stderr);
    }
  }
 private:
  const Opts& o_;
  std::vector<kw_env*> envs_;  // per entry of o_.devices (same policies, same indices)
 public:
  kw_metrics* metrics_ = nullptr;  // GET /metrics (owned by main)
 private:
  std::mutex qm_;
  std::condition_variable qcv_;
  std::deque<Job*> q_;
  std::mutex wm_;  // workers: idle count and the batches handed over
  std::condition_variable wcv_;
  int idle_ = 0;
  std::deque<std::vector<Job*>> work_;
};

// ---- HTTP/1.1 (Content-Length and chunked bodies, keep-alive)
struct Conn {
  int fd;
  std::string in;
  bool read_more() {
    char b[65536];
    const ssize_t n = recv(fd, b, sizeof(b), 0);
    if (n <= 0) return false;
    in.append(b, (size_t)n);
    return true;
  }
  bool send_all(const std::string& s) {
    size_t o = 0;
    while (o < s.size()) {
      const ssize_t n = send(fd, s.data() + o, s.size() - o, MSG_NOSIGNAL);
      if (n <= 0) return false;
      o += (size_t)n;
    }
    return true;
  }
};

std::string lower(std::string s) {
  for (char& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t"), e = s.find_last_not_of(" \t\r");
  return a == std::string::npos ? std::string() : s.substr(a, e - a + 1);
}

bool percent_decode(const std::string& s, std::string* out) {  // axum Path extractor
  out->clear();
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%') {
      if (i + 2 >= s.size() || !isxdigit((unsigned char)s[i + 1]) || !isxdigit((unsigned char)s[i + 2])) return false;
      *out += (char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16);
      i += 2;
    } else {
      *out += s[i];
    }
  }
  return true;
}

const char* reason(int s) {
  switch (s) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    default: return "Internal Server Error";
  }
}

void serve(Server* srv, int fd) {
  Conn c{fd, {}};
  for (;;) {
    size_t he;
    while ((he = c.in.find("\r\n\r\n")) == std::string::npos) {
      if (c.in.size() > (1u << 20) || !c.read_more()) {
        close(fd);
        return;
      }
    }
    // request line and headers, parsed in place (no stream objects per request)
    const std::string_view head(c.in.data(), he);
    size_t le = head.find("\r\n");
    const std::string_view rline = head.substr(0, le);
    const size_t s1 = rline.find(' '), s2 = s1 == std::string_view::npos ? s1 : rline.find(' ', s1 + 1);
    const std::string method(rline.substr(0, s1));
    const std::string target(s1 == std::string_view::npos ? std::string_view() : rline.substr(s1 + 1, s2 - s1 - 1));
    const std::string version(s2 == std::string_view::npos ? std::string_view() : rline.substr(s2 + 1));
    std::string ctype;
    long long clen = -1;
    bool chunked = false, keep = version != "HTTP/1.0";
    for (size_t at = le == std::string_view::npos ? head.size() : le + 2; at < head.size();) {
      size_t end = head.find("\r\n", at);
      if (end == std::string_view::npos) end = head.size();
      const std::string_view line = head.substr(at, end - at);
      at = end + 2;
      const size_t colon = line.find(':');
      if (colon == std::string_view::npos) continue;
      const std::string k = lower(trim(std::string(line.substr(0, colon)))), v = trim(std::string(line.substr(colon + 1)));
      if (k == "content-length") clen = atoll(v.c_str());
      else if (k == "content-type") ctype = lower(v);
      else if (k == "transfer-encoding") chunked = lower(v).find("chunked") != std::string::npos;
      else if (k == "connection") keep = lower(v) != "close" && (keep || lower(v) == "keep-alive");
    }
    c.in.erase(0, he + 4);
    std::string body;
    bool too_large = false;
    size_t drained = 0;
    constexpr size_t kDrainCap = (size_t)64 << 20;  // an oversized body is drained up to 64 MiB, else the connection drops
    if (chunked) {
      for (;;) {
        size_t le;
        while ((le = c.in.find("\r\n")) == std::string::npos) {
          if (c.in.size() > 64 || !c.read_more()) return (void)close(fd);
        }
        const std::string hex = c.in.substr(0, c.in.find_first_of(";\r"));
        if (hex.empty() || hex.size() > 8 || hex.find_first_not_of("0123456789abcdefABCDEF") != std::string::npos)
          return (void)close(fd);
        const size_t n = strtoul(hex.c_str(), nullptr, 16);  // < 2^32: no overflow below
        if (body.size() + n > srv->max_body()) too_large = true;
        if (too_large && drained + n > kDrainCap) return (void)close(fd);
        while (c.in.size() < le + 2 + n + 2)
          if (!c.read_more()) return (void)close(fd);
        if (too_large) drained += n;  // past the limit: read and discard, then answer 413
        else body.append(c.in, le + 2, n);
        c.in.erase(0, le + 2 + n + 2);
        if (n == 0) break;
      }
      if (too_large) body.clear();
    } else if (clen > 0) {
      if ((unsigned long long)clen > srv->max_body()) {
        too_large = true;
        if ((unsigned long long)clen > kDrainCap) return (void)close(fd);
        size_t left = (size_t)clen;  // read and discard the body so the client sees the answer
        while (left > 0) {
          if (c.in.empty() && !c.read_more()) return (void)close(fd);
          const size_t k = std::min(left, c.in.size());
          c.in.erase(0, k);
          left -= k;
        }
      } else {
        while ((long long)c.in.size() < clen)
          if (!c.read_more()) return (void)close(fd);
        body = c.in.substr(0, (size_t)clen);
        c.in.erase(0, (size_t)clen);
      }
    }
    // routing (src/lib.rs:206-225)
    Reply rep;
    const std::string path = target.substr(0, target.find('?'));
    Route route = R_VALIDATE;
    std::string rest;
    bool known = true;
    if (path.rfind("/validate/", 0) == 0) {
      route = R_VALIDATE;
      rest = path.substr(10);
    } else if (path.rfind("/audit/", 0) == 0) {
      route = R_AUDIT;
      rest = path.substr(7);
    } else if (path.rfind("/validate_raw/", 0) == 0) {
      route = R_RAW;
      rest = path.substr(14);
    } else {
      known = false;
    }
    std::string policy;
    if (path == "/readiness") {
      rep.status = method == "GET" ? 200 : 405;
      rep.ctype.clear();
    } else if (path == "/metrics") {  // the reference pushes OTLP; kwhost exposes the same series
      rep.status = method == "GET" ? 200 : 405;
      rep.ctype.clear();
      if (method == "GET" && srv->metrics_) {
        size_t need = 0;
        kw_metrics_render(srv->metrics_, nullptr, 0, &need);
        std::vector<char> mb(need + 1);
        kw_metrics_render(srv->metrics_, mb.data(), mb.size(), &need);
        rep.body.assign(mb.data(), strnlen(mb.data(), mb.size()));
        rep.ctype = "text/plain; version=0.0.4";
      }
    } else if (!known || rest.empty() || rest.find('/') != std::string::npos || !percent_decode(rest, &policy)) {
      rep.status = 404;
      rep.ctype.clear();
    } else if (method != "POST") {
      rep.status = 405;
      rep.ctype.clear();
    } else if (!(ctype.rfind("application/json", 0) == 0 ||
                 (ctype.rfind("application/", 0) == 0 && ctype.find("+json") != std::string::npos))) {
      rep = rejection(route, 415, "Expected request with `Content-Type: application/json`");
    } else if (too_large) {  // DefaultBodyLimit: the body is not read, the connection closes after the answer
      rep = rejection(route, 413, "Failed to buffer the request body: length limit exceeded");
      keep = false;
    } else {
      Job j;
      j.route = route;
      j.policy = std::move(policy);
      j.body = std::move(body);
      srv->submit(&j);
      std::unique_lock<std::mutex> lk(j.m);
      j.cv.wait(lk, [&] { return j.done; });
      rep = std::move(j.reply);
    }
    std::string out = "HTTP/1.1 " + std::to_string(rep.status) + " " + reason(rep.status) + "\r\n";
    if (!rep.ctype.empty()) out += "content-type: " + rep.ctype + "\r\n";
    out += "content-length: " + std::to_string(rep.body.size()) + "\r\n";
    if (!keep) out += "connection: close\r\n";
    out += "\r\n" + rep.body;
    if (too_large) keep = false;
    if (!c.send_all(out) || !keep) {
      close(fd);
      return;
    }
  }
}

int usage() {
  fprintf(stderr,
          "usage: kwhost --policies policies.yml [--addr A] [--port P] [--device D | --devices D0,D1,..] [--max-batch N]\n"
          "              [--max-wait-us T] [--workers W] [--max-body-bytes B] [--stats-ms N]\n"
          "              [--always-accept-admission-reviews-on-namespace NS] [--continue-on-errors] [--no-device]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
    const char* v = nullptr;
    if (a == "--policies" && (v = val())) o.policies = v;
    else if (a == "--addr" && (v = val())) o.addr = v;
    else if (a == "--port" && (v = val())) o.port = atoi(v);
    else if (a == "--device" && (v = val())) o.device = atoi(v);
    else if (a == "--devices" && (v = val())) {
      o.devices.clear();
      for (const char* c = v; *c;) {
        o.devices.push_back(atoi(c));
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
      }
    }
    else if (a == "--max-batch" && (v = val())) o.max_batch = std::max(1, atoi(v));
    else if (a == "--max-wait-us" && (v = val())) o.max_wait_us = std::max(0, atoi(v));
    else if (a == "--workers" && (v = val())) o.workers = std::max(1, atoi(v));
    else if (a == "--stats-ms" && (v = val())) o.stats_ms = std::max(0, atoi(v));
    else if (a == "--max-body-bytes" && (v = val())) o.max_body = (size_t)std::max(0ll, atoll(v));
    else if (a == "--always-accept-admission-reviews-on-namespace" && (v = val())) o.always_ns = v;
    else if (a == "--continue-on-errors") o.continue_on_errors = true;
    else if (a == "--no-device") o.no_device = true;
    else return usage();
  }
  if (o.policies.empty()) return usage();
  if (o.devices.empty()) o.devices.push_back(o.device);
  if (o.devices.size() > StageStats::kMaxDev) return usage();
  o.device = o.devices[0];
  std::ifstream f(o.policies, std::ios::binary);
  if (!f) {
    fprintf(stderr, "kwhost: cannot read %s\n", o.policies.c_str());
    return 1;
  }
  const std::string doc((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  kw_env_options eo;
  memset(&eo, 0, sizeof(eo));
  eo.continue_on_errors = o.continue_on_errors ? 1 : 0;
  eo.always_accept_namespace = o.always_ns.empty() ? nullptr : o.always_ns.c_str();
  eo.device = o.no_device ? -1 : o.device;
  kw_env* env = nullptr;
  char err[2048] = {0};
  const size_t first = doc.find_first_not_of(" \t\r\n");
  const bool is_json = first != std::string::npos && doc[first] == '{';
  if (int rc = is_json ? kw_env_build(doc.data(), doc.size(), &eo, &env, err, sizeof(err))
                       : kw_env_build_yaml(doc.data(), doc.size(), &eo, &env, err, sizeof(err))) {
    fprintf(stderr, "kwhost: %s (code %d)\n", err, rc);
    return 1;
  }
  // the other devices' environments: the first one's blob, deserialized there
  std::vector<kw_env*> envs = {env};
  if (o.devices.size() > 1 && !o.no_device) {
    size_t need = 0;
    kw_env_serialize(env, nullptr, 0, &need);
    std::vector<char> blob(need);
    if (int rc = kw_env_serialize(env, blob.data(), blob.size(), &need)) {
      fprintf(stderr, "kwhost: cannot serialize the environment (code %d)\n", rc);
      return 1;
    }
    for (size_t d = 1; d < o.devices.size(); ++d) {
      kw_env* e = nullptr;
      if (int rc = kw_env_deserialize(blob.data(), blob.size(), o.devices[d], &e, err, sizeof(err))) {
        fprintf(stderr, "kwhost: device %d: %s (code %d)\n", o.devices[d], err, rc);
        return 1;
      }
      envs.push_back(e);
    }
  } else {
    while (envs.size() < o.devices.size()) envs.push_back(env);
  }
  const int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa;
  memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)o.port);
  if (inet_pton(AF_INET, o.addr.c_str(), &sa.sin_addr) != 1 || bind(ls, (sockaddr*)&sa, sizeof(sa)) != 0 ||
      listen(ls, 1024) != 0) {
    fprintf(stderr, "kwhost: cannot listen on %s:%d: %s\n", o.addr.c_str(), o.port, strerror(errno));
    return 1;
  }
  signal(SIGPIPE, SIG_IGN);
  Server srv(o, envs);
  srv.metrics_ = kw_metrics_create();
  srv.start();
  if (o.stats_ms > 0) std::thread(&Server::stats_loop, &srv).detach();
  fprintf(stderr, "kwhost: %d policies on %zu device pipeline(s), listening on %s:%d\n", kw_env_policy_count(env),
          o.devices.size(), o.addr.c_str(), o.port);
  for (;;) {
    const int fd = accept(ls, nullptr, nullptr);
    if (fd < 0) continue;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::thread(serve, &srv, fd).detach();
  }
}
