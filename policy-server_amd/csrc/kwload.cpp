// kwload — closed-loop HTTP load generator for kwhost (the serving measurement, SURVEY §8(d) mode 4).
//
// C keep-alive connections, one thread each, POST synthetic AdmissionReview documents (libkwsynth,
// the bench's own workload generator) to /validate/<policy> (or /audit, /validate_raw) back to back
// for --warmup + --duration seconds; requests completed inside the measured window are counted and
// their latency (send -> full response read) recorded. Prints one JSON line: req/s, latency
// percentiles (p50/p90/p99/p99.9/max, ms), HTTP status counts, and the allowed fraction.
//
// Usage: kwload --port P --policy ID [--addr 127.0.0.1] [--route validate|audit|validate_raw]
//   [--connections 64] [--duration 10] [--warmup 2] [--config 4] [--docs 4096] [--seed 1]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

extern "C" {
struct kws_batch;
kws_batch* kws_generate(int config, uint64_t n, uint64_t seed, uint64_t row0);
void kws_free(kws_batch* b);
int kws_json(const kws_batch* b, uint64_t row, char* buf, size_t cap, size_t* need);
}

namespace {

using Clock = std::chrono::steady_clock;

struct Opts {
  std::string addr = "127.0.0.1", policy, route = "validate";
  int port = 3000, connections = 64, config = 4, docs = 4096;
  double duration = 10, warmup = 2;
  uint64_t seed = 1;
};

struct Result {
  std::vector<uint32_t> lat_us;
  std::map<int, uint64_t> status;
  uint64_t allowed = 0, answered = 0, errors = 0;
};

std::string pct_encode(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      o += (char)c;
    } else {
      char b[4];
      snprintf(b, sizeof(b), "%%%02X", c);
      o += b;
    }
  }
  return o;
}

int connect_to(const Opts& o) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  sockaddr_in sa;
  memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)o.port);
  inet_pton(AF_INET, o.addr.c_str(), &sa.sin_addr);
  if (connect(fd, (sockaddr*)&sa, sizeof(sa)) != 0) {
    close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

// One request/response exchange on a keep-alive connection; returns the status (0 on I/O error).
int exchange(int fd, const std::string& req, std::string* buf, std::string* body) {
  size_t o = 0;
  while (o < req.size()) {
    const ssize_t n = send(fd, req.data() + o, req.size() - o, MSG_NOSIGNAL);
    if (n <= 0) return 0;
    o += (size_t)n;
  }
  size_t he;
  char tmp[65536];
  while ((he = buf->find("\r\n\r\n")) == std::string::npos) {
    const ssize_t n = recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return 0;
    buf->append(tmp, (size_t)n);
  }
  const int status = atoi(buf->c_str() + 9);  // "HTTP/1.1 200 OK"
  size_t clen = 0;
  for (size_t p = buf->find("\r\n"); p < he; p = buf->find("\r\n", p + 2)) {
    if (strncasecmp(buf->c_str() + p + 2, "content-length:", 15) == 0) clen = strtoul(buf->c_str() + p + 17, nullptr, 10);
  }
  while (buf->size() < he + 4 + clen) {
    const ssize_t n = recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return 0;
    buf->append(tmp, (size_t)n);
  }
  body->assign(*buf, he + 4, clen);
  buf->erase(0, he + 4 + clen);
  return status;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
    if (!v) {
      fprintf(stderr, "kwload: %s needs a value\n", a.c_str());
      return 2;
    }
    ++i;
    if (a == "--addr") o.addr = v;
    else if (a == "--port") o.port = atoi(v);
    else if (a == "--policy") o.policy = v;
    else if (a == "--route") o.route = v;
    else if (a == "--connections") o.connections = std::max(1, atoi(v));
    else if (a == "--duration") o.duration = atof(v);
    else if (a == "--warmup") o.warmup = atof(v);
    else if (a == "--config") o.config = atoi(v);
    else if (a == "--docs") o.docs = std::max(1, atoi(v));
    else if (a == "--seed") o.seed = strtoull(v, nullptr, 10);
    else {
      fprintf(stderr, "kwload: unknown option %s\n", a.c_str());
      return 2;
    }
  }
  if (o.policy.empty() || (o.route != "validate" && o.route != "audit" && o.route != "validate_raw")) {
    fprintf(stderr, "usage: kwload --port P --policy ID [--route validate|audit|validate_raw] [--connections C]\n"
                    "              [--duration S] [--warmup S] [--config N] [--docs N] [--seed S] [--addr A]\n");
    return 2;
  }
  // the requests: full HTTP messages, built once (a RawReview body is the same document: its
  // extra kind/apiVersion members are ignored by RawReviewRequest)
  kws_batch* syn = kws_generate(o.config, (uint64_t)o.docs, o.seed, 0);
  if (!syn) {
    fprintf(stderr, "kwload: cannot generate config %d\n", o.config);
    return 1;
  }
  std::vector<std::string> reqs((size_t)o.docs);
  uint64_t body_bytes = 0;
  const std::string head = "POST /" + o.route + "/" + pct_encode(o.policy) +
                           " HTTP/1.1\r\nhost: kwhost\r\ncontent-type: application/json\r\ncontent-length: ";
  std::vector<char> jb(1 << 16);
  for (int r = 0; r < o.docs; ++r) {
    size_t need = 0;
    if (kws_json(syn, (uint64_t)r, jb.data(), jb.size(), &need) != 0) {
      jb.resize(need);
      kws_json(syn, (uint64_t)r, jb.data(), jb.size(), &need);
    }
    const std::string body(jb.data(), need - 1);
    body_bytes += body.size();
    reqs[(size_t)r] = head + std::to_string(body.size()) + "\r\n\r\n" + body;
  }
  kws_free(syn);

  const auto t0 = Clock::now();
  const auto t_meas = t0 + std::chrono::microseconds((int64_t)(o.warmup * 1e6));
  const auto t_end = t_meas + std::chrono::microseconds((int64_t)(o.duration * 1e6));
  std::vector<Result> res((size_t)o.connections);
  std::atomic<int> failed_connect{0};
  auto client = [&](int c) {
    Result& R = res[(size_t)c];
    R.lat_us.reserve(1 << 16);
    int fd = connect_to(o);
    if (fd < 0) {
      ++failed_connect;
      return;
    }
    std::string buf, body;
    size_t k = (size_t)c * 7919u % reqs.size();
    for (;;) {
      const auto s = Clock::now();
      if (s >= t_end) break;
      const int st = exchange(fd, reqs[k], &buf, &body);
      const auto e = Clock::now();
      k = (k + 1) % reqs.size();
      if (st == 0) {  // I/O error: reconnect
        close(fd);
        buf.clear();
        if (s >= t_meas) ++R.errors;
        fd = connect_to(o);
        if (fd < 0) return;
        continue;
      }
      if (s < t_meas || e > t_end) continue;  // only exchanges wholly inside the window
      R.lat_us.push_back((uint32_t)std::chrono::duration_cast<std::chrono::microseconds>(e - s).count());
      ++R.status[st];
      if (st == 200) {
        ++R.answered;
        if (body.find("\"allowed\":true") != std::string::npos) ++R.allowed;
      }
    }
    close(fd);
  };
  std::vector<std::thread> th;
  for (int c = 0; c < o.connections; ++c) th.emplace_back(client, c);
  for (auto& t : th) t.join();

  std::vector<uint32_t> lat;
  std::map<int, uint64_t> status;
  uint64_t allowed = 0, answered = 0, errors = 0;
  for (const Result& R : res) {
    lat.insert(lat.end(), R.lat_us.begin(), R.lat_us.end());
    for (const auto& kv : R.status) status[kv.first] += kv.second;
    allowed += R.allowed;
    answered += R.answered;
    errors += R.errors;
  }
  std::sort(lat.begin(), lat.end());
  auto q = [&](double p) {
    if (lat.empty()) return 0.0;
    const size_t i = std::min(lat.size() - 1, (size_t)(p * (double)lat.size()));
    return lat[i] / 1000.0;
  };
  double mean = 0;
  for (uint32_t x : lat) mean += x;
  mean = lat.empty() ? 0 : mean / (double)lat.size() / 1000.0;
  std::string st = "{";
  for (const auto& kv : status) st += (st.size() > 1 ? "," : "") + ("\"" + std::to_string(kv.first) + "\":" + std::to_string(kv.second));
  st += "}";
  printf("{\"tool\": \"kwload\", \"route\": \"%s\", \"policy\": \"%s\", \"connections\": %d, \"duration_s\": %.3f, "
         "\"requests\": %zu, \"req_per_s\": %.1f, \"latency_ms\": {\"mean\": %.3f, \"p50\": %.3f, \"p90\": %.3f, "
         "\"p99\": %.3f, \"p999\": %.3f, \"max\": %.3f}, \"status\": %s, \"io_errors\": %llu, \"failed_connects\": %d, "
         "\"allowed_fraction\": %.4f, \"workload\": {\"config\": %d, \"distinct_docs\": %d, \"mean_body_bytes\": %.1f}}\n",
         o.route.c_str(), o.policy.c_str(), o.connections, o.duration, lat.size(), (double)lat.size() / o.duration, mean,
         q(0.5), q(0.9), q(0.99), q(0.999), lat.empty() ? 0.0 : lat.back() / 1000.0, st.c_str(),
         (unsigned long long)errors, failed_connect.load(), answered ? (double)allowed / (double)answered : 0.0, o.config,
         o.docs, (double)body_bytes / o.docs);
  return 0;
}
