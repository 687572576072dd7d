// fmt_bench — host cost of kwhost's per-request stages without a GPU ("profile
// response formatting"): flatten (kw_batch_from_json) and the service epilogue + response JSON
// (kw_format_response_doc), on synthetic AdmissionReviews of a bench config, verdict words from the
// host walk (kw_debug_host_walk, the slot compiler's sequential form of the device walk).
//   build: make scripts/fmt_bench      run: scripts/fmt_bench [policies.yml] [policy] [config] [rows] [batch]
// Prints one JSON line: microseconds per request of each stage, and the verdict mix.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/kwgpu.h"

extern "C" {
struct kws_batch;
kws_batch* kws_generate(int config, uint64_t n, uint64_t seed, uint64_t row0);
int kws_json(const kws_batch* b, uint64_t row, char* buf, size_t cap, size_t* need);
void kws_free(kws_batch* b);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const char* yml = argc > 1 ? argv[1] : "configs/c4_64.yml";
  const char* pol = argc > 2 ? argv[2] : "psp-capabilities-00";
  const int cfg = argc > 3 ? atoi(argv[3]) : 4;
  const uint64_t n = argc > 4 ? strtoull(argv[4], nullptr, 10) : 20000;
  const uint64_t per = argc > 5 ? strtoull(argv[5], nullptr, 10) : 64;  // kwhost's micro-batch size
  FILE* f = fopen(yml, "rb");
  if (!f) return fprintf(stderr, "cannot open %s\n", yml), 1;
  std::string text;
  char tmp[65536];
  for (size_t m; (m = fread(tmp, 1, sizeof(tmp), f)) > 0;) text.append(tmp, m);
  fclose(f);
  kw_env_options o{1, "kubewarden", -1};
  kw_env* env = nullptr;
  char err[512];
  if (kw_env_build_yaml(text.data(), text.size(), &o, &env, err, sizeof(err)) != KW_OK) return fprintf(stderr, "%s\n", err), 1;
  int32_t idx = -1;
  if (kw_env_lookup(env, pol, strlen(pol), &idx) != KW_OK) return fprintf(stderr, "no policy %s\n", pol), 1;
  kws_batch* sb = kws_generate(cfg, n, 1234, 0);
  std::vector<std::string> docs(n);
  for (uint64_t r = 0; r < n; ++r) {
    size_t need = 0;
    kws_json(sb, r, nullptr, 0, &need);
    docs[r].resize(need);
    kws_json(sb, r, docs[r].data(), need, &need);
    docs[r].resize(strnlen(docs[r].data(), docs[r].size()));
  }
  kws_free(sb);
  double t_flat = 0, t_walk = 0, t_fmt = 0;
  uint64_t bytes = 0, allowed = 0, patched = 0, rejected = 0;
  std::vector<char> buf(4096);
  for (uint64_t r0 = 0; r0 < n; r0 += per) {
    const uint64_t m = std::min(per, n - r0);
    std::vector<const char*> p(m);
    std::vector<size_t> l(m);
    for (uint64_t k = 0; k < m; ++k) p[k] = docs[r0 + k].data(), l[k] = docs[r0 + k].size();
    double t = now_us();
    kw_batch* b = nullptr;
    int64_t bad = -1;
    if (kw_batch_from_json(p.data(), l.data(), m, KW_DOC_ADMISSION_REVIEW, &b, &bad, err, sizeof(err)) != KW_OK)
      return fprintf(stderr, "flatten: %s\n", err), 1;
    t_flat += now_us() - t;
    std::vector<uint32_t> v(m);
    t = now_us();
    if (kw_debug_host_walk(env, b, &idx, 1, KW_ORIGIN_VALIDATE, v.data()) != KW_OK) return fprintf(stderr, "walk\n"), 1;
    t_walk += now_us() - t;
    t = now_us();
    for (uint64_t k = 0; k < m; ++k) {
      size_t need = 0;
      int rc = kw_format_response_doc(env, b, k, idx, v[k], nullptr, p[k], l[k], KW_DOC_ADMISSION_REVIEW, buf.data(), buf.size(), &need);
      if (rc == KW_E_NOSPACE) {
        buf.resize(need + 1);
        rc = kw_format_response_doc(env, b, k, idx, v[k], nullptr, p[k], l[k], KW_DOC_ADMISSION_REVIEW, buf.data(), buf.size(), &need);
      }
      if (rc != KW_OK) return fprintf(stderr, "format rc %d\n", rc), 1;
      bytes += need;
    }
    t_fmt += now_us() - t;
    for (uint32_t w : v) {
      allowed += (w & KW_F_ALLOWED) != 0;
      patched += (w & KW_F_PATCH) != 0;
      rejected += !(w & KW_F_ALLOWED);
    }
    kw_batch_destroy(b);
  }
  printf("{\"policy\": \"%s\", \"config\": %d, \"rows\": %llu, \"batch\": %llu, \"us_per_request\": {\"flatten\": %.3f, "
         "\"host_walk\": %.3f, \"format\": %.3f}, \"mean_response_bytes\": %.1f, \"allowed\": %.4f, \"patched\": %.4f, "
         "\"rejected\": %.4f}\n",
         pol, cfg, (unsigned long long)n, (unsigned long long)per, t_flat / n, t_walk / n, t_fmt / n, (double)bytes / n,
         (double)allowed / n, (double)patched / n, (double)rejected / n);
  kw_env_destroy(env);
  return 0;
}
