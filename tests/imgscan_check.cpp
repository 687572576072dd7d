// Host check of the tile kernel's image-reference scan (policy-server_amd/csrc/imgscan.hpp, the
// exact code the kernel runs: four bytes a step with per-byte match masks) against a byte loop
// restating the normalisation rules (oracle orc_image_parts): every ImageRef field,
// on random references built from the tokens the rules test (registries, "docker.io",
// "localhost", ':', '/', '@', '.', non-ASCII, NUL) amid noise bytes of neighbouring strings.
// Built and run by tests/test_imgscan.py:  clang++ -O2 -std=c++17 -I policy-server_amd/csrc
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "imgscan.hpp"

using namespace kw;

static ImageRef reference(const uint8_t* s, uint32_t b, uint32_t e) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t at = NONE, s0 = NONE, s1 = NONE, lc = NONE;
  bool dc = false;
  for (uint32_t q = b; q < e; ++q) {
    const uint8_t c = s[q];
    if (c == '@') {
      at = q;
      break;
    }
    if (c == '/') {
      if (s0 == NONE) s0 = q;
      else if (s1 == NONE) s1 = q;
    } else if (c == ':') {
      lc = q;
      if (s0 == NONE) dc = true;
    } else if (c == '.') {
      if (s0 == NONE) dc = true;
    }
  }
  auto eq = [&](uint32_t x, uint32_t y, const char* t) {
    return y - x == strlen(t) && memcmp(s + x, t, y - x) == 0;
  };
  ImageRef r;
  r.b = b;
  r.e = e;
  r.at = at;
  r.slash0 = s0;
  r.name_end = at != NONE ? at : e;
  r.is_reg = s0 != NONE && (dc || eq(b, s0, "localhost"));
  r.rest_b = r.is_reg ? s0 + 1 : b;
  r.colon = (lc != NONE && lc >= r.rest_b) ? lc : NONE;
  r.path_end = r.colon != NONE ? r.colon : r.name_end;
  const uint32_t fs = r.is_reg ? s1 : s0;
  r.path_slash = fs != NONE && fs < r.path_end;
  r.is_docker = !r.is_reg || eq(b, s0, "docker.io");
  r.eff_tag = r.colon != NONE || at == NONE;
  return r;
}

static bool same(const ImageRef& x, const ImageRef& y) {
  return x.b == y.b && x.e == y.e && x.at == y.at && x.slash0 == y.slash0 && x.rest_b == y.rest_b && x.colon == y.colon &&
         x.path_end == y.path_end && x.name_end == y.name_end && x.is_reg == y.is_reg && x.path_slash == y.path_slash &&
         x.is_docker == y.is_docker && x.eff_tag == y.eff_tag;
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 400000;
  std::mt19937 g(7);
  const char* tok[] = {"docker.io", "localhost", "ghcr.io", "quay.io", "a", "bc", ".", ":", "/", "/", "@", "sha256",
                       "x:y", "\x80", "<NUL>", "library", "v1.2.3", "my-corp.example:5000", "latest"};
  const int ntok = sizeof(tok) / sizeof(tok[0]);
  alignas(16) uint8_t buf[512];
  long bad = 0;
  for (long it = 0; it < iters; ++it) {
    // fill the buffer with noise (neighbouring strings), then place one reference at b
    for (auto& c : buf) c = (uint8_t)"@/:.ab\x80"[g() % 7];
    std::string ref;
    const int n = (int)(g() % 14);
    for (int k = 0; k < n; ++k) {
      const int t = (int)(g() % ntok);
      if (t == 14) ref.push_back('\0');
      else ref += tok[t];
    }
    if (ref.size() > 200) ref.resize(200);
    const uint32_t b = g() % 200, e = b + (uint32_t)ref.size();
    memcpy(buf + b, ref.data(), ref.size());
    const ImageRef want = reference(buf, b, e);
    const ImageRef got = parse_image(buf, b, e);
    if (!same(want, got)) {
      if (bad < 5) printf("mismatch b=%u e=%u ref='%s'\n", b, e, ref.c_str());
      ++bad;
    }
  }
  printf("checked %ld mismatches %ld\n", iters, bad);
  return bad ? 1 : 0;
}
