// imgscan.hpp — image-reference scan of trusted-repos normalisation (oracle:
// orc_image_parts), shared by the tile kernel (kernels.hip: strings staged in LDS, or HBM pools) and
// the host checker that compares it with a byte loop (tests/imgscan_check.cpp, CPU suite).
#pragma once
#include <cstdint>

#include "kwdev.hpp"  // KW_HD

#ifndef KW_ALIGNBIT  // device align_bytes as v_alignbit_b32
#define KW_ALIGNBIT 1
#endif

namespace kw {

KW_HD inline uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__) && KW_ALIGNBIT
  return __builtin_amdgcn_alignbit(hi, lo, 8u * sh);  // one v_alignbit_b32 (sh < 4), not a 64-bit shift
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
#endif
}
KW_HD inline uint32_t img_min(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Literal fragments of image normalisation; constexpr + unrolled loops turn them into immediates.
constexpr char kDockerIo[] = "docker.io";
constexpr char kLibrary[] = "library/";
constexpr char kLatest[] = "latest";
constexpr char kLocalhost[] = "localhost";

template <int N>
KW_HD inline bool equals_const(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e, const char (&s)[N]) {
  if ((int)(e - b) != N - 1) return false;
#pragma unroll
  for (int i = 0; i < N - 1; ++i)
    if (bytes[b + (uint32_t)i] != (uint8_t)s[i]) return false;
  return true;
}

// Parsed image reference (DESIGN.md §2 trusted-repos; oracle: orc_image_parts).
struct ImageRef {
  uint32_t b, e, at, slash0, rest_b, colon, path_end, name_end;
  bool is_reg, path_slash, is_docker, eff_tag;
};

KW_HD inline ImageRef parse_image(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t at = NONE, slash0 = NONE, slash1 = NONE, last_colon = NONE;
  bool dotcolon = false;
  // four bytes a step: per-byte match masks (bit 7 of each byte) of '@', '/', ':' and '.', exact
  // (no borrow between bytes), restricted to the string and cut at the first '@'
  auto eqb = [](uint32_t x, uint32_t c4) -> uint32_t {
    const uint32_t y = x ^ c4;
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
  };
  for (uint32_t p0 = b & ~3u; p0 < e; p0 += 4u) {
    const uint32_t w = *(const uint32_t*)(bytes + p0);
    const uint32_t lo = p0 < b ? b - p0 : 0u, hi = img_min(4u, e - p0);  // valid bytes [lo, hi)
    const uint32_t vm = (0x80808080u << (8u * lo)) & (hi >= 4u ? 0xffffffffu : ((1u << (8u * hi)) - 1u));
    uint32_t m_at = eqb(w, 0x40404040u) & vm, m_sl = eqb(w, 0x2f2f2f2fu) & vm;
    uint32_t m_co = eqb(w, 0x3a3a3a3au) & vm, m_dt = eqb(w, 0x2e2e2e2eu) & vm;
    if (m_at) {  // the digest starts here: nothing at or after the '@' counts
      const uint32_t keep = (1u << __builtin_ctz(m_at)) - 1u;
      at = p0 + (uint32_t)__builtin_ctz(m_at) / 8u;
      m_sl &= keep;
      m_co &= keep;
      m_dt &= keep;
    }
    if (m_co) last_colon = p0 + (31u - (uint32_t)__builtin_clz(m_co)) / 8u;
    if (slash0 == NONE) {
      const uint32_t before = m_sl ? (1u << __builtin_ctz(m_sl)) - 1u : 0xffffffffu;  // bytes before the first '/'
      if ((m_co | m_dt) & before) dotcolon = true;
      if (m_sl) {
        slash0 = p0 + (uint32_t)__builtin_ctz(m_sl) / 8u;
        m_sl &= m_sl - 1u;
      }
    }
    if (slash1 == NONE && m_sl) slash1 = p0 + (uint32_t)__builtin_ctz(m_sl) / 8u;
    if (m_at) break;
  }
  ImageRef r;
  r.b = b;
  r.e = e;
  r.at = at;
  r.slash0 = slash0;
  r.name_end = at != NONE ? at : e;
  r.is_reg = slash0 != NONE && (dotcolon || equals_const(bytes, b, slash0, kLocalhost));
  r.rest_b = r.is_reg ? slash0 + 1 : b;
  r.colon = (last_colon != NONE && last_colon >= r.rest_b) ? last_colon : NONE;
  r.path_end = r.colon != NONE ? r.colon : r.name_end;
  const uint32_t first_slash_rest = r.is_reg ? slash1 : slash0;
  r.path_slash = first_slash_rest != NONE && first_slash_rest < r.path_end;
  r.is_docker = !r.is_reg || equals_const(bytes, b, slash0, kDockerIo);
  r.eff_tag = r.colon != NONE || at == NONE;
  return r;
}

}  // namespace kw
