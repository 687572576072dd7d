// imgscan.hpp — image-reference scan of trusted-repos normalisation (oracle:
// orc_image_parts), shared by the tile kernel (kernels.hip: strings staged in LDS, or HBM pools) and
// the host checker that compares it with a byte loop (tests/imgscan_check.cpp, CPU suite).
#pragma once
#include <cstdint>

#include "kwdev.hpp"  // KW_HD

#ifndef KW_ALIGNBIT  // device align_bytes as v_alignbit_b32
#define KW_ALIGNBIT 1
#endif
#ifndef KW_XAD  // image scan: per-byte equality masks through v_xad_u32
#define KW_XAD 1
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

// Little-endian word of s[4k, 4k + 4) (bytes past the string are 0).
template <int N>
constexpr uint32_t const_word(const char (&s)[N], int k) {
  uint32_t w = 0;
  for (int i = 0; i < 4; ++i)
    if (4 * k + i < N - 1) w |= (uint32_t)(uint8_t)s[4 * k + i] << (8 * i);
  return w;
}

// equals_const for the 9-byte constants, branch-free: three word loads from the aligned-down start
// (they stay within the string's 16 bytes of zero padding), no dependent byte chain.
template <int N>
KW_HD inline bool equals_const9(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e, const char (&s)[N]) {
  static_assert(N - 1 == 9, "9-byte constants");
  const uint32_t* q = (const uint32_t*)(bytes + (b & ~3u));
  const uint32_t sh = b & 3u;
  const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const uint32_t x0 = align_bytes(q1, q0, sh), x1 = align_bytes(q2, q1, sh), x2 = align_bytes(q3, q2, sh);
  return ((uint32_t)(e - b == 9u) & (uint32_t)(x0 == const_word(s, 0)) & (uint32_t)(x1 == const_word(s, 1)) &
          (uint32_t)((x2 & 0xffu) == const_word(s, 2))) != 0u;
}

// Parsed image reference (DESIGN.md §2 trusted-repos; oracle: orc_image_parts).
struct ImageRef {
  uint32_t b, e, at, slash0, rest_b, colon, path_end, name_end;
  bool is_reg, path_slash, is_docker, eff_tag;
};

KW_HD inline ImageRef parse_image(const uint8_t* __restrict__ bytes, uint32_t b, uint32_t e) {
  const uint32_t NONE = 0xffffffffu;
  uint32_t at = NONE, slash0 = NONE, slash1 = NONE, co_p = NONE, co_m = 0u;
  bool dotcolon = false;
  // four bytes a step: per-byte match masks (bit 7 of each byte) of '@', '/', ':' and '.', exact
  // (no carry between bytes: both operands of the add are below 0x80 per byte), restricted to the
  // string and cut at the first '@'. xm = the word's low 7 bits.
  // vmx: the valid bytes whose bit 7 is clear (a byte with bit 7 set never matches)
  const uint32_t k7f = 0x7F7F7F7Fu;
  auto eqm = [&](uint32_t xm, uint32_t c4, uint32_t vmx) -> uint32_t {
#if defined(__HIP_DEVICE_COMPILE__) && KW_XAD
    // one v_xad_u32 ((a ^ b) + c); left to itself the compiler rewrites (x & 0x7F) ^ c as
    // (x ^ c) & 0x7F and spends an add and an or per character class on it
    uint32_t t;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(t) : "v"(xm), "s"(c4), "v"(k7f));
    return ~t & vmx;
#else
    return ~((xm ^ c4) + k7f) & vmx;
#endif
  };
  uint32_t vm = 0x80808080u << (8u * (b & 3u));  // the first word: bytes before b excluded
  // the last word (p0 == pe): bytes from e on excluded
  const uint32_t pe = (e - 1u) & ~3u, tail = 0xffffffffu >> (8u * ((0u - e) & 3u));
  for (uint32_t p0 = b & ~3u; p0 < e; p0 += 4u) {
    const uint32_t w = *(const uint32_t*)(bytes + p0);
    const uint32_t xm = w & 0x7F7F7F7Fu, vmx = vm & ~w & (p0 == pe ? tail : 0xffffffffu);
    uint32_t m_at = eqm(xm, 0x40404040u, vmx), m_sl = eqm(xm, 0x2f2f2f2fu, vmx);
    uint32_t m_co = eqm(xm, 0x3a3a3a3au, vmx), m_dt = eqm(xm, 0x2e2e2e2eu, vmx);
    vm = 0x80808080u;
    if (m_at) {  // the digest starts here: nothing at or after the '@' counts
      const uint32_t keep = (1u << __builtin_ctz(m_at)) - 1u;
      at = p0 + (uint32_t)__builtin_ctz(m_at) / 8u;
      m_sl &= keep;
      m_co &= keep;
      m_dt &= keep;
    }
    if (m_co) {  // the last word holding a ':' (its position is taken once, after the scan)
      co_p = p0;
      co_m = m_co;
    }
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
  const uint32_t last_colon = co_m ? co_p + (31u - (uint32_t)__builtin_clz(co_m)) / 8u : NONE;
  ImageRef r;
  r.b = b;
  r.e = e;
  r.at = at;
  r.slash0 = slash0;
  r.name_end = at != NONE ? at : e;
  r.is_reg = slash0 != NONE && (dotcolon || equals_const9(bytes, b, slash0, kLocalhost));
  r.rest_b = r.is_reg ? slash0 + 1 : b;
  r.colon = (last_colon != NONE && last_colon >= r.rest_b) ? last_colon : NONE;
  r.path_end = r.colon != NONE ? r.colon : r.name_end;
  const uint32_t first_slash_rest = r.is_reg ? slash1 : slash0;
  r.path_slash = first_slash_rest != NONE && first_slash_rest < r.path_end;
  r.is_docker = !r.is_reg || equals_const9(bytes, b, slash0, kDockerIo);
  r.eff_tag = r.colon != NONE || at == NONE;
  return r;
}

}  // namespace kw
