// mbls_soa.hpp — HBM layouts shared by the kernel translation units: big-endian wire words,
// digit-major SoA field elements (digit d of element i at base[d * n + i]: one coalesced
// 256-byte access per digit row of a wave) and the lane layout of the lane-group kernels.
#pragma once
#include "mbls_pairing.hpp"

namespace mbls_soa {
using namespace mbls;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

template <int NW>
__device__ __forceinline__ void load_be(const uint8_t* p, uint32_t (&w)[NW]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int j = 0; j < NW / 4; ++j) {
    const uint4 v = q[j];
    w[4 * j + 0] = bswap32(v.x);
    w[4 * j + 1] = bswap32(v.y);
    w[4 * j + 2] = bswap32(v.z);
    w[4 * j + 3] = bswap32(v.w);
  }
}
template <int NW>
__device__ __forceinline__ void store_be(uint8_t* p, const uint32_t (&w)[NW]) {
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int j = 0; j < NW / 4; ++j)
    q[j] = make_uint4(bswap32(w[4 * j]), bswap32(w[4 * j + 1]), bswap32(w[4 * j + 2]), bswap32(w[4 * j + 3]));
}

__device__ __forceinline__ void st_fp(uint32_t* base, size_t n, size_t i, int d0, const fp& a) {
#pragma unroll
  for (int d = 0; d < NL; ++d) base[(size_t)(d0 + d) * n + i] = a.v[d];
}
__device__ __forceinline__ fp ld_fp(const uint32_t* base, size_t n, size_t i, int d0) {
  fp a;
#pragma unroll
  for (int d = 0; d < NL; ++d) a.v[d] = base[(size_t)(d0 + d) * n + i];
  return a;
}
__device__ __forceinline__ void st_g2(uint32_t* base, size_t n, size_t i, const aff<fp2>& a) {
  st_fp(base, n, i, 0, a.x.c0);
  st_fp(base, n, i, NL, a.x.c1);
  st_fp(base, n, i, 2 * NL, a.y.c0);
  st_fp(base, n, i, 3 * NL, a.y.c1);
}
__device__ __forceinline__ aff<fp2> ld_g2(const uint32_t* base, size_t n, size_t i) {
  aff<fp2> a;
  a.x.c0 = ld_fp(base, n, i, 0);
  a.x.c1 = ld_fp(base, n, i, NL);
  a.y.c0 = ld_fp(base, n, i, 2 * NL);
  a.y.c1 = ld_fp(base, n, i, 3 * NL);
  return a;
}
__device__ __forceinline__ aff<fp> ld_g1(const uint32_t* base, size_t n, size_t i) {
  return {ld_fp(base, n, i, 0), ld_fp(base, n, i, NL)};
}

__device__ __forceinline__ aff<fp> neg_g1_gen() { return {fp_from(k::G1X), fp_from(k::G1Y_NEG)}; }

__device__ __forceinline__ void st_fp12(uint32_t* base, size_t n, size_t i, const fp12& f) {
  const fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    st_fp(base, n, i, 2 * j * NL, c[j]->c0);
    st_fp(base, n, i, (2 * j + 1) * NL, c[j]->c1);
  }
}
__device__ __forceinline__ fp12 ld_fp12(const uint32_t* base, size_t n, size_t i) {
  fp12 f;
  fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    c[j]->c0 = ld_fp(base, n, i, 2 * j * NL);
    c[j]->c1 = ld_fp(base, n, i, (2 * j + 1) * NL);
  }
  return f;
}

// coefficient of w^k of a one-lane st_fp12 value (k < 6; zero for the lane groups' pad lanes
// 6, 7): w^(2j) is component j, w^(2j+1) component 3 + j
__device__ __forceinline__ fp2 ld_fp12_coef(const uint32_t* base, size_t n, size_t i, int k) {
  const int j = k >= 6 ? 0 : (k & 1) ? 3 + (k >> 1) : (k >> 1);
  const fp2 c = {ld_fp(base, n, i, 2 * j * NL), ld_fp(base, n, i, (2 * j + 1) * NL)};
  return fp2_select(k < 6, c, fp2_zero());
}

__device__ __forceinline__ void st_lane(uint32_t* base, size_t nl, size_t l, const fp2& a) {
  st_fp(base, nl, l, 0, a.c0);
  st_fp(base, nl, l, NL, a.c1);
}
__device__ __forceinline__ fp2 ld_lane(const uint32_t* base, size_t nl, size_t l) {
  return {ld_fp(base, nl, l, 0), ld_fp(base, nl, l, NL)};
}
}  // namespace mbls_soa
