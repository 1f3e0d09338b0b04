// mbls_fp.hpp — BLS12-381 base field Fp for gfx950.
//
// Representation: one element per lane, 14 radix-2^28 digits (little-endian) in 32-bit
// VGPRs, Montgomery form with R = 2^392.  Why radix 2^28 on CDNA4 (measured, see
// DESIGN.md §3 and profiles/): `v_mad_u64_u32` issues at ~half the simple-VALU rate while
// `v_addc_co_u32` carry chains cost as much as a mad, so a 32-bit CIOS spends half its
// issue slots on carries.  With 28-bit digits a whole Montgomery column (<= 28 products of
// <= 60 bits) accumulates in one 64-bit register with no carry handling at all: one mad per
// digit product, 3 cheap ops per column.  Measured 6.9e10 Fp-mul/s/GPU vs 5.3e10 for CIOS-32.
//
// Replaces blst's mul_mont_384 / sqr_mont_384 / add_mod_384 / sub_mod_384 (blst 0.3.11,
// reached from native/bls_nif/src/lib.rs through lighthouse `bls`); re-derived, not ported.
//
// Invariants ("normalized, weakly reduced"): every digit < 2^28 and value < 2p.  All public
// functions take and return such values; `fp_canon` gives the unique representative < p.
// fp_mul additionally accepts digits < 2^30 (sums of up to four normalized values) as long
// as a*b < p*2^392, which is what the `_lazy` helpers rely on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mbls_constants.hpp"

#define MBLS_HD __host__ __device__ __forceinline__
// coarse out-of-line boundary (keeps code size and compile time bounded for the pairing /
// hash kernels; struct arguments of such functions are passed in memory, so only use it for
// functions whose body is >> their argument size)
#define MBLS_NI __host__ __device__ __noinline__ inline

namespace mbls {

constexpr int NL = 14;
constexpr uint32_t M28 = 0x0fffffffu;

struct fp {
  uint32_t v[NL];
};

MBLS_HD uint32_t p_digit(int i) { return k::P_RAW[i]; }

MBLS_HD fp fp_from(const uint32_t (&t)[NL]) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = t[i];
  return r;
}
MBLS_HD fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = 0;
  return r;
}
MBLS_HD fp fp_one() { return fp_from(k::ONE); }

// ---------------------------------------------------------------------------------------
// Montgomery product, product scanning (FIPS order).  Each column's products are split over
// three independent 64-bit accumulators (even / odd a*b terms, m*p terms) so the mad
// chains can overlap: at low occupancy a single serial chain per column leaves the
// v_mad_u64_u32 latency exposed.  Bounds per accumulator are smaller than the serial sum's.
// ---------------------------------------------------------------------------------------
MBLS_HD fp fp_mul_inl(const fp& a, const fp& b) {
  uint32_t m[NL];
  fp t;
  uint64_t acc = 0;
#pragma unroll
  for (int kk = 0; kk < NL; ++kk) {
    uint64_t s0 = acc, s1 = 0, s2 = 0;
#pragma unroll
    for (int i = 0; i <= kk; ++i) {
      if (i & 1)
        s1 += (uint64_t)a.v[i] * b.v[kk - i];
      else
        s0 += (uint64_t)a.v[i] * b.v[kk - i];
    }
#pragma unroll
    for (int i = 0; i < kk; ++i) s2 += (uint64_t)m[i] * p_digit(kk - i);
    uint64_t s = s0 + s1 + s2;
    m[kk] = ((uint32_t)s * k::N0) & M28;
    s += (uint64_t)m[kk] * p_digit(0);
    acc = s >> 28;
  }
#pragma unroll
  for (int kk = NL; kk < 2 * NL - 1; ++kk) {
    uint64_t s0 = acc, s1 = 0, s2 = 0;
#pragma unroll
    for (int i = kk - NL + 1; i < NL; ++i) {
      if (i & 1)
        s1 += (uint64_t)a.v[i] * b.v[kk - i];
      else
        s0 += (uint64_t)a.v[i] * b.v[kk - i];
    }
#pragma unroll
    for (int i = kk - NL + 1; i < NL; ++i) s2 += (uint64_t)m[i] * p_digit(kk - i);
    const uint64_t s = s0 + s1 + s2;
    t.v[kk - NL] = (uint32_t)s & M28;
    acc = s >> 28;
  }
  t.v[NL - 1] = (uint32_t)acc;
  return t;
}

// Squaring over pre-doubled digits: cross products once (105 + 196 mads instead of 392), each
// column in two accumulators (a_i a_j terms, m*p terms).  Measured r01 (tools/g1_variants.hip,
// profiles/r01_g1_variants.txt): 2.2% faster key validation than doubling the 64-bit cross
// sums.  Digits < 2^30: 2 a_i < 2^31, a column's cross terms < 7 * 2^61 + 2^60 + 2^36, the
// m*p terms < 14 * 2^56, their sum < 2^64.
MBLS_HD fp fp_sqr_inl(const fp& a) {
  uint32_t m[NL], a2[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) a2[i] = a.v[i] << 1;
  fp t;
  uint64_t acc = 0;
#pragma unroll
  for (int kk = 0; kk < NL; ++kk) {
    uint64_t s0 = acc, s2 = 0;
#pragma unroll
    for (int i = 0; i < kk - i; ++i) s0 += (uint64_t)a2[i] * a.v[kk - i];
    if ((kk & 1) == 0) s0 += (uint64_t)a.v[kk / 2] * a.v[kk / 2];
#pragma unroll
    for (int i = 0; i < kk; ++i) s2 += (uint64_t)m[i] * p_digit(kk - i);
    uint64_t s = s0 + s2;
    m[kk] = ((uint32_t)s * k::N0) & M28;
    s += (uint64_t)m[kk] * p_digit(0);
    acc = s >> 28;
  }
#pragma unroll
  for (int kk = NL; kk < 2 * NL - 1; ++kk) {
    uint64_t s0 = acc, s2 = 0;
#pragma unroll
    for (int i = kk - NL + 1; i < kk - i; ++i) s0 += (uint64_t)a2[i] * a.v[kk - i];
    if ((kk & 1) == 0) s0 += (uint64_t)a.v[kk / 2] * a.v[kk / 2];
#pragma unroll
    for (int i = kk - NL + 1; i < NL; ++i) s2 += (uint64_t)m[i] * p_digit(kk - i);
    const uint64_t s = s0 + s2;
    t.v[kk - NL] = (uint32_t)s & M28;
    acc = s >> 28;
  }
  t.v[NL - 1] = (uint32_t)acc;
  return t;
}

// Sum of two Montgomery products with ONE reduction: (a b + c d) R^-1 mod p, in [0, 2p).
// Operands a, c normalized (digits < 2^28), b, d digits < 2^30, a b + c d < p R (R/p > 2^11).
// Columns: 28 products < 2^58 + 14 m*p terms < 2^56 + carry < 2^63.  Four accumulators per
// column (a b even / odd terms, c d, m p) keep the mad chains short.  An Fp2 product is two
// of these (mbls_fp2.hpp fp2_mul): 4 x 196 + 2 x 196 mads, the same as Karatsuba's three
// Montgomery products, but no normalized additions.
MBLS_HD fp fp_mul2_inl(const fp& a, const fp& b, const fp& c, const fp& d) {
  uint32_t m[NL];
  fp t;
  uint64_t acc = 0;
#pragma unroll
  for (int kk = 0; kk < NL; ++kk) {
    uint64_t s0 = acc, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int i = 0; i <= kk; ++i) {
      if (i & 1)
        s1 += (uint64_t)a.v[i] * b.v[kk - i];
      else
        s0 += (uint64_t)a.v[i] * b.v[kk - i];
      s2 += (uint64_t)c.v[i] * d.v[kk - i];
    }
#pragma unroll
    for (int i = 0; i < kk; ++i) s3 += (uint64_t)m[i] * p_digit(kk - i);
    uint64_t s = (s0 + s1) + (s2 + s3);
    m[kk] = ((uint32_t)s * k::N0) & M28;
    s += (uint64_t)m[kk] * p_digit(0);
    acc = s >> 28;
  }
#pragma unroll
  for (int kk = NL; kk < 2 * NL - 1; ++kk) {
    uint64_t s0 = acc, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int i = kk - NL + 1; i < NL; ++i) {
      if (i & 1)
        s1 += (uint64_t)a.v[i] * b.v[kk - i];
      else
        s0 += (uint64_t)a.v[i] * b.v[kk - i];
      s2 += (uint64_t)c.v[i] * d.v[kk - i];
      s3 += (uint64_t)m[i] * p_digit(kk - i);
    }
    const uint64_t s = (s0 + s1) + (s2 + s3);
    t.v[kk - NL] = (uint32_t)s & M28;
    acc = s >> 28;
  }
  t.v[NL - 1] = (uint32_t)acc;
  return t;
}

// 4p with raised digits: digit-wise a + P4B - b never borrows for normalized b < 2p.
// n = digits of 4p; d_0 = n_0 + 2^28, d_i = n_i + 2^28 - 1 (0 < i < 13), d_13 = n_13 - 1
// (the same value: the added 2^28 (2^28 - 1) ... telescopes to 0).  Digits < 2^29.
struct pbig_t {
  uint32_t v[NL];
};
constexpr pbig_t p4_big() {
  pbig_t r{};
  uint64_t c = 0;
  uint32_t n[NL] = {};
  for (int i = 0; i < NL; ++i) {
    const uint64_t x = (uint64_t)k::P_RAW[i] * 4u + c;
    n[i] = (uint32_t)(x & M28);
    c = x >> 28;
  }
  for (int i = 0; i < NL; ++i) r.v[i] = i == 0 ? n[i] + (1u << 28) : i < NL - 1 ? n[i] + (1u << 28) - 1u : n[i] - 1u;
  return r;
}
constexpr pbig_t P4B = p4_big();

// a - b + 4p without normalization: value in (2p, 6p), digits < 3 * 2^28.  For a, b
// normalized (< 2p); only as the second operand of a multiply.
MBLS_HD fp fp_sub_lazy(const fp& a, const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + P4B.v[i] - b.v[i];
  return s;
}
// 4p - b (value in (2p, 4p], digits < 2^29): the negation as a multiply operand
MBLS_HD fp fp_neg_lazy(const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = P4B.v[i] - b.v[i];
  return s;
}

// Out-of-line forms for the large kernels (pairing, hash-to-curve): scalar arguments keep
// the operands in VGPRs (no byval scratch), and the call keeps code size I-cache friendly.
#if defined(__HIP_DEVICE_COMPILE__) && defined(MBLS_FP_OUTLINE)
#define MBLS_A14(p)                                                                                        \
  uint32_t p##0, uint32_t p##1, uint32_t p##2, uint32_t p##3, uint32_t p##4, uint32_t p##5, uint32_t p##6, \
      uint32_t p##7, uint32_t p##8, uint32_t p##9, uint32_t p##10, uint32_t p##11, uint32_t p##12, uint32_t p##13
#define MBLS_U14(x) \
  x.v[0], x.v[1], x.v[2], x.v[3], x.v[4], x.v[5], x.v[6], x.v[7], x.v[8], x.v[9], x.v[10], x.v[11], x.v[12], x.v[13]
__device__ __noinline__ inline fp fp_mul_call(MBLS_A14(a), MBLS_A14(b)) {
  const fp x = {{a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13}};
  const fp y = {{b0, b1, b2, b3, b4, b5, b6, b7, b8, b9, b10, b11, b12, b13}};
  return fp_mul_inl(x, y);
}
__device__ __noinline__ inline fp fp_sqr_call(MBLS_A14(a)) {
  const fp x = {{a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, a12, a13}};
  return fp_sqr_inl(x);
}
MBLS_HD fp fp_mul(const fp& a, const fp& b) { return fp_mul_call(MBLS_U14(a), MBLS_U14(b)); }
MBLS_HD fp fp_sqr(const fp& a) { return fp_sqr_call(MBLS_U14(a)); }
MBLS_HD fp fp_mul2(const fp& a, const fp& b, const fp& c, const fp& d) { return fp_mul2_inl(a, b, c, d); }
#elif !defined(__HIP_DEVICE_COMPILE__)
// host build (test harness only): out of line to keep compile time bounded.  With
// MBLS_HOST_COUNT (tests/hostsim) every product is counted: the work model of the bench's
// rooflines is frozen from these counts of the device algorithms (tools/work_model.py).
#ifdef MBLS_HOST_COUNT
inline thread_local uint64_t g_host_mul = 0, g_host_sqr = 0, g_host_mul2 = 0;
#define MBLS_HOST_TICK(c) (++(c))
#else
#define MBLS_HOST_TICK(c) ((void)0)
#endif
__host__ __noinline__ inline fp fp_mul_host(const fp& a, const fp& b) {
  MBLS_HOST_TICK(g_host_mul);
  return fp_mul_inl(a, b);
}
__host__ __noinline__ inline fp fp_sqr_host(const fp& a) {
  MBLS_HOST_TICK(g_host_sqr);
  return fp_sqr_inl(a);
}
__host__ __noinline__ inline fp fp_mul2_host(const fp& a, const fp& b, const fp& c, const fp& d) {
  MBLS_HOST_TICK(g_host_mul2);
  return fp_mul2_inl(a, b, c, d);
}
MBLS_HD fp fp_mul(const fp& a, const fp& b) { return fp_mul_host(a, b); }
MBLS_HD fp fp_sqr(const fp& a) { return fp_sqr_host(a); }
MBLS_HD fp fp_mul2(const fp& a, const fp& b, const fp& c, const fp& d) { return fp_mul2_host(a, b, c, d); }
#else
MBLS_HD fp fp_mul(const fp& a, const fp& b) { return fp_mul_inl(a, b); }
MBLS_HD fp fp_sqr(const fp& a) { return fp_sqr_inl(a); }
MBLS_HD fp fp_mul2(const fp& a, const fp& b, const fp& c, const fp& d) { return fp_mul2_inl(a, b, c, d); }
#endif

// ---------------------------------------------------------------------------------------
// Lazy reduction: a sum of products reduced once.  fpcols holds the 27 column sums of
// schoolbook products; cols_redc returns (sum) R^-1 mod p in [0, 2p), the value the separate
// Montgomery products would add up to, with one reduction (196 mads) instead of one per
// product.  Operand digits must be < 2^28 (normalized values): a product then adds < 14 * 2^56
// to a column, so up to 12 products plus the reduction's 14 m*p terms and the carry stay
// < 2^63.5; the sum's value < 12 (2p)^2 < p R keeps the result < 2p.
// ---------------------------------------------------------------------------------------
struct fpcols {
  uint64_t c[2 * NL - 1];
};
MBLS_HD void cols_zero(fpcols& a) {
#pragma unroll
  for (int i = 0; i < 2 * NL - 1; ++i) a.c[i] = 0;
}
MBLS_HD void cols_mad(fpcols& acc, const fp& a, const fp& b) {
#pragma unroll
  for (int i = 0; i < NL; ++i)
#pragma unroll
    for (int j = 0; j < NL; ++j) acc.c[i + j] += (uint64_t)a.v[i] * b.v[j];
}
MBLS_HD fp cols_redc(const fpcols& acc) {
  uint32_t m[NL];
  fp t;
  uint64_t carry = 0;
#pragma unroll
  for (int kk = 0; kk < NL; ++kk) {
    uint64_t s = acc.c[kk] + carry;
#pragma unroll
    for (int i = 0; i < kk; ++i) s += (uint64_t)m[i] * p_digit(kk - i);
    m[kk] = ((uint32_t)s * k::N0) & M28;
    s += (uint64_t)m[kk] * p_digit(0);
    carry = s >> 28;
  }
#pragma unroll
  for (int kk = NL; kk < 2 * NL - 1; ++kk) {
    uint64_t s = acc.c[kk] + carry;
#pragma unroll
    for (int i = kk - NL + 1; i < NL; ++i) s += (uint64_t)m[i] * p_digit(kk - i);
    t.v[kk - NL] = (uint32_t)s & M28;
    carry = s >> 28;
  }
  t.v[NL - 1] = (uint32_t)carry;
  return t;
}

// ---------------------------------------------------------------------------------------
// Additive group (normalized, weakly reduced results)
// ---------------------------------------------------------------------------------------

// s in [0, 4p) with digits possibly >= 2^28 (unnormalized, signed-safe) -> normalized < 2p
MBLS_HD fp fp_norm_sub2p(fp s) {
  // signed carry propagation
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int32_t d = (int32_t)s.v[i] + c;
    c = d >> 28;  // arithmetic shift = floor division
    s.v[i] = (uint32_t)d & M28;
  }
  // conditional subtract 2p
  fp d;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int32_t x = (int32_t)s.v[i] - (int32_t)k::P2_RAW[i] + br;
    br = x >> 28;
    d.v[i] = (uint32_t)x & M28;
  }
  // br == -1 means s < 2p: keep s
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = br ? s.v[i] : d.v[i];
  return r;
}

MBLS_HD fp fp_add(const fp& a, const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + b.v[i];
  return fp_norm_sub2p(s);
}
MBLS_HD fp fp_dbl(const fp& a) { return fp_add(a, a); }

MBLS_HD fp fp_sub(const fp& a, const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + k::P2_RAW[i] - b.v[i];  // wraps as signed
  return fp_norm_sub2p(s);
}

MBLS_HD fp fp_neg(const fp& a) { return fp_sub(fp_zero(), a); }

// Lazy sum (no normalization): digits < 2^29, value < 4p.  Only as fp_mul/fp_sqr input.
MBLS_HD fp fp_add_lazy(const fp& a, const fp& b) {
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + b.v[i];
  return s;
}

MBLS_HD fp fp_mul3(const fp& a) { return fp_add(fp_dbl(a), a); }
MBLS_HD fp fp_mul4(const fp& a) { return fp_dbl(fp_dbl(a)); }
MBLS_HD fp fp_mul8(const fp& a) { return fp_dbl(fp_mul4(a)); }
MBLS_HD fp fp_mul12(const fp& a) { return fp_mul4(fp_mul3(a)); }

// ---------------------------------------------------------------------------------------
// Lazy linear combinations (the key-validation ladder).
//
// fp_mul/fp_sqr accept digits < 2^30 (a column then holds < 14*2^60 + 14*2^56 + 2^36
// < 2^64) and return a value < 2p whenever the product of the input VALUES is < p*R
// (R = 2^392, so R/p ~ 2^11.3: e.g. 20p x 6p is fine).  So a sum or difference that only
// feeds a multiply needs no conditional subtraction: form it digit-wise in int32 with a
// multiple of p added to keep it non-negative, then one signed carry pass (fp_carry) leaves
// digits < 2^28 and a value in [0, k p).  Callers track the k bounds (mbls_curve.hpp jac_*).
// ---------------------------------------------------------------------------------------
struct pmul_t {
  int32_t v[NL];
};
constexpr pmul_t p_times(uint32_t m) {  // digits of m*p, m < 2^11
  pmul_t r{};
  uint64_t c = 0;
  for (int i = 0; i < NL; ++i) {
    const uint64_t x = (uint64_t)k::P_RAW[i] * m + c;
    r.v[i] = (int32_t)(x & M28);
    c = x >> 28;
  }
  return r;
}

// signed carry pass: digit-wise combination (|d_i| < 2^31 - 2^4) of value in [0, 2^392)
MBLS_HD fp fp_carry(const int32_t (&d)[NL]) {
  fp r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    const int32_t x = d[i] + c;
    c = x >> 28;  // arithmetic shift = floor division
    r.v[i] = (uint32_t)x & M28;
  }
  r.v[NL - 1] = (uint32_t)(d[NL - 1] + c);
  return r;
}

// a + b + c without normalisation (digits < 3 * 2^28; only as a multiply input)
MBLS_HD fp fp_add3_lazy(const fp& a, const fp& b, const fp& c) {
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + b.v[i] + c.v[i];
  return s;
}

// a mod p reduced to [0, 2p) for any a with digits < 2^30 and value < 2^11 p: a * R / R
MBLS_HD fp fp_shrink(const fp& a) { return fp_mul(a, fp_from(k::ONE)); }

// unique representative < p
MBLS_HD fp fp_canon(const fp& a) {
  fp d;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int32_t x = (int32_t)a.v[i] - (int32_t)k::P_RAW[i] + br;
    br = x >> 28;
    d.v[i] = (uint32_t)x & M28;
  }
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = br ? a.v[i] : d.v[i];
  return r;
}

MBLS_HD bool fp_is_zero(const fp& a) {
  const fp c = fp_canon(a);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) acc |= c.v[i];
  return acc == 0;
}
MBLS_HD bool fp_eq(const fp& a, const fp& b) { return fp_is_zero(fp_sub(a, b)); }

MBLS_HD fp fp_select(bool c, const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}
MBLS_HD fp fp_cneg(const fp& a, bool neg) { return fp_select(neg, fp_neg(a), a); }

MBLS_HD fp fp_to_mont(const fp& a) { return fp_mul(a, fp_from(k::R2)); }
MBLS_HD fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.v[0] = 1;
  return fp_canon(fp_mul(a, one));
}

// a^e for a fixed public exponent (little-endian 32-bit words), left-to-right binary.
// Branches depend only on the exponent, so they are wave-uniform.
template <int NW>
MBLS_HD fp fp_pow_words(const fp& a, const uint32_t (&e)[NW]) {
  fp r = a;
  int top = 31;
  while (top > 0 && !((e[NW - 1] >> top) & 1u)) --top;
#pragma unroll 1
  for (int w = NW - 1; w >= 0; --w) {
    const uint32_t word = e[w];
    const int start = (w == NW - 1) ? top - 1 : 31;
#pragma unroll 1
    for (int b = start; b >= 0; --b) {
      r = fp_sqr(r);
      if ((word >> b) & 1u) r = fp_mul(r, a);
    }
  }
  return r;
}

// a^e by a width-3 sliding window over a schedule generated offline (tools/gen_constants.py):
// table a, a^3, a^5, a^7; ~110 multiplies instead of ~228 for the binary method on these
// dense exponents.  Schedule entries are uniform, so every branch is wave-uniform.
template <int NS>
MBLS_HD fp fp_pow_win3(const fp& a, const int16_t (&sched)[NS][2], int first) {
  const fp a2 = fp_sqr(a);
  const fp t0 = a;
  const fp t1 = fp_mul(t0, a2);
  const fp t2 = fp_mul(t1, a2);
  const fp t3 = fp_mul(t2, a2);
  fp r = fp_select(first == 0, t0, fp_select(first == 1, t1, fp_select(first == 2, t2, t3)));
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const int nsq = sched[s][0], idx = sched[s][1];
#pragma unroll 1
    for (int q = 0; q < nsq; ++q) r = fp_sqr(r);
    if (idx >= 0) r = fp_mul(r, fp_select(idx == 0, t0, fp_select(idx == 1, t1, fp_select(idx == 2, t2, t3))));
  }
  return r;
}

// Width-4 form for the key kernel's square root (its registers are free at that point):
// table a, a^3, ..., a^15, 78 + 8 multiplies instead of 106 + 4 for (p+1)/4.  The table index
// of a step is wave uniform, so the switch is a scalar branch, not a select chain.
template <int NS>
MBLS_HD fp fp_pow_win4(const fp& a, const int16_t (&sched)[NS][2], int first) {
  const fp a2 = fp_sqr(a);
  const fp t0 = a, t1 = fp_mul(t0, a2), t2 = fp_mul(t1, a2), t3 = fp_mul(t2, a2), t4 = fp_mul(t3, a2),
           t5 = fp_mul(t4, a2), t6 = fp_mul(t5, a2), t7 = fp_mul(t6, a2);
  auto pick = [&](int i) -> fp {
    switch (i) {
      case 0: return t0;
      case 1: return t1;
      case 2: return t2;
      case 3: return t3;
      case 4: return t4;
      case 5: return t5;
      case 6: return t6;
      default: return t7;
    }
  };
  fp r = pick(first);
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const int nsq = sched[s][0], idx = sched[s][1];
#pragma unroll 1
    for (int q = 0; q < nsq; ++q) r = fp_sqr(r);
    if (idx >= 0) r = fp_mul(r, pick(idx));
  }
  return r;
}

// a^(p-2) by the width-3 window (~456 sequential Fp products): kept for cross-checks
MBLS_NI fp fp_inv_fermat(const fp& a) { return fp_pow_win3(a, k::WIN_INV, k::WIN_INV_FIRST); }  // 0 -> 0

// ---------------------------------------------------------------------------------------
// Inversion by Bernstein-Yang divsteps ("safegcd", Fast constant-time gcd computation and
// modular inversion, 2019), constant time: a fixed 40 batches of 28 divsteps = 1,120 >= the
// proven bound floor((49 d + 57) / 17) = 1,101 for d = 381 bits (f = p, 0 <= g < p), no
// data-dependent branch, so it is also safe where the input depends on a secret (Sign).
// Each batch runs 28 divsteps on the low 32 bits of (f, g) with the 2x2 transition matrix in
// int32 (|entries| <= 2^28), then applies the matrix to the full signed radix-2^28 f, g
// (exact division by 2^28) and to the cofactors d, e (f = d a, g = e a mod p) with one
// Montgomery-style digit (m = -(u d + v e) p^-1 mod 2^28) so that the division is exact mod p.
// ~30 k instructions against ~376 k issue slots for the 456 products of a^(p-2): the inverse
// sits on the latency-bound G2 chains (SSWU, affine conversions, the final exponentiation).
// ---------------------------------------------------------------------------------------
struct sfp {  // signed radix-2^28 integer: digits 0..12 in [0, 2^28), digit 13 signed
  int32_t v[NL];
};
// (u x + v y) / 2^28 for x, y signed; the low 28 bits of u x + v y must be zero
MBLS_HD sfp sfp_lincomb_shift(const sfp& x, const sfp& y, int32_t u, int32_t v) {
  sfp r;
  int64_t acc = (int64_t)u * x.v[0] + (int64_t)v * y.v[0];
  acc >>= 28;  // exact: the low digit is zero
#pragma unroll
  for (int j = 1; j < NL; ++j) {
    acc += (int64_t)u * x.v[j] + (int64_t)v * y.v[j];
    r.v[j - 1] = (int32_t)((uint32_t)acc & M28);
    acc >>= 28;
  }
  r.v[NL - 1] = (int32_t)acc;
  return r;
}
// (u x + v y + m p) / 2^28 with m chosen so the sum is divisible by 2^28 (x, y signed)
MBLS_HD sfp sfp_lincomb_modp(const sfp& x, const sfp& y, int32_t u, int32_t v) {
  sfp r;
  int64_t acc = (int64_t)u * x.v[0] + (int64_t)v * y.v[0];
  const int64_t m = (int64_t)(((uint32_t)acc * k::N0) & M28);
  acc += m * (int64_t)p_digit(0);
  acc >>= 28;
#pragma unroll
  for (int j = 1; j < NL; ++j) {
    acc += (int64_t)u * x.v[j] + (int64_t)v * y.v[j] + m * (int64_t)p_digit(j);
    r.v[j - 1] = (int32_t)((uint32_t)acc & M28);
    acc >>= 28;
  }
  r.v[NL - 1] = (int32_t)acc;
  return r;
}
MBLS_NI fp fp_inv(const fp& a_mont) {
  const fp a = fp_canon(a_mont);  // 0 <= a < p (0 -> 0, as a^(p-2))
  sfp f, g, d, e;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    f.v[i] = (int32_t)p_digit(i);
    g.v[i] = (int32_t)a.v[i];
    d.v[i] = 0;
    e.v[i] = i == 0 ? 1 : 0;
  }
  int32_t delta = 1;
#pragma unroll 1
  for (int batch = 0; batch < 40; ++batch) {
    uint32_t fl = (uint32_t)f.v[0] | ((uint32_t)f.v[1] << 28), gl = (uint32_t)g.v[0] | ((uint32_t)g.v[1] << 28);
    // 2^i (f_i, g_i) = (u f + v g, q f + r g) on the low bits
    uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
    for (int i = 0; i < 28; ++i) {
      const uint32_t sw = (uint32_t)((-delta) >> 31) & (0u - (gl & 1u));  // delta > 0 and g odd
      const uint32_t tf = fl, tu = u, tv = v;
      fl = sw ? gl : fl;
      gl = sw ? 0u - tf : gl;
      u = sw ? q : u;
      v = sw ? r : v;
      q = sw ? 0u - tu : q;
      r = sw ? 0u - tv : r;
      delta = sw ? -delta : delta;
      const uint32_t odd = 0u - (gl & 1u);
      gl += fl & odd;
      q += u & odd;
      r += v & odd;
      delta += 1;
      gl >>= 1;
      u <<= 1;
      v <<= 1;
    }
    const sfp f2 = sfp_lincomb_shift(f, g, (int32_t)u, (int32_t)v);
    const sfp g2 = sfp_lincomb_shift(f, g, (int32_t)q, (int32_t)r);
    const sfp d2 = sfp_lincomb_modp(d, e, (int32_t)u, (int32_t)v);
    const sfp e2 = sfp_lincomb_modp(d, e, (int32_t)q, (int32_t)r);
    f = f2;
    g = g2;
    d = d2;
    e = e2;
  }
  // f = +-1 now (a != 0), d = f a^-1 with |d| < 41 p: a^-1 = sign(f) d.  Bring it to a
  // non-negative multiple-of-p offset (+ 64 p), normalize the digits, then two Montgomery
  // products by R^2 turn the plain inverse of the Montgomery value a = x R into x^-1 R.
  const bool neg = f.v[NL - 1] < 0;
  constexpr pmul_t P64 = p_times(64);
  int32_t s[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) s[i] = (neg ? -d.v[i] : d.v[i]) + P64.v[i];
  const fp inv_plain = fp_carry(s);  // value in (23 p, 105 p), digits < 2^28
  const fp r2 = fp_from(k::R2);
  return fp_mul(fp_mul(inv_plain, r2), r2);
}

// ---------------------------------------------------------------------------------------
// Byte conversion (big-endian 48-byte field elements as in the ZCash encoding)
// ---------------------------------------------------------------------------------------

// 12 big-endian 32-bit words (already byte-swapped to host order, w[0] most significant)
// -> radix-2^28 digits (plain, not Montgomery).  Top 3 bits of w[0] must be cleared.
MBLS_HD fp fp_from_be_words(const uint32_t (&w)[12]) {
  // little-endian 32-bit limbs
  uint32_t l[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) l[i] = w[11 - i];
  fp r;
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    const int bit = 28 * d;
    const int li = bit >> 5, sh = bit & 31;
    uint64_t x = l[li < 12 ? li : 11] >> sh;
    if (li + 1 < 12 && sh > 4) x |= (uint64_t)l[li + 1] << (32 - sh);
    r.v[d] = (li < 12) ? ((uint32_t)x & M28) : 0u;
  }
  return r;
}

// plain (canonical, < p) digits -> 12 big-endian words
MBLS_HD void fp_to_be_words(const fp& a, uint32_t (&w)[12]) {
  uint32_t l[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int bit = 32 * i;
    const int d = bit / 28, sh = bit % 28;
    uint64_t x = (uint64_t)a.v[d] >> sh;
    if (d + 1 < NL) x |= (uint64_t)a.v[d + 1] << (28 - sh);
    if (d + 2 < NL && sh > 24) x |= (uint64_t)a.v[d + 2] << (56 - sh);
    l[i] = (uint32_t)x;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) w[i] = l[11 - i];
}

// plain value comparisons
MBLS_HD bool fp_raw_lt_p(const fp& a) {
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) br = ((int32_t)a.v[i] - (int32_t)k::P_RAW[i] + br) >> 28;
  return br != 0;
}
// a (plain, canonical) > (p-1)/2 ?
MBLS_HD bool fp_raw_gt_half(const fp& a) {
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) br = ((int32_t)k::HALF_P_RAW[i] - (int32_t)a.v[i] + br) >> 28;
  return br != 0;
}
MBLS_HD bool fp_raw_is_zero(const fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) acc |= a.v[i];
  return acc == 0;
}

}  // namespace mbls
