// mbls_lazy.hpp — lazily reduced Fp / Fp2 values with compile-time bounds, for the G2 and
// pairing formulas.
//
// Why: in those formulas a normalized addition (carry pass + conditional subtraction of 2p +
// select, ~112 instructions per Fp) costs a fifth of a Montgomery product, and a G2 / Fp12 step
// has dozens of them — they were about half of the lane-group Miller loop's instructions and a
// third of the one-lane pairing's (profiles/r02_isa_mix.txt).  Here a sum or difference is one
// digit-wise pass plus a ONE-SHOT carry (every digit's overflow moved up one digit in parallel,
// no serial chain), and its value is only bounded, not reduced: it may exceed 2p.  Such values
// feed multiplications (which accept them and return normalized values) or further lazy ops;
// `reduce` brings one back below 2p in ~70 instructions when a formula's output must be
// normalized.
//
// Safety by construction: `lz<B>` / `lz2<B>` carry the bound B (value < B p per coefficient) in
// the type; every operation computes its result's bound at compile time and the products
// static_assert that the Montgomery reduction's input stays below p R (R / p > 2^11.3, budget
// 2400 p^2).  Digits of a lazy value are < 2^28 + 16 (one-shot carry of sums of a few digits).
//
// Replaces the add_mod / sub_mod / mul_by_3 / mul_by_8 / mul_by_b chains inside blst's G2 and
// Fp12 formulas (reached from lighthouse verify / aggregate_verify, native/bls_nif/src/lib.rs);
// re-derived.
#pragma once
#include "mbls_fp2.hpp"

namespace mbls {

// ---- big-digit multiples of p -----------------------------------------------------------
// K p with every digit raised so that a + KPB - b never borrows for b with digits < 2^28 + 16
// and value < (K - 1) p: d_0 = n_0 + 2^29, d_i = n_i + 2^29 - 2 (0 < i < 13), d_13 = n_13 - 2,
// n the digits of K p (the added terms telescope to 0).  Digits < 2^30.
constexpr pbig_t pk_big(uint32_t K) {
  pbig_t r{};
  uint64_t c = 0;
  uint32_t n[NL] = {};
  for (int i = 0; i < NL; ++i) {
    const uint64_t x = (uint64_t)k::P_RAW[i] * K + c;
    n[i] = (uint32_t)(x & M28);
    c = x >> 28;
  }
  for (int i = 0; i < NL; ++i)
    r.v[i] = i == 0 ? n[i] + (1u << 29) : i < NL - 1 ? n[i] + (1u << 29) - 2u : n[i] - 2u;
  return r;
}
template <int K>
struct PKB {
  static constexpr pbig_t v = pk_big(K);
};

// one-shot carry: digit i keeps its low 28 bits plus digit i-1's overflow (all digits in
// parallel); the top digit keeps everything.  Input digits < 2^32, output digits < 2^28 + 16.
MBLS_HD fp fp_cn(const fp& s) {
  fp r;
  r.v[0] = s.v[0] & M28;
#pragma unroll
  for (int i = 1; i < NL - 1; ++i) r.v[i] = (s.v[i] & M28) + (s.v[i - 1] >> 28);
  r.v[NL - 1] = s.v[NL - 1] + (s.v[NL - 2] >> 28);
  return r;
}

// a mod p reduced to [0, 2p) for a lazy value (digits < 2^28 + 16, value < 2400 p): subtract
// q p with q = floor(a_13 / (floor(p / 2^364) + 1)) <= a / p, so the result is >= 0 and
// < p + 2 * 2^364 + a_13 * 2^364 / P' < 2p (P' = p / 2^364 ~ 1.07e5).  Digit-wise in 64 bits
// (a_i - q p_i), then a signed carry pass.
MBLS_HD fp fp_reduce(const fp& a) {
  constexpr uint32_t PT = k::P_RAW[NL - 1] + 1u;  // floor(p / 2^364) + 1 (p's low digits are nonzero)
  const uint32_t q = a.v[NL - 1] / PT;             // constant divisor: a multiply-shift
  fp r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    const int64_t y = (int64_t)a.v[i] - (int64_t)q * (int64_t)k::P_RAW[i] + c;
    r.v[i] = (uint32_t)y & M28;
    c = y >> 28;  // arithmetic: floor
  }
  // the value is in [0, 2p): the top digit is what remains, non-negative and < 2^18
  r.v[NL - 1] = (uint32_t)((int64_t)a.v[NL - 1] - (int64_t)q * (int64_t)k::P_RAW[NL - 1] + c);
  return r;
}

// Sum of N Montgomery products with ONE reduction, (sum_j a_j b_j) R^-1 mod p in [0, 2p):
// a_j digits < 2^28 + 16, b_j digits < 2^30, sum < 2400 p^2.  N <= 3: a column holds at most
// 14 N products < 2^58 + 14 reduction terms < 2^56 + the carry, < 2^64.
template <int N>
MBLS_HD fp fp_muln_inl(const fp (&a)[N], const fp (&b)[N]) {
  static_assert(N >= 1 && N <= 3, "column bound");
  uint32_t m[NL];
  fp t;
  uint64_t acc = 0;
#pragma unroll
  for (int kk = 0; kk < 2 * NL - 1; ++kk) {
    uint64_t s0 = acc, s1 = 0, s2 = 0;
    const int lo = kk < NL ? 0 : kk - NL + 1, hi = kk < NL ? kk : NL - 1;
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int i = lo; i <= hi; ++i) {
        if (j == 1) s1 += (uint64_t)a[j].v[i] * b[j].v[kk - i];
        else s0 += (uint64_t)a[j].v[i] * b[j].v[kk - i];
      }
#pragma unroll
    for (int i = (kk < NL ? 0 : kk - NL + 1); i < (kk < NL ? kk : NL); ++i) s2 += (uint64_t)m[i] * p_digit(kk - i);
    uint64_t s = s0 + s1 + s2;
    if (kk < NL) {
      m[kk] = ((uint32_t)s * k::N0) & M28;
      s += (uint64_t)m[kk] * p_digit(0);
      acc = s >> 28;
    } else {
      t.v[kk - NL] = (uint32_t)s & M28;
      acc = s >> 28;
    }
  }
  t.v[NL - 1] = (uint32_t)acc;
  return t;
}

template <int B>
struct lz {
  fp v;
  static constexpr int bound = B;
};
template <int B>
struct lz2 {
  fp2 v;
  static constexpr int bound = B;
};
using nz = lz<2>;
using nz2 = lz2<2>;

MBLS_HD nz2 nrm(const fp2& a) { return {a}; }  // a normalized value (< 2p)
MBLS_HD nz nrm(const fp& a) { return {a}; }

// ---- Fp -----------------------------------------------------------------------------------
template <int A, int C>
MBLS_HD lz<A + C> operator+(const lz<A>& a, const lz<C>& b) {
  static_assert(A + C <= 4096, "bound");
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v.v[i] + b.v.v[i];
  return {fp_cn(s)};
}
template <int C>
constexpr int ksub() {
  int k = 2;
  while (k <= C) k *= 2;
  return k;
}
template <int A, int C>
MBLS_HD lz<A + ksub<C>()> operator-(const lz<A>& a, const lz<C>& b) {
  constexpr int K = ksub<C>();
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v.v[i] + PKB<K>::v.v[i] - b.v.v[i];
  return {fp_cn(s)};
}
template <int C>
MBLS_HD lz<ksub<C>()> neg(const lz<C>& b) {
  constexpr int K = ksub<C>();
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = PKB<K>::v.v[i] - b.v.v[i];
  return {fp_cn(s)};
}
// small constant multiple (c <= 12: digits (2^28 + 16) c < 2^32)
template <int c, int A>
MBLS_HD lz<c * A> smul(const lz<A>& a) {
  static_assert(c >= 1 && c <= 12, "small constant");
  fp s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v.v[i] * (uint32_t)c;
  return {fp_cn(s)};
}
template <int A>
MBLS_HD nz reduce(const lz<A>& a) {
  static_assert(A <= 2400, "reduce bound");
  return {fp_reduce(a.v)};
}
template <int A, int C>
MBLS_HD nz mul(const lz<A>& a, const lz<C>& b) {
  static_assert(A * C <= 2400, "Montgomery input bound");
  return {fp_mul(a.v, b.v)};
}

// ---- Fp2 ----------------------------------------------------------------------------------
template <int A, int C>
MBLS_HD lz2<A + C> operator+(const lz2<A>& a, const lz2<C>& b) {
  const lz<A> a0{a.v.c0}, a1{a.v.c1};
  const lz<C> b0{b.v.c0}, b1{b.v.c1};
  return {{(a0 + b0).v, (a1 + b1).v}};
}
template <int A, int C>
MBLS_HD lz2<A + ksub<C>()> operator-(const lz2<A>& a, const lz2<C>& b) {
  const lz<A> a0{a.v.c0}, a1{a.v.c1};
  const lz<C> b0{b.v.c0}, b1{b.v.c1};
  return {{(a0 - b0).v, (a1 - b1).v}};
}
template <int C>
MBLS_HD lz2<ksub<C>()> neg(const lz2<C>& b) {
  return {{neg(lz<C>{b.v.c0}).v, neg(lz<C>{b.v.c1}).v}};
}
template <int c, int A>
MBLS_HD lz2<c * A> smul(const lz2<A>& a) {
  return {{smul<c>(lz<A>{a.v.c0}).v, smul<c>(lz<A>{a.v.c1}).v}};
}
// times xi = 1 + u: (a0 - a1, a0 + a1)
template <int A>
MBLS_HD lz2<A + ksub<A>()> mul_xi(const lz2<A>& a) {
  const lz<A> a0{a.v.c0}, a1{a.v.c1};
  return {{(a0 - a1).v, (a0 + a1).v}};
}
// times 3b' = 12 xi (the G2 curve constant of the RCB formulas)
template <int A>
MBLS_HD lz2<12 * (A + ksub<A>())> mul_b3(const lz2<A>& a) {
  return smul<12>(mul_xi(a));
}
template <int A>
MBLS_HD nz2 reduce(const lz2<A>& a) {
  static_assert(A <= 2400, "reduce bound");
  return {{fp_reduce(a.v.c0), fp_reduce(a.v.c1)}};
}
template <int A>
MBLS_HD lz2<A> sel(bool c, const lz2<A>& a, const lz2<A>& b) {
  return {fp2_select(c, a.v, b.v)};
}
template <int A, int C>
MBLS_HD lz2<(A > C ? A : C)> sel(bool c, const lz2<A>& a, const lz2<C>& b) {
  return {fp2_select(c, a.v, b.v)};
}
// widen the bound (free): makes two values selectable / summable into one type
template <int W, int A>
MBLS_HD lz2<W> widen(const lz2<A>& a) {
  static_assert(W >= A, "widen");
  return {a.v};
}

// Fp2 product of lazy operands: (a0 b0 + a1 (32p - b1)) + (a0 b1 + a1 b0) u, one reduction
// per coefficient (fp_mul2).  Bound: A (C + 32) p^2 <= 2400 p^2; b1 < 31 p for the raised 32p.
template <int A, int C>
MBLS_HD nz2 mul(const lz2<A>& a, const lz2<C>& b) {
  static_assert(C < 32 && A * (C + 32) <= 2400, "Fp2 product bound");
  fp nb1;
#pragma unroll
  for (int i = 0; i < NL; ++i) nb1.v[i] = PKB<32>::v.v[i] - b.v.c1.v[i];  // digits < 2^30
  return {{fp_mul2(a.v.c0, b.v.c0, a.v.c1, nb1), fp_mul2(a.v.c0, b.v.c1, a.v.c1, b.v.c0)}};
}
// (a0 + a1)(a0 - a1 + K p) + 2 a0 a1 u
template <int A>
MBLS_HD nz2 sqr(const lz2<A>& a) {
  constexpr int K = ksub<A>();
  static_assert(2 * A * (A + K) <= 2400, "Fp2 square bound");
  fp s, d, a2;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    s.v[i] = a.v.c0.v[i] + a.v.c1.v[i];                      // digits < 2^29 + 32
    d.v[i] = a.v.c0.v[i] + PKB<K>::v.v[i] - a.v.c1.v[i];     // digits < 2^30 + 2^28 + 16
    a2.v[i] = a.v.c0.v[i] << 1;                              // digits < 2^29 + 32
  }
  return {{fp_mul(s, fp_cn(d)), fp_mul(a2, a.v.c1)}};
}
// Fp2 times an Fp value
template <int A, int C>
MBLS_HD nz2 mul(const lz2<A>& a, const lz<C>& s) {
  static_assert(A * C <= 2400, "bound");
  return {{fp_mul(a.v.c0, s.v), fp_mul(a.v.c1, s.v)}};
}

// value / 2 for a lazy value (odd: + p first): < (A + 1) p / 2
template <int A>
MBLS_HD lz2<(A + 2) / 2> half(const lz2<A>& a) {
  auto h = [](const fp& x) {
    const uint32_t odd = x.v[0] & 1u;
    fp t;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const uint32_t y = x.v[i] + (odd ? k::P_RAW[i] : 0u) + c;
      c = y >> 28;
      t.v[i] = y & M28;
    }
    t.v[NL - 1] |= c << 28;  // value < 2^392: the top digit holds the rest
    fp r;
#pragma unroll
    for (int i = 0; i < NL - 1; ++i) r.v[i] = (t.v[i] >> 1) | ((t.v[i + 1] & 1u) << 27);
    r.v[NL - 1] = t.v[NL - 1] >> 1;
    return r;
  };
  return {{h(a.v.c0), h(a.v.c1)}};
}

// Lazy sums of Fp2 products (fpcols, reduced once by fp2_cols_redc): re/im += a b, or a b xi
// when `xi`.  Signs and the twist are folded into the second operand as lazy values:
//   a b    = (a0 b0 + a1 (-b1))               + (a0 b1 + a1 b0) u
//   a b xi = (a0 (b0 - b1) + a1 (-(b0 + b1))) + (a0 (b0 + b1) + a1 (b0 - b1)) u
// b normalized: the folded operands are < 8p, so 6 calls with a < A p add < 6 * 2 * 8 A p^2 to
// an accumulator pair (the reduction needs < 2400 p^2: A <= 25); digits < 2^28 + 16 keep 12
// products + 14 reduction terms per column < 2^64.
template <int A>
MBLS_HD void cols_mad2(fpcols& re, fpcols& im, const lz2<A>& a, const nz2& b, bool xi) {
  static_assert(6 * 2 * 8 * A <= 2400, "lazy column sum bound");
  const lz<2> b0{b.v.c0}, b1{b.v.c1};
  const lz<4> s = b0 + b1;
  const lz<6> d = b0 - b1;
  const fp r0 = fp_select(xi, d.v, b0.v), r1 = neg(lz<4>{fp_select(xi, s.v, b1.v)}).v;
  const fp i0 = fp_select(xi, s.v, b1.v), i1 = fp_select(xi, d.v, b0.v);
  cols_mad(re, a.v.c0, r0);
  cols_mad(re, a.v.c1, r1);
  cols_mad(im, a.v.c0, i0);
  cols_mad(im, a.v.c1, i1);
}

}  // namespace mbls
