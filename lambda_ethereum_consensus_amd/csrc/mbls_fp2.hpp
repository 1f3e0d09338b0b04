// mbls_fp2.hpp — Fp2 = Fp[u]/(u^2 + 1) on top of the radix-2^28 Fp.
// Replaces blst's *_fp2 routines (mul_fp2, sqr_fp2, sqrt_fp2, reciprocal_fp2); re-derived.
#pragma once
#include "mbls_fp.hpp"

namespace mbls {

struct fp2 {
  fp c0, c1;
};

MBLS_HD fp2 fp2_from(const uint32_t (&a)[NL], const uint32_t (&b)[NL]) { return {fp_from(a), fp_from(b)}; }
MBLS_HD fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
MBLS_HD fp2 fp2_one() { return {fp_one(), fp_zero()}; }

MBLS_HD fp2 fp2_add(const fp2& a, const fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
MBLS_HD fp2 fp2_sub(const fp2& a, const fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
MBLS_HD fp2 fp2_dbl(const fp2& a) { return {fp_dbl(a.c0), fp_dbl(a.c1)}; }
MBLS_HD fp2 fp2_neg(const fp2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
MBLS_HD fp2 fp2_conj(const fp2& a) { return {a.c0, fp_neg(a.c1)}; }

// Schoolbook with one reduction per coefficient (fp_mul2_inl):
//   (a0 b0 + a1 (4p - b1)) + (a0 b1 + a1 b0) u
// Same multiply-adds as Karatsuba's three products and no normalized additions: ~26% fewer
// instructions per Fp2 product.  Sums: a0 b0 + a1 (4p - b1) < 12 p^2, a0 b1 + a1 b0 < 8 p^2.
MBLS_HD fp2 fp2_mul(const fp2& a, const fp2& b) {
  return {fp_mul2(a.c0, b.c0, a.c1, fp_neg_lazy(b.c1)), fp_mul2(a.c0, b.c1, a.c1, b.c0)};
}
// (a0 + a1)(a0 - a1) + 2 a0 a1 u; a0 - a1 as a0 - a1 + 4p (< 6p): (4p)(6p) < p R
MBLS_HD fp2 fp2_sqr(const fp2& a) {
  const fp t0 = fp_mul(fp_add_lazy(a.c0, a.c1), fp_sub_lazy(a.c0, a.c1));
  const fp t1 = fp_mul(fp_add_lazy(a.c0, a.c0), a.c1);
  return {t0, t1};
}
// Lazy sums of Fp2 products (mbls_fp.hpp fpcols): re/im += a b, or a b xi when `xi` (a
// select, so lanes may differ).  Schoolbook over Fp with the signs folded into the second
// operand (residues mod p: -b1 as 2p - b1), so every column term is a non-negative mad:
//   a b    = (a0 b0 + a1 (-b1))        + (a0 b1 + a1 b0) u
//   a b xi = (a0 (b0 - b1) + a1 (-(b0 + b1))) + (a0 (b0 + b1) + a1 (b0 - b1)) u
// a, b normalized (digits < 2^28); at most 6 calls per accumulator pair (12 products each).
MBLS_HD void fp2_cols_mad(fpcols& re, fpcols& im, const fp2& a, const fp2& b, bool xi) {
  const fp s = fp_add(b.c0, b.c1), d = fp_sub(b.c0, b.c1);
  const fp r0 = fp_select(xi, d, b.c0), r1 = fp_neg(fp_select(xi, s, b.c1));
  const fp i0 = fp_select(xi, s, b.c1), i1 = fp_select(xi, d, b.c0);
  cols_mad(re, a.c0, r0);
  cols_mad(re, a.c1, r1);
  cols_mad(im, a.c0, i0);
  cols_mad(im, a.c1, i1);
}
MBLS_HD fp2 fp2_cols_redc(const fpcols& re, const fpcols& im) { return {cols_redc(re), cols_redc(im)}; }

MBLS_HD fp2 fp2_mul_fp(const fp2& a, const fp& s) { return {fp_mul(a.c0, s), fp_mul(a.c1, s)}; }
// times xi = 1 + u: (a0 - a1) + (a0 + a1) u
MBLS_HD fp2 fp2_mul_xi(const fp2& a) { return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }
// times u: -a1 + a0 u
MBLS_HD fp2 fp2_mul_u(const fp2& a) { return {fp_neg(a.c1), a.c0}; }
MBLS_HD fp2 fp2_mul3(const fp2& a) { return {fp_mul3(a.c0), fp_mul3(a.c1)}; }

MBLS_HD bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
MBLS_HD bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
MBLS_HD fp2 fp2_select(bool c, const fp2& a, const fp2& b) { return {fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)}; }
MBLS_HD fp2 fp2_canon(const fp2& a) { return {fp_canon(a.c0), fp_canon(a.c1)}; }

MBLS_HD fp fp2_norm(const fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

// 1/(a0 + a1 u) = (a0 - a1 u) / (a0^2 + a1^2); 0 -> 0
MBLS_NI fp2 fp2_inv(const fp2& a) {
  const fp t = fp_inv(fp2_norm(a));
  return {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
}

template <int NW>
MBLS_HD fp2 fp2_pow_words(const fp2& a, const uint32_t (&e)[NW]) {
  fp2 r = a;
  int top = 31;
  while (top > 0 && !((e[NW - 1] >> top) & 1u)) --top;
#pragma unroll 1
  for (int w = NW - 1; w >= 0; --w) {
    const uint32_t word = e[w];
    const int start = (w == NW - 1) ? top - 1 : 31;
#pragma unroll 1
    for (int b = start; b >= 0; --b) {
      r = fp2_sqr(r);
      if ((word >> b) & 1u) r = fp2_mul(r, a);
    }
  }
  return r;
}

// Fp: a^((p-3)/4).  For a QR a != 0: t^2 a = 1 and sqrt(a) = t a.
MBLS_NI fp fp_pm3_4(const fp& a) { return fp_pow_win3(a, k::WIN_PM3_4, k::WIN_PM3_4_FIRST); }

// Fp square root (p = 3 mod 4): a^((p+1)/4).  Returns true and r with r^2 = a if a is a
// square.  Inline form for the key kernel, out-of-line form for everyone else.
MBLS_HD bool fp_sqrt_inl(fp& r, const fp& a) {
  r = fp_pow_win4(a, k::WIN4_SQRT, k::WIN4_SQRT_FIRST);
  return fp_eq(fp_sqr(r), a);
}
MBLS_NI bool fp_sqrt(fp& r, const fp& a) { return fp_sqrt_inl(r, a); }

// Fp2 square root through the norm (p = 3 mod 4).  gamma = sqrt(a0^2 + a1^2) in Fp (the one
// exponentiation that also decides whether a is a square), delta = (a0 + gamma) / 2,
// t = delta^((p-3)/4): if delta is a residue (t^2 delta = 1) a root is (t delta, a1 t / 2),
// otherwise (t^2 delta = -1) it is (-a1 t / 2, t delta) -- both satisfy x0^2 - x1^2 = a0 and
// 2 x0 x1 = a1 given gamma^2 = a0^2 + a1^2.  So a second exponentiation for (a0 - gamma) / 2
// is never needed (before: taken by a wave whenever any of its lanes needed it).  a1 = 0 uses
// gamma = a0 (delta = a0: a non-residue a0 then gives (0, sqrt(-a0))).  Any root is fine: the
// callers fix the sign from the encoding flag / sgn0.  `gamma` may come from elsewhere (the
// SSWU map derives g(x2)'s from g(x1)'s, mbls_h2c.hpp).
MBLS_HD fp2 fp2_sqrt_from_gamma(const fp2& a, const fp& gamma_in) {
  const fp inv2 = fp_from(k::INV2);
  const fp gamma = fp_select(fp_is_zero(a.c1), a.c0, gamma_in);
  const fp delta = fp_mul(fp_add(a.c0, gamma), inv2);
  const fp t = fp_pm3_4(delta);
  const fp td = fp_mul(t, delta);
  const bool qr = fp_eq(fp_mul(t, td), fp_one());
  const fp h = fp_mul(fp_mul(a.c1, t), inv2);  // a1 t / 2
  return {fp_select(qr, td, fp_neg(h)), fp_select(qr, h, td)};
}
// The same root of a = U / e (U in Fp2, e in Fp, e != 0) without inverting e: with
// gamma' = gamma e (gamma'^2 = norm(U)) and d' = (U0 + gamma') / 2 = delta e, one exponentiation
// T = (d' e)^((p-3)/4) gives chi = T^2 d' e = +-1, (d' T)^2 = chi delta and
// 1 / (e d' T) = chi T, so the two cases above become (d' T, U1 T / 2) and (-U1 T / 2, d' T).
// Two Fp products more than fp2_sqrt_from_gamma, one inversion less for the SSWU map.
MBLS_HD fp2 fp2_sqrt_ratio_from_gamma(const fp2& u, const fp& e, const fp& gamma_in) {
  const fp inv2 = fp_from(k::INV2);
  const fp gamma = fp_select(fp_is_zero(u.c1), u.c0, gamma_in);
  const fp d = fp_mul(fp_add(u.c0, gamma), inv2);
  const fp t = fp_pm3_4(fp_mul(d, e));
  const fp td = fp_mul(t, d);
  const bool qr = fp_eq(fp_mul(fp_mul(t, td), e), fp_one());
  const fp h = fp_mul(fp_mul(u.c1, t), inv2);  // U1 T / 2
  return {fp_select(qr, td, fp_neg(h)), fp_select(qr, h, td)};
}
MBLS_NI bool fp2_sqrt(fp2& r, const fp2& a) {
  fp gamma;
  const bool sq = fp_sqrt(gamma, fp2_norm(a));  // a is a square iff its norm is
  r = fp2_sqrt_from_gamma(a, gamma);
  return sq && fp2_eq(fp2_sqr(r), a);
}

// a is a square in Fp2 iff its norm is a square in Fp (Legendre symbol via exponent).
MBLS_NI bool fp2_is_square(const fp2& a) {
  const fp n = fp2_norm(a);
  const fp l = fp_pow_win3(n, k::WIN_LEGENDRE, k::WIN_LEGENDRE_FIRST);
  return fp_is_zero(n) || fp_eq(l, fp_one());
}

// RFC 9380 sgn0 for Fp2 (on canonical plain values)
MBLS_HD uint32_t fp2_sgn0(const fp2& a) {
  const fp x0 = fp_from_mont(a.c0), x1 = fp_from_mont(a.c1);
  const uint32_t s0 = x0.v[0] & 1u;
  const uint32_t z0 = fp_raw_is_zero(x0) ? 1u : 0u;
  const uint32_t s1 = x1.v[0] & 1u;
  return s0 | (z0 & s1);
}

// ZCash / blst G2 y-sign flag: im != 0 ? im > (p-1)/2 : re > (p-1)/2
MBLS_HD bool fp2_sgn_zcash(const fp2& a) {
  const fp x0 = fp_from_mont(a.c0), x1 = fp_from_mont(a.c1);
  return fp_raw_is_zero(x1) ? fp_raw_gt_half(x0) : fp_raw_gt_half(x1);
}

}  // namespace mbls
