// mbls_pairing.hpp — Fp6/Fp12 tower, optimal-ate Miller loop and final exponentiation.
//
// Fp6 = Fp2[v]/(v^3 - (1+u)), Fp12 = Fp6[w]/(w^2 - v); coefficient (i, j) of
// fp12{c_i}.c_j multiplies w^(2j+i).  Replaces blst's miller_loop_n / final_exp (reached
// from lighthouse verify / fast_aggregate_verify / aggregate_verify,
// native/bls_nif/src/lib.rs:59,81,99,118); re-derived:
//  * T kept in homogeneous projective coordinates on the M-type twist; lines scaled by
//    Fp2 factors (killed by the final exponentiation) into the sparse shape
//    c0 + (c2 x_P) w^2 + (c3 y_P) w^3, multiplied in with a 13-Fp2-mul sparse product.
//  * final exponentiation: easy part (p^6-1)(p^2+1), hard part by Hayashida–Hayasaka–
//    Teruya: 3(p^4-p^2+1)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3, i.e. the result is the cube of
//    the reduced pairing — verdicts ("== 1") are unchanged since gcd(3, r) = 1.
#pragma once
#include "mbls_curve.hpp"

namespace mbls {

// Call boundaries of the Miller steps (T passed by reference, the line returned in memory)
// and of the cyclotomic squaring: inlined into the loops by default (T / f stay in registers).
// Measured r01 (profiles/r01_pipeline_experiments.txt): gossip 916k -> 987k verify/s,
// deposit AV 116k -> 125k sets/s, cold / warm epoch unchanged.
// the Miller loop's Fp12 squaring and sparse line product: inlined too (gossip 992k -> 1023k
// verify/s, deposit AV 122.6k -> 128.1k sets/s, r01)
// Fp6 / Fp12 general products stay out of line: inlining them measured gossip +1.8%, deposit
// AV +1.2% (r01) for a 6x longer build of the one-lane translation unit (~6 min).
// fp12_mul stays a call: inlining it alone grew the one-lane verdict's
// scratch past what three queues can hold resident and the cold epoch fell to 16-17k sets/s
// (gossip 1.02M -> 0.64M), r01.
#define MBLS_MSTEP_FN __host__ __device__ __forceinline__
#define MBLS_CYC_FN __host__ __device__ __forceinline__
#define MBLS_F12_FN __host__ __device__ __forceinline__
#define MBLS_F12M_FN MBLS_NI
#define MBLS_F6_FN MBLS_NI

struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

MBLS_HD fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }
MBLS_HD fp6 fp6_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }
MBLS_HD fp6 fp6_add(const fp6& a, const fp6& b) { return {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
MBLS_HD fp6 fp6_sub(const fp6& a, const fp6& b) { return {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
MBLS_HD fp6 fp6_neg(const fp6& a) { return {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
// times v: (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2
MBLS_HD fp6 fp6_mul_v(const fp6& a) { return {fp2_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba over Fp2 with the sums and differences lazily reduced (mbls_lazy.hpp): each
// coefficient is reduced once at the end
MBLS_F6_FN fp6 fp6_mul(const fp6& a, const fp6& b) {
  const nz2 a0 = nrm(a.c0), a1 = nrm(a.c1), a2 = nrm(a.c2), b0 = nrm(b.c0), b1 = nrm(b.c1), b2 = nrm(b.c2);
  const nz2 t0 = mul(a0, b0), t1 = mul(a1, b1), t2 = mul(a2, b2);
  const fp2 c0 = reduce(t0 + mul_xi(mul(a1 + a2, b1 + b2) - (t1 + t2))).v;
  const fp2 c1 = reduce(mul(a0 + a1, b0 + b1) - (t0 + t1) + mul_xi(t2)).v;
  const fp2 c2 = reduce(mul(a0 + a2, b0 + b2) - (t0 + t2) + t1).v;
  return {c0, c1, c2};
}
// Chung–Hasan SQR2
MBLS_NI fp6 fp6_sqr(const fp6& a) {
  const fp2 s0 = fp2_sqr(a.c0);
  const fp2 s1 = fp2_dbl(fp2_mul(a.c0, a.c1));
  const fp2 s2 = fp2_sqr(fp2_add(fp2_sub(a.c0, a.c1), a.c2));
  const fp2 s3 = fp2_dbl(fp2_mul(a.c1, a.c2));
  const fp2 s4 = fp2_sqr(a.c2);
  return {fp2_add(s0, fp2_mul_xi(s3)), fp2_add(s1, fp2_mul_xi(s4)), fp2_sub(fp2_add(fp2_add(s1, s2), s3), fp2_add(s0, s4))};
}
MBLS_NI fp6 fp6_inv(const fp6& a) {
  const fp2 c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  const fp2 c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  const fp2 c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  const fp2 t = fp2_add(fp2_mul(a.c0, c0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2))));
  const fp2 ti = fp2_inv(t);
  return {fp2_mul(c0, ti), fp2_mul(c1, ti), fp2_mul(c2, ti)};
}

MBLS_HD fp12 fp12_one() { return {fp6_one(), fp6_zero()}; }
// Fp6 product of lazy operands (< A p) with lazy, unreduced outputs, so the Fp12 products can
// combine three of them before one reduction per coefficient (mbls_lazy.hpp)
struct lz6 {
  lz2<28> c0;
  lz2<16> c1;
  lz2<12> c2;
};
template <int A>
MBLS_HD lz6 fp6_mul_lz(const lz2<A>& a0, const lz2<A>& a1, const lz2<A>& a2, const lz2<A>& b0, const lz2<A>& b1,
                       const lz2<A>& b2) {
  const nz2 t0 = mul(a0, b0), t1 = mul(a1, b1), t2 = mul(a2, b2);
  return {t0 + mul_xi(mul(a1 + a2, b1 + b2) - (t1 + t2)), mul(a0 + a1, b0 + b1) - (t0 + t1) + mul_xi(t2),
          mul(a0 + a2, b0 + b2) - (t0 + t2) + t1};
}
template <int A>
MBLS_HD lz6 fp6_mul_lz(const lz2<A> (&a)[3], const lz2<A> (&b)[3]) {
  return fp6_mul_lz(a[0], a[1], a[2], b[0], b[1], b[2]);
}
// (a0 + a1 w)(b0 + b1 w) = (t0 + v t1) + ((a0 + a1)(b0 + b1) - t0 - t1) w (Karatsuba over Fp6)
MBLS_F12M_FN fp12 fp12_mul(const fp12& a, const fp12& b) {
  const nz2 A0[3] = {nrm(a.c0.c0), nrm(a.c0.c1), nrm(a.c0.c2)}, A1[3] = {nrm(a.c1.c0), nrm(a.c1.c1), nrm(a.c1.c2)};
  const nz2 B0[3] = {nrm(b.c0.c0), nrm(b.c0.c1), nrm(b.c0.c2)}, B1[3] = {nrm(b.c1.c0), nrm(b.c1.c1), nrm(b.c1.c2)};
  const lz6 t0 = fp6_mul_lz(A0, B0), t1 = fp6_mul_lz(A1, B1);
  const lz2<4> AS[3] = {A0[0] + A1[0], A0[1] + A1[1], A0[2] + A1[2]}, BS[3] = {B0[0] + B1[0], B0[1] + B1[1], B0[2] + B1[2]};
  const lz6 s = fp6_mul_lz(AS, BS);
  return {{reduce(t0.c0 + mul_xi(t1.c2)).v, reduce(t0.c1 + t1.c0).v, reduce(t0.c2 + t1.c1).v},
          {reduce(s.c0 - t0.c0 - t1.c0).v, reduce(s.c1 - t0.c1 - t1.c1).v, reduce(s.c2 - t0.c2 - t1.c2).v}};
}
// complex squaring: (a0 + a1 w)^2 = (a0 + a1)(a0 + v a1) - t - v t + 2 t w,  t = a0 a1
MBLS_F12_FN fp12 fp12_sqr(const fp12& a) {
  const nz2 A0[3] = {nrm(a.c0.c0), nrm(a.c0.c1), nrm(a.c0.c2)}, A1[3] = {nrm(a.c1.c0), nrm(a.c1.c1), nrm(a.c1.c2)};
  const lz6 t = fp6_mul_lz(A0, A1);
  // a0 + a1 and a0 + v a1 (v (x0, x1, x2) = (xi x2, x0, x1)), both widened to one bound
  const lz2<8> S[3] = {widen<8>(A0[0] + A1[0]), widen<8>(A0[1] + A1[1]), widen<8>(A0[2] + A1[2])};
  const lz2<8> V[3] = {A0[0] + mul_xi(A1[2]), widen<8>(A0[1] + A1[0]), widen<8>(A0[2] + A1[1])};
  const lz6 s = fp6_mul_lz(S, V);
  return {{reduce(s.c0 - t.c0 - mul_xi(t.c2)).v, reduce(s.c1 - t.c1 - t.c0).v, reduce(s.c2 - t.c2 - t.c1).v},
          {reduce(smul<2>(t.c0)).v, reduce(smul<2>(t.c1)).v, reduce(smul<2>(t.c2)).v}};
}
MBLS_HD fp12 fp12_conj(const fp12& a) { return {a.c0, fp6_neg(a.c1)}; }
MBLS_NI fp12 fp12_inv(const fp12& a) {
  const fp6 t = fp6_inv(fp6_sub(fp6_sqr(a.c0), fp6_mul_v(fp6_sqr(a.c1))));
  return {fp6_mul(a.c0, t), fp6_neg(fp6_mul(a.c1, t))};
}
MBLS_NI bool fp12_is_one(const fp12& a) {
  return fp2_eq(a.c0.c0, fp2_one()) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}

// Frobenius x -> x^(p^e): coefficient of w^k becomes conj^e(c) * gamma_e[k]
#define MBLS_G(e, kk) fp2_from(k::FROB##e##_##kk##_C0, k::FROB##e##_##kk##_C1)
MBLS_NI fp12 fp12_frob(const fp12& a) {
  return {{fp2_conj(a.c0.c0), fp2_mul(fp2_conj(a.c0.c1), MBLS_G(1, 2)), fp2_mul(fp2_conj(a.c0.c2), MBLS_G(1, 4))},
          {fp2_mul(fp2_conj(a.c1.c0), MBLS_G(1, 1)), fp2_mul(fp2_conj(a.c1.c1), MBLS_G(1, 3)),
           fp2_mul(fp2_conj(a.c1.c2), MBLS_G(1, 5))}};
}
MBLS_NI fp12 fp12_frob2(const fp12& a) {
  return {{a.c0.c0, fp2_mul(a.c0.c1, MBLS_G(2, 2)), fp2_mul(a.c0.c2, MBLS_G(2, 4))},
          {fp2_mul(a.c1.c0, MBLS_G(2, 1)), fp2_mul(a.c1.c1, MBLS_G(2, 3)), fp2_mul(a.c1.c2, MBLS_G(2, 5))}};
}
#undef MBLS_G

// (a + b t)^2 in Fp4 = Fp2[t]/(t^2 - xi): (a^2 + xi b^2, 2ab = (a + b)^2 - a^2 - b^2), lazy
MBLS_HD void fp4_sqr(lz2<8>& c0, lz2<10>& c1, const nz2& a, const nz2& b) {
  const nz2 t0 = sqr(a), t1 = sqr(b);
  c0 = mul_xi(t1) + t0;
  c1 = sqr(a + b) - (t0 + t1);
}

// Squaring in the cyclotomic subgroup (Granger–Scott 2010): view Fp12 as Fp4[w]/(w^3 - t),
// t = w^3, f = A + B w + C w^2 with A = c(w^0) + c(w^3) t, B = c(w^1) + c(w^4) t,
// C = c(w^2) + c(w^5) t; then f^2 = (3A^2 - 2conj A) + (3t C^2 + 2conj B) w + (3B^2 - 2conj C) w^2.
// 9 Fp2 squarings instead of the generic 2 Fp6 products; every output coefficient is one
// lazy combination 3 s +- 2 z, reduced once.  Valid only for f^(p^6+1)... = 1, i.e. after the
// easy part of the final exponentiation.
MBLS_CYC_FN fp12 fp12_cyclotomic_sqr(const fp12& f) {
  const nz2 z0 = nrm(f.c0.c0), z4 = nrm(f.c0.c1), z3 = nrm(f.c0.c2), z2 = nrm(f.c1.c0), z1 = nrm(f.c1.c1),
            z5 = nrm(f.c1.c2);
  lz2<8> a0, a2, a4;
  lz2<10> a1, a3, a5;
  fp4_sqr(a0, a1, z0, z1);
  fp4_sqr(a2, a3, z2, z3);
  fp4_sqr(a4, a5, z4, z5);
  const fp2 r0 = reduce(smul<3>(a0) - smul<2>(z0)).v;
  const fp2 r1 = reduce(smul<3>(a1) + smul<2>(z1)).v;
  const fp2 r4 = reduce(smul<3>(a2) - smul<2>(z4)).v;
  const fp2 r5 = reduce(smul<3>(a3) + smul<2>(z5)).v;
  const fp2 r2 = reduce(smul<3>(mul_xi(a5)) + smul<2>(z2)).v;
  const fp2 r3 = reduce(smul<3>(a4) - smul<2>(z3)).v;
  return {{r0, r4, r3}, {r2, r1, r5}};
}

// g^|x| for g in the cyclotomic subgroup (|x| = 0xd201000000010000)
MBLS_NI fp12 fp12_pow_xabs(const fp12& g) {
  fp12 r = g;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = fp12_cyclotomic_sqr(r);
    if ((k::X_ABS >> b) & 1ull) r = fp12_mul(r, g);
  }
  return r;
}
// g^x with x < 0: conj(g^|x|) (inverse = conjugate in the cyclotomic subgroup)
MBLS_HD fp12 fp12_pow_x(const fp12& g) { return fp12_conj(fp12_pow_xabs(g)); }

MBLS_NI fp12 final_exp(const fp12& f) {
  // easy part
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));  // f^(p^6 - 1)
  t = fp12_mul(fp12_frob2(t), t);                 // ^(p^2 + 1)
  // hard part: t^((x-1)^2 (x+p) (x^2+p^2-1) + 3)
  fp12 a = fp12_mul(fp12_pow_x(t), fp12_conj(t));  // t^(x-1)
  a = fp12_mul(fp12_pow_x(a), fp12_conj(a));        // t^((x-1)^2)
  fp12 b = fp12_mul(fp12_pow_x(a), fp12_frob(a));   // a^(x+p)
  fp12 c = fp12_pow_x(fp12_pow_x(b));               // b^(x^2)
  c = fp12_mul(fp12_mul(c, fp12_frob2(b)), fp12_conj(b));  // b^(x^2 + p^2 - 1)
  const fp12 t3 = fp12_mul(fp12_cyclotomic_sqr(t), t);
  return fp12_mul(c, t3);
}

// ---------------------------------------------------------------------------------------
// Miller loop
// ---------------------------------------------------------------------------------------
// f * (l0 + l1 v + (l4 v) w) with l0 = c0, l1 = c2 x_P, l4 = c3 y_P: t0 = f.c0 (l0 + l1 v),
// t1 = f.c1 (l4 v), s = (f.c0 + f.c1)(l0 + (l1 + l4) v); result (t0 + v t1) + (s - t0 - t1) w.
// 13 Fp2 products, every sum lazy, each output coefficient reduced once.
MBLS_F12_FN fp12 fp12_mul_line(const fp12& f, const fp2& l0, const fp2& l1, const fp2& l4) {
  const nz2 L0 = nrm(l0), L1 = nrm(l1), L4 = nrm(l4);
  const nz2 a0 = nrm(f.c0.c0), a1 = nrm(f.c0.c1), a2 = nrm(f.c0.c2);
  const nz2 b0 = nrm(f.c1.c0), b1 = nrm(f.c1.c1), b2 = nrm(f.c1.c2);
  const nz2 u0 = mul(a0, L0), u1 = mul(a1, L1);
  const lz2<8> t00 = u0 + mul_xi(mul(a2, L1));
  const lz2<10> t01 = mul(a0 + a1, L0 + L1) - (u0 + u1);
  const lz2<4> t02 = u1 + mul(a2, L0);
  const lz2<6> t10 = mul_xi(mul(b2, L4));
  const nz2 t11 = mul(b0, L4), t12 = mul(b1, L4);
  const lz2<4> c0 = a0 + b0, c1 = a1 + b1, c2 = a2 + b2, m = L1 + L4;
  const nz2 w0 = mul(c0, L0), w1 = mul(c1, m);
  const lz2<8> s0 = w0 + mul_xi(mul(c2, m));
  const lz2<10> s1 = mul(c0 + c1, L0 + m) - (w0 + w1);
  const lz2<4> s2 = w1 + mul(c2, L0);
  return {{reduce(t00 + mul_xi(t12)).v, reduce(t01 + t10).v, reduce(t02 + t11).v},
          {reduce(s0 - t00 - t10).v, reduce(s1 - t01 - t11).v, reduce(s2 - t02 - t12).v}};
}
// Miller steps with T lazily reduced (g2lz, mbls_curve.hpp) and the line's coefficients lazy:
// the doubling shares X^2, Y^2, Z^2, YZ, XY between the tangent and 2T (9 Fp2 products instead
// of 11), the addition shares y_Q Z and x_Q Z.  The line meets P through products (lazy
// inputs are fine there); only l0 at an affine P is reduced.
struct line_lz {
  lz2<6> c0;   // f *= c0 + (c2 x_P) w^2 + (c3 y_P) w^3 (projective P: c0 Z_P)
  lz2<16> c2;
  lz2<12> c3;
};
// doubling step: tangent at T (c0 = Y^2 - 3b' Z^2, c2 = -3X^2, c3 = 2YZ), T <- 2T (RCB Alg. 9)
MBLS_MSTEP_FN line_lz miller_dbl(g2lz& t) {
  const nz2 xx = sqr(t.x), yy = sqr(t.y), zz = sqr(t.z), yz = mul(t.y, t.z), xy = mul(t.x, t.y);
  const nz2 t2 = reduce(mul_b3(zz));  // 3b' Z^2
  line_lz l;
  l.c0 = yy - t2;
  l.c2 = widen<16>(neg(smul<3>(xx)));
  l.c3 = widen<12>(smul<2>(yz));
  const lz2<16> z8 = smul<8>(yy);
  const lz2<10> t0m = yy - smul<3>(t2);
  const lz2<4> y3s = yy + t2;
  t = {widen<8>(smul<2>(mul(t0m, xy))), widen<8>(mul(t2, z8) + mul(t0m, y3s)), widen<8>(mul(yz, z8))};
  return l;
}
// addition step with affine Q: theta = Y - y_Q Z, kappa = X - x_Q Z,
// c0 = theta x_Q - kappa y_Q, c2 = -theta, c3 = kappa;  T <- T + Q (RCB Alg. 8)
MBLS_MSTEP_FN line_lz miller_add(g2lz& t, const aff<fp2>& q) {
  const nz2 qx = nrm(q.x), qy = nrm(q.y);
  const nz2 yqz = mul(qy, t.z), xqz = mul(qx, t.z);
  const lz2<12> theta = t.y - yqz, kappa = t.x - xqz;
  line_lz l;
  l.c0 = mul(theta, qx) - mul(kappa, qy);
  l.c2 = neg(theta);
  l.c3 = kappa;
  const nz2 t0 = mul(t.x, qx), t1 = mul(t.y, qy);
  const lz2<10> t3 = mul(qx + qy, t.x + t.y) - (t0 + t1);
  const lz2<10> t4 = yqz + t.y;
  const nz2 y3b = reduce(mul_b3(xqz + t.x));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2 = reduce(mul_b3(t.z));
  const lz2<4> z3 = t1 + t2;
  const lz2<6> t1m = t1 - t2;
  t = {widen<8>(mul(t3, t1m) - mul(t4, y3b)), widen<8>(mul(t1m, z3) + mul(y3b, t03)),
       widen<8>(mul(z3, t4) + mul(t03, t3))};
  return l;
}
MBLS_HD fp12 fp12_mul_line_at(const fp12& f, const line_lz& l, const aff<fp>& p) {
  return fp12_mul_line(f, reduce(l.c0).v, mul(l.c2, nrm(p.x)).v, mul(l.c3, nrm(p.y)).v);
}
// P = (X : Y : Z) projective: the line scaled by Z (an Fp factor, killed by the final
// exponentiation), so a projective key sum needs no inversion
MBLS_HD fp12 fp12_mul_line_at(const fp12& f, const line_lz& l, const proj<fp>& p) {
  return fp12_mul_line(f, mul(l.c0, nrm(p.z)).v, mul(l.c2, nrm(p.x)).v, mul(l.c3, nrm(p.y)).v);
}

// f_{|x|,Q}(P) conjugated (x < 0), single pair (P affine or projective)
template <class P>
MBLS_NI fp12 miller_loop_1(const P& p, const aff<fp2>& q) {
  g2lz t = g2lz_from(q);
  fp12 f = fp12_one();
  bool first = true;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (!first) f = fp12_sqr(f);
    f = fp12_mul_line_at(f, miller_dbl(t), p);
    first = false;
    if ((k::X_ABS >> b) & 1ull) f = fp12_mul_line_at(f, miller_add(t, q), p);
  }
  return fp12_conj(f);
}

// product of two Miller loops sharing the squarings (P1 affine or projective)
template <class P1>
MBLS_NI fp12 miller_loop_2(const P1& p1, const aff<fp2>& q1, const aff<fp>& p2, const aff<fp2>& q2) {
  g2lz t1 = g2lz_from(q1), t2 = g2lz_from(q2);
  fp12 f = fp12_one();
  bool first = true;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (!first) f = fp12_sqr(f);
    first = false;
    f = fp12_mul_line_at(f, miller_dbl(t1), p1);
    f = fp12_mul_line_at(f, miller_dbl(t2), p2);
    if ((k::X_ABS >> b) & 1ull) {
      f = fp12_mul_line_at(f, miller_add(t1, q1), p1);
      f = fp12_mul_line_at(f, miller_add(t2, q2), p2);
    }
  }
  return fp12_conj(f);
}

}  // namespace mbls
