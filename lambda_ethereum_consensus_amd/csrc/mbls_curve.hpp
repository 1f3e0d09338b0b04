// mbls_curve.hpp — G1 (E: y^2 = x^3 + 4 over Fp) and G2 (E': y^2 = x^3 + 4(1+u) over Fp2).
//
// Points are homogeneous projective (X:Y:Z) with the Renes–Costello–Batina complete
// formulas for a = 0 (RCB 2016, Algorithms 7/8/9): no exceptional cases, no branches, so
// aggregation of arbitrary (duplicate, opposite) keys needs no special handling on a SIMD.
// Identity = (0:1:0).
//
// Replaces blst's POINTonE1/E2 add/double/dadd, the in_G1/in_G2 membership tests and the
// ZCash (un)compression used by lighthouse `PublicKey::deserialize`,
// `Signature::deserialize` and `serialize` (native/bls_nif/src/lib.rs:20-140).
#pragma once
#include "mbls_fp2.hpp"
#include "mbls_lazy.hpp"

namespace mbls {

// ----- field-generic helpers ------------------------------------------------------------
MBLS_HD fp f_add(const fp& a, const fp& b) { return fp_add(a, b); }
MBLS_HD fp f_sub(const fp& a, const fp& b) { return fp_sub(a, b); }
MBLS_HD fp f_mul(const fp& a, const fp& b) { return fp_mul(a, b); }
MBLS_HD fp f_sqr(const fp& a) { return fp_sqr(a); }
MBLS_HD fp f_neg(const fp& a) { return fp_neg(a); }
MBLS_HD bool f_is_zero(const fp& a) { return fp_is_zero(a); }
MBLS_HD bool f_eq(const fp& a, const fp& b) { return fp_eq(a, b); }
MBLS_HD fp f_select(bool c, const fp& a, const fp& b) { return fp_select(c, a, b); }
MBLS_HD fp f_mul_b3(const fp& a) { return fp_mul12(a); }  // 3b = 12
MBLS_HD void f_set_zero(fp& a) { a = fp_zero(); }
MBLS_HD void f_set_one(fp& a) { a = fp_one(); }

MBLS_HD fp2 f_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
MBLS_HD fp2 f_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
MBLS_HD fp2 f_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
MBLS_HD fp2 f_sqr(const fp2& a) { return fp2_sqr(a); }
MBLS_HD fp2 f_neg(const fp2& a) { return fp2_neg(a); }
MBLS_HD bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
MBLS_HD bool f_eq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
MBLS_HD fp2 f_select(bool c, const fp2& a, const fp2& b) { return fp2_select(c, a, b); }
MBLS_HD fp2 f_mul_b3(const fp2& a) {  // 3b' = 12(1+u)
  const fp2 t = fp2_mul_xi(a);
  return {fp_mul12(t.c0), fp_mul12(t.c1)};
}
MBLS_HD void f_set_zero(fp2& a) { a = fp2_zero(); }
MBLS_HD void f_set_one(fp2& a) { a = fp2_one(); }

template <class F>
struct proj {
  F x, y, z;
};
template <class F>
struct aff {
  F x, y;
};

template <class F>
MBLS_HD proj<F> pt_identity() {
  proj<F> r;
  f_set_zero(r.x);
  f_set_one(r.y);
  f_set_zero(r.z);
  return r;
}
template <class F>
MBLS_HD proj<F> pt_from_affine(const aff<F>& a) {
  proj<F> r;
  r.x = a.x;
  r.y = a.y;
  f_set_one(r.z);
  return r;
}
template <class F>
MBLS_HD bool pt_is_identity(const proj<F>& p) {
  return f_is_zero(p.z);
}
template <class F>
MBLS_HD proj<F> pt_neg(const proj<F>& p) {
  return {p.x, f_neg(p.y), p.z};
}
template <class F>
MBLS_HD proj<F> pt_select(bool c, const proj<F>& a, const proj<F>& b) {
  return {f_select(c, a.x, b.x), f_select(c, a.y, b.y), f_select(c, a.z, b.z)};
}

// RCB Algorithm 7 (complete addition, a = 0)
template <class F>
MBLS_HD proj<F> pt_add_t(const proj<F>& p, const proj<F>& q) {
  F t0 = f_mul(p.x, q.x);
  F t1 = f_mul(p.y, q.y);
  F t2 = f_mul(p.z, q.z);
  F t3 = f_mul(f_add(p.x, p.y), f_add(q.x, q.y));
  F t4 = f_add(t0, t1);
  t3 = f_sub(t3, t4);
  t4 = f_mul(f_add(p.y, p.z), f_add(q.y, q.z));
  F x3 = f_add(t1, t2);
  t4 = f_sub(t4, x3);
  x3 = f_mul(f_add(p.x, p.z), f_add(q.x, q.z));
  F y3 = f_add(t0, t2);
  y3 = f_sub(x3, y3);
  x3 = f_add(t0, t0);
  t0 = f_add(x3, t0);
  t2 = f_mul_b3(t2);
  F z3 = f_add(t1, t2);
  t1 = f_sub(t1, t2);
  y3 = f_mul_b3(y3);
  x3 = f_mul(t4, y3);
  t2 = f_mul(t3, t1);
  x3 = f_sub(t2, x3);
  y3 = f_mul(y3, t0);
  t1 = f_mul(t1, z3);
  y3 = f_add(t1, y3);
  t0 = f_mul(t0, t3);
  z3 = f_mul(z3, t4);
  z3 = f_add(z3, t0);
  return {x3, y3, z3};
}

// RCB Algorithm 8 (mixed addition, q affine, a = 0)
template <class F>
MBLS_HD proj<F> pt_add_affine_t(const proj<F>& p, const aff<F>& q) {
  F t0 = f_mul(p.x, q.x);
  F t1 = f_mul(p.y, q.y);
  F t3 = f_mul(f_add(q.x, q.y), f_add(p.x, p.y));
  F t4 = f_add(t0, t1);
  t3 = f_sub(t3, t4);
  t4 = f_add(f_mul(q.y, p.z), p.y);
  F y3 = f_add(f_mul(q.x, p.z), p.x);
  F x3 = f_add(t0, t0);
  t0 = f_add(x3, t0);
  F t2 = f_mul_b3(p.z);
  F z3 = f_add(t1, t2);
  t1 = f_sub(t1, t2);
  y3 = f_mul_b3(y3);
  x3 = f_mul(t4, y3);
  t2 = f_mul(t3, t1);
  x3 = f_sub(t2, x3);
  y3 = f_mul(y3, t0);
  t1 = f_mul(t1, z3);
  y3 = f_add(t1, y3);
  t0 = f_mul(t0, t3);
  z3 = f_mul(z3, t4);
  z3 = f_add(z3, t0);
  return {x3, y3, z3};
}

// RCB Algorithm 9 (doubling, a = 0)
template <class F>
MBLS_HD proj<F> pt_dbl_t(const proj<F>& p) {
  F t0 = f_sqr(p.y);
  F z3 = f_add(t0, t0);
  z3 = f_add(z3, z3);
  z3 = f_add(z3, z3);
  F t1 = f_mul(p.y, p.z);
  F t2 = f_sqr(p.z);
  t2 = f_mul_b3(t2);
  F x3 = f_mul(t2, z3);
  F y3 = f_add(t0, t2);
  z3 = f_mul(t1, z3);
  t1 = f_add(t2, t2);
  t2 = f_add(t1, t2);
  t0 = f_sub(t0, t2);
  y3 = f_mul(t0, y3);
  y3 = f_add(x3, y3);
  t1 = f_mul(p.x, p.y);
  x3 = f_mul(t0, t1);
  x3 = f_add(x3, x3);
  return {x3, y3, z3};
}

// G1 ops inline (the key-validation kernel is throughput bound on them); G2 ops out of line
// (their Fp2 bodies are large and they sit inside long loops).
MBLS_HD proj<fp> pt_add(const proj<fp>& p, const proj<fp>& q) { return pt_add_t(p, q); }
MBLS_HD proj<fp> pt_add_affine(const proj<fp>& p, const aff<fp>& q) { return pt_add_affine_t(p, q); }
MBLS_HD proj<fp> pt_dbl(const proj<fp>& p) { return pt_dbl_t(p); }
// G2 group law on one lane: inlined into the ladders by default (the running point then stays
// in registers instead of scratch).  Measured r01, 2 runs each: gossip 900k / 903k -> 918k /
// 921k verify/s, deposit AV 116.9k / 117.4k -> 122.1k / 122.2k sets/s, cold and warm epoch
// unchanged.
#define MBLS_G2PT_FN __host__ __device__ __forceinline__
MBLS_G2PT_FN proj<fp2> pt_add(const proj<fp2>& p, const proj<fp2>& q) { return pt_add_t(p, q); }
MBLS_G2PT_FN proj<fp2> pt_add_affine(const proj<fp2>& p, const aff<fp2>& q) { return pt_add_affine_t(p, q); }
MBLS_G2PT_FN proj<fp2> pt_dbl(const proj<fp2>& p) { return pt_dbl_t(p); }

// [|x|] * q for the BLS parameter |x| = 0xd201000000010000 (left-to-right, wave-uniform).
template <class F>
MBLS_HD proj<F> pt_mul_xabs(const proj<F>& q) {
  proj<F> r = q;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = pt_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = pt_add(r, q);
  }
  return r;
}
template <class F>
MBLS_HD proj<F> pt_mul_xabs_affine(const aff<F>& q) {
  proj<F> r = pt_from_affine(q);
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = pt_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = pt_add_affine(r, q);
  }
  return r;
}

// ---------------------------------------------------------------------------------------
// G2 group law with lazily reduced coordinates (mbls_lazy.hpp): every coordinate < 8p, the
// sums and differences of the RCB formulas formed lazily, only the 3b' multiples reduced.
// The ladders below (membership [|x|] Q, cofactor clearing, the Miller loops' T) keep their
// running point in this form and reduce once at the end.
// ---------------------------------------------------------------------------------------
struct g2lz {
  lz2<8> x, y, z;
};
MBLS_HD g2lz g2lz_from(const proj<fp2>& p) { return {{p.x}, {p.y}, {p.z}}; }
MBLS_HD g2lz g2lz_from(const aff<fp2>& q) { return {{q.x}, {q.y}, {fp2_one()}}; }
MBLS_HD proj<fp2> g2lz_reduce(const g2lz& t) { return {reduce(t.x).v, reduce(t.y).v, reduce(t.z).v}; }

// RCB Algorithm 9 (as pt_dbl_t)
MBLS_HD g2lz g2lz_dbl(const g2lz& t) {
  const nz2 yy = sqr(t.y), zz = sqr(t.z), yz = mul(t.y, t.z), xy = mul(t.x, t.y);
  const nz2 t2 = reduce(mul_b3(zz));
  const lz2<16> z8 = smul<8>(yy);
  const lz2<10> t0m = yy - smul<3>(t2);
  const lz2<4> y3s = yy + t2;
  return {widen<8>(smul<2>(mul(t0m, xy))), widen<8>(mul(t2, z8) + mul(t0m, y3s)), widen<8>(mul(yz, z8))};
}
// RCB Algorithm 7 (as pt_add_t)
MBLS_HD g2lz g2lz_add(const g2lz& p, const g2lz& q) {
  const nz2 t0 = mul(p.x, q.x), t1 = mul(p.y, q.y), t2 = mul(p.z, q.z);
  const lz2<10> t3 = mul(p.x + p.y, q.x + q.y) - (t0 + t1);
  const lz2<10> t4 = mul(p.y + p.z, q.y + q.z) - (t1 + t2);
  const nz2 y3 = reduce(mul_b3(mul(p.x + p.z, q.x + q.z) - (t0 + t2)));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2b = reduce(mul_b3(t2));
  const lz2<4> z3 = t1 + t2b;
  const lz2<6> t1m = t1 - t2b;
  return {widen<8>(mul(t3, t1m) - mul(t4, y3)), widen<8>(mul(t1m, z3) + mul(y3, t03)),
          widen<8>(mul(z3, t4) + mul(t03, t3))};
}
// RCB Algorithm 8 (as pt_add_affine_t): q affine, normalized
MBLS_HD g2lz g2lz_add_affine(const g2lz& p, const aff<fp2>& q) {
  const nz2 qx = nrm(q.x), qy = nrm(q.y);
  const nz2 t0 = mul(p.x, qx), t1 = mul(p.y, qy);
  const lz2<10> t3 = mul(qx + qy, p.x + p.y) - (t0 + t1);
  const lz2<10> t4 = mul(qy, p.z) + p.y;
  const nz2 y3b = reduce(mul_b3(mul(qx, p.z) + p.x));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2 = reduce(mul_b3(p.z));
  const lz2<4> z3 = t1 + t2;
  const lz2<6> t1m = t1 - t2;
  return {widen<8>(mul(t3, t1m) - mul(t4, y3b)), widen<8>(mul(t1m, z3) + mul(y3b, t03)),
          widen<8>(mul(z3, t4) + mul(t03, t3))};
}

// [|x|] q with the running point lazily reduced (63 doublings, 5 additions); result normalized
MBLS_NI proj<fp2> g2_mul_xabs(const proj<fp2>& q) {
  const g2lz ql = g2lz_from(q);
  g2lz r = ql;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = g2lz_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = g2lz_add(r, ql);
  }
  return g2lz_reduce(r);
}
MBLS_NI proj<fp2> g2_mul_xabs_affine(const aff<fp2>& q) {
  g2lz r = g2lz_from(q);
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = g2lz_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = g2lz_add_affine(r, q);
  }
  return g2lz_reduce(r);
}

// [|x|] q on Jacobian coordinates (r05): x = X / Z^2, y = Y / Z^3.  The doubling (dbl-2009-l for
// a = 0: five Fp2 squarings and two Fp2 products) costs 32 reduced Fp-product units against 44
// for the complete projective doubling above, 63 times per [|x|].  The five additions
// (add-2007-bl) decide their exceptional cases exactly -- R = Q (doubling), R = -Q (the
// identity), R the identity (Q) -- so the result is the point g2_mul_xabs returns for every
// input, small-order points included.  The identity is (1 : 1 : 0), a fixed point of the
// doubling.  Used by hash_to_G2's cofactor clearing (two [|x|] per hash, MBLS_H2C_JAC).
struct g2jz {
  lz2<16> x, z;
  nz2 y;
};
struct g2jq {  // a fixed addend: reduced Jacobian coordinates with Z^2 and Z^3
  nz2 x, y, z, zz, zzz;
};
MBLS_HD g2jz g2jz_dbl(const g2jz& t) {
  const nz2 A = sqr(t.x), B = sqr(t.y), C = sqr(B);
  const nz2 S1 = sqr(t.x + B);
  const nz2 D = reduce(smul<2>(S1 - (A + C)));  // 4 X B
  const lz2<6> E = smul<3>(A);
  const nz2 F = sqr(E);
  const lz2<10> X3 = F - smul<2>(D);
  const nz2 Y3 = reduce(mul(E, D - X3) - smul<8>(C));
  const lz2<4> Z3 = smul<2>(mul(t.y, t.z));
  return {widen<16>(X3), widen<16>(Z3), Y3};
}
MBLS_HD g2jz g2jz_add(const g2jz& r, const g2jq& q) {
  const nz2 z1z1 = sqr(r.z);
  const nz2 u1 = mul(r.x, q.zz), u2 = mul(q.x, z1z1);
  const nz2 s1 = mul(q.zzz, r.y), s2 = mul(q.y, mul(r.z, z1z1));
  const nz2 h = reduce(u2 - u1), hr = reduce(s2 - s1);
  const nz2 I = sqr(smul<2>(h));
  const nz2 J = mul(h, I), V = mul(u1, I);
  const lz2<4> rr = smul<2>(hr);
  const lz2<10> X3 = sqr(rr) - (J + smul<2>(V));
  const nz2 Y3 = reduce(mul(rr, V - X3) - smul<2>(mul(s1, J)));
  const lz2<4> Z3 = smul<2>(mul(mul(r.z, q.z), h));
  g2jz out{widen<16>(X3), widen<16>(Z3), Y3};
  const bool r_inf = fp2_is_zero(reduce(r.z).v), h0 = fp2_is_zero(h.v), hr0 = fp2_is_zero(hr.v);
  if (h0 && !r_inf) {  // R = +-Q: rare, lane-divergent
    if (hr0) {
      out = g2jz_dbl(r);
    } else {
      out.x = widen<16>(nrm(fp2_one()));
      out.y = nrm(fp2_one());
      out.z = widen<16>(nrm(fp2_zero()));
    }
  }
  if (r_inf) out = {widen<16>(q.x), widen<16>(q.z), q.y};
  return out;
}
MBLS_NI proj<fp2> g2_mul_xabs_jac(const proj<fp2>& p) {
  if (fp2_is_zero(p.z)) return p;  // the identity
  const nz2 X = nrm(p.x), Y = nrm(p.y), Z = nrm(p.z);
  const nz2 zz = sqr(Z);
  const g2jq q{mul(X, Z), mul(Y, zz), Z, zz, mul(zz, Z)};  // (X : Y : Z) -> (X Z : Y Z^2 : Z)
  g2jz r{widen<16>(q.x), widen<16>(q.z), q.y};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = g2jz_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = g2jz_add(r, q);
  }
  // back to homogeneous: (X Z : Y : Z^3); the identity (1 : 1 : 0) -> (0 : 1 : 0)
  const nz2 rz = reduce(r.z);
  return {mul(r.x, rz).v, r.y.v, mul(sqr(rz), rz).v};
}

// projective equality X1 Z2 == X2 Z1 and Y1 Z2 == Y2 Z1 (identity handled: (0:1:0))
template <class F>
MBLS_HD bool pt_eq(const proj<F>& p, const proj<F>& q) {
  return f_eq(f_mul(p.x, q.z), f_mul(q.x, p.z)) && f_eq(f_mul(p.y, q.z), f_mul(q.y, p.z));
}

// affine conversion (identity -> (0,0) with the flag returned false)
MBLS_HD bool pt_to_affine(aff<fp>& a, const proj<fp>& p) {
  const fp zi = fp_inv(p.z);
  a.x = fp_mul(p.x, zi);
  a.y = fp_mul(p.y, zi);
  return !fp_is_zero(p.z);
}
MBLS_HD bool pt_to_affine(aff<fp2>& a, const proj<fp2>& p) {
  const fp2 zi = fp2_inv(p.z);
  a.x = fp2_mul(p.x, zi);
  a.y = fp2_mul(p.y, zi);
  return !fp2_is_zero(p.z);
}

// ---------------------------------------------------------------------------------------
// Membership tests
// ---------------------------------------------------------------------------------------

// Jacobian G1 points (x = X/Z^2, y = Y/Z^3) for the doubling-heavy membership ladder,
// with lazy reduction (mbls_fp.hpp fp_carry): sums and differences that only feed a
// multiply skip the conditional subtraction.  Invariant between operations: digits < 2^28,
// X < 26p, Y < 18p, Z < 2p (Z is always a multiply output).  Every multiply below has an
// input-value product < 2^11 p^2 (bounds in the comments, in units of p).
//
// Exceptional cases.  dbl-2009-l is exact on E1 (odd group order: no point has Y = 0).  The
// additions (madd-2007-bl, add-2007-bl) are incomplete: P = +-Q or an identity input gives
// Z3 = 0, and Z = 0 then stays 0 through every later dbl/add, so the final check (which
// requires Z != 0) rejects.  For P in G1 the ladders only form [k]P +- P with 2 <= k < 2^64
// < r, so no exceptional case occurs and the test is exact; for P not in G1 the correct
// answer is "reject" anyway.  So the verdict equals Scott's test on every point of E1(Fp).
struct jac1 {
  fp x, y, z;
};
namespace lazy {
constexpr pmul_t P4 = p_times(4), P6 = p_times(6), P8 = p_times(8), P16 = p_times(16), P24 = p_times(24),
                 P26 = p_times(26), P36 = p_times(36);
}
// dbl-2009-l (a = 0): 2M + 5S.  D = 2 Dh with Dh = T - A - C.
MBLS_HD jac1 jac_dbl(const jac1& p) {
  const fp a = fp_sqr(p.x);                         // 26^2
  const fp b = fp_sqr(p.y);                         // 18^2
  const fp c = fp_sqr(b);                           // 2^2
  const fp t = fp_sqr(fp_add_lazy(p.x, b));         // 28^2
  const fp e = fp_add3_lazy(a, a, a);               // E = 3A < 6p, digits < 2^30
  const fp f = fp_sqr(e);                           // 6^2
  int32_t d[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)t.v[i] - (int32_t)a.v[i] - (int32_t)c.v[i] + lazy::P4.v[i];
  const fp dh = fp_carry(d);                        // Dh + 4p in (0, 6p)
#pragma unroll
  for (int i = 0; i < NL; ++i)  // X3 = F - 2D = F - 4 Dh  in (0, 26p)
    d[i] = (int32_t)f.v[i] - (int32_t)(dh.v[i] << 2) + lazy::P24.v[i];
  const fp x3 = fp_carry(d);
#pragma unroll
  for (int i = 0; i < NL; ++i)  // D - X3 in (0, 38p)
    d[i] = 2 * (int32_t)dh.v[i] - (int32_t)x3.v[i] + lazy::P26.v[i];
  const fp pm = fp_mul(e, fp_carry(d));             // 6 x 38
#pragma unroll
  for (int i = 0; i < NL; ++i)  // Y3 = E (D - X3) - 8C  in (0, 18p)
    d[i] = (int32_t)pm.v[i] - (int32_t)(c.v[i] << 3) + lazy::P16.v[i];
  const fp y3 = fp_carry(d);
  const fp z3 = fp_mul(fp_add_lazy(p.y, p.y), p.z);  // 36 x 2
  return {x3, y3, z3};
}
// madd-2007-bl, q affine (< p): 7M + 3S
MBLS_HD jac1 jac_madd(const jac1& p, const aff<fp>& q) {
  int32_t d[NL];
  const fp z1z1 = fp_sqr(p.z);                      // 2^2
  const fp u2 = fp_mul(q.x, z1z1);                  // 1 x 2
  const fp s2 = fp_mul(q.y, fp_mul(p.z, z1z1));     // 1 x 2
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)u2.v[i] - (int32_t)p.x.v[i] + lazy::P26.v[i];
  const fp h = fp_carry(d);                         // H = U2 - X1 in (0, 28p)
  const fp hh = fp_sqr(h);                          // 28^2
  fp i4;
#pragma unroll
  for (int i = 0; i < NL; ++i) i4.v[i] = hh.v[i] << 2;  // I = 4HH < 8p, digits < 2^30
  const fp j = fp_mul(h, i4);                       // 28 x 8
  const fp v = fp_mul(p.x, i4);                     // 26 x 8
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = 2 * ((int32_t)s2.v[i] - (int32_t)p.y.v[i]) + lazy::P36.v[i];
  const fp r = fp_carry(d);                         // r = 2(S2 - Y1) in (0, 40p)
  const fp r2 = fp_sqr(r);                          // 40^2
#pragma unroll
  for (int i = 0; i < NL; ++i)  // X3 = r^2 - J - 2V  in [0, 8p)
    d[i] = (int32_t)r2.v[i] - (int32_t)j.v[i] - 2 * (int32_t)v.v[i] + lazy::P6.v[i];
  const fp x3 = fp_carry(d);
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)v.v[i] - (int32_t)x3.v[i] + lazy::P8.v[i];
  const fp t0 = fp_mul(r, fp_carry(d));             // 40 x 10
  const fp t1 = fp_mul(p.y, j);                     // 18 x 2
#pragma unroll
  for (int i = 0; i < NL; ++i)  // Y3 = r (V - X3) - 2 Y1 J  in [0, 6p)
    d[i] = (int32_t)t0.v[i] - 2 * (int32_t)t1.v[i] + lazy::P4.v[i];
  const fp y3 = fp_carry(d);
  const fp z3 = fp_mul(fp_add_lazy(p.z, p.z), h);   // Z3 = 2 Z1 H: 4 x 28
  return {x3, y3, z3};
}
// add-2007-bl against a fixed q with q.z^2 and q.z^3 precomputed: 10M + 2S
struct jac1_base {
  fp x, y, z, zz, zzz;
};
MBLS_HD jac1_base jac_base(const jac1& q) {
  const fp zz = fp_sqr(q.z);
  return {q.x, q.y, q.z, zz, fp_mul(zz, q.z)};
}
MBLS_HD jac1 jac_add(const jac1& p, const jac1_base& q) {
  int32_t d[NL];
  const fp z1z1 = fp_sqr(p.z);                      // 2^2
  const fp u1 = fp_mul(p.x, q.zz);                  // 26 x 2
  const fp u2 = fp_mul(q.x, z1z1);                  // 26 x 2
  const fp s1 = fp_mul(p.y, q.zzz);                 // 18 x 2
  const fp s2 = fp_mul(q.y, fp_mul(p.z, z1z1));     // 18 x 2
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)u2.v[i] - (int32_t)u1.v[i] + lazy::P4.v[i];
  const fp h = fp_carry(d);                         // H = U2 - U1 in (0, 6p)
  const fp h2 = fp_add_lazy(h, h);                  // 2H < 12p, digits < 2^29
  const fp ii = fp_sqr(h2);                         // I = (2H)^2: 12^2
  const fp j = fp_mul(h, ii);                       // J = H I: 6 x 2
  const fp v = fp_mul(u1, ii);                      // V = U1 I: 2 x 2
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = 2 * ((int32_t)s2.v[i] - (int32_t)s1.v[i]) + lazy::P4.v[i];
  const fp r = fp_carry(d);                         // r = 2(S2 - S1) in (0, 8p)
  const fp r2 = fp_sqr(r);                          // 8^2
#pragma unroll
  for (int i = 0; i < NL; ++i)  // X3 = r^2 - J - 2V  in [0, 8p)
    d[i] = (int32_t)r2.v[i] - (int32_t)j.v[i] - 2 * (int32_t)v.v[i] + lazy::P6.v[i];
  const fp x3 = fp_carry(d);
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)v.v[i] - (int32_t)x3.v[i] + lazy::P8.v[i];
  const fp t0 = fp_mul(r, fp_carry(d));             // 8 x 10
  const fp t1 = fp_mul(s1, j);                      // 2 x 2
#pragma unroll
  for (int i = 0; i < NL; ++i)  // Y3 = r (V - X3) - 2 S1 J  in [0, 6p)
    d[i] = (int32_t)t0.v[i] - 2 * (int32_t)t1.v[i] + lazy::P4.v[i];
  const fp y3 = fp_carry(d);
  const fp z3 = fp_mul(fp_mul(p.z, q.z), h2);       // Z3 = 2 Z1 Z2 H: 2 x 12
  return {x3, y3, z3};
}

// [|x|] q for the BLS parameter |x| = 0xd201000000010000 (63 doublings, 5 additions)
MBLS_HD jac1 jac_mul_xabs_affine(const aff<fp>& q) {
  jac1 r = {q.x, q.y, fp_from(k::ONE)};
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = jac_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = jac_madd(r, q);
  }
  return r;
}
MBLS_HD jac1 jac_mul_xabs(const jac1& q) {
  const jac1_base qb = jac_base(q);
  jac1 r = q;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = jac_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = jac_add(r, qb);
  }
  return r;
}

// G1: phi(P) == [-x^2] P with phi(x, y) = (beta x, y) (Scott 2021; exact for BLS12-381 and
// equivalent to blst's POINTonE1_in_G1).  [x^2] = [|x|][|x|] since the signs cancel.
// With Q = [x^2] P in Jacobian form: phi(P) == -Q  <=>  X == beta x Z^2, Y == -y Z^3, Z != 0.
MBLS_HD bool g1_in_subgroup(const aff<fp>& p) {
  const jac1 q = jac_mul_xabs(jac_mul_xabs_affine(p));
  const fp zz = fp_sqr(q.z);
  const fp bx = fp_mul(fp_from(k::BETA), p.x);
  const fp ex = fp_mul(bx, zz);                      // < 2p
  const fp ey = fp_mul(p.y, fp_mul(zz, q.z));        // y Z^3 < 2p
  int32_t d[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)q.x.v[i] - (int32_t)ex.v[i] + lazy::P4.v[i];
  const bool okx = fp_is_zero(fp_shrink(fp_carry(d)));  // X - beta x Z^2 (in (0, 30p)) == 0 mod p
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)q.y.v[i] + (int32_t)ey.v[i];
  const bool oky = fp_is_zero(fp_shrink(fp_carry(d)));  // Y + y Z^3 (in [0, 20p)) == 0 mod p
  return okx && oky && !fp_is_zero(q.z);
}

// G2 psi endomorphism: (x, y) -> (conj(x) cx, conj(y) cy)
MBLS_NI proj<fp2> g2_psi(const proj<fp2>& p) {
  const fp2 cx = fp2_from(k::PSI_CX_C0, k::PSI_CX_C1), cy = fp2_from(k::PSI_CY_C0, k::PSI_CY_C1);
  return {fp2_mul(fp2_conj(p.x), cx), fp2_mul(fp2_conj(p.y), cy), fp2_conj(p.z)};
}

// G2: psi(Q) == [x] Q = -[|x|] Q (Scott 2021; equivalent to blst's POINTonE2_in_G2)
MBLS_NI bool g2_in_subgroup(const aff<fp2>& q) {
  const proj<fp2> qp = pt_from_affine(q);
  const proj<fp2> xq = pt_neg(g2_mul_xabs_affine(q));
  return pt_eq(g2_psi(qp), xq);
}

// ---------------------------------------------------------------------------------------
// ZCash compressed encoding (as blst POINTonE1_Uncompress_Z / POINTonE2_Uncompress_Z)
// ---------------------------------------------------------------------------------------
enum : int32_t {
  DEC_OK = 0,
  DEC_BAD_ENCODING = 1,
  DEC_NOT_ON_CURVE = 2,
  DEC_NOT_IN_GROUP = 3,
  DEC_INFINITY = 4,  // well-formed infinity encoding (0xc0 00..)
};

// w: the 48 bytes as 12 big-endian 32-bit words (w[0] holds bytes 0..3, byte 0 in bits 31..24)
MBLS_HD int32_t g1_uncompress(aff<fp>& out, const uint32_t (&w)[12]) {
  const uint32_t b0 = w[0] >> 24;
  if (!(b0 & 0x80u)) return DEC_BAD_ENCODING;
  if (b0 & 0x40u) {
    uint32_t rest = w[0] & 0x3fffffffu;
#pragma unroll
    for (int i = 1; i < 12; ++i) rest |= w[i];
    return rest == 0 ? DEC_INFINITY : DEC_BAD_ENCODING;
  }
  uint32_t xw[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) xw[i] = w[i];
  xw[0] &= 0x1fffffffu;
  const fp xr = fp_from_be_words(xw);
  if (!fp_raw_lt_p(xr)) return DEC_BAD_ENCODING;
  const fp x = fp_to_mont(xr);
  const fp rhs = fp_add(fp_mul(fp_sqr(x), x), fp_from(k::B1));
  fp y;
  if (!fp_sqrt_inl(y, rhs)) return DEC_NOT_ON_CURVE;
  const bool want = (b0 >> 5) & 1u;
  const bool have = fp_raw_gt_half(fp_from_mont(y));
  y = fp_cneg(y, want != have);
  out.x = x;
  out.y = y;
  if (fp_raw_is_zero(xr)) return DEC_NOT_IN_GROUP;  // (0, +-2) has order 3
  return DEC_OK;
}

// 96 bytes as 24 big-endian words: x.c1 in w[0..11] (flags in the top byte), x.c0 in w[12..23]
MBLS_NI int32_t g2_uncompress(aff<fp2>& out, const uint32_t (&w)[24]) {
  const uint32_t b0 = w[0] >> 24;
  if (!(b0 & 0x80u)) return DEC_BAD_ENCODING;
  if (b0 & 0x40u) {
    uint32_t rest = w[0] & 0x3fffffffu;
#pragma unroll
    for (int i = 1; i < 24; ++i) rest |= w[i];
    return rest == 0 ? DEC_INFINITY : DEC_BAD_ENCODING;
  }
  uint32_t w1[12], w0[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    w1[i] = w[i];
    w0[i] = w[12 + i];
  }
  w1[0] &= 0x1fffffffu;
  const fp x1r = fp_from_be_words(w1), x0r = fp_from_be_words(w0);
  if (!fp_raw_lt_p(x1r) || !fp_raw_lt_p(x0r)) return DEC_BAD_ENCODING;
  const fp2 x = {fp_to_mont(x0r), fp_to_mont(x1r)};
  const fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_from(k::B2_C0, k::B2_C1));
  fp2 y;
  if (!fp2_sqrt(y, rhs)) return DEC_NOT_ON_CURVE;
  const bool want = (b0 >> 5) & 1u;
  const bool have = fp2_sgn_zcash(y);
  if (want != have) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  return DEC_OK;
}

// compress an affine G1 point (Montgomery coords) or the identity
MBLS_HD void g1_compress(uint32_t (&w)[12], const aff<fp>& a, bool is_identity) {
  if (is_identity) {
#pragma unroll
    for (int i = 0; i < 12; ++i) w[i] = 0;
    w[0] = 0xc0000000u;
    return;
  }
  const fp x = fp_from_mont(a.x), y = fp_from_mont(a.y);
  fp_to_be_words(x, w);
  w[0] |= 0x80000000u | (fp_raw_gt_half(y) ? 0x20000000u : 0u);
}

MBLS_HD void g2_compress(uint32_t (&w)[24], const aff<fp2>& a, bool is_identity) {
  if (is_identity) {
#pragma unroll
    for (int i = 0; i < 24; ++i) w[i] = 0;
    w[0] = 0xc0000000u;
    return;
  }
  uint32_t w1[12], w0[12];
  fp_to_be_words(fp_from_mont(a.x.c1), w1);
  fp_to_be_words(fp_from_mont(a.x.c0), w0);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    w[i] = w1[i];
    w[12 + i] = w0[i];
  }
  w[0] |= 0x80000000u | (fp2_sgn_zcash(a.y) ? 0x20000000u : 0u);
}

}  // namespace mbls
