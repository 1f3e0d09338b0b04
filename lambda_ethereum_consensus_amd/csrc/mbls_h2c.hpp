// mbls_h2c.hpp — hash_to_curve BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380 §8.8.2) on gfx950.
//
// Specialised for the path's inputs: 32-byte messages (Hash256 signing roots, the only
// length the reference NIF accepts: native/bls_nif/src/lib.rs:25,59,79,99,118) and the PoP
// DST `BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`.  The constant parts of every SHA-256
// input block are precomputed by tools/gen_constants.py, so each lane only feeds its
// message words.  Replaces blst's Hash_to_G2 (expand_message_xmd, map_to_g2 / SSWU,
// isogeny_map_to_E2, clear_cofactor); re-derived from the RFC.
#pragma once
#include "mbls_curve.hpp"

namespace mbls {

// ----- SHA-256 ---------------------------------------------------------------------------
MBLS_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

MBLS_NI void sha256_compress(uint32_t (&st)[8], const uint32_t* blk /* 16 BE words */) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + k::SHA256_K[i] + wi;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

MBLS_HD void sha256_init(uint32_t (&st)[8]) {
  st[0] = 0x6a09e667u;
  st[1] = 0xbb67ae85u;
  st[2] = 0x3c6ef372u;
  st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu;
  st[5] = 0x9b05688cu;
  st[6] = 0x1f83d9abu;
  st[7] = 0x5be0cd19u;
}

// 2-block message: 8 variable words followed by 24 constant (padded) words
MBLS_HD void sha256_two_blocks(uint32_t (&st)[8], const uint32_t (&head)[8], const uint32_t (&tail)[24]) {
  uint32_t blk[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) blk[i] = head[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) blk[8 + i] = tail[i];
  sha256_compress(st, blk);
#pragma unroll
  for (int i = 0; i < 16; ++i) blk[i] = tail[8 + i];
  sha256_compress(st, blk);
}

// generic SHA-256 of a short byte string (host-side test helper; not on the device path)
inline void sha256_bytes(const uint8_t* msg, int len, uint8_t* out32) {
  uint8_t buf[1024 + 128] = {0};
  for (int i = 0; i < len; ++i) buf[i] = msg[i];
  buf[len] = 0x80;
  int total = len + 1;
  while (total % 64 != 56) buf[total++] = 0;
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) buf[total++] = (uint8_t)(bits >> (56 - 8 * i));
  uint32_t st[8];
  sha256_init(st);
  for (int off = 0; off < total; off += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) {
      const uint8_t* q = buf + off + 4 * i;
      w[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
    sha256_compress(st, w);
  }
  for (int i = 0; i < 8; ++i) {
    out32[4 * i] = st[i] >> 24;
    out32[4 * i + 1] = st[i] >> 16;
    out32[4 * i + 2] = st[i] >> 8;
    out32[4 * i + 3] = st[i];
  }
}

// expand_message_xmd(msg32, DST_POP, 256): out = 64 big-endian words (b_1 || ... || b_8)
MBLS_NI void expand_message_xmd_msg32(uint32_t (&out)[64], const uint32_t (&msg)[8]) {
  uint32_t b0[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b0[i] = k::SHA256_ZPAD_STATE[i];
  sha256_two_blocks(b0, msg, k::XMD_B0_TAIL);
  uint32_t bi[8];
  sha256_init(bi);
  sha256_two_blocks(bi, b0, k::XMD_BI_TAIL1);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = bi[j];
#pragma unroll
  for (int i = 2; i <= 8; ++i) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = b0[j] ^ bi[j];
    sha256_init(bi);
    switch (i) {  // compile-time after unrolling
      case 2: sha256_two_blocks(bi, x, k::XMD_BI_TAIL2); break;
      case 3: sha256_two_blocks(bi, x, k::XMD_BI_TAIL3); break;
      case 4: sha256_two_blocks(bi, x, k::XMD_BI_TAIL4); break;
      case 5: sha256_two_blocks(bi, x, k::XMD_BI_TAIL5); break;
      case 6: sha256_two_blocks(bi, x, k::XMD_BI_TAIL6); break;
      case 7: sha256_two_blocks(bi, x, k::XMD_BI_TAIL7); break;
      default: sha256_two_blocks(bi, x, k::XMD_BI_TAIL8); break;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) out[8 * (i - 1) + j] = bi[j];
  }
}

// 8 big-endian words (256-bit value) -> radix-2^28 digits (plain)
MBLS_HD fp fp_from_be_words8(const uint32_t* w) {
  uint32_t full[12];
#pragma unroll
  for (int i = 0; i < 4; ++i) full[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) full[4 + i] = w[i];
  return fp_from_be_words(full);
}

// hash_to_field: 64-byte big-endian chunk -> Montgomery Fp (value mod p)
MBLS_HD fp fp_from_64_bytes(const uint32_t* w16) {
  const fp hi = fp_from_be_words8(w16), lo = fp_from_be_words8(w16 + 8);
  return fp_add(fp_mul(lo, fp_from(k::R2)), fp_mul(hi, fp_from(k::H2F_C)));
}

// ----- simplified SWU on E2': y^2 = x^3 + A' x + B' (RFC 9380 §6.6.2) --------------------
// With x2 = Z u^2 x1, g(x2) = (Z u^2)^3 g(x1) and exactly one of the two is a square (x1 from
// the exceptional case is always one).  One Fp exponentiation r = n1^((p+1)/4) of
// n1 = norm(g(x1)) gives both norm roots: r if n1 is a residue, else r^2 = -n1 and
// norm(g(x2)) = w^3 n1 (w = norm(Z u^2) = 5 norm(u)^2, -w and -n1 residues) has the root
// w sqrt(-5) norm(u) r.
// No inversion either (r03): x1 = N / D stays a fraction (N = (-B/A)(den + 1), D = den, or
// B/(ZA) over 1 when den = 0), g(x1) = U / V with U = N (N^2 + A D^2) + B D^3, V = D^3, and the
// root is taken of the ratio U conj(V) / norm(V) (fp2_sqrt_ratio_from_gamma: the inverse of the
// Fp denominator rides on the (p-3)/4 power).  norm(U conj(V)) = norm(g(x1)) norm(V)^2 has the
// same residuosity, and g(x2) scales U by (Z u^2)^3 as before.  y comes out affine (sgn0 needs
// it), x as N / D, and iso3_map takes the fraction.  So the map costs two exponentiations
// (norm root, the ratio's (p-3)/4 power) instead of up to seven.
struct sswu_pt {
  fp2 xn, xd, y;  // a point of E2': x = xn / xd, y affine
};
MBLS_NI aff<fp2> map_to_curve_sswu_two_roots(const fp2& u);
#if defined(MBLS_HOST_COUNT) && !defined(__HIP_DEVICE_COMPILE__)
inline thread_local uint64_t g_host_sswu_fallback = 0;  // tests/hostsim: the guard never fires
#endif
MBLS_NI sswu_pt map_to_curve_sswu(const fp2& u) {
  const fp2 A = fp2_from(k::SSWU_A_C0, k::SSWU_A_C1), B = fp2_from(k::SSWU_B_C0, k::SSWU_B_C1);
  const fp2 Z = fp2_from(k::SSWU_Z_C0, k::SSWU_Z_C1);
  const fp2 zu2 = fp2_mul(Z, fp2_sqr(u));
  const fp2 zu4 = fp2_sqr(zu2);
  const fp2 den = fp2_add(zu4, zu2);
  const bool den0 = fp2_is_zero(den);
  const fp2 n = fp2_select(den0, fp2_from(k::SSWU_B_DIV_ZA_C0, k::SSWU_B_DIV_ZA_C1),
                           fp2_mul(fp2_from(k::SSWU_MB_DIV_A_C0, k::SSWU_MB_DIV_A_C1), fp2_add(den, fp2_one())));
  const fp2 d = fp2_select(den0, fp2_one(), den);
  const fp2 d2 = fp2_sqr(d), d3 = fp2_mul(d2, d);
  const fp2 gu = fp2_add(fp2_mul(n, fp2_add(fp2_sqr(n), fp2_mul(A, d2))), fp2_mul(B, d3));  // g(x1) D^3
  const fp2 u1 = fp2_mul(gu, fp2_conj(d3));  // g(x1) = u1 / e
  const fp e = fp2_norm(d3);
  fp r;
  const bool sq1 = fp_sqrt(r, fp2_norm(u1));
  const fp g2 = fp_mul(fp_mul(fp2_norm(zu2), fp_from(k::SQRT_M5)), fp_mul(fp2_norm(u), r));
  const fp2 a = fp2_select(sq1, u1, fp2_mul(fp2_mul(zu4, zu2), u1));  // g(x) e
  fp2 y = fp2_sqrt_ratio_from_gamma(a, e, fp_select(sq1, r, g2));
  const fp2 x = fp2_select(sq1, n, fp2_mul(zu2, n));
  if (!fp2_eq(fp2_mul_fp(fp2_sqr(y), e), a)) {  // never: the identities above
#if defined(MBLS_HOST_COUNT) && !defined(__HIP_DEVICE_COMPILE__)
    ++g_host_sswu_fallback;
#endif
    const aff<fp2> q = map_to_curve_sswu_two_roots(u);
    return {q.x, fp2_one(), q.y};
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return {x, d, y};
}
// the textbook form (two Fp2 square roots); only the guard above can reach it
MBLS_NI aff<fp2> map_to_curve_sswu_two_roots(const fp2& u) {
  const fp2 A = fp2_from(k::SSWU_A_C0, k::SSWU_A_C1), B = fp2_from(k::SSWU_B_C0, k::SSWU_B_C1);
  const fp2 Z = fp2_from(k::SSWU_Z_C0, k::SSWU_Z_C1);
  const fp2 zu2 = fp2_mul(Z, fp2_sqr(u));
  const fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  const bool den0 = fp2_is_zero(den);
  fp2 x1 = fp2_mul(fp2_from(k::SSWU_MB_DIV_A_C0, k::SSWU_MB_DIV_A_C1), fp2_add(fp2_one(), fp2_inv(den)));
  x1 = fp2_select(den0, fp2_from(k::SSWU_B_DIV_ZA_C0, k::SSWU_B_DIV_ZA_C1), x1);
  const fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  fp2 y;
  fp2 x = x1;
  if (!fp2_sqrt(y, gx1)) {
    x = fp2_mul(zu2, x1);
    const fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x), A), x), B);
    fp2_sqrt(y, gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return {x, y};
}

// ----- 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3), projective output, no inversion ------
// Input x = s / d (map_to_curve_sswu): the four polynomials homogenised in (s, d),
// XN = x_num d^3, XD = x_den d^2, YN = y_num d^3, YD = y_den d^3, so that
// x' = XN / (XD d) and y' = y YN / YD  ->  (XN YD : y YN XD d : XD d YD).
MBLS_NI proj<fp2> iso3_map(const sswu_pt& p) {
  const fp2 s = p.xn, d = p.xd;
  const fp2 s2 = fp2_sqr(s), s3 = fp2_mul(s2, s), d2 = fp2_sqr(d), d3 = fp2_mul(d2, d);
  const fp2 sd = fp2_mul(s, d), s2d = fp2_mul(s2, d), sd2 = fp2_mul(sd, d);
#define MBLS_K2(n) fp2_from(k::n##_C0, k::n##_C1)
  const fp2 xn = fp2_add(fp2_add(fp2_mul(MBLS_K2(ISO_XNUM3), s3), fp2_mul(MBLS_K2(ISO_XNUM2), s2d)),
                         fp2_add(fp2_mul(MBLS_K2(ISO_XNUM1), sd2), fp2_mul(MBLS_K2(ISO_XNUM0), d3)));
  const fp2 xd = fp2_add(fp2_add(s2, fp2_mul(MBLS_K2(ISO_XDEN1), sd)), fp2_mul(MBLS_K2(ISO_XDEN0), d2));
  const fp2 yn = fp2_add(fp2_add(fp2_mul(MBLS_K2(ISO_YNUM3), s3), fp2_mul(MBLS_K2(ISO_YNUM2), s2d)),
                         fp2_add(fp2_mul(MBLS_K2(ISO_YNUM1), sd2), fp2_mul(MBLS_K2(ISO_YNUM0), d3)));
  const fp2 yd = fp2_add(fp2_add(s3, fp2_mul(MBLS_K2(ISO_YDEN2), s2d)),
                         fp2_add(fp2_mul(MBLS_K2(ISO_YDEN1), sd2), fp2_mul(MBLS_K2(ISO_YDEN0), d3)));
#undef MBLS_K2
  const fp2 xdd = fp2_mul(xd, d);
  return {fp2_mul(xn, yd), fp2_mul(fp2_mul(p.y, yn), xdd), fp2_mul(xdd, yd)};
}

// ----- clear_cofactor (RFC 9380 Appendix G.3; equals h_eff * P) -------------------------
// [x]P, x < 0: on Jacobian coordinates (r05; the complete projective ladder it replaced measured
// 3-4% slower on deposit / gossip, profiles/r05_ab_h2c_jacobian.txt)
MBLS_NI proj<fp2> pt_mul_x(const proj<fp2>& p) { return pt_neg(g2_mul_xabs_jac(p)); }

MBLS_NI proj<fp2> clear_cofactor_g2(const proj<fp2>& P) {
  proj<fp2> t1 = pt_mul_x(P);
  proj<fp2> t2 = g2_psi(P);
  proj<fp2> t3 = g2_psi(g2_psi(pt_dbl(P)));
  t3 = pt_add(t3, pt_neg(t2));
  t2 = pt_add(t1, t2);
  t2 = pt_mul_x(t2);
  t3 = pt_add(t3, t2);
  t3 = pt_add(t3, pt_neg(t1));
  return pt_add(t3, pt_neg(P));
}

// hash_to_G2(msg32) with the PoP DST; projective result
MBLS_NI proj<fp2> hash_to_g2_msg32(const uint32_t (&msg)[8]) {
  uint32_t ub[64];
  expand_message_xmd_msg32(ub, msg);
  const fp2 u0 = {fp_from_64_bytes(ub + 0), fp_from_64_bytes(ub + 16)};
  const fp2 u1 = {fp_from_64_bytes(ub + 32), fp_from_64_bytes(ub + 48)};
  const proj<fp2> q0 = iso3_map(map_to_curve_sswu(u0));
  const proj<fp2> q1 = iso3_map(map_to_curve_sswu(u1));
  return clear_cofactor_g2(pt_add(q0, q1));
}

}  // namespace mbls
