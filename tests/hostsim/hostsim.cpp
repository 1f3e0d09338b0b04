// TEST INFRASTRUCTURE ONLY — host build of the device arithmetic headers.
//
// The kernels' field/curve/pairing code is written `__host__ __device__`; this file
// compiles the very same headers for the CPU so `tests/test_hostsim_*.py` can compare them
// against the Python oracle in this GPU-less container.  It is never linked into the
// product (`libmbls.so` dispatches to HIP kernels only) and exports no `Bls` entry point.
#include <cstdint>
#include <cstring>

#define MBLS_HOST_COUNT 1

#include "mbls_curve.hpp"
#include "mbls_h2c.hpp"
#include "mbls_pairing.hpp"

using namespace mbls;

namespace {
void be_to_words(const uint8_t* b, uint32_t* w, int nwords) {
  for (int i = 0; i < nwords; ++i)
    w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
}
void words_to_be(const uint32_t* w, uint8_t* b, int nwords) {
  for (int i = 0; i < nwords; ++i) {
    b[4 * i] = w[i] >> 24;
    b[4 * i + 1] = w[i] >> 16;
    b[4 * i + 2] = w[i] >> 8;
    b[4 * i + 3] = w[i];
  }
}
// 48-byte big-endian plain value (< p) -> Montgomery fp
fp load_fp(const uint8_t* b) {
  uint32_t w[12];
  be_to_words(b, w, 12);
  return fp_to_mont(fp_from_be_words(w));
}
void store_fp(const fp& a, uint8_t* b) {
  uint32_t w[12];
  fp_to_be_words(fp_from_mont(a), w);
  words_to_be(w, b, 12);
}
fp2 load_fp2(const uint8_t* b) { return {load_fp(b), load_fp(b + 48)}; }  // c0 || c1
void store_fp2(const fp2& a, uint8_t* b) {
  store_fp(a.c0, b);
  store_fp(a.c1, b + 48);
}
void store_fp12(const fp12& f, uint8_t* b) {  // 6 Fp2 coefficients of w^0..w^5 order c0.c0,c0.c1,c0.c2,c1.c0,...
  const fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) store_fp2(*c[i], b + 96 * i);
}
fp12 load_fp12(const uint8_t* b) {
  fp12 f;
  fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) *c[i] = load_fp2(b + 96 * i);
  return f;
}
}  // namespace

extern "C" {

// op: 0 add 1 sub 2 mul 3 sqr 4 inv 5 neg 6 sqrt (returns 0 if non-residue)
int hs_fp_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const fp x = load_fp(a), y = load_fp(b);
  fp r;
  int ok = 1;
  switch (op) {
    case 0: r = fp_add(x, y); break;
    case 1: r = fp_sub(x, y); break;
    case 2: r = fp_mul(x, y); break;
    case 3: r = fp_sqr(x); break;
    case 4: r = fp_inv(x); break;
    case 5: r = fp_neg(x); break;
    case 6: ok = fp_sqrt(r, x); break;
    default: return -1;
  }
  store_fp(r, out);
  return ok;
}

// Fp inverse of raw Montgomery digits (weakly reduced inputs, [p, 2p) included): the divstep
// inversion the kernels use (which = 0) or the a^(p-2) exponentiation it replaced (which = 1)
int hs_fp_inv_raw(int which, const uint32_t* a, uint32_t* out) {
  fp x;
  for (int i = 0; i < NL; ++i) x.v[i] = a[i];
  const fp r = which ? fp_inv_fermat(x) : fp_inv(x);
  for (int i = 0; i < NL; ++i) out[i] = r.v[i];
  return 0;
}

// op: 0 add 1 sub 2 mul 3 sqr 4 inv 5 neg 6 sqrt 7 mul_xi 8 is_square
int hs_fp2_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const fp2 x = load_fp2(a), y = load_fp2(b);
  fp2 r = fp2_zero();
  int ok = 1;
  switch (op) {
    case 0: r = fp2_add(x, y); break;
    case 1: r = fp2_sub(x, y); break;
    case 2: r = fp2_mul(x, y); break;
    case 3: r = fp2_sqr(x); break;
    case 4: r = fp2_inv(x); break;
    case 5: r = fp2_neg(x); break;
    case 6: ok = fp2_sqrt(r, x); break;
    case 7: r = fp2_mul_xi(x); break;
    case 8: ok = fp2_is_square(x); break;
    default: return -1;
  }
  store_fp2(r, out);
  return ok;
}

// Raw Montgomery digits in and out (28 x u32: c0 then c1), so tests can feed the weakly
// reduced representatives [p, 2p) and extreme digit patterns the canonical loaders never make.
// op: 0 mul 1 sqr 2 add 3 sub 4 mul_xi 5 neg
int hs_fp2_raw(int op, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  fp2 x, y;
  for (int i = 0; i < NL; ++i) {
    x.c0.v[i] = a[i];
    x.c1.v[i] = a[NL + i];
    y.c0.v[i] = b[i];
    y.c1.v[i] = b[NL + i];
  }
  fp2 r;
  switch (op) {
    case 0: r = fp2_mul(x, y); break;
    case 1: r = fp2_sqr(x); break;
    case 2: r = fp2_add(x, y); break;
    case 3: r = fp2_sub(x, y); break;
    case 4: r = fp2_mul_xi(x); break;
    case 5: r = fp2_neg(x); break;
    default: return -1;
  }
  for (int i = 0; i < NL; ++i) {
    out[i] = r.c0.v[i];
    out[NL + i] = r.c1.v[i];
  }
  return 1;
}

// lazy sum of n (<= 6) Fp2 products, times xi where xi[t]: sum_t (xi^e_t) a_t b_t, reduced once
int hs_fp2_sop(int n, const uint8_t* a, const uint8_t* b, const uint8_t* xi, uint8_t* out) {
  if (n < 0 || n > 6) return -1;
  fpcols re, im;
  cols_zero(re);
  cols_zero(im);
  for (int t = 0; t < n; ++t) fp2_cols_mad(re, im, load_fp2(a + 96 * t), load_fp2(b + 96 * t), xi[t] != 0);
  store_fp2(fp2_cols_redc(re, im), out);
  return 1;
}

int hs_g1_uncompress(const uint8_t* in48, uint8_t* x, uint8_t* y) {
  uint32_t w[12];
  be_to_words(in48, w, 12);
  aff<fp> a;
  a.x = fp_zero();
  a.y = fp_zero();
  const int32_t st = g1_uncompress(a, w);
  store_fp(a.x, x);
  store_fp(a.y, y);
  return st;
}
int hs_g1_in_subgroup(const uint8_t* x, const uint8_t* y) { return g1_in_subgroup({load_fp(x), load_fp(y)}); }

// op 0: P + Q (projective complete add), 1: P + Q (mixed), 2: 2P, 3: [|x|]P; result affine
int hs_g1_op(int op, const uint8_t* px, const uint8_t* py, const uint8_t* qx, const uint8_t* qy, uint8_t* rx, uint8_t* ry) {
  const aff<fp> p = {load_fp(px), load_fp(py)}, q = {load_fp(qx), load_fp(qy)};
  proj<fp> r;
  switch (op) {
    case 0: r = pt_add(pt_from_affine(p), pt_from_affine(q)); break;
    case 1: r = pt_add_affine(pt_from_affine(p), q); break;
    case 2: r = pt_dbl(pt_from_affine(p)); break;
    case 3: r = pt_mul_xabs_affine(p); break;
    default: return -1;
  }
  aff<fp> a;
  const bool fin = pt_to_affine(a, r);
  store_fp(a.x, rx);
  store_fp(a.y, ry);
  return fin;
}
void hs_g1_compress(const uint8_t* x, const uint8_t* y, int is_inf, uint8_t* out48) {
  uint32_t w[12];
  g1_compress(w, {load_fp(x), load_fp(y)}, is_inf != 0);
  words_to_be(w, out48, 12);
}

int hs_g2_uncompress(const uint8_t* in96, uint8_t* x, uint8_t* y) {
  uint32_t w[24];
  be_to_words(in96, w, 24);
  aff<fp2> a;
  a.x = fp2_zero();
  a.y = fp2_zero();
  const int32_t st = g2_uncompress(a, w);
  store_fp2(a.x, x);
  store_fp2(a.y, y);
  return st;
}
int hs_g2_in_subgroup(const uint8_t* x, const uint8_t* y) { return g2_in_subgroup({load_fp2(x), load_fp2(y)}); }
int hs_g2_op(int op, const uint8_t* px, const uint8_t* py, const uint8_t* qx, const uint8_t* qy, uint8_t* rx, uint8_t* ry) {
  const aff<fp2> p = {load_fp2(px), load_fp2(py)}, q = {load_fp2(qx), load_fp2(qy)};
  proj<fp2> r;
  switch (op) {
    case 0: r = pt_add(pt_from_affine(p), pt_from_affine(q)); break;
    case 1: r = pt_add_affine(pt_from_affine(p), q); break;
    case 2: r = pt_dbl(pt_from_affine(p)); break;
    case 3: r = pt_mul_xabs_affine(p); break;
    case 4: r = g2_psi(pt_from_affine(p)); break;
    case 5: r = g2_mul_xabs_jac(pt_from_affine(p)); break;  // hash_to_G2's Jacobian [|x|] ladder
    case 6: r = g2_mul_xabs(pt_from_affine(p)); break;      // the complete projective one
    default: return -1;
  }
  aff<fp2> a;
  const bool fin = pt_to_affine(a, r);
  store_fp2(a.x, rx);
  store_fp2(a.y, ry);
  return fin;
}
void hs_g2_compress(const uint8_t* x, const uint8_t* y, int is_inf, uint8_t* out96) {
  uint32_t w[24];
  g2_compress(w, {load_fp2(x), load_fp2(y)}, is_inf != 0);
  words_to_be(w, out96, 24);
}

// hash_to_G2 with the PoP DST of a 32-byte message; result affine
int hs_hash_to_g2(const uint8_t* msg32, uint8_t* x, uint8_t* y) {
  uint32_t w[8];
  be_to_words(msg32, w, 8);
  const proj<fp2> h = hash_to_g2_msg32(w);
  aff<fp2> a;
  const bool fin = pt_to_affine(a, h);
  store_fp2(a.x, x);
  store_fp2(a.y, y);
  return fin;
}
// expand_message_xmd(msg32, DST_POP, 256)
void hs_expand_xmd(const uint8_t* msg32, uint8_t* out256) {
  uint32_t w[8], o[64];
  be_to_words(msg32, w, 8);
  expand_message_xmd_msg32(o, w);
  words_to_be(o, out256, 64);
}
// map_to_curve_sswu + iso3 of one field element u (c0||c1 plain), affine result
#if !defined(__HIP_DEVICE_COMPILE__)
// times the SSWU map fell back to its two-root form (must stay 0)
uint64_t hs_sswu_fallbacks(void) { return g_host_sswu_fallback; }
#endif

void hs_map_to_curve(const uint8_t* u, uint8_t* x, uint8_t* y) {
  const proj<fp2> q = iso3_map(map_to_curve_sswu(load_fp2(u)));
  aff<fp2> a;
  pt_to_affine(a, q);
  store_fp2(a.x, x);
  store_fp2(a.y, y);
}

// sha256 of a short message
void hs_sha256(const uint8_t* msg, int len, uint8_t* out32) { sha256_bytes(msg, len, out32); }

// Miller loop + final exponentiation of one pair (affine inputs); out = 6*96 bytes
void hs_pairing(const uint8_t* px, const uint8_t* py, const uint8_t* qx, const uint8_t* qy, uint8_t* out) {
  const aff<fp> p = {load_fp(px), load_fp(py)};
  const aff<fp2> q = {load_fp2(qx), load_fp2(qy)};
  const fp12 f = final_exp(miller_loop_1(p, q));
  store_fp12(f, out);
}
void hs_miller_only_final_exp(const uint8_t* fin, uint8_t* out) { store_fp12(final_exp(load_fp12(fin)), out); }

// Fp12 ops: 0 mul 1 sqr 2 inv 3 frobenius(p) 4 cyclotomic sqr 5 conj
void hs_fp12_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const fp12 x = load_fp12(a), y = load_fp12(b);
  fp12 r;
  switch (op) {
    case 0: r = fp12_mul(x, y); break;
    case 1: r = fp12_sqr(x); break;
    case 2: r = fp12_inv(x); break;
    case 3: r = fp12_frob(x); break;
    case 4: r = fp12_cyclotomic_sqr(x); break;
    case 5: r = fp12_conj(x); break;
    default: r = x;
  }
  store_fp12(r, out);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Work model: Fp products of each phase of one valid (pk, msg, sig) verify as
// the DEVICE algorithms compute them (one-lane forms).  out[2k] = multiplications, out[2k+1]
// = squarings of phase k: 0 pk decompress, 1 G1 membership, 2 signature decompress, 3 G2
// membership, 4 hash_to_G2, 5 one-pair Miller loop, 6 final exponentiation, 7 two-pair Miller
// loop (shared squarings), 8 one G1 mixed addition (aggregation), 9 one Fp12 product.
// Returns 0, or the failing phase + 1.
int hs_count_phases(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig96, uint64_t* out) {
  // a two-product sum with one reduction (fp_mul2: 588 mads) counts as 1.5 multiplications, so
  // an Fp2 product stays 3 of them
  uint64_t* m = &g_host_mul;
  uint64_t* q = &g_host_sqr;
  uint64_t* m2 = &g_host_mul2;
  uint64_t m0, q0, m20;
  int phase = 0;
  auto begin = [&] { m0 = *m; q0 = *q; m20 = *m2; };
  auto end = [&] { out[2 * phase] = *m - m0 + 3 * (*m2 - m20) / 2; out[2 * phase + 1] = *q - q0; ++phase; };
  uint32_t w[24];
  be_to_words(pk48, w, 12);
  uint32_t w12[12];
  for (int i = 0; i < 12; ++i) w12[i] = w[i];
  aff<fp> p;
  begin();
  if (g1_uncompress(p, w12) != DEC_OK) return 1;
  end();
  begin();
  if (!g1_in_subgroup(p)) return 2;
  end();
  be_to_words(sig96, w, 24);
  aff<fp2> s;
  begin();
  if (g2_uncompress(s, w) != DEC_OK) return 3;
  end();
  begin();
  if (!g2_in_subgroup(s)) return 4;
  end();
  uint32_t mw[8];
  be_to_words(msg32, mw, 8);
  aff<fp2> h;
  begin();
  pt_to_affine(h, hash_to_g2_msg32(mw));
  end();
  begin();
  const fp12 f1 = miller_loop_1(p, h);
  end();
  begin();
  (void)final_exp(f1);
  end();
  begin();
  const aff<fp> ng = {fp_from(k::G1X), fp_from(k::G1Y_NEG)};
  (void)miller_loop_2(p, h, ng, s);
  end();
  begin();
  (void)pt_add_affine(pt_from_affine(p), p);
  end();
  begin();
  (void)fp12_mul(f1, f1);
  end();
  return 0;
}
#endif

}  // extern "C"
