// mbls_k_g2.hip — G2-side kernels: signature decode + G2 membership, hash_to_G2, the
// pairing verdicts for verify / fast_aggregate_verify / aggregate_verify, sign, and
// signature aggregation.
//
// Built with MBLS_FP_OUTLINE: the Fp multiply is a scalar-argument call, so these long
// kernels (Miller loop + final exponentiation, SSWU + cofactor clearing) stay I-cache sized.
// Replaces the blst calls behind lighthouse Signature::deserialize / verify /
// fast_aggregate_verify / eth_fast_aggregate_verify / aggregate_verify / sign / aggregate
// (native/bls_nif/src/lib.rs:14-119).
#define MBLS_FP_OUTLINE 1
#include "mbls_h2c.hpp"
#include "mbls_kernels.h"
#include "mbls_pairing.hpp"
#include "mbls_pairing_lg.hpp"

using namespace mbls;

namespace {

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

}  // namespace

// One lane per set: the signature-side Miller loop f_{|x|,sigma}(-g1) (conjugated), which
// depends only on the signature and so runs on the aux stream while the keys are being
// validated.  Sets whose signature is not a usable G2 point store 1 (an infinite signature
// is skipped by blst's pairing aggregation: e(-g1, O) = 1).
extern "C" __global__ __launch_bounds__(64) void mbls_k_sig_miller(const int32_t* __restrict__ sig_st,
                                                                  const uint32_t* __restrict__ sig_xy, uint32_t n_sets,
                                                                  uint32_t* __restrict__ fsig) {
  // latency-critical per-set chain: win issue arbitration against the co-resident
  // throughput-bound key-validation waves (static priority, MI355X_MICROARCH §Two waves)
  __builtin_amdgcn_s_setprio(3);
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  fp12 f = fp12_one();
  if (sig_st[s] == MBLS_DEC_OK) f = miller_loop_1(neg_g1_gen(), ld_g2(sig_xy, n_sets, s));
  st_fp12(fsig, n_sets, s, f);
}

// One lane per signature: NONE (all-zero) detection, ZCash G2 decode, optional G2
// membership (blst sig_groupcheck=true in verify paths; aggregate does no group check).
extern "C" __global__ __launch_bounds__(64) void mbls_k_g2_sig_decode(const uint8_t* __restrict__ sigs, uint32_t n,
                                                                     int32_t group_check,
                                                                     const int32_t* __restrict__ pre,
                                                                     int32_t* __restrict__ st,
                                                                     uint32_t* __restrict__ xy) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (pre && pre[i] != MBLS_DEC_OK) {  // host-detected (wrong length -> BLST_BAD_ENCODING)
    st[i] = pre[i];
    return;
  }
  uint32_t w[24];
  load_be<24>(sigs + (size_t)i * 96, w);
  uint32_t any = 0;
#pragma unroll
  for (int j = 0; j < 24; ++j) any |= w[j];
  aff<fp2> a;
  a.x = fp2_zero();
  a.y = fp2_zero();
  int32_t s;
  if (any == 0) {
    s = MBLS_DEC_NONE;
  } else {
    s = g2_uncompress(a, w);
    if (s == MBLS_DEC_OK && group_check && !g2_in_subgroup(a)) s = MBLS_DEC_SIG_NOT_IN_G2;
  }
  st[i] = s;
  st_g2(xy, n, i, a);
}

// One lane per message: H(m) = hash_to_G2(m, DST_POP), affine.
extern "C" __global__ __launch_bounds__(64) void mbls_k_hash_to_g2(const uint8_t* __restrict__ msgs, uint32_t n,
                                                                  uint32_t* __restrict__ hxy) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  load_be<8>(msgs + (size_t)i * 32, w);
  aff<fp2> a;
  pt_to_affine(a, hash_to_g2_msg32(w));
  st_g2(hxy, n, i, a);
}

// One lane per set: fast_aggregate_verify / eth_fast_aggregate_verify / verify verdict with
// the reference's precedence (signature decode error, then the first key error, then the
// boolean rules of lighthouse GenericAggregateSignature + blst).
// key_off == nullptr means one key per set (Bls.verify).  fsig (optional): the precomputed
// signature-side Miller values of mbls_k_sig_miller; without it the loop runs here.
extern "C" __global__ __launch_bounds__(64) void mbls_k_fav_verdict(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy, const uint32_t* __restrict__ fsig,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, int32_t eth_variant, const int32_t* __restrict__ set_pre,
    int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  const int32_t ss = sig_st[s];
  const int32_t ps = pk_st[s];
  const int32_t sp = set_pre ? set_pre[s] : 0;  // host message-level outcome (-7), after key errors
  const uint32_t nk = key_off ? key_off[s + 1] - key_off[s] : 1u;
  int32_t out;
  if (ss == MBLS_DEC_BAD_ENCODING || ss == MBLS_DEC_NOT_ON_CURVE) {
    out = mbls_sig_code(ss);
  } else if (mbls_is_pk_error(ps)) {
    out = mbls_pk_code(ps);
  } else if (sp != 0) {
    out = sp;
  } else if (nk == 0) {
    out = (eth_variant && ss == MBLS_DEC_INFINITY) ? 1 : 0;
  } else if (ss == MBLS_DEC_NONE || ps == MBLS_AGG_INFINITY || ss == MBLS_DEC_SIG_NOT_IN_G2) {
    out = 0;
  } else {
    const aff<fp> p = ld_g1(pk_xy, n_sets, s);
    const aff<fp2> h = ld_g2(h_xy, n_sets, s);
    fp12 f = miller_loop_1(p, h);
    if (fsig) {
      f = fp12_mul(f, ld_fp12(fsig, n_sets, s));  // precomputed e(-g1, sigma) Miller value (1 if infinite)
    } else if (ss != MBLS_DEC_INFINITY) {       // blst skips an infinite signature: e(-g1, O) = 1
      f = fp12_mul(f, miller_loop_1(neg_g1_gen(), ld_g2(sig_xy, n_sets, s)));
    }
    out = fp12_is_one(final_exp(f)) ? 1 : 0;
  }
  status[s] = out;
}

// ----- lane-group forms (mbls_pairing_lg.hpp): 8 sets per wave, lane k of a group holds the
// coefficient of w^k.  Per-lane Fp12 values are stored lane-major: dword d of lane l of
// n_lanes at base[d * n_lanes + l] (coalesced). ------------------------------------------
namespace {
__device__ __forceinline__ void st_lane(uint32_t* base, size_t nl, size_t l, const fp2& a) {
  st_fp(base, nl, l, 0, a.c0);
  st_fp(base, nl, l, NL, a.c1);
}
__device__ __forceinline__ fp2 ld_lane(const uint32_t* base, size_t nl, size_t l) {
  return {ld_fp(base, nl, l, 0), ld_fp(base, nl, l, NL)};
}
}  // namespace

// The signature-side Miller value of mbls_k_sig_miller, one set per 8-lane group.
extern "C" __global__ __launch_bounds__(64) void mbls_k_sig_miller_lg(const int32_t* __restrict__ sig_st,
                                                                     const uint32_t* __restrict__ sig_xy,
                                                                     uint32_t n_sets, uint32_t* __restrict__ fsig) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;  // tail groups compute on a copy, store nothing
  fp2 f = lg::x12_one();
  if (sig_st[s] == MBLS_DEC_OK) f = lg::miller_lg(pt_from_affine(neg_g1_gen()), ld_g2(sig_xy, n_sets, s));
  if (g < n_sets) st_lane(fsig, (size_t)n_sets * 8, (size_t)g * 8 + lg::gk(), f);
}

// mbls_k_fav_verdict (same precedence and boolean rules) with the pairing on 8-lane groups;
// pk_xy holds the projective per-set key sums of mbls_k_g1_aggregate, fsig (required) the
// values of mbls_k_sig_miller_lg.
extern "C" __global__ __launch_bounds__(64) void mbls_k_fav_verdict_lg(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ h_xy,
    uint32_t n_sets, int32_t eth_variant, const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const int32_t ss = sig_st[s];
  const int32_t ps = pk_st[s];
  const int32_t sp = set_pre ? set_pre[s] : 0;
  const uint32_t nk = key_off ? key_off[s + 1] - key_off[s] : 1u;
  int32_t out = -1000;
  if (ss == MBLS_DEC_BAD_ENCODING || ss == MBLS_DEC_NOT_ON_CURVE) {
    out = mbls_sig_code(ss);
  } else if (mbls_is_pk_error(ps)) {
    out = mbls_pk_code(ps);
  } else if (sp != 0) {
    out = sp;
  } else if (nk == 0) {
    out = (eth_variant && ss == MBLS_DEC_INFINITY) ? 1 : 0;
  } else if (ss == MBLS_DEC_NONE || ps == MBLS_AGG_INFINITY || ss == MBLS_DEC_SIG_NOT_IN_G2) {
    out = 0;
  }
  if (out == -1000) {  // group uniform: every lane of the group has the same set
    const proj<fp> pk = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL), ld_fp(pk_xy, n_sets, s, 2 * NL)};
    fp2 f = lg::miller_lg(pk, ld_g2(h_xy, n_sets, s));
    f = lg::x12_mul(f, ld_lane(fsig, (size_t)n_sets * 8, (size_t)s * 8 + lg::gk()));
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (g < n_sets && lg::gk() == 0) status[g] = out;
}

// One lane per (key, message) pair: the Miller value f_{|x|,H(m)}(pk) (conjugated), written
// in the lane layout of the lane-group kernels (pair j, coefficient k at row 8 j + k).  A pair
// whose key did not decode stores 1 (its set is decided by the key error anyway).
extern "C" __global__ __launch_bounds__(64) void mbls_k_miller_pairs(const int32_t* __restrict__ key_st,
                                                                    const uint32_t* __restrict__ key_xy,
                                                                    const uint32_t* __restrict__ h_xy,
                                                                    uint32_t n_pairs, uint32_t* __restrict__ fpair) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_pairs) return;
  fp12 f = fp12_one();
  if (key_st[j] == MBLS_DEC_OK) f = miller_loop_1(ld_g1(key_xy, n_pairs, j), ld_g2(h_xy, n_pairs, j));
  const fp2* c[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};  // w^0 .. w^5
  const size_t nl = (size_t)n_pairs * 8;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    st_fp(fpair, nl, (size_t)j * 8 + k, 0, c[k]->c0);
    st_fp(fpair, nl, (size_t)j * 8 + k, NL, c[k]->c1);
  }
#pragma unroll
  for (int k = 6; k < 8; ++k) {
    st_fp(fpair, nl, (size_t)j * 8 + k, 0, fp_zero());
    st_fp(fpair, nl, (size_t)j * 8 + k, NL, fp_zero());
  }
}

// aggregate_verify verdicts (mbls_k_av_verdict's precedence and rules) from per-pair Miller
// values (mbls_k_miller_pairs) and the signature-side values (mbls_k_sig_miller_lg): one set
// per 8-lane group, product of the set's pair values, then the lane-group final exponentiation.
extern "C" __global__ __launch_bounds__(64) void mbls_k_av_verdict_lg(
    const int32_t* __restrict__ key_st, uint32_t n_pairs, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ fpair,
    uint32_t n_sets, const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const int32_t ss = sig_st[s];
  const uint32_t lo = key_off[s], hi = key_off[s + 1];
  int32_t out = -1000;
  if (ss == MBLS_DEC_BAD_ENCODING || ss == MBLS_DEC_NOT_ON_CURVE) out = mbls_sig_code(ss);
  if (out == -1000) {
    for (uint32_t j = lo; j < hi; ++j) {
      const int32_t ks = key_st[j];
      if (ks != MBLS_DEC_OK) {
        out = mbls_pk_code(ks);
        break;
      }
    }
  }
  if (out == -1000 && set_pre && set_pre[s] != 0) out = set_pre[s] == MBLS_SET_FALSE ? 0 : set_pre[s];
  if (out == -1000 && (hi == lo || ss == MBLS_DEC_NONE || ss == MBLS_DEC_SIG_NOT_IN_G2)) out = 0;
  if (out == -1000) {  // group uniform
    const int k = lg::gk();
    // an infinite signature is skipped by blst (its stored value is 1)
    fp2 f = ld_lane(fsig, (size_t)n_sets * 8, (size_t)s * 8 + k);
    const size_t nl = (size_t)n_pairs * 8;
#pragma unroll 1
    for (uint32_t j = lo; j < hi; ++j) f = lg::x12_mul(f, ld_lane(fpair, nl, (size_t)j * 8 + k));
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (g < n_sets && lg::gk() == 0) status[g] = out;
}

// One lane per set: aggregate_verify.  Pair j of set s = (key j, message j) for
// key_off[s] <= j < key_off[s+1]; h_xy holds H(m_j) per pair.
extern "C" __global__ __launch_bounds__(64) void mbls_k_av_verdict(
    const int32_t* __restrict__ key_st, const uint32_t* __restrict__ key_xy, uint32_t n_pairs,
    const uint32_t* __restrict__ key_off, const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, const int32_t* __restrict__ set_pre,
    int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  const int32_t ss = sig_st[s];
  const uint32_t lo = key_off[s], hi = key_off[s + 1];
  int32_t out = -1000;
  if (ss == MBLS_DEC_BAD_ENCODING || ss == MBLS_DEC_NOT_ON_CURVE) out = mbls_sig_code(ss);
  if (out == -1000) {
    for (uint32_t j = lo; j < hi; ++j) {
      const int32_t ks = key_st[j];
      if (ks != MBLS_DEC_OK) {
        out = mbls_pk_code(ks);
        break;
      }
    }
  }
  // host message-level outcome: -7 (message length) or MBLS_SET_FALSE (count mismatch)
  if (out == -1000 && set_pre && set_pre[s] != 0) out = set_pre[s] == MBLS_SET_FALSE ? 0 : set_pre[s];
  if (out == -1000) {
    if (hi == lo || ss == MBLS_DEC_NONE || ss == MBLS_DEC_SIG_NOT_IN_G2) {
      out = 0;
    } else {
      fp12 f = fp12_one();
      for (uint32_t j = lo; j < hi; ++j) f = fp12_mul(f, miller_loop_1(ld_g1(key_xy, n_pairs, j), ld_g2(h_xy, n_pairs, j)));
      if (ss != MBLS_DEC_INFINITY) f = fp12_mul(f, miller_loop_1(neg_g1_gen(), ld_g2(sig_xy, n_sets, s)));
      out = fp12_is_one(final_exp(f)) ? 1 : 0;
    }
  }
  status[s] = out;
}

// One lane per (sk, msg): sigma = sk * H(m), compressed.  The secret key has been range
// checked on the host (0 < sk < r, lighthouse SecretKey::deserialize).  Constant-time
// double-and-always-add over 256 bits.
extern "C" __global__ __launch_bounds__(64) void mbls_k_sign(const uint8_t* __restrict__ sk32,
                                                            const uint8_t* __restrict__ msgs, uint32_t n,
                                                            uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t m[8], sk[8];
  load_be<8>(msgs + (size_t)i * 32, m);
  load_be<8>(sk32 + (size_t)i * 32, sk);
  const proj<fp2> h = hash_to_g2_msg32(m);
  proj<fp2> r = pt_identity<fp2>();
#pragma unroll 1
  for (int b = 255; b >= 0; --b) {
    r = pt_dbl(r);
    const proj<fp2> t = pt_add(r, h);
    const bool bit = (sk[7 - (b >> 5)] >> (b & 31)) & 1u;
    r = pt_select(bit, t, r);
  }
  aff<fp2> a;
  const bool fin = pt_to_affine(a, r);
  uint32_t w[24];
  g2_compress(w, a, !fin);
  store_be<24>(out96 + (size_t)i * 96, w);
}

// One lane per set: Bls.aggregate — sum of the decoded signatures (NONE skipped, no group
// check, first undecodable signature is the error), compressed.
extern "C" __global__ __launch_bounds__(64) void mbls_k_g2_aggregate(const int32_t* __restrict__ sig_st,
                                                                    const uint32_t* __restrict__ sig_xy,
                                                                    uint32_t n_sigs, const uint32_t* __restrict__ off,
                                                                    uint32_t n_sets, uint8_t* __restrict__ out96,
                                                                    int32_t* __restrict__ status) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  const uint32_t lo = off[s], hi = off[s + 1];
  int32_t out = 2;  // MBLS_OK
  if (hi == lo) out = -8;  // Empty signature vector
  for (uint32_t j = lo; j < hi && out == 2; ++j) {
    const int32_t st = sig_st[j];
    if (st == MBLS_DEC_BAD_ENCODING || st == MBLS_DEC_NOT_ON_CURVE) out = mbls_sig_code(st);
  }
  uint32_t w[24];
#pragma unroll
  for (int j = 0; j < 24; ++j) w[j] = 0;
  if (out == 2) {
    proj<fp2> acc = pt_identity<fp2>();
    for (uint32_t j = lo; j < hi; ++j)
      if (sig_st[j] == MBLS_DEC_OK) acc = pt_add_affine(acc, ld_g2(sig_xy, n_sigs, j));
    aff<fp2> a;
    const bool fin = pt_to_affine(a, acc);
    g2_compress(w, a, !fin);
  }
  store_be<24>(out96 + (size_t)s * 96, w);
  status[s] = out;
}

// ----- host launch wrappers ---------------------------------------------------------------
namespace mbls_launch {
static inline dim3 grid64(uint32_t n) { return dim3((n + 63) / 64); }
hipError_t g2_sig_decode(const uint8_t* sigs, uint32_t n, int32_t group_check, const int32_t* pre, int32_t* st,
                         uint32_t* xy, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G2_SIG_DECODE, s);
  hipLaunchKernelGGL(mbls_k_g2_sig_decode, grid64(n), dim3(64), 0, s, sigs, n, group_check, pre, st, xy);
  return hipGetLastError();
}
hipError_t hash_to_g2(const uint8_t* msgs, uint32_t n, uint32_t* hxy, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_HASH_TO_G2, s);
  hipLaunchKernelGGL(mbls_k_hash_to_g2, grid64(n), dim3(64), 0, s, msgs, n, hxy);
  return hipGetLastError();
}
hipError_t sig_miller(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sets, uint32_t* fsig, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_SIG_MILLER, s);
  hipLaunchKernelGGL(mbls_k_sig_miller, grid64(n_sets), dim3(64), 0, s, sig_st, sig_xy, n_sets, fsig);
  return hipGetLastError();
}
hipError_t fav_verdict(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                       const uint32_t* sig_xy, const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets,
                       int32_t eth_variant, const int32_t* set_pre, int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_FAV_VERDICT, s);
  hipLaunchKernelGGL(mbls_k_fav_verdict, grid64(n_sets), dim3(64), 0, s, pk_st, pk_xy, key_off, sig_st, sig_xy, fsig,
                     h_xy, n_sets, eth_variant, set_pre, status);
  return hipGetLastError();
}
hipError_t sig_miller_lg(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sets, uint32_t* fsig,
                         hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_SIG_MILLER, s);
  hipLaunchKernelGGL(mbls_k_sig_miller_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, sig_st, sig_xy, n_sets, fsig);
  return hipGetLastError();
}
hipError_t fav_verdict_lg(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                          const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets, int32_t eth_variant,
                          const int32_t* set_pre, int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_FAV_VERDICT, s);
  hipLaunchKernelGGL(mbls_k_fav_verdict_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, pk_st, pk_xy, key_off, sig_st,
                     fsig, h_xy, n_sets, eth_variant, set_pre, status);
  return hipGetLastError();
}
hipError_t miller_pairs(const int32_t* key_st, const uint32_t* key_xy, const uint32_t* h_xy, uint32_t n_pairs,
                        uint32_t* fpair, hipStream_t s) {
  if (n_pairs == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_MILLER_PAIRS, s);
  hipLaunchKernelGGL(mbls_k_miller_pairs, grid64(n_pairs), dim3(64), 0, s, key_st, key_xy, h_xy, n_pairs, fpair);
  return hipGetLastError();
}
hipError_t av_verdict_lg(const int32_t* key_st, uint32_t n_pairs, const uint32_t* key_off, const int32_t* sig_st,
                         const uint32_t* fsig, const uint32_t* fpair, uint32_t n_sets, const int32_t* set_pre,
                         int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_AV_VERDICT, s);
  hipLaunchKernelGGL(mbls_k_av_verdict_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, key_st, n_pairs, key_off, sig_st,
                     fsig, fpair, n_sets, set_pre, status);
  return hipGetLastError();
}
hipError_t av_verdict(const int32_t* key_st, const uint32_t* key_xy, uint32_t n_pairs, const uint32_t* key_off,
                      const int32_t* sig_st, const uint32_t* sig_xy, const uint32_t* h_xy, uint32_t n_sets,
                      const int32_t* set_pre, int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_AV_VERDICT, s);
  hipLaunchKernelGGL(mbls_k_av_verdict, grid64(n_sets), dim3(64), 0, s, key_st, key_xy, n_pairs, key_off, sig_st,
                     sig_xy, h_xy, n_sets, set_pre, status);
  return hipGetLastError();
}
hipError_t sign(const uint8_t* sk32, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_SIGN, s);
  hipLaunchKernelGGL(mbls_k_sign, grid64(n), dim3(64), 0, s, sk32, msgs, n, out96);
  return hipGetLastError();
}
hipError_t g2_aggregate(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sigs, const uint32_t* off,
                        uint32_t n_sets, uint8_t* out96, int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G2_AGGREGATE, s);
  hipLaunchKernelGGL(mbls_k_g2_aggregate, grid64(n_sets), dim3(64), 0, s, sig_st, sig_xy, n_sigs, off, n_sets, out96,
                     status);
  return hipGetLastError();
}
}  // namespace mbls_launch
