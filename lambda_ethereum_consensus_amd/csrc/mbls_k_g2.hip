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
#include "mbls_soa.hpp"

using namespace mbls;

using namespace mbls_soa;

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
hipError_t miller_pairs(const int32_t* key_st, const uint32_t* key_xy, const uint32_t* h_xy, uint32_t n_pairs,
                        uint32_t* fpair, hipStream_t s) {
  if (n_pairs == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_MILLER_PAIRS, s);
  hipLaunchKernelGGL(mbls_k_miller_pairs, grid64(n_pairs), dim3(64), 0, s, key_st, key_xy, h_xy, n_pairs, fpair);
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
