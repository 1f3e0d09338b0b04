// mbls_k_lg.hip — the lane-group pairing kernels (mbls_pairing_lg.hpp: one set per 8-lane
// group): signature-side Miller values, fast_aggregate_verify and aggregate_verify verdicts.
// Their own translation unit so that every function they call is compiled under the same
// occupancy bound (a callee shared with the 512-VGPR single-lane kernels would be compiled
// for the largest budget, and a kernel's allocation is the maximum over its callees).
#define MBLS_FP_OUTLINE 1
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "mbls_kernels.h"
#include "mbls_pairing_lg.hpp"
#include "mbls_soa.hpp"

#define MBLS_LG_BLOCKS_PER_CU 1

using namespace mbls;
using namespace mbls_soa;

// ----- lane-group forms (mbls_pairing_lg.hpp): 8 sets per wave, lane k of a group holds the
// coefficient of w^k.  Per-lane Fp12 values are stored lane-major: dword d of lane l of
// n_lanes at base[d * n_lanes + l] (coalesced). ------------------------------------------
// The signature-side Miller value of mbls_k_sig_miller, one set per 8-lane group.
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_sig_miller_lg(const int32_t* __restrict__ sig_st,
                                                                     const uint32_t* __restrict__ sig_xy,
                                                                     uint32_t n_sets, uint32_t* __restrict__ fsig,
                                                                     const int32_t* __restrict__ rlc_ok) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  if (rlc_ok && *rlc_ok) return;  // the batch check passed: no per-set pairing is needed
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;  // tail groups compute on a copy, store nothing
  fp2 f = lg::x12_one();
  if (sig_st[s] == MBLS_DEC_OK) f = lg::miller_lg(pt_from_affine(neg_g1_gen()), ld_g2(sig_xy, n_sets, s));
  if (g < n_sets) st_lane(fsig, (size_t)n_sets * 8, (size_t)g * 8 + lg::gk(), f);
}

// mbls_k_fav_verdict (same precedence and boolean rules) with the pairing on 8-lane groups;
// pk_xy holds the projective per-set key sums of mbls_k_g1_aggregate; fsig (optional) the
// signature-side values of mbls_k_sig_miller_lg, else both Miller loops run here together.
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_fav_verdict_lg(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy, const uint32_t* __restrict__ fsig,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, int32_t eth_variant, const int32_t* __restrict__ set_pre,
    const int32_t* __restrict__ rlc_ok, int32_t* __restrict__ status, int32_t fsig_onelane) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const uint32_t nk = key_off ? key_off[s + 1] - key_off[s] : 1u;
  int32_t out = mbls_fav_precheck(sig_st[s], pk_st[s], set_pre ? set_pre[s] : 0, nk, eth_variant);
  if (out == MBLS_NEEDS_PAIRING && rlc_ok && *rlc_ok) out = 1;  // covered by the batch check
  if (out == MBLS_NEEDS_PAIRING) {  // group uniform: every lane of the group has the same set
    // (Bls.verify, no key_off: a decoded affine key, 28 rows)
    const proj<fp> pk = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL),
                         key_off ? ld_fp(pk_xy, n_sets, s, 2 * NL) : fp_one()};
    fp2 f;
    if (fsig) {  // signature side precomputed by mbls_k_sig_miller_lg (or, fsig_onelane, by
                 // the one-lane mbls_k_sig_miller: a deferred cold verdict, mbls_engine.cpp)
      f = lg::miller_lg(pk, ld_g2(h_xy, n_sets, s));
      f = lg::x12_mul(f, fsig_onelane ? ld_fp12_coef(fsig, n_sets, s, lg::gk())
                                      : ld_lane(fsig, (size_t)n_sets * 8, (size_t)s * 8 + lg::gk()));
    } else {  // both pairs in one loop (shared squarings); an infinite signature is skipped
      f = lg::miller2_lg(pk, ld_g2(h_xy, n_sets, s), pt_from_affine(neg_g1_gen()), ld_g2(sig_xy, n_sets, s),
                         sig_st[s] == MBLS_DEC_OK);
    }
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (g < n_sets && lg::gk() == 0) status[g] = out;
}

// mbls_k_fav_verdict_lg on 16-lane groups (4 sets per wave, mbls_pairing_lg.hpp): the Fp12
// values hold one Fp component per lane, the Miller steps run in duplicate on the two 8-lane
// halves.  Same inputs, precedence and outputs.
__device__ __forceinline__ fp ld_fsig16(const uint32_t* fsig, uint32_t n_sets, uint32_t s, int onelane) {
  const int c = lg::hc(), k = c >> 1, h = c & 1;
  if (onelane) {  // st_fp12 layout: w^(2j) is component j, w^(2j+1) component 3 + j
    const int j = k >= 6 ? 0 : (k & 1) ? 3 + (k >> 1) : (k >> 1);
    return lg::pad16(ld_fp(fsig, n_sets, s, (2 * j + h) * NL));
  }
  return ld_fp(fsig, (size_t)n_sets * 8, (size_t)s * 8 + k, h * NL);  // lane layout (pad lanes hold 0)
}
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_fav_verdict_lg16(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy, const uint32_t* __restrict__ fsig,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, int32_t eth_variant, const int32_t* __restrict__ set_pre,
    const int32_t* __restrict__ rlc_ok, int32_t* __restrict__ status, int32_t fsig_onelane) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 4);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const uint32_t nk = key_off ? key_off[s + 1] - key_off[s] : 1u;
  int32_t out = mbls_fav_precheck(sig_st[s], pk_st[s], set_pre ? set_pre[s] : 0, nk, eth_variant);
  if (out == MBLS_NEEDS_PAIRING && rlc_ok && *rlc_ok) out = 1;
  if (out == MBLS_NEEDS_PAIRING) {  // group uniform
    // (Bls.verify, no key_off: a decoded affine key, 28 rows)
    const proj<fp> pk = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL),
                         key_off ? ld_fp(pk_xy, n_sets, s, 2 * NL) : fp_one()};
    fp f;
    if (fsig) {
      f = lg::miller16(pk, ld_g2(h_xy, n_sets, s));
      f = lg::x16_mul(f, ld_fsig16(fsig, n_sets, s, fsig_onelane));
    } else {
      f = lg::miller2_16(pk, ld_g2(h_xy, n_sets, s), pt_from_affine(neg_g1_gen()), ld_g2(sig_xy, n_sets, s),
                         sig_st[s] == MBLS_DEC_OK);
    }
    out = lg::x16_is_one(lg::x16_final_exp(f)) ? 1 : 0;
  }
  if (g < n_sets && lg::hc() == 0) status[g] = out;
}

// aggregate_verify verdicts (mbls_k_av_verdict's precedence and rules) from per-pair Miller
// values (mbls_k_miller_pairs) and the signature-side values (mbls_k_sig_miller_lg): one set
// per 8-lane group, product of the set's pair values, then the lane-group final exponentiation.
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_av_verdict_lg(
    const int32_t* __restrict__ key_st, uint32_t n_pairs, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ fpair,
    uint32_t n_sets, const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
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

// hash_to_G2 of one message per 8-lane group (lane-group form of mbls_k_hash_to_g2 for
// latency-bound batches): affine H(m) in the same SoA layout
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_hash_to_g2_lg(
    const uint8_t* __restrict__ msgs, uint32_t n, uint32_t* __restrict__ hxy) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n ? g : n - 1;
  uint32_t w[8];
  load_be<8>(msgs + (size_t)s * 32, w);
  aff<fp2> a;
  pt_to_affine(a, lg::hash_to_g2_lg(w));
  if (g < n && lg::gk() == 0) st_g2(hxy, n, s, a);
}

// The G2 side of a latency-critical FAV call in one launch, two kinds of blocks side by side:
// blocks [0, nb) hash one message per group (as mbls_k_hash_to_g2_lg); blocks [nb, 2 nb)
// decode one signature per group (as mbls_k_g2_sig_decode with the group check; the psi test's
// [x] sigma in lane-parallel rounds) and, when fsig is given, run its signature-side Miller
// loop (as mbls_k_sig_miller_lg).  The two chains overlap instead of running back to back.
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_g2_prep_lg(
    const uint8_t* __restrict__ sigs, const int32_t* __restrict__ sig_pre, const uint8_t* __restrict__ msgs,
    uint32_t n, int32_t* __restrict__ sig_st, uint32_t* __restrict__ sig_xy, uint32_t* __restrict__ hxy,
    uint32_t* __restrict__ fsig, uint32_t parts) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t nb = (n + 7) / 8;
  // parts: 1 hash blocks only, 2 signature blocks only, 3 both (hash blocks first)
  const bool hash_part = parts == 3 ? blockIdx.x < nb : parts == 1;  // block (wave) uniform
  const uint32_t g = (hash_part || parts != 3 ? blockIdx.x : blockIdx.x - nb) * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n ? g : n - 1;
  const int k = lg::gk();
  if (hash_part) {
    uint32_t w[8];
    load_be<8>(msgs + (size_t)s * 32, w);
    aff<fp2> a;
    pt_to_affine(a, lg::hash_to_g2_lg(w));
    if (g < n && k == 0) st_g2(hxy, n, s, a);
    return;
  }
  aff<fp2> a;
  a.x = fp2_zero();
  a.y = fp2_zero();
  int32_t st;
  if (sig_pre && sig_pre[s] != MBLS_DEC_OK) {
    st = sig_pre[s];
  } else {
    uint32_t w[24];
    load_be<24>(sigs + (size_t)s * 96, w);
    uint32_t any = 0;
#pragma unroll
    for (int j = 0; j < 24; ++j) any |= w[j];
    if (any == 0) {
      st = MBLS_DEC_NONE;
    } else {
      st = g2_uncompress(a, w);
      if (st == MBLS_DEC_OK) {  // group uniform
        const proj<fp2> q = pt_from_affine(a);
        if (!pt_eq(g2_psi(q), lg::g2_mul_x_lg(q))) st = MBLS_DEC_SIG_NOT_IN_G2;
      }
    }
  }
  if (g < n && k == 0) {
    sig_st[s] = st;
    st_g2(sig_xy, n, s, a);
  }
  if (fsig) {
    fp2 f = lg::x12_one();
    if (st == MBLS_DEC_OK) f = lg::miller_lg(pt_from_affine(neg_g1_gen()), a);
    if (g < n) st_lane(fsig, (size_t)n * 8, (size_t)g * 8 + k, f);
  }
}

// mbls_k_g2_prep_lg on 16-lane groups (4 sets per wave): the hash and decode chains run their
// 8-lane code in duplicate on the two halves, the signature-side Miller loop in the 16-lane
// form; fsig is written in the same lane layout (lane (k, h) stores component h of w^k).
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_g2_prep_lg16(
    const uint8_t* __restrict__ sigs, const int32_t* __restrict__ sig_pre, const uint8_t* __restrict__ msgs,
    uint32_t n, int32_t* __restrict__ sig_st, uint32_t* __restrict__ sig_xy, uint32_t* __restrict__ hxy,
    uint32_t* __restrict__ fsig, uint32_t parts) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t nb = (n + 3) / 4;
  // parts: 1 hash blocks only, 2 signature blocks only, 3 both (hash blocks first)
  const bool hash_part = parts == 3 ? blockIdx.x < nb : parts == 1;  // block (wave) uniform
  const uint32_t g = (hash_part || parts != 3 ? blockIdx.x : blockIdx.x - nb) * 4u + (threadIdx.x >> 4);
  const uint32_t s = g < n ? g : n - 1;
  const int c = lg::hc();
  if (hash_part) {
    uint32_t w[8];
    load_be<8>(msgs + (size_t)s * 32, w);
    aff<fp2> a;
    pt_to_affine(a, lg::hash_to_g2_lg(w));
    if (g < n && c == 0) st_g2(hxy, n, s, a);
    return;
  }
  aff<fp2> a;
  a.x = fp2_zero();
  a.y = fp2_zero();
  int32_t st;
  if (sig_pre && sig_pre[s] != MBLS_DEC_OK) {
    st = sig_pre[s];
  } else {
    uint32_t w[24];
    load_be<24>(sigs + (size_t)s * 96, w);
    uint32_t any = 0;
#pragma unroll
    for (int j = 0; j < 24; ++j) any |= w[j];
    if (any == 0) {
      st = MBLS_DEC_NONE;
    } else {
      st = g2_uncompress(a, w);
      if (st == MBLS_DEC_OK) {  // group uniform
        const proj<fp2> q = pt_from_affine(a);
        if (!pt_eq(g2_psi(q), lg::g2_mul_x_lg(q))) st = MBLS_DEC_SIG_NOT_IN_G2;
      }
    }
  }
  if (g < n && c == 0) {
    sig_st[s] = st;
    st_g2(sig_xy, n, s, a);
  }
  if (fsig) {
    fp f = lg::x16_one();
    if (st == MBLS_DEC_OK) f = lg::miller16(pt_from_affine(neg_g1_gen()), a);
    if (g < n) st_fp(fsig, (size_t)n * 8, (size_t)g * 8 + (c >> 1), (c & 1) * NL, f);
  }
}

// ----- the latency chain split in three (r03, mbls_engine.cpp dev_fav) ----------------------
// A latency-critical cold call used to run H(m) beside the signature chain (g2_prep_lg), then
// the key-side Miller loop and the final exponentiation in one verdict kernel, so the key-side
// loop waited for the longer of the two prep chains.  Split: the key-side Miller value
// f_{|x|,H(m)}(apk) is computed as soon as H(m) and the key sums exist (its own stream), beside
// the signature chain (decode + psi check + signature-side Miller loop), and a final kernel
// multiplies the two Miller values and runs the final exponentiation.  Same field elements as
// mbls_k_fav_verdict_lg(16) with fsig: the product is taken in the other order.
// Key-side Miller values in the lane layout of fsig (8-lane: lane k holds the Fp2 coefficient of
// w^k; 16-lane: lane (k, h) stores component h of w^k at the same place); 1 where the set's key
// sum is not a usable point (the verdict's precheck decides those sets).
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_key_miller_lg(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ h_xy,
    uint32_t n_sets, uint32_t* __restrict__ fpk) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  fp2 f = lg::x12_one();
  if (pk_st[s] == MBLS_DEC_OK) {  // group uniform
    const proj<fp> pk = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL), ld_fp(pk_xy, n_sets, s, 2 * NL)};
    f = lg::miller_lg(pk, ld_g2(h_xy, n_sets, s));
  }
  if (g < n_sets) st_lane(fpk, (size_t)n_sets * 8, (size_t)g * 8 + lg::gk(), f);
}
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_key_miller_lg16(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ h_xy,
    uint32_t n_sets, uint32_t* __restrict__ fpk) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 4);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const int c = lg::hc();
  fp f = lg::x16_one();
  if (pk_st[s] == MBLS_DEC_OK) {  // group uniform
    const proj<fp> pk = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL), ld_fp(pk_xy, n_sets, s, 2 * NL)};
    f = lg::miller16(pk, ld_g2(h_xy, n_sets, s));
  }
  if (g < n_sets) st_fp(fpk, (size_t)n_sets * 8, (size_t)g * 8 + (c >> 1), (c & 1) * NL, f);
}
// verdict from the two Miller values (precedence and rules of mbls_k_fav_verdict_lg)
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_fav_final_lg(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ key_off, const int32_t* __restrict__ sig_st,
    const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ fpk, uint32_t n_sets, int32_t eth_variant,
    const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const uint32_t nk = key_off[s + 1] - key_off[s];
  int32_t out = mbls_fav_precheck(sig_st[s], pk_st[s], set_pre ? set_pre[s] : 0, nk, eth_variant);
  if (out == MBLS_NEEDS_PAIRING) {  // group uniform
    const size_t nl = (size_t)n_sets * 8, l = (size_t)s * 8 + lg::gk();
    const fp2 f = lg::x12_mul(ld_lane(fpk, nl, l), ld_lane(fsig, nl, l));
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (g < n_sets && lg::gk() == 0) status[g] = out;
}
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_fav_final_lg16(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ key_off, const int32_t* __restrict__ sig_st,
    const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ fpk, uint32_t n_sets, int32_t eth_variant,
    const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 4);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  const uint32_t nk = key_off[s + 1] - key_off[s];
  int32_t out = mbls_fav_precheck(sig_st[s], pk_st[s], set_pre ? set_pre[s] : 0, nk, eth_variant);
  if (out == MBLS_NEEDS_PAIRING) {  // group uniform
    const fp f = lg::x16_mul(ld_fsig16(fpk, n_sets, s, 0), ld_fsig16(fsig, n_sets, s, 0));
    out = lg::x16_is_one(lg::x16_final_exp(f)) ? 1 : 0;
  }
  if (g < n_sets && lg::hc() == 0) status[g] = out;
}

// ----- random-linear-combination batch check ---------------------------
// prod_s e([r_s] apk_s, H(m_s)) * e(-g1, sum_s [r_s] sigma_s) == 1 over the candidate sets
// (those mbls_fav_precheck leaves to a pairing), r_s 64-bit from a per-call secret seed.

// Miller value of ([r_s] apk_s, H(m_s)) per candidate set, 1 otherwise; group n_sets computes
// the signature side e(-g1, Q) for Q = sum [r_s] sigma_s (projective, 1 if Q = O).  Output:
// n_sets + 1 values in lane layout.
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_rlc_miller_lg(
    const int32_t* __restrict__ cand, const uint32_t* __restrict__ p_xy, const uint32_t* __restrict__ h_xy,
    const uint32_t* __restrict__ q_sum, uint32_t n_sets, uint32_t* __restrict__ fr) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t s = g < n_sets ? g : n_sets - 1;
  fp2 f = lg::x12_one();
  if (g == n_sets) {  // group uniform
    const proj<fp2> q = {{ld_fp(q_sum, 1, 0, 0), ld_fp(q_sum, 1, 0, NL)},
                         {ld_fp(q_sum, 1, 0, 2 * NL), ld_fp(q_sum, 1, 0, 3 * NL)},
                         {ld_fp(q_sum, 1, 0, 4 * NL), ld_fp(q_sum, 1, 0, 5 * NL)}};
    aff<fp2> qa;
    if (pt_to_affine(qa, q)) f = lg::miller_lg(pt_from_affine(neg_g1_gen()), qa);
  } else if (cand[s]) {
    const proj<fp> p = {ld_fp(p_xy, n_sets, s, 0), ld_fp(p_xy, n_sets, s, NL), ld_fp(p_xy, n_sets, s, 2 * NL)};
    f = lg::miller_lg(p, ld_g2(h_xy, n_sets, s));
  }
  if (g <= n_sets) st_lane(fr, (size_t)(n_sets + 1) * 8, (size_t)g * 8 + lg::gk(), f);
}

// product of lane-layout values in chunks of 16: out[c] = prod in[16 c .. 16 c + 15]
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_rlc_prod_lg(
    const uint32_t* __restrict__ in, uint32_t n_in, uint32_t* __restrict__ out, uint32_t n_out) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t c = blockIdx.x * 8u + (threadIdx.x >> 3);
  const uint32_t cc = c < n_out ? c : n_out - 1;
  const int k = lg::gk();
  const uint32_t lo = cc * 16u, hi = min(lo + 16u, n_in);
  fp2 f = ld_lane(in, (size_t)n_in * 8, (size_t)lo * 8 + k);
#pragma unroll 1
  for (uint32_t j = lo + 1; j < hi; ++j) f = lg::x12_mul(f, ld_lane(in, (size_t)n_in * 8, (size_t)j * 8 + k));
  if (c < n_out) st_lane(out, (size_t)n_out * 8, (size_t)c * 8 + k, f);
}

// one group: the final exponentiation of the batch product == 1 -> *ok
extern "C" __global__ __launch_bounds__(64, MBLS_LG_BLOCKS_PER_CU) void mbls_k_rlc_final_lg(
    const uint32_t* __restrict__ fprod, int32_t* __restrict__ ok) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  if (threadIdx.x >= 8) return;  // one group
  const bool pass = lg::x12_is_one(lg::x12_final_exp(ld_lane(fprod, 8, lg::gk())));
  if (threadIdx.x == 0) *ok = pass ? 1 : 0;
}

// ----- host launch wrappers ---------------------------------------------------------------
namespace mbls_launch {
// the 6-lane verdict (mbls_k_lg6.hip, its own translation unit)
hipError_t fav_verdict_lg6(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                           const uint32_t* sig_xy, const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets,
                           int32_t eth_variant, const int32_t* set_pre, const int32_t* rlc_ok, int32_t* status,
                           hipStream_t s, int32_t fsig_onelane);
hipError_t av_verdict_lg6(const int32_t* key_st, uint32_t n_pairs, const uint32_t* key_off, const int32_t* sig_st,
                          const uint32_t* fsig, const uint32_t* fpair, uint32_t n_sets, const int32_t* set_pre,
                          int32_t* status, hipStream_t s);
hipError_t g2_prep_lg6(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                       uint32_t* sig_xy, uint32_t* hxy, uint32_t* fsig, hipStream_t s, uint32_t parts);
hipError_t key_miller_lg6(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* h_xy, uint32_t n_sets,
                          uint32_t* fpk, hipStream_t s);
hipError_t fav_final_lg6(const int32_t* pk_st, const uint32_t* key_off, const int32_t* sig_st, const uint32_t* fsig,
                         const uint32_t* fpk, uint32_t n_sets, int32_t eth_variant, const int32_t* set_pre,
                         int32_t* status, hipStream_t s);
size_t lane_group6_private_bytes();
// MBLS_LG6=0: the 8-lane verdicts on padded 8-lane groups
static bool use_lg6() {
  static const bool on = [] {
    const char* v = std::getenv("MBLS_LG6");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  return on;
}
// MBLS_LG6_CHAIN=1 (experiment): the lane-group prep, key-side Miller loop and final kernel on
// 6-lane groups too.  Measured r03 (profiles/r03_lg6_chain_ab.txt): one mainnet block 6.50 vs
// 6.44 ms, host end-to-end 64.6-77.0k vs 65.5-78.3k sets/s -- latency-bound chains gain nothing
// from fewer SIMDs per set, so they keep the 8-lane form.
static bool use_lg6_chain() {
  static const bool on = [] {
    const char* v = std::getenv("MBLS_LG6_CHAIN");
    return v && std::strcmp(v, "1") == 0;
  }();
  return on && use_lg6();
}
hipError_t sig_miller_lg(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sets, uint32_t* fsig,
                         const int32_t* rlc_ok, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_SIG_MILLER, s);
  hipLaunchKernelGGL(mbls_k_sig_miller_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, sig_st, sig_xy, n_sets, fsig,
                     rlc_ok);
  return hipGetLastError();
}
hipError_t fav_verdict_lg(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                          const uint32_t* sig_xy, const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets,
                          int32_t eth_variant, const int32_t* set_pre, const int32_t* rlc_ok, int32_t* status,
                          hipStream_t s, int32_t fsig_onelane) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_FAV_VERDICT, s);
  // 16-lane groups halve the per-lane chain but double the waves and the duplicated 8-lane
  // step work: they win where the verdict is latency bound -- batches of <= 1,024 sets and the
  // deferred verdict a caller is waiting for (fsig_onelane) -- and lose on pipelined throughput
  // batches.  Measured r02 (20 steps): one mainnet block 9.70 -> 8.52 ms, warm epoch (2,048-set
  // calls) 560k -> 436k sets/s if forced.  MBLS_LG16=1 / =0 forces either form.
  static const int lg16_env = [] {
    const char* v = std::getenv("MBLS_LG16");
    return v ? (std::strcmp(v, "0") == 0 ? 0 : 1) : -1;
  }();
  const bool lg16 = lg16_env >= 0 ? lg16_env == 1 : (n_sets <= 1024 || fsig_onelane);
  // the 8-lane form on 6-lane groups (mbls_k_lg6.hip: ten sets per wave, no pad lanes) unless
  // MBLS_LG6=0 (padded 8-lane groups); each form has its own counter (r05)
  const bool lg6 = use_lg6();
  mbls_prof::Scope prof_form_(lg16  ? mbls_prof::K_FAV_VERDICT_LG16
                              : lg6 ? mbls_prof::K_FAV_VERDICT_LG6
                                    : mbls_prof::K_FAV_VERDICT_LG8,
                              s);
  if (lg16)
    hipLaunchKernelGGL(mbls_k_fav_verdict_lg16, dim3((n_sets + 3) / 4), dim3(64), 0, s, pk_st, pk_xy, key_off, sig_st,
                       sig_xy, fsig, h_xy, n_sets, eth_variant, set_pre, rlc_ok, status, fsig_onelane);
  else if (lg6)
    return fav_verdict_lg6(pk_st, pk_xy, key_off, sig_st, sig_xy, fsig, h_xy, n_sets, eth_variant, set_pre, rlc_ok,
                           status, s, fsig_onelane);
  else
    hipLaunchKernelGGL(mbls_k_fav_verdict_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, pk_st, pk_xy, key_off, sig_st,
                       sig_xy, fsig, h_xy, n_sets, eth_variant, set_pre, rlc_ok, status, fsig_onelane);
  return hipGetLastError();
}
hipError_t av_verdict_lg(const int32_t* key_st, uint32_t n_pairs, const uint32_t* key_off, const int32_t* sig_st,
                         const uint32_t* fsig, const uint32_t* fpair, uint32_t n_sets, const int32_t* set_pre,
                         int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_AV_VERDICT, s);
  if (use_lg6()) return av_verdict_lg6(key_st, n_pairs, key_off, sig_st, fsig, fpair, n_sets, set_pre, status, s);
  hipLaunchKernelGGL(mbls_k_av_verdict_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, key_st, n_pairs, key_off, sig_st,
                     fsig, fpair, n_sets, set_pre, status);
  return hipGetLastError();
}
hipError_t g2_prep_lg(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                      uint32_t* sig_xy, uint32_t* hxy, uint32_t* fsig, hipStream_t s, uint32_t parts) {
  if (n == 0 || parts == 0) return hipSuccess;
  const uint32_t copies = parts == 3 ? 2 : 1;
  mbls_prof::Scope prof_(mbls_prof::K_G2_PREP, s);
  // 16-lane groups under MBLS_LG16_PREP=1 (the signature-side Miller loop in the 16-lane form;
  // measured r02: no gain, the hash and decode chains set the kernel's length: 4.51 vs 4.47 ms
  // per mainnet block, and the warm epoch loses)
  static const bool lg16 = [] {
    const char* v = std::getenv("MBLS_LG16_PREP");
    return v && std::strcmp(v, "1") == 0;
  }();
  if (lg16)
    hipLaunchKernelGGL(mbls_k_g2_prep_lg16, dim3(copies * ((n + 3) / 4)), dim3(64), 0, s, sigs, sig_pre, msgs, n,
                       sig_st, sig_xy, hxy, fsig, parts);
  else if (use_lg6_chain())  // 6-lane groups (mbls_k_lg6.hip; the lane layout's pad slots written as zero)
    return g2_prep_lg6(sigs, sig_pre, msgs, n, sig_st, sig_xy, hxy, fsig, s, parts);
  else
    hipLaunchKernelGGL(mbls_k_g2_prep_lg, dim3(copies * ((n + 7) / 8)), dim3(64), 0, s, sigs, sig_pre, msgs, n, sig_st,
                       sig_xy, hxy, fsig, parts);
  return hipGetLastError();
}
// 16-lane groups for the split chain's kernels where fav_verdict_lg would pick them
static bool split_lg16(uint32_t n_sets) {
  static const int lg16_env = [] {
    const char* v = std::getenv("MBLS_LG16");
    return v ? (std::strcmp(v, "0") == 0 ? 0 : 1) : -1;
  }();
  return lg16_env >= 0 ? lg16_env == 1 : n_sets <= 1024;
}
hipError_t key_miller_lg(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* h_xy, uint32_t n_sets,
                         uint32_t* fpk, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_KEY_MILLER, s);
  if (split_lg16(n_sets))
    hipLaunchKernelGGL(mbls_k_key_miller_lg16, dim3((n_sets + 3) / 4), dim3(64), 0, s, pk_st, pk_xy, h_xy, n_sets, fpk);
  else if (use_lg6_chain())
    return key_miller_lg6(pk_st, pk_xy, h_xy, n_sets, fpk, s);
  else
    hipLaunchKernelGGL(mbls_k_key_miller_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, pk_st, pk_xy, h_xy, n_sets, fpk);
  return hipGetLastError();
}
hipError_t fav_final_lg(const int32_t* pk_st, const uint32_t* key_off, const int32_t* sig_st, const uint32_t* fsig,
                        const uint32_t* fpk, uint32_t n_sets, int32_t eth_variant, const int32_t* set_pre,
                        int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_FAV_VERDICT, s);
  const bool lg16 = split_lg16(n_sets);
  mbls_prof::Scope prof_form_(lg16                ? mbls_prof::K_FAV_VERDICT_LG16
                              : use_lg6_chain() ? mbls_prof::K_FAV_VERDICT_LG6
                                                : mbls_prof::K_FAV_VERDICT_LG8,
                              s);
  if (lg16)
    hipLaunchKernelGGL(mbls_k_fav_final_lg16, dim3((n_sets + 3) / 4), dim3(64), 0, s, pk_st, key_off, sig_st, fsig, fpk,
                       n_sets, eth_variant, set_pre, status);
  else if (use_lg6_chain())
    return fav_final_lg6(pk_st, key_off, sig_st, fsig, fpk, n_sets, eth_variant, set_pre, status, s);
  else
    hipLaunchKernelGGL(mbls_k_fav_final_lg, dim3((n_sets + 7) / 8), dim3(64), 0, s, pk_st, key_off, sig_st, fsig, fpk,
                       n_sets, eth_variant, set_pre, status);
  return hipGetLastError();
}
hipError_t hash_to_g2_lg(const uint8_t* msgs, uint32_t n, uint32_t* hxy, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_HASH_TO_G2, s);
  hipLaunchKernelGGL(mbls_k_hash_to_g2_lg, dim3((n + 7) / 8), dim3(64), 0, s, msgs, n, hxy);
  return hipGetLastError();
}
hipError_t rlc_check(const RlcBufs& b, const uint32_t* h_xy, uint32_t n_sets, const uint32_t* q_sum,
                     hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_RLC, s);
  hipLaunchKernelGGL(mbls_k_rlc_miller_lg, dim3((n_sets + 8) / 8), dim3(64), 0, s, b.cand, b.p_xy, h_xy, q_sum, n_sets,
                     b.fr);
  // product tree in chunks of 16, ping-ponging between fr and fr_tmp
  uint32_t* in = b.fr;
  uint32_t* out = b.fr_tmp;
  uint32_t n = n_sets + 1;
  while (n > 1) {
    const uint32_t m = (n + 15) / 16;
    hipLaunchKernelGGL(mbls_k_rlc_prod_lg, dim3((m + 7) / 8), dim3(64), 0, s, in, n, out, m);
    std::swap(in, out);
    n = m;
  }
  hipLaunchKernelGGL(mbls_k_rlc_final_lg, dim3(1), dim3(64), 0, s, in, b.ok);
  return hipGetLastError();
}
size_t lane_group_private_bytes() {
  const void* const kernels[] = {
      reinterpret_cast<const void*>(mbls_k_sig_miller_lg),
      reinterpret_cast<const void*>(mbls_k_fav_verdict_lg),
      reinterpret_cast<const void*>(mbls_k_fav_verdict_lg16),
      reinterpret_cast<const void*>(mbls_k_av_verdict_lg),
      reinterpret_cast<const void*>(mbls_k_hash_to_g2_lg),
      reinterpret_cast<const void*>(mbls_k_g2_prep_lg),
      reinterpret_cast<const void*>(mbls_k_g2_prep_lg16),
      reinterpret_cast<const void*>(mbls_k_rlc_miller_lg),
      reinterpret_cast<const void*>(mbls_k_rlc_prod_lg),
      reinterpret_cast<const void*>(mbls_k_rlc_final_lg),
      reinterpret_cast<const void*>(mbls_k_key_miller_lg),
      reinterpret_cast<const void*>(mbls_k_key_miller_lg16),
      reinterpret_cast<const void*>(mbls_k_fav_final_lg),
      reinterpret_cast<const void*>(mbls_k_fav_final_lg16),
  };
  size_t m = lane_group6_private_bytes();
  for (const void* k : kernels) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k) == hipSuccess) m = std::max(m, a.localSizeBytes);
  }
  return m;
}
}  // namespace mbls_launch
