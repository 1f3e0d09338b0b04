// mbls_k_lg6.hip — the fast_aggregate_verify verdict on 6-lane groups (mbls_pairing_lg.hpp with
// MBLS_LG_GROUP = 6): lane k of a group owns the Fp2 coefficient of w^k of every Fp12 value, as
// in the 8-lane form, but the two pad lanes are gone, so a wave carries ten sets instead of eight
// (lanes 60..63 form a tail group that computes on a copy and stores nothing).  Per lane the
// instruction stream is the 8-lane one: the same latency per set, 20% less SIMD time per set.
// That is what bounds a pipelined table (warm) epoch, whose verdicts are ~70% of its
// instructions (r03 PMC, profiles/r03_pmc_sq.json).  Its own translation unit: the group size
// is a compile-time property of every lane-group routine.  Replaces, per set, blst's
// miller_loop_n + final_exp behind lighthouse fast_aggregate_verify (native/bls_nif/src/lib.rs:99,118).
#define MBLS_LG_GROUP 6
#ifndef MBLS_LG_FP_INLINE
#define MBLS_FP_OUTLINE 1
#endif
#include <algorithm>

#include "mbls_kernels.h"
#include "mbls_pairing_lg.hpp"
#include "mbls_soa.hpp"

using namespace mbls;
using namespace mbls_soa;

namespace {
constexpr uint32_t kSetsPerWave = 10;
}

// mbls_k_fav_verdict_lg on 6-lane groups: same inputs, precedence and outputs.  The Miller
// steps of this form take P affine (mbls_pairing_lg.hpp), so the projective key sum is
// normalised first: one constant-time inversion per set, ~1% of the verdict's instructions.
extern "C" __global__ __launch_bounds__(64, 1) void mbls_k_fav_verdict_lg6(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy, const uint32_t* __restrict__ fsig,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, int32_t eth_variant, const int32_t* __restrict__ set_pre,
    const int32_t* __restrict__ rlc_ok, int32_t* __restrict__ status, int32_t fsig_onelane) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const bool live = threadIdx.x < 6u * kSetsPerWave;  // group uniform
  const uint32_t g = blockIdx.x * kSetsPerWave + threadIdx.x / 6u;
  const uint32_t s = (live && g < n_sets) ? g : n_sets - 1;  // tail groups compute on a copy
  const uint32_t nk = key_off ? key_off[s + 1] - key_off[s] : 1u;
  int32_t out = mbls_fav_precheck(sig_st[s], pk_st[s], set_pre ? set_pre[s] : 0, nk, eth_variant);
  if (out == MBLS_NEEDS_PAIRING && rlc_ok && *rlc_ok) out = 1;
  if (out == MBLS_NEEDS_PAIRING) {  // group uniform
    const fp z = ld_fp(pk_xy, n_sets, s, 2 * NL);
    const fp zi = fp_inv(z);  // the key sum is not the identity here (the precheck decided those)
    const proj<fp> pk = {fp_mul(ld_fp(pk_xy, n_sets, s, 0), zi), fp_mul(ld_fp(pk_xy, n_sets, s, NL), zi), fp_one()};
    fp2 f;
    if (fsig) {
      f = lg::miller_lg(pk, ld_g2(h_xy, n_sets, s));
      f = lg::x12_mul(f, fsig_onelane ? ld_fp12_coef(fsig, n_sets, s, lg::gk())
                                      : ld_lane(fsig, (size_t)n_sets * 8, (size_t)s * 8 + lg::gk()));
    } else {
      f = lg::miller2_lg(pk, ld_g2(h_xy, n_sets, s), pt_from_affine(neg_g1_gen()), ld_g2(sig_xy, n_sets, s),
                         sig_st[s] == MBLS_DEC_OK);
    }
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (live && g < n_sets && lg::gk() == 0) status[g] = out;
}

// mbls_k_av_verdict_lg on 6-lane groups (aggregate_verify verdicts from the per-pair Miller values
// of mbls_k_miller_pairs and the signature-side values; same precedence and outputs)
extern "C" __global__ __launch_bounds__(64, 1) void mbls_k_av_verdict_lg6(
    const int32_t* __restrict__ key_st, uint32_t n_pairs, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ fpair,
    uint32_t n_sets, const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const bool live = threadIdx.x < 6u * kSetsPerWave;  // group uniform
  const uint32_t g = blockIdx.x * kSetsPerWave + threadIdx.x / 6u;
  const uint32_t s = (live && g < n_sets) ? g : n_sets - 1;
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
  if (live && g < n_sets && lg::gk() == 0) status[g] = out;
}

namespace mbls_launch {
hipError_t av_verdict_lg6(const int32_t* key_st, uint32_t n_pairs, const uint32_t* key_off, const int32_t* sig_st,
                          const uint32_t* fsig, const uint32_t* fpair, uint32_t n_sets, const int32_t* set_pre,
                          int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(mbls_k_av_verdict_lg6, dim3((n_sets + kSetsPerWave - 1) / kSetsPerWave), dim3(64), 0, s, key_st,
                     n_pairs, key_off, sig_st, fsig, fpair, n_sets, set_pre, status);
  return hipGetLastError();
}
hipError_t fav_verdict_lg6(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                           const uint32_t* sig_xy, const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets,
                           int32_t eth_variant, const int32_t* set_pre, const int32_t* rlc_ok, int32_t* status,
                           hipStream_t s, int32_t fsig_onelane) {
  hipLaunchKernelGGL(mbls_k_fav_verdict_lg6, dim3((n_sets + kSetsPerWave - 1) / kSetsPerWave), dim3(64), 0, s, pk_st,
                     pk_xy, key_off, sig_st, sig_xy, fsig, h_xy, n_sets, eth_variant, set_pre, rlc_ok, status,
                     fsig_onelane);
  return hipGetLastError();
}
size_t lane_group6_private_bytes() {
  size_t m = 0;
  for (const void* k : {reinterpret_cast<const void*>(mbls_k_fav_verdict_lg6),
                        reinterpret_cast<const void*>(mbls_k_av_verdict_lg6)}) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k) == hipSuccess) m = std::max(m, a.localSizeBytes);
  }
  return m;
}
}  // namespace mbls_launch
