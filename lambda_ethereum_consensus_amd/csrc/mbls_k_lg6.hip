// mbls_k_lg6.hip — the 8-lane-group kernels on 6-lane groups (mbls_pairing_lg.hpp with
// MBLS_LG_GROUP = 6): lane k of a group owns the Fp2 coefficient of w^k of every Fp12 value, as
// in the 8-lane form, but the two pad lanes are gone, so a wave carries ten sets instead of eight
// (lanes 60..63 form a tail group that computes on a copy and stores nothing).  Per lane the
// instruction stream is the 8-lane one: the same latency per set, 20% less SIMD time per set.
// That is what bounds a pipelined table (warm) epoch, whose verdicts are ~70% of its
// instructions (r03 PMC, profiles/r03_pmc_sq.json).  Its own translation unit: the group size
// is a compile-time property of every lane-group routine.  Replaces, per set, blst's
// miller_loop_n + final_exp behind lighthouse fast_aggregate_verify (native/bls_nif/src/lib.rs:99,118).
#define MBLS_LG_GROUP 6
#define MBLS_FP_OUTLINE 1
#include <algorithm>

#include "mbls_kernels.h"
#include "mbls_pairing_lg.hpp"
#include "mbls_soa.hpp"

using namespace mbls;
using namespace mbls_soa;

namespace {
constexpr uint32_t kSetsPerWave = 10;
}
// waves per SIMD the 6-lane kernels must fit (1: up to 512 registers; 2: 256, spilling to
// scratch).  Applied to every kernel of this translation unit: the outlined Miller loop / final
// exponentiation they share are compiled once, under the occupancy all their callers agree on.
#define MBLS_LG6_WAVES 1
#define MBLS_LG6_OCC __attribute__((amdgpu_waves_per_eu(MBLS_LG6_WAVES, MBLS_LG6_WAVES)))


// The 6-lane verdict's joint Miller loop (lg::miller2_trio_sel) behind a call boundary that keeps
// the kernel's and the loop's registers apart: this lane's P and the address of its pair's Q in
// argument registers (28 + 4 VGPRs), not both pairs' points by reference through scratch (r05:
// the by-reference form wrote and read back 960 B per lane per verdict, ~25 MB per 2,048-set
// launch).
#define MBLS_LG6_A14(p)                                                                                    \
  uint32_t p##0, uint32_t p##1, uint32_t p##2, uint32_t p##3, uint32_t p##4, uint32_t p##5, uint32_t p##6, \
      uint32_t p##7, uint32_t p##8, uint32_t p##9, uint32_t p##10, uint32_t p##11, uint32_t p##12, uint32_t p##13
#define MBLS_LG6_U14(x) \
  x.v[0], x.v[1], x.v[2], x.v[3], x.v[4], x.v[5], x.v[6], x.v[7], x.v[8], x.v[9], x.v[10], x.v[11], x.v[12], x.v[13]
__device__ __noinline__ fp2 miller2_trio_lane(MBLS_LG6_A14(x), MBLS_LG6_A14(y), const uint32_t* __restrict__ qxy,
                                              uint32_t n, uint32_t s_use2) {
  const aff<fp> p = {{{x0, x1, x2, x3, x4, x5, x6, x7, x8, x9, x10, x11, x12, x13}},
                     {{y0, y1, y2, y3, y4, y5, y6, y7, y8, y9, y10, y11, y12, y13}}};
  return lg::miller2_trio_sel(p, ld_g2(qxy, n, s_use2 & 0x7fffffffu), (s_use2 >> 31) != 0u);
}

// mbls_k_fav_verdict_lg on 6-lane groups: same inputs, precedence and outputs.  The Miller
// steps of this form take P affine (mbls_pairing_lg.hpp), so the projective key sum is
// normalised first: one constant-time inversion per set, ~1% of the verdict's instructions.
extern "C" __global__ __launch_bounds__(64) MBLS_LG6_OCC void mbls_k_fav_verdict_lg6(
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
    proj<fp> pk = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL), fp_one()};
    if (key_off) {  // a per-set key sum (projective); Bls.verify (no key_off): a decoded affine key
      const fp zi = fp_inv(ld_fp(pk_xy, n_sets, s, 2 * NL));  // not the identity (the precheck decided those)
      pk.x = fp_mul(pk.x, zi);
      pk.y = fp_mul(pk.y, zi);
    }
    fp2 f;
    if (fsig) {
      f = lg::miller_lg(pk, ld_g2(h_xy, n_sets, s));
      f = lg::x12_mul(f, fsig_onelane ? ld_fp12_coef(fsig, n_sets, s, lg::gk())
                                      : ld_lane(fsig, (size_t)n_sets * 8, (size_t)s * 8 + lg::gk()));
    } else {
      // lanes 0..2 of the group: (pk, H(m)); lanes 3..5: (-g1, signature)
      const bool second = lg::gk() >= 3;
      const aff<fp> g1n = neg_g1_gen();
      const fp px = fp_select(second, g1n.x, pk.x), py = fp_select(second, g1n.y, pk.y);
      f = miller2_trio_lane(MBLS_LG6_U14(px), MBLS_LG6_U14(py), second ? sig_xy : h_xy, n_sets,
                            s | (sig_st[s] == MBLS_DEC_OK ? 0x80000000u : 0u));
    }
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (live && g < n_sets && lg::gk() == 0) status[g] = out;
}

// mbls_k_av_verdict_lg on 6-lane groups (aggregate_verify verdicts from the per-pair Miller values
// of mbls_k_miller_pairs and the signature-side values; same precedence and outputs)
extern "C" __global__ __launch_bounds__(64) MBLS_LG6_OCC void mbls_k_av_verdict_lg6(
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

// ----- the split latency chain and the lane-group prep on 6-lane groups (host batch calls of
// > 1,024 sets: mbls_engine.cpp dev_fav with `latency`) ---------------------------------------
// Lane-layout outputs keep the 8-slot stride of the other forms (slot 8 s + k); slots 6 and 7,
// which a 16-lane consumer reads as the zero pad, are written with zeros here too.
namespace {
__device__ __forceinline__ void st_lane6(uint32_t* buf, uint32_t n_sets, uint32_t s, const fp2& f) {
  const int k = lg::gk();
  st_lane(buf, (size_t)n_sets * 8, (size_t)s * 8 + k, f);
  if (k < 2) st_lane(buf, (size_t)n_sets * 8, (size_t)s * 8 + 6 + k, fp2_zero());
}
}  // namespace

// mbls_k_g2_prep_lg on 6-lane groups (parts: 1 hash blocks, 2 signature blocks, 3 both)
extern "C" __global__ __launch_bounds__(64) MBLS_LG6_OCC void mbls_k_g2_prep_lg6(
    const uint8_t* __restrict__ sigs, const int32_t* __restrict__ sig_pre, const uint8_t* __restrict__ msgs,
    uint32_t n, int32_t* __restrict__ sig_st, uint32_t* __restrict__ sig_xy, uint32_t* __restrict__ hxy,
    uint32_t* __restrict__ fsig, uint32_t parts) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t nb = (n + kSetsPerWave - 1) / kSetsPerWave;
  const bool hash_part = parts == 3 ? blockIdx.x < nb : parts == 1;  // block (wave) uniform
  const bool live = threadIdx.x < 6u * kSetsPerWave;                 // group uniform
  const uint32_t g = (hash_part || parts != 3 ? blockIdx.x : blockIdx.x - nb) * kSetsPerWave + threadIdx.x / 6u;
  const bool mine = live && g < n;
  const uint32_t s = mine ? g : n - 1;
  const int k = lg::gk();
  if (hash_part) {
    uint32_t w[8];
    load_be<8>(msgs + (size_t)s * 32, w);
    aff<fp2> a;
    pt_to_affine(a, lg::hash_to_g2_lg(w));
    if (mine && k == 0) st_g2(hxy, n, s, a);
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
  if (mine && k == 0) {
    sig_st[s] = st;
    st_g2(sig_xy, n, s, a);
  }
  if (fsig) {
    fp2 f = lg::x12_one();
    if (st == MBLS_DEC_OK) f = lg::miller_lg(pt_from_affine(neg_g1_gen()), a);  // P affine: -g1
    if (mine) st_lane6(fsig, n, s, f);
  }
}

// mbls_k_key_miller_lg on 6-lane groups: the key sum normalised first (P affine, see above)
extern "C" __global__ __launch_bounds__(64) MBLS_LG6_OCC void mbls_k_key_miller_lg6(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ h_xy,
    uint32_t n_sets, uint32_t* __restrict__ fpk) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const bool live = threadIdx.x < 6u * kSetsPerWave;
  const uint32_t g = blockIdx.x * kSetsPerWave + threadIdx.x / 6u;
  const bool mine = live && g < n_sets;
  const uint32_t s = mine ? g : n_sets - 1;
  fp2 f = lg::x12_one();
  if (pk_st[s] == MBLS_DEC_OK) {  // group uniform; a valid sum is not the identity
    const fp zi = fp_inv(ld_fp(pk_xy, n_sets, s, 2 * NL));
    const proj<fp> pk = {fp_mul(ld_fp(pk_xy, n_sets, s, 0), zi), fp_mul(ld_fp(pk_xy, n_sets, s, NL), zi), fp_one()};
    f = lg::miller_lg(pk, ld_g2(h_xy, n_sets, s));
  }
  if (mine) st_lane6(fpk, n_sets, s, f);
}

// mbls_k_fav_final_lg on 6-lane groups
extern "C" __global__ __launch_bounds__(64) MBLS_LG6_OCC void mbls_k_fav_final_lg6(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ key_off, const int32_t* __restrict__ sig_st,
    const uint32_t* __restrict__ fsig, const uint32_t* __restrict__ fpk, uint32_t n_sets, int32_t eth_variant,
    const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const bool live = threadIdx.x < 6u * kSetsPerWave;
  const uint32_t g = blockIdx.x * kSetsPerWave + threadIdx.x / 6u;
  const bool mine = live && g < n_sets;
  const uint32_t s = mine ? g : n_sets - 1;
  const uint32_t nk = key_off[s + 1] - key_off[s];
  int32_t out = mbls_fav_precheck(sig_st[s], pk_st[s], set_pre ? set_pre[s] : 0, nk, eth_variant);
  if (out == MBLS_NEEDS_PAIRING) {  // group uniform
    const size_t nl = (size_t)n_sets * 8, l = (size_t)s * 8 + lg::gk();
    const fp2 f = lg::x12_mul(ld_lane(fpk, nl, l), ld_lane(fsig, nl, l));
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (mine && lg::gk() == 0) status[g] = out;
}

namespace mbls_launch {
hipError_t g2_prep_lg6(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                       uint32_t* sig_xy, uint32_t* hxy, uint32_t* fsig, hipStream_t s, uint32_t parts) {
  const uint32_t copies = parts == 3 ? 2 : 1;
  hipLaunchKernelGGL(mbls_k_g2_prep_lg6, dim3(copies * ((n + kSetsPerWave - 1) / kSetsPerWave)), dim3(64), 0, s, sigs,
                     sig_pre, msgs, n, sig_st, sig_xy, hxy, fsig, parts);
  return hipGetLastError();
}
hipError_t key_miller_lg6(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* h_xy, uint32_t n_sets,
                          uint32_t* fpk, hipStream_t s) {
  hipLaunchKernelGGL(mbls_k_key_miller_lg6, dim3((n_sets + kSetsPerWave - 1) / kSetsPerWave), dim3(64), 0, s, pk_st,
                     pk_xy, h_xy, n_sets, fpk);
  return hipGetLastError();
}
hipError_t fav_final_lg6(const int32_t* pk_st, const uint32_t* key_off, const int32_t* sig_st, const uint32_t* fsig,
                         const uint32_t* fpk, uint32_t n_sets, int32_t eth_variant, const int32_t* set_pre,
                         int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(mbls_k_fav_final_lg6, dim3((n_sets + kSetsPerWave - 1) / kSetsPerWave), dim3(64), 0, s, pk_st,
                     key_off, sig_st, fsig, fpk, n_sets, eth_variant, set_pre, status);
  return hipGetLastError();
}
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
                        reinterpret_cast<const void*>(mbls_k_av_verdict_lg6), reinterpret_cast<const void*>(mbls_k_g2_prep_lg6),
                        reinterpret_cast<const void*>(mbls_k_key_miller_lg6),
                        reinterpret_cast<const void*>(mbls_k_fav_final_lg6)}) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k) == hipSuccess) m = std::max(m, a.localSizeBytes);
  }
  return m;
}
}  // namespace mbls_launch
