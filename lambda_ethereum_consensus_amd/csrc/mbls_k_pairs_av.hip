// mbls_k_pairs_av.hip — the one-lane aggregate_verify kernels: per-(key, message) Miller
// values and the aggregate_verify verdict.  Their own translation unit (split from
// mbls_k_pair.hip) so the large pairing units compile side by side.
//
// Built with MBLS_FP_OUTLINE: the Fp multiply is a scalar-argument call, so these long
// kernels (Miller loop + final exponentiation, SSWU + cofactor clearing) stay I-cache sized.
// Replaces the blst calls behind lighthouse Signature::deserialize / verify /
// fast_aggregate_verify / eth_fast_aggregate_verify / aggregate_verify / sign / aggregate
// (native/bls_nif/src/lib.rs:14-119).
#define MBLS_FP_OUTLINE 1
// waves per SIMD the one-lane kernels must fit (1: up to 512 registers, the SIMD to itself)
#ifndef MBLS_G2_WAVES
#define MBLS_G2_WAVES 1  // 2 (256 registers, spills): epoch 82.9k -> 66.1k sets/s, r01
#endif
#include <utility>
#include "mbls_h2c.hpp"
#include "mbls_kernels.h"
#include "mbls_pairing.hpp"
#include "mbls_soa.hpp"

using namespace mbls;

using namespace mbls_soa;

// One lane per (key, message) pair: the Miller value f_{|x|,H(m)}(pk) (conjugated), written
// in the lane layout of the lane-group kernels (pair j, coefficient k at row 8 j + k).  A pair
// whose key did not decode stores 1 (its set is decided by the key error anyway).
// Lane t takes pairs 2t and 2t + 1.  When both belong to one set, one 2-pair Miller loop with
// shared squarings gives their product (stored at slot 2t, one at 2t + 1; aggregate_verify
// multiplies a set's slots): 20% fewer Fp multiplies per pair than two loops.  Otherwise
// (a set boundary between them) each slot gets its own loop.
__device__ __forceinline__ void st_pair_value(uint32_t* fpair, size_t nl, uint32_t j, const fp12& f) {
  const fp2* c[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};  // w^0 .. w^5
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
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_miller_pairs(
    const int32_t* __restrict__ key_st, const uint32_t* __restrict__ key_xy, const uint32_t* __restrict__ h_xy,
    uint32_t n_pairs, const uint32_t* __restrict__ key_off, uint32_t n_sets, uint32_t* __restrict__ fpair) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j0 = 2 * t, j1 = j0 + 1;
  if (j0 >= n_pairs) return;
  // set of pair j0: the last s with key_off[s] <= j0
  uint32_t lo = 0, hi = n_sets;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (key_off[mid] <= j0) lo = mid; else hi = mid;
  }
  const bool has1 = j1 < n_pairs;
  const bool same = has1 && j1 < key_off[lo + 1];
  const bool ok0 = key_st[j0] == MBLS_DEC_OK, ok1 = has1 && key_st[j1] == MBLS_DEC_OK;
  const size_t nl = (size_t)n_pairs * 8;
  if (same && ok0 && ok1) {
    st_pair_value(fpair, nl, j0, miller_loop_2(ld_g1(key_xy, n_pairs, j0), ld_g2(h_xy, n_pairs, j0),
                                               ld_g1(key_xy, n_pairs, j1), ld_g2(h_xy, n_pairs, j1)));
    st_pair_value(fpair, nl, j1, fp12_one());
  } else {
    // a pair whose key did not decode stores 1 (its set is decided by the key error anyway)
    st_pair_value(fpair, nl, j0, ok0 ? miller_loop_1(ld_g1(key_xy, n_pairs, j0), ld_g2(h_xy, n_pairs, j0)) : fp12_one());
    if (has1)
      st_pair_value(fpair, nl, j1,
                    ok1 ? miller_loop_1(ld_g1(key_xy, n_pairs, j1), ld_g2(h_xy, n_pairs, j1)) : fp12_one());
  }
}

// One lane per set: aggregate_verify.  Pair j of set s = (key j, message j) for
// key_off[s] <= j < key_off[s+1]; h_xy holds H(m_j) per pair.
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_av_verdict(
    const int32_t* __restrict__ key_st, const uint32_t* __restrict__ key_xy, uint32_t n_pairs,
    const uint32_t* __restrict__ key_off, const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, const int32_t* __restrict__ set_pre,
    int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
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

// ----- host launch wrappers ---------------------------------------------------------------
namespace mbls_launch {
static inline dim3 grid64(uint32_t n) { return dim3((n + 63) / 64); }
hipError_t miller_pairs(const int32_t* key_st, const uint32_t* key_xy, const uint32_t* h_xy, uint32_t n_pairs,
                        const uint32_t* key_off, uint32_t n_sets, uint32_t* fpair, hipStream_t s) {
  if (n_pairs == 0 || n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_MILLER_PAIRS, s);
  hipLaunchKernelGGL(mbls_k_miller_pairs, grid64((n_pairs + 1) / 2), dim3(64), 0, s, key_st, key_xy, h_xy, n_pairs,
                     key_off, n_sets, fpair);
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
}  // namespace mbls_launch
