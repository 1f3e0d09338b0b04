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
#define MBLS_G2_WAVES 1  // 2 (256 registers, spills): epoch 82.9k -> 66.1k sets/s, r01
#include <utility>
#include "mbls_h2c.hpp"
#include "mbls_kernels.h"
#include "mbls_pairing.hpp"
#include "mbls_soa.hpp"

using namespace mbls;

using namespace mbls_soa;

// The two-pair Miller loop of mbls_k_miller_pairs with both running points in LDS (r05,
// MBLS_PAIRS_LDS).  One lane holds f (168 dwords), both running points (2 x 84) and both P (2 x
// 28): more than its 512 registers, so the loop spilled ~5.5 KB per lane per iteration to
// scratch (45.8 GB per 131,072-lane launch, profiles/r05_pmc_traffic_deposit.json) and waited on
// the reloads 32% of its wave-cycles (profiles/r05_pmc_stall_deposit.json).  The two T now live
// in LDS, reduced (< 2p, 28-bit digits) and packed 14 digits -> 13 dwords: 156 dwords per lane,
// 39 KiB per one-wave workgroup, four per CU -- the occupancy the registers allow anyway.  A
// compiler-only memory barrier before each read keeps them there instead of forwarded back into
// registers.  Measured (deposit_av, 20 steps): the second T and both P unpacked in LDS 209-210k
// -> 214-215k sets/s, both T packed 214k -> 219k (profiles/r05_ab_pairs_lds.txt).
namespace pav {
constexpr int kW = 13;  // dwords per packed Fp
__shared__ uint32_t s_t[2 * 6 * kW * 64];
__device__ __forceinline__ void fence() { __asm__ volatile("" ::: "memory"); }
__device__ __forceinline__ void put(int row, const fp& a) {
  uint64_t acc = 0;
  int bits = 0, o = 0;
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    acc |= (uint64_t)a.v[d] << bits;
    bits += 28;
    if (bits >= 32) {
      s_t[(row + o++) * 64 + threadIdx.x] = (uint32_t)acc;
      acc >>= 32;
      bits -= 32;
    }
  }
  s_t[(row + o) * 64 + threadIdx.x] = (uint32_t)acc;  // o == 12: the last 8 bits (value < 2^392)
}
__device__ __forceinline__ fp get(int row) {
  fp a;
  uint64_t acc = 0;
  int bits = 0, o = 0;
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    if (bits < 28) {
      acc |= (uint64_t)s_t[(row + o++) * 64 + threadIdx.x] << bits;
      bits += 32;
    }
    a.v[d] = (uint32_t)acc & M28;
    acc >>= 28;
    bits -= 28;
  }
  return a;
}
__device__ __forceinline__ void put_t(int j, const g2lz& t) {
  const nz2 x = reduce(t.x), y = reduce(t.y), z = reduce(t.z);
  const int r = j * 6 * kW;
  put(r, x.v.c0), put(r + kW, x.v.c1), put(r + 2 * kW, y.v.c0), put(r + 3 * kW, y.v.c1), put(r + 4 * kW, z.v.c0),
      put(r + 5 * kW, z.v.c1);
}
__device__ __forceinline__ g2lz get_t(int j) {
  fence();
  const int r = j * 6 * kW;
  return {{{get(r), get(r + kW)}}, {{get(r + 2 * kW), get(r + 3 * kW)}}, {{get(r + 4 * kW), get(r + 5 * kW)}}};
}
}  // namespace pav

__device__ __noinline__ fp12 miller_loop_2_lds(const aff<fp>& p1, const aff<fp2>& q1, const aff<fp>& p2,
                                               const aff<fp2>& q2) {
  pav::put_t(0, g2lz_from(q1));
  pav::put_t(1, g2lz_from(q2));
  fp12 f = fp12_one();
  bool first = true;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (!first) f = fp12_sqr(f);
    first = false;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      g2lz t = pav::get_t(j);
      const line_lz l = miller_dbl(t);
      pav::put_t(j, t);
      f = fp12_mul_line_at(f, l, j ? p2 : p1);
    }
    if ((k::X_ABS >> b) & 1ull) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        g2lz t = pav::get_t(j);
        const line_lz l = miller_add(t, j ? q2 : q1);
        pav::put_t(j, t);
        f = fp12_mul_line_at(f, l, j ? p2 : p1);
      }
    }
  }
  return fp12_conj(f);
}

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
    st_pair_value(fpair, nl, j0, miller_loop_2_lds(ld_g1(key_xy, n_pairs, j0), ld_g2(h_xy, n_pairs, j0),
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
