// mbls_k_av6.hip — aggregate_verify on 6-lane groups with joint Miller loops (r05).
//
// Reference: Bls.aggregate_verify/3 -> native/bls_nif/src/lib.rs:62-82 -> blst aggregate_verify:
// prod_i e(pk_i, H(m_i)) == e(g1, sigma), i.e. prod_i e(pk_i, H(m_i)) * e(-g1, sigma) == 1.
//
// r04 ran the key pairs on one lane per pair couple (mbls_k_miller_pairs: 37 ms per 16,384 x 16
// batch, its 5,248-byte frames moving 45.8 GB per launch), the signature pair in its own lane-group
// kernel, and multiplied 9 values per set before the final exponentiation.  Here a set's pairs --
// the signature pair (-g1, sigma) first, then (pk_j, H(m_j)) in list order -- are cut into groups
// of kPairs = 4, and a 6-lane group runs ONE Miller loop over its group's pairs: the Fp12
// squaring of each iteration is shared by the four (16 x 16 + 1 pairs: 107 lane products per
// iteration per set instead of 123), each couple of pairs steps on the two trios of the group
// (mbls_pairing_lg.hpp dbl_step_trio / add_step_trio: lanes 0..2 the first pair's T, 3..5 the
// second's).  The two running points of a group live in registers as "current" and "other" and
// swap after each couple's step, so the step code is emitted once; P and Q are read from global
// memory where a step needs them (L2-resident), not held.  A second kernel multiplies a set's group
// values (5 for 17 pairs) and runs the final exponentiation.  Group g's set and chunk come from an
// exclusive scan of ceil((n_s + 1) / kPairs) (mbls_k_av_group_plan); the pairs grid is sized for
// the bound n_pairs / kPairs + n_sets and the groups past the scan's total return at once.
#define MBLS_LG_GROUP 6
#define MBLS_FP_OUTLINE 1
#include <algorithm>

#include "mbls_av6.h"
#include "mbls_kernels.h"
#include "mbls_pairing_lg.hpp"
#include "mbls_soa.hpp"

using namespace mbls;
using namespace mbls_soa;

namespace {
constexpr uint32_t kSetsPerWave = 10;  // groups per 64-lane wave (lanes 60..63: a tail group)
constexpr uint32_t kPairs = 4;         // pairs per group (two couples)
constexpr uint32_t kPlanThreads = 1024;
}  // namespace

// grp_off[s] = sum over t < s of ceil((n_t + 1) / kPairs), grp_off[n_sets] = the total: one
// workgroup, each thread scanning a contiguous run of sets
extern "C" __global__ __launch_bounds__(kPlanThreads) void mbls_k_av_group_plan(const uint32_t* __restrict__ key_off,
                                                                                 uint32_t n_sets,
                                                                                 uint32_t* __restrict__ grp_off) {
  __shared__ uint32_t part[kPlanThreads];
  const uint32_t t = threadIdx.x, per = (n_sets + kPlanThreads - 1) / kPlanThreads;
  const uint32_t lo = std::min(n_sets, t * per), hi = std::min(n_sets, lo + per);
  uint32_t sum = 0;
  for (uint32_t s = lo; s < hi; ++s) sum += (key_off[s + 1] - key_off[s] + kPairs) / kPairs;
  part[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < kPlanThreads; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;  // exclusive prefix of this thread's run
  for (uint32_t s = lo; s < hi; ++s) {
    grp_off[s] = run;
    run += (key_off[s + 1] - key_off[s] + kPairs) / kPairs;
  }
  if (t == kPlanThreads - 1) grp_off[n_sets] = part[t];
}

namespace {
// Pair i of set s's list: 0 = (-g1, sigma), i >= 1 = (pk_{key_off[s] + i - 1}, H(m_same)).
struct PairSrc {
  const int32_t* key_st;
  const uint32_t* key_xy;
  const uint32_t* h_xy;
  uint32_t n_pairs;
  const int32_t* sig_st;
  const uint32_t* sig_xy;
  uint32_t n_sets;
};
// valid pairs contribute; an invalid key (its set is decided by the key error), a signature that
// is not a decoded subgroup point (decided by the precheck) or the infinity signature (blst skips
// it: its pairing is 1) contribute nothing
__device__ __forceinline__ bool pair_valid(const PairSrc& a, uint32_t s, uint32_t i, uint32_t k0) {
  return i == 0 ? a.sig_st[s] == MBLS_DEC_OK : a.key_st[k0 + i - 1] == MBLS_DEC_OK;
}
__device__ __forceinline__ lg::pt_lg pair_p(const PairSrc& a, uint32_t i, uint32_t k0) {
  const aff<fp> p = i == 0 ? neg_g1_gen() : ld_g1(a.key_xy, a.n_pairs, k0 + i - 1);
  return lg::pt_lg_from(pt_from_affine(p));
}
__device__ __forceinline__ aff<fp2> pair_q(const PairSrc& a, uint32_t s, uint32_t i, uint32_t k0) {
  return i == 0 ? ld_g2(a.sig_xy, a.n_sets, s) : ld_g2(a.h_xy, a.n_pairs, k0 + i - 1);
}
}  // namespace

// One 6-lane group per (set, chunk of kPairs pairs): the product of the chunk's Miller values,
// conjugated (x < 0), in the lane layout (slot 8 g + k; slots 6, 7 written as zero).
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void mbls_k_av_pairs_lg6(
    const int32_t* __restrict__ key_st, const uint32_t* __restrict__ key_xy, const uint32_t* __restrict__ h_xy,
    uint32_t n_pairs, const uint32_t* __restrict__ key_off, uint32_t n_sets, const int32_t* __restrict__ sig_st,
    const uint32_t* __restrict__ sig_xy, const uint32_t* __restrict__ grp_off, uint32_t* __restrict__ fgrp) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t n_grp = grp_off[n_sets];
  const uint32_t first = blockIdx.x * kSetsPerWave;
  if (first >= n_grp) return;  // wave uniform: past the scan's total
  const bool live = threadIdx.x < 6u * kSetsPerWave;
  const uint32_t gq = first + threadIdx.x / 6u;
  const bool mine = live && gq < n_grp;
  const uint32_t g = mine ? gq : n_grp - 1;  // tail groups compute on a copy
  // set of group g: the last s with grp_off[s] <= g
  uint32_t lo = 0, hi = n_sets;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (grp_off[mid] <= g) lo = mid; else hi = mid;
  }
  const uint32_t s = lo, k0 = key_off[s], n_list = key_off[s + 1] - k0 + 1;
  const uint32_t i0 = (g - grp_off[s]) * kPairs, i1 = std::min(n_list, i0 + kPairs);
  const PairSrc src{key_st, key_xy, h_xy, n_pairs, sig_st, sig_xy, n_sets};
  const bool second = lg::gk() >= 3;  // trio of the lane: the couple's first or second pair
  const int g0 = lg::gbase(), g1 = lg::gbase() + 3;
  // couple c = pairs (i0 + 2c, i0 + 2c + 1); a missing or invalid pair's lines are skipped
  // (all flags group uniform).  Couple values live in scalars, picked by c with selects: a
  // runtime-indexed array would go to scratch.
  const uint32_t a0 = i0, a1 = i0 + 2;
  const bool u00 = a0 < i1 && pair_valid(src, s, a0, k0), u01 = a0 + 1 < i1 && pair_valid(src, s, a0 + 1, k0);
  const bool u10 = a1 < i1 && pair_valid(src, s, a1, k0), u11 = a1 + 1 < i1 && pair_valid(src, s, a1 + 1, k0);
  const uint32_t m0 = std::min(second ? a0 + 1 : a0, n_list - 1), m1 = std::min(second ? a1 + 1 : a1, n_list - 1);
  const bool two = a1 < i1;  // group uniform: the second couple exists
  lg::tlz cur = lg::tlz_from(pair_q(src, s, m0, k0));
  lg::tlz oth = lg::tlz_from(pair_q(src, s, m1, k0));
  fp2 f = lg::x12_one();
#pragma unroll 1
  for (int bit = 62; bit >= 0; --bit) {
    if (bit != 62) f = lg::x12_sqr(f);
    const bool add = (k::X_ABS >> bit) & 1ull;
#pragma unroll 1
    for (int st = 0; st < (add ? 4 : 2); ++st) {  // doubling of couples 0, 1; then, on a set bit, their additions
      const int c = st & 1;
      if (c == 0 || two) {
        const uint32_t m = c ? m1 : m0;
        const bool ua = c ? u10 : u00, ub = c ? u11 : u01;
        const lg::line_lg l = st < 2 ? lg::dbl_step_trio(cur, pair_p(src, m, k0))
                                     : lg::add_step_trio(cur, pair_q(src, s, m, k0), pair_p(src, m, k0));
        if (ua) {
          const lg::line_lg q = lg::pull(l, g0);
          f = lg::x12_mul_line(f, q.l0, q.l2, q.l3);
        }
        if (ub) {
          const lg::line_lg q = lg::pull(l, g1);
          f = lg::x12_mul_line(f, q.l0, q.l2, q.l3);
        }
      }
      if (two) {  // couple 1's running point takes the registers of the next step
        const lg::tlz t = cur;
        cur = oth;
        oth = t;
      }
    }
  }
  f = lg::x12_conj(f);
  if (mine) {
    const int k = lg::gk();
    st_lane(fgrp, (size_t)n_grp * 8, (size_t)g * 8 + k, f);
    if (k < 2) st_lane(fgrp, (size_t)n_grp * 8, (size_t)g * 8 + 6 + k, fp2_zero());
  }
}

// aggregate_verify verdicts from the group values: same precedence and outputs as
// mbls_k_av_verdict_lg6 (signature decode errors, then the first bad key in list order, then the
// host's message rules, then the boolean rules), the pairing check over the product of the set's
// group values (the signature pair included).
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void mbls_k_av_verdict_grp_lg6(
    const int32_t* __restrict__ key_st, const uint32_t* __restrict__ key_off, const int32_t* __restrict__ sig_st,
    const uint32_t* __restrict__ grp_off, const uint32_t* __restrict__ fgrp, uint32_t n_sets,
    const int32_t* __restrict__ set_pre, int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const bool live = threadIdx.x < 6u * kSetsPerWave;
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
    const uint32_t n_grp = grp_off[n_sets], a = grp_off[s], b = grp_off[s + 1];
    const size_t nl = (size_t)n_grp * 8;
    fp2 f = ld_lane(fgrp, nl, (size_t)a * 8 + k);
#pragma unroll 1
    for (uint32_t j = a + 1; j < b; ++j) f = lg::x12_mul(f, ld_lane(fgrp, nl, (size_t)j * 8 + k));
    out = lg::x12_is_one(lg::x12_final_exp(f)) ? 1 : 0;
  }
  if (live && g < n_sets && lg::gk() == 0) status[g] = out;
}

namespace mbls_launch {
uint32_t av_groups_bound(uint32_t n_pairs, uint32_t n_sets) {
  // sum of ceil((n_s + 1) / kPairs) <= (n_pairs + n_sets) / kPairs + n_sets
  return (uint32_t)(((uint64_t)n_pairs + n_sets) / kPairs + n_sets + 1);
}
hipError_t av_pairs_lg6(const int32_t* key_st, const uint32_t* key_xy, const uint32_t* h_xy, uint32_t n_pairs,
                        const uint32_t* key_off, uint32_t n_sets, const int32_t* sig_st, const uint32_t* sig_xy,
                        uint32_t* grp_off, uint32_t* fgrp, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_MILLER_PAIRS, s);
  hipLaunchKernelGGL(mbls_k_av_group_plan, dim3(1), dim3(kPlanThreads), 0, s, key_off, n_sets, grp_off);
  const uint32_t bound = av_groups_bound(n_pairs, n_sets);
  hipLaunchKernelGGL(mbls_k_av_pairs_lg6, dim3((bound + kSetsPerWave - 1) / kSetsPerWave), dim3(64), 0, s, key_st,
                     key_xy, h_xy, n_pairs, key_off, n_sets, sig_st, sig_xy, grp_off, fgrp);
  return hipGetLastError();
}
hipError_t av_verdict_grp_lg6(const int32_t* key_st, const uint32_t* key_off, const int32_t* sig_st,
                              const uint32_t* grp_off, const uint32_t* fgrp, uint32_t n_sets, const int32_t* set_pre,
                              int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_AV_VERDICT, s);
  hipLaunchKernelGGL(mbls_k_av_verdict_grp_lg6, dim3((n_sets + kSetsPerWave - 1) / kSetsPerWave), dim3(64), 0, s,
                     key_st, key_off, sig_st, grp_off, fgrp, n_sets, set_pre, status);
  return hipGetLastError();
}
}  // namespace mbls_launch
