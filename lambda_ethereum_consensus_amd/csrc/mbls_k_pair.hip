// mbls_k_pair.hip — the one-lane pairing kernels of verify / fast_aggregate_verify:
// signature-side Miller values and the verdicts (Miller loops + final exponentiation).  Their
// own translation unit (split from mbls_k_g2.hip; aggregate_verify's in mbls_k_pairs_av.hip) so
// the large units compile side by side.
//
// Built with MBLS_FP_OUTLINE: the Fp multiply is a scalar-argument call, so these long
// kernels (Miller loop + final exponentiation, SSWU + cofactor clearing) stay I-cache sized.
// Replaces the blst calls behind lighthouse Signature::deserialize / verify /
// fast_aggregate_verify / eth_fast_aggregate_verify / aggregate_verify / sign / aggregate
// (native/bls_nif/src/lib.rs:14-119).
#define MBLS_FP_OUTLINE 1
// waves per SIMD the one-lane kernels must fit (1: up to 512 registers, the SIMD to itself)
#define MBLS_G2_WAVES 1  // 2 (256 registers, spills): epoch 82.9k -> 66.1k sets/s, r01
#include <algorithm>
#include <utility>
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
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_sig_miller(const int32_t* __restrict__ sig_st,
                                                                  const uint32_t* __restrict__ sig_xy, uint32_t n_sets,
                                                                  uint32_t* __restrict__ fsig) {
  // latency-critical per-set chain: win issue arbitration against the co-resident
  // throughput-bound key-validation waves (static priority, MI355X_MICROARCH §Two waves)
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  fp12 f = fp12_one();
  if (sig_st[s] == MBLS_DEC_OK) f = miller_loop_1(neg_g1_gen(), ld_g2(sig_xy, n_sets, s));
  st_fp12(fsig, n_sets, s, f);
}

// One lane per set: fast_aggregate_verify / eth_fast_aggregate_verify / verify verdict with
// the reference's precedence (signature decode error, then the first key error, then the
// boolean rules of lighthouse GenericAggregateSignature + blst).
// key_off == nullptr means one key per set (Bls.verify).  fsig (optional): the precomputed
// signature-side Miller values of mbls_k_sig_miller; without it the loop runs here.
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_fav_verdict(
    const int32_t* __restrict__ pk_st, const uint32_t* __restrict__ pk_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy, const uint32_t* __restrict__ fsig,
    const uint32_t* __restrict__ h_xy, uint32_t n_sets, int32_t eth_variant, const int32_t* __restrict__ set_pre,
    int32_t* __restrict__ status) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
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
    // Bls.verify: decoded affine keys (28 rows); fast_aggregate_verify (key_off set): the
    // projective per-set key sums of mbls_k_g1_aggregate (42 rows)
    const aff<fp2> h = ld_g2(h_xy, n_sets, s);
    fp12 f;
    if (key_off) {
      const proj<fp> p = {ld_fp(pk_xy, n_sets, s, 0), ld_fp(pk_xy, n_sets, s, NL), ld_fp(pk_xy, n_sets, s, 2 * NL)};
      if (fsig)  // precomputed e(-g1, sigma) Miller value (1 if infinite)
        f = fp12_mul(miller_loop_1(p, h), ld_fp12(fsig, n_sets, s));
      else if (ss != MBLS_DEC_INFINITY)  // both pairs, shared squarings
        f = miller_loop_2(p, h, neg_g1_gen(), ld_g2(sig_xy, n_sets, s));
      else  // blst skips an infinite signature: e(-g1, O) = 1
        f = miller_loop_1(p, h);
    } else {
      const aff<fp> p = ld_g1(pk_xy, n_sets, s);
      if (fsig)
        f = fp12_mul(miller_loop_1(p, h), ld_fp12(fsig, n_sets, s));
      else if (ss != MBLS_DEC_INFINITY)
        f = miller_loop_2(p, h, neg_g1_gen(), ld_g2(sig_xy, n_sets, s));
      else
        f = miller_loop_1(p, h);
    }
    out = fp12_is_one(final_exp(f)) ? 1 : 0;
  }
  status[s] = out;
}

// ----- host launch wrappers ---------------------------------------------------------------
namespace mbls_launch {
static inline dim3 grid64(uint32_t n) { return dim3((n + 63) / 64); }
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
  mbls_prof::Scope prof1_(mbls_prof::K_FAV_VERDICT_1L, s);
  hipLaunchKernelGGL(mbls_k_fav_verdict, grid64(n_sets), dim3(64), 0, s, pk_st, pk_xy, key_off, sig_st, sig_xy, fsig,
                     h_xy, n_sets, eth_variant, set_pre, status);
  return hipGetLastError();
}
static size_t private_bytes(const void* k) {
  hipFuncAttributes a{};
  return hipFuncGetAttributes(&a, k) == hipSuccess ? a.localSizeBytes : 0;
}
size_t onelane_pair_private_bytes() {
  return std::max(private_bytes(reinterpret_cast<const void*>(mbls_k_fav_verdict)),
                  private_bytes(reinterpret_cast<const void*>(mbls_k_sig_miller)));
}
}  // namespace mbls_launch
