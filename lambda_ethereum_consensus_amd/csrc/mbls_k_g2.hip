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

#include "mbls_g2_onelane.hpp"
using mbls_g2_onelane::hash_one;
using mbls_g2_onelane::sig_decode_one;


// (the one-lane signature decode and H(m) kernels, mbls_k_g2_sig_decode / mbls_k_hash_to_g2, are
// in mbls_k_g2w.hip: compiled for two waves per SIMD)
extern "C" __global__ void mbls_k_g2_sig_decode(const uint8_t* __restrict__ sigs, uint32_t n, int32_t group_check,
                                                const int32_t* __restrict__ pre, int32_t* __restrict__ st,
                                                uint32_t* __restrict__ xy);
extern "C" __global__ void mbls_k_hash_to_g2(const uint8_t* __restrict__ msgs, uint32_t n, uint32_t* __restrict__ hxy);

// The one-lane G2 prep of a verify / fast_aggregate_verify batch in ONE launch: blocks [0, nb)
// hash the messages (the longer chain, dispatched first), blocks [nb, 2 nb) decode and
// group-check the signatures -- the two independent chains of a call side by side instead of
// back to back on its stream (r03: a pipelined table epoch is bound by the G2 streams' time
// per call, decode 2.7 ms + H(m) 6.4 ms per 2,048 sets back to back).
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_g2_prep_1l(
    const uint8_t* __restrict__ sigs, const int32_t* __restrict__ sig_pre, const uint8_t* __restrict__ msgs,
    uint32_t n, int32_t* __restrict__ sig_st, uint32_t* __restrict__ sig_xy, uint32_t* __restrict__ hxy) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t nb = (n + 63) / 64;
  const bool hash_part = blockIdx.x < nb;  // block uniform
  const uint32_t i = (hash_part ? blockIdx.x : blockIdx.x - nb) * 64u + threadIdx.x;
  if (i >= n) return;
  if (hash_part)
    hash_one(msgs, n, i, hxy);
  else
    sig_decode_one(sigs, n, i, 1, sig_pre, sig_st, sig_xy);
}

// ----- random-linear-combination batch check, single-lane parts ---------
namespace {
__device__ __forceinline__ void st_g2p(uint32_t* base, size_t n, size_t i, const proj<fp2>& p) {
  st_fp(base, n, i, 0, p.x.c0);
  st_fp(base, n, i, NL, p.x.c1);
  st_fp(base, n, i, 2 * NL, p.y.c0);
  st_fp(base, n, i, 3 * NL, p.y.c1);
  st_fp(base, n, i, 4 * NL, p.z.c0);
  st_fp(base, n, i, 5 * NL, p.z.c1);
}
__device__ __forceinline__ proj<fp2> ld_g2p(const uint32_t* base, size_t n, size_t i) {
  return {{ld_fp(base, n, i, 0), ld_fp(base, n, i, NL)},
          {ld_fp(base, n, i, 2 * NL), ld_fp(base, n, i, 3 * NL)},
          {ld_fp(base, n, i, 4 * NL), ld_fp(base, n, i, 5 * NL)}};
}
__device__ __forceinline__ proj<fp2> shfl_xor_g2(const proj<fp2>& p, int m) {
  proj<fp2> r;
  fp* dst[6] = {&r.x.c0, &r.x.c1, &r.y.c0, &r.y.c1, &r.z.c0, &r.z.c1};
  const fp* src[6] = {&p.x.c0, &p.x.c1, &p.y.c0, &p.y.c1, &p.z.c0, &p.z.c1};
#pragma unroll
  for (int c = 0; c < 6; ++c)
#pragma unroll
    for (int d = 0; d < NL; ++d) dst[c]->v[d] = __shfl_xor(src[c]->v[d], m);
  return r;
}
}  // namespace

// Per set: whether a pairing decides it (mbls_fav_precheck), its scalar r_s = r0 + r1 x with
// (r0, r1) = SHA-256(seed || s)[0..8) as two 32-bit halves (injective: |x| > 2^63, so 2^64
// distinct scalars mod r), [r_s] apk_s and [r_s] sigma_s (identity outside the combination and
// for infinite signatures, whose pairs blst skips).  On G2, psi acts as [x]: [r_s] sigma =
// [r0] sigma + [r1] psi(sigma), a 32-bit joint ladder; on G1 the 97-bit signed integer
// r0 - r1 |x| is used directly.  Waves 0 .. nw-1 do the G1 halves, waves nw .. 2nw-1 the G2
// halves (wave-uniform split: the two run side by side).  Constant-time ladders, RCB formulas.
namespace {
__device__ __forceinline__ void rlc_scalar(uint4 seed_lo, uint4 seed_hi, uint32_t s, uint32_t& r0, uint32_t& r1) {
  uint32_t blk[16] = {seed_lo.x, seed_lo.y, seed_lo.z, seed_lo.w, seed_hi.x, seed_hi.y, seed_hi.z, seed_hi.w,
                      s,         0x80000000u, 0u,       0u,        0u,        0u,        0u,        36u * 8u};
  uint32_t h[8];
  sha256_init(h);
  sha256_compress(h, blk);
  r0 = h[0];
  r1 = h[1];
  if ((r0 | r1) == 0) r0 = 1;
}
}  // namespace

extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_rlc_scale(
    const int32_t* __restrict__ set_st, const uint32_t* __restrict__ set_xy, const uint32_t* __restrict__ key_off,
    const int32_t* __restrict__ sig_st, const uint32_t* __restrict__ sig_xy, uint32_t n_sets, int32_t eth,
    const int32_t* __restrict__ set_pre, uint4 seed_lo, uint4 seed_hi, int32_t* __restrict__ cand,
    uint32_t* __restrict__ p_xy, uint32_t* __restrict__ q_xy) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t nw = (n_sets + 63) / 64;
  const bool g2_half = blockIdx.x >= nw;
  const uint32_t s = (g2_half ? blockIdx.x - nw : blockIdx.x) * 64u + threadIdx.x;
  if (s >= n_sets) return;
  const int32_t ss = sig_st[s];
  const uint32_t nk = key_off[s + 1] - key_off[s];
  const bool c = mbls_fav_precheck(ss, set_st[s], set_pre ? set_pre[s] : 0, nk, eth) == MBLS_NEEDS_PAIRING;
  uint32_t r0, r1;
  rlc_scalar(seed_lo, seed_hi, s, r0, r1);
  if (!g2_half) {
    cand[s] = c ? 1 : 0;
    // t = r0 - r1 |x| as a signed 97-bit integer: |t| in 32-bit words (w2 w1 w0), sign
    const uint64_t lo = (uint64_t)r1 * (uint32_t)k::X_ABS, hi = (uint64_t)r1 * (uint32_t)(k::X_ABS >> 32);
    // m = r1 |x| = hi << 32 + lo (96 bits) as three words
    const uint64_t mid = (lo >> 32) + (hi & 0xffffffffull);
    uint32_t m0 = (uint32_t)lo, m1 = (uint32_t)mid, m2 = (uint32_t)((hi >> 32) + (mid >> 32));
    // |t| = m - r0 (m >= r0 unless r1 = 0), negative sign
    const bool neg = m2 | m1 | (m0 > r0);
    uint32_t t0, t1, t2;
    if (neg) {
      const uint64_t d0 = (uint64_t)m0 - r0;
      t0 = (uint32_t)d0;
      const uint64_t d1 = (uint64_t)m1 - (uint32_t)((d0 >> 63) & 1u);
      t1 = (uint32_t)d1;
      t2 = m2 - (uint32_t)((d1 >> 63) & 1u);
    } else {
      t0 = r0 - m0;
      t1 = 0;
      t2 = 0;
    }
    proj<fp> p = pt_identity<fp>();
    if (c) p = {ld_fp(set_xy, n_sets, s, 0), ld_fp(set_xy, n_sets, s, NL), ld_fp(set_xy, n_sets, s, 2 * NL)};
    proj<fp> rp = pt_identity<fp>();
    const uint32_t tw[3] = {t0, t1, t2};
#pragma unroll 1
    for (int b = 95; b >= 0; --b) {
      rp = pt_dbl(rp);
      rp = pt_select((tw[b >> 5] >> (b & 31)) & 1u, pt_add(rp, p), rp);
    }
    if (neg) rp = pt_neg(rp);
    st_fp(p_xy, n_sets, s, 0, rp.x);
    st_fp(p_xy, n_sets, s, NL, rp.y);
    st_fp(p_xy, n_sets, s, 2 * NL, rp.z);
  } else {
    proj<fp2> q = pt_identity<fp2>();
    if (c && ss == MBLS_DEC_OK) q = pt_from_affine(ld_g2(sig_xy, n_sets, s));
    const proj<fp2> qp = g2_psi(q);  // [x] q
    const proj<fp2> qq = pt_add(q, qp);
    proj<fp2> rq = pt_identity<fp2>();
#pragma unroll 1
    for (int b = 31; b >= 0; --b) {
      rq = pt_dbl(rq);
      const uint32_t sel = ((r0 >> b) & 1u) | (((r1 >> b) & 1u) << 1);
      const proj<fp2> add = pt_select(sel == 3, qq, pt_select(sel == 2, qp, q));
      rq = pt_select(sel != 0, pt_add(rq, add), rq);
    }
    st_g2p(q_xy, n_sets, s, rq);
  }
}

// One wave per 64 points: sum (butterfly of complete additions), lane 0 stores the partial.
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_rlc_sum_g2(const uint32_t* __restrict__ in, uint32_t n_in,
                                                                  uint32_t* __restrict__ out, uint32_t n_out) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  proj<fp2> acc = i < n_in ? ld_g2p(in, n_in, i) : pt_identity<fp2>();
#pragma unroll 1
  for (int m = 1; m < 64; m <<= 1) acc = pt_add(acc, shfl_xor_g2(acc, m));
  if (threadIdx.x == 0 && blockIdx.x < n_out) st_g2p(out, n_out, blockIdx.x, acc);
}

// One lane per (sk, msg): sigma = sk * H(m), compressed.  The secret key has been range
// checked on the host (0 < sk < r, lighthouse SecretKey::deserialize).  Constant-time
// double-and-always-add over 256 bits.
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_sign(const uint8_t* __restrict__ sk32,
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
extern "C" __global__ __launch_bounds__(64, MBLS_G2_WAVES) void mbls_k_g2_aggregate(const int32_t* __restrict__ sig_st,
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
hipError_t g2_prep_1l(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                      uint32_t* sig_xy, uint32_t* hxy, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G2_PREP, s);
  hipLaunchKernelGGL(mbls_k_g2_prep_1l, dim3(2 * ((n + 63) / 64)), dim3(64), 0, s, sigs, sig_pre, msgs, n, sig_st,
                     sig_xy, hxy);
  return hipGetLastError();
}
hipError_t g2_prep_split(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                         uint32_t* sig_xy, uint32_t* hxy, hipStream_t s) {
  // the same two chains as g2_prep_1l, as the two-wave kernels of mbls_k_g2w.hip, back to back
  hipError_t rc = hash_to_g2(msgs, n, hxy, s);
  return rc == hipSuccess ? g2_sig_decode(sigs, n, 1, sig_pre, sig_st, sig_xy, s) : rc;
}
hipError_t rlc_scale(const int32_t* set_st, const uint32_t* set_xy, const uint32_t* key_off, const int32_t* sig_st,
                     const uint32_t* sig_xy, uint32_t n_sets, int32_t eth, const int32_t* set_pre,
                     const uint32_t (&seed)[8], const RlcBufs& b, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_RLC, s);
  const uint4 lo = make_uint4(seed[0], seed[1], seed[2], seed[3]), hi = make_uint4(seed[4], seed[5], seed[6], seed[7]);
  hipLaunchKernelGGL(mbls_k_rlc_scale, dim3(2 * ((n_sets + 63) / 64)), dim3(64), 0, s, set_st, set_xy, key_off, sig_st,
                     sig_xy, n_sets, eth, set_pre, lo, hi, b.cand, b.p_xy, b.q_xy);
  return hipGetLastError();
}
// sum of n projective G2 points in q_xy (64 per wave and level); *result = the 1-point row set
hipError_t rlc_sum_g2(uint32_t* q_xy, uint32_t* q_tmp, uint32_t n, uint32_t** result, hipStream_t s) {
  uint32_t* in = q_xy;
  uint32_t* out = q_tmp;
  do {
    const uint32_t m = (n + 63) / 64;
    hipLaunchKernelGGL(mbls_k_rlc_sum_g2, dim3(m), dim3(64), 0, s, in, n, out, m);
    std::swap(in, out);
    n = m;
  } while (n > 1);
  *result = in;
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
size_t onelane_g2_private_bytes() {
  size_t m = 0;
  for (const void* k : {reinterpret_cast<const void*>(mbls_k_g2_sig_decode), reinterpret_cast<const void*>(mbls_k_hash_to_g2),
                        reinterpret_cast<const void*>(mbls_k_g2_prep_1l)}) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k) == hipSuccess) m = std::max(m, a.localSizeBytes);
  }
  return m;
}
}  // namespace mbls_launch
