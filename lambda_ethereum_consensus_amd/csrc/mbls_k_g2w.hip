// mbls_k_g2w.hip — the one-lane signature decode and H(m) = hash_to_G2(m, DST_POP) kernels of
// the aggregate_verify batches (and of Bls.aggregate's decode), in their own translation unit so
// that they are compiled for two waves per SIMD (256 registers) while the other one-lane kernels
// keep a whole SIMD (mbls_k_g2.hip): with two waves a SIMD hides one wave's scratch reloads
// behind the other's arithmetic (stall PMC pass: H(m) waits on s_waitcnt 23% of its wave-cycles
// at one wave, profiles/r05_pmc_stall_deposit.json).  r05: a deposit batch's 262,144-message
// H(m) 38.5 -> 29 ms and its 16,384 signature decodes 8.6 -> 4.0 ms beside the key kernel,
// deposit AV 201k -> 212k sets/s; the same occupancy for the fused prep (mbls_k_g2_prep_1l)
// costs the warm epoch 21% (profiles/r05_ab_g2_waves.txt).  Replaces blst's signature
// deserialization and hash_to_curve behind lighthouse aggregate_verify / aggregate
// (native/bls_nif/src/lib.rs:31-51,62-82).
#define MBLS_FP_OUTLINE 1
#define MBLS_G2W_WAVES 2
#include "mbls_g2_onelane.hpp"

using namespace mbls;
using namespace mbls_soa;
using mbls_g2_onelane::hash_one;
using mbls_g2_onelane::sig_decode_one;

extern "C" __global__ __launch_bounds__(64, MBLS_G2W_WAVES) void mbls_k_g2_sig_decode(
    const uint8_t* __restrict__ sigs, uint32_t n, int32_t group_check, const int32_t* __restrict__ pre,
    int32_t* __restrict__ st, uint32_t* __restrict__ xy) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sig_decode_one(sigs, n, i, group_check, pre, st, xy);
}

extern "C" __global__ __launch_bounds__(64, MBLS_G2W_WAVES) void mbls_k_hash_to_g2(const uint8_t* __restrict__ msgs,
                                                                                 uint32_t n, uint32_t* __restrict__ hxy) {
  __builtin_amdgcn_s_setprio(MBLS_G2_PRIO);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  hash_one(msgs, n, i, hxy);
}

namespace mbls_launch {
hipError_t g2_sig_decode(const uint8_t* sigs, uint32_t n, int32_t group_check, const int32_t* pre, int32_t* st,
                         uint32_t* xy, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G2_SIG_DECODE, s);
  hipLaunchKernelGGL(mbls_k_g2_sig_decode, dim3((n + 63) / 64), dim3(64), 0, s, sigs, n, group_check, pre, st, xy);
  return hipGetLastError();
}
hipError_t hash_to_g2(const uint8_t* msgs, uint32_t n, uint32_t* hxy, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_HASH_TO_G2, s);
  hipLaunchKernelGGL(mbls_k_hash_to_g2, dim3((n + 63) / 64), dim3(64), 0, s, msgs, n, hxy);
  return hipGetLastError();
}
}  // namespace mbls_launch
