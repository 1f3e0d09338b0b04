// mbls_g2_onelane.hpp — the per-lane bodies of the one-lane G2 kernels shared by
// mbls_k_g2.hip (the fused prep: one wave per SIMD) and mbls_k_g2w.hip (aggregate_verify's
// signature decode and H(m): two waves per SIMD).
#pragma once
#include "mbls_h2c.hpp"
#include "mbls_kernels.h"
#include "mbls_soa.hpp"

namespace mbls_g2_onelane {
using namespace mbls;
using namespace mbls_soa;
// One lane per signature: NONE (all-zero) detection, ZCash G2 decode, optional G2
// membership (blst sig_groupcheck=true in verify paths; aggregate does no group check).
__device__ __forceinline__ void sig_decode_one(const uint8_t* __restrict__ sigs, uint32_t n, uint32_t i,
                                               int32_t group_check, const int32_t* __restrict__ pre,
                                               int32_t* __restrict__ st, uint32_t* __restrict__ xy) {
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
// H(m) = hash_to_G2(m, DST_POP) of message i, affine
__device__ __forceinline__ void hash_one(const uint8_t* __restrict__ msgs, uint32_t n, uint32_t i,
                                         uint32_t* __restrict__ hxy) {
  uint32_t w[8];
  load_be<8>(msgs + (size_t)i * 32, w);
  aff<fp2> a;
  pt_to_affine(a, hash_to_g2_msg32(w));
  st_g2(hxy, n, i, a);
}
}  // namespace mbls_g2_onelane
