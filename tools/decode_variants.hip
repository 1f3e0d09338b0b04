// Occupancy / code-shape experiment for the key-validation kernel (tools/, not product).
// Build variants: -DOUTLINE (out-of-line Fp multiply), -DWAVES=2 (launch bounds).
// Keys come from libmbls's SkToPk kernel; output: ms per 2^20 keys and a checksum.
#ifdef OUTLINE
#define MBLS_FP_OUTLINE 1
#endif
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/mbls.h"
#include "mbls_curve.hpp"

#ifndef WAVES
#define WAVES 1
#endif

using namespace mbls;

__global__ __launch_bounds__(256, WAVES) void k_decode(const uint8_t* __restrict__ pks, uint32_t n,
                                                       int32_t* __restrict__ st, uint32_t* __restrict__ xy) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[12];
  const uint4* q = reinterpret_cast<const uint4*>(pks + (size_t)i * 48);
  for (int j = 0; j < 3; ++j) {
    const uint4 v = q[j];
    w[4 * j] = __builtin_bswap32(v.x);
    w[4 * j + 1] = __builtin_bswap32(v.y);
    w[4 * j + 2] = __builtin_bswap32(v.z);
    w[4 * j + 3] = __builtin_bswap32(v.w);
  }
  aff<fp> a;
  a.x = fp_zero();
  a.y = fp_zero();
  int32_t s = g1_uncompress(a, w);
  if (s == DEC_OK && !g1_in_subgroup(a)) s = DEC_NOT_IN_GROUP;
  st[i] = s;
  for (int d = 0; d < NL; ++d) {
    xy[(size_t)d * n + i] = a.x.v[d];
    xy[(size_t)(NL + d) * n + i] = a.y.v[d];
  }
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 20);
  mbls_init(0);
  std::vector<uint8_t> sk(32 * (size_t)n, 0);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t v = 0x1234567890abcdefULL + 7919ULL * i;
    for (int b = 0; b < 8; ++b) sk[32 * (size_t)i + 31 - b] = (uint8_t)(v >> (8 * b));
    sk[32 * (size_t)i + 1] = 0x42;
  }
  uint8_t *d_sk = (uint8_t*)mbls_dev_malloc(sk.size()), *d_pk = (uint8_t*)mbls_dev_malloc(48 * (size_t)n);
  mbls_dev_memcpy_h2d(d_sk, sk.data(), sk.size());
  mbls_dev_sk_to_pk(d_sk, n, d_pk, nullptr);
  mbls_dev_synchronize(nullptr);
  int32_t* st;
  uint32_t* xy;
  hipMalloc(&st, 4 * (size_t)n);
  hipMalloc(&xy, 4 * 28 * (size_t)n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_decode, dim3((n + 255) / 256), dim3(256), 0, 0, d_pk, n, st, xy);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_decode, dim3((n + 255) / 256), dim3(256), 0, 0, d_pk, n, st, xy);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  std::vector<int32_t> hs(n);
  hipMemcpy(hs.data(), st, 4 * (size_t)n, hipMemcpyDeviceToHost);
  long ok = 0;
  for (auto v : hs) ok += (v == 0);
  printf("{\"variant\": \"%s waves=%d\", \"keys\": %u, \"ms\": %.3f, \"valid\": %ld}\n",
#ifdef OUTLINE
         "outline",
#else
         "inline",
#endif
         WAVES, n, best, ok);
  return 0;
}
