// Fp Montgomery-multiply throughput on gfx950 (tools/, not product): the radix-2^28 product of
// mbls_fp.hpp (NL = 14 digits).  Each lane iterates x <- x*y (dependent chain) over 4 independent
// chains, 16 waves per CU; lane 0's chain 0 is recomputed on the host with the same header (its
// functions are __host__ __device__) and must match bit for bit.
// (r05: the buffers are sized from NL.  The r01 version of this harness still had the CIOS-32
// layout of 12 limbs hard-coded and indexed past its buffers with 14 digits -- an illegal
// address fault on the first r05 run; profiles/r01_fp_rates_radix28.json came from a build of
// the time that was not committed.)
// build: hipcc --offload-arch=gfx950 -O3 -I lambda_ethereum_consensus_amd/csrc -o tools/fp_rates_radix28 tools/fp_rates.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "mbls_fp.hpp"

using namespace mbls;

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

// in: 2 NL digit rows of n (x, y); out: NL rows of n
__global__ __launch_bounds__(256) void k_chain(uint32_t* out, const uint32_t* in, int n, int iters) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  fp x0, x1, x2, x3, y;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    x0.v[i] = in[(size_t)i * n + g];
    y.v[i] = in[(size_t)(i + NL) * n + g];
  }
  x1 = fp_add(x0, y);
  x2 = fp_add(x1, y);
  x3 = fp_add(x2, y);
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
    x0 = fp_mul(x0, y);
    x1 = fp_mul(x1, y);
    x2 = fp_mul(x2, y);
    x3 = fp_mul(x3, y);
  }
  // all four chains reach the output (the host check recomputes the xor of them), so none is
  // dead code (r05: a first version compared a sum's digits with an impossible value, which the
  // compiler proved false and dropped three chains -- 2.6e11 "Fp-mul/s", 4x the mad peak allows)
#pragma unroll
  for (int i = 0; i < NL; ++i) out[(size_t)i * n + g] = x0.v[i] ^ x1.v[i] ^ x2.v[i] ^ x3.v[i];
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int n = prop.multiProcessorCount * 256 * 4;  // 16 waves per CU
  const int iters = 256;
  const size_t in_words = (size_t)n * 2 * NL, out_words = (size_t)n * NL;
  uint32_t *in = nullptr, *out = nullptr;
  CHECK(hipMalloc(&in, sizeof(uint32_t) * in_words));
  CHECK(hipMalloc(&out, sizeof(uint32_t) * out_words));
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * in_words);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < in_words; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const int digit = (int)((i / n) % NL);
    // digits < 2^28; the top digit < 2^16 keeps the value < 2^380 < p
    h[i] = (uint32_t)s & (digit == NL - 1 ? 0xffffu : M28);
  }
  CHECK(hipMemcpy(in, h, sizeof(uint32_t) * in_words, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, out, in, n, 4);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, out, in, n, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  // host check of lane 0: the four chains, xor-folded as the kernel stores them
  fp c[4], y;
  for (int i = 0; i < NL; ++i) {
    c[0].v[i] = h[(size_t)i * n];
    y.v[i] = h[(size_t)(i + NL) * n];
  }
  c[1] = fp_add(c[0], y);
  c[2] = fp_add(c[1], y);
  c[3] = fp_add(c[2], y);
  for (int it = 0; it < iters; ++it)
    for (auto& x : c) x = fp_mul(x, y);
  uint32_t o[NL];
  for (int i = 0; i < NL; ++i) CHECK(hipMemcpy(&o[i], out + (size_t)i * n, 4, hipMemcpyDeviceToHost));
  int match = 1;
  for (int i = 0; i < NL; ++i) match &= o[i] == (c[0].v[i] ^ c[1].v[i] ^ c[2].v[i] ^ c[3].v[i]);
  const double muls = (double)n * iters * 4;
  printf("{\"variant\": \"radix28\", \"ms\": %.3f, \"fp_mul_per_s\": %.4e, \"host_match\": %d}\n", best,
         muls / (best * 1e-3), match);
  free(h);
  return match ? 0 : 1;
}
