// Fp Montgomery-multiply throughput on gfx950 (tools/, not product).
// Each lane iterates x <- x*y (dependent chain) over 4 independent chains.
// build: hipcc --offload-arch=gfx950 -O3 [-DMBLS_FP_ROW_LOOP] -I lambda_ethereum_consensus_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include "mbls_fp.hpp"

using namespace mbls;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

__global__ void k_chain(uint32_t* out, const uint32_t* in, int n, int iters) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  fp x0, x1, x2, x3, y;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    x0.v[i] = in[i * n + g];
    y.v[i] = in[(i + NL) * n + g];
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
  x0 = fp_add(fp_add(x0, x1), fp_add(x2, x3));
#pragma unroll
  for (int i = 0; i < NL; ++i) out[i * n + g] = x0.v[i];
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int n = prop.multiProcessorCount * 256 * 4;  // 16 waves per CU
  const int iters = 256;
  uint32_t *in, *out;
  CHECK(hipMalloc(&in, sizeof(uint32_t) * n * 24));
  CHECK(hipMalloc(&out, sizeof(uint32_t) * n * 12));
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * n * 24);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n * 24; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const int limb = (i / n) % 12;
    h[i] = (uint32_t)s & (limb == 11 ? 0x0fffffffu : 0xffffffffu);  // < p
  }
  CHECK(hipMemcpy(in, h, sizeof(uint32_t) * n * 24, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, out, in, n, 4);
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
  const double muls = (double)n * iters * 4;
  // checksum of lane 0 output for cross-variant comparison
  uint32_t o[12];
  for (int i = 0; i < 12; ++i) CHECK(hipMemcpy(&o[i], out + i * n, 4, hipMemcpyDeviceToHost));
  printf("{\"variant\": \"%s\", \"ms\": %.3f, \"fp_mul_per_s\": %.4e, \"lane0\": \"",
#ifdef MBLS_FP_ROW_LOOP
         "row_loop",
#else
         "unrolled",
#endif
         best, muls / (best * 1e-3));
  for (int i = 11; i >= 0; --i) printf("%08x", o[i]);
  printf("\", \"in_x\": \"");
  for (int i = 11; i >= 0; --i) printf("%08x", h[i * n]);
  printf("\", \"in_y\": \"");
  for (int i = 11; i >= 0; --i) printf("%08x", h[(i + 12) * n]);
  printf("\"}\n");
  return 0;
}
