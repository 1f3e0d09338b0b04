// Integer/FP64 issue-rate microbenchmark for gfx950 (MI355X).
//
// Calibrates the INT32 multiply-add roofline used by bench.py (SURVEY.md §8d asks for an
// unrolled independent v_mad_u64_u32 measurement instead of the assumed 16 MAC/clk/CU).
// Each lane runs 8 independent dependency chains of ONE instruction; we report ns per
// wave-instruction per SIMD and the implied chip-wide lane-ops/s.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/isa_rates tools/isa_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ void k_mad_u64(uint64_t* out, uint32_t seed) {
  uint64_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = seed * 3 + threadIdx.x, y = seed ^ 0x9e3779b9u;
  for (int i = 0; i < ITERS; ++i) {
#define S(k) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a##k) : "v"(x), "v"(y) : "vcc");
    REP8(S)
#undef S
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

#define SIMPLE_KERNEL(NAME, ASM)                                                              \
  __global__ void NAME(uint64_t* out, uint32_t seed) {                                       \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,     \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint32_t x = seed * 3 + threadIdx.x;                                                     \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(ASM : "+v"(a0) : "v"(x) : "vcc"); asm volatile(ASM : "+v"(a1) : "v"(x) : "vcc"); \
      asm volatile(ASM : "+v"(a2) : "v"(x) : "vcc"); asm volatile(ASM : "+v"(a3) : "v"(x) : "vcc"); \
      asm volatile(ASM : "+v"(a4) : "v"(x) : "vcc"); asm volatile(ASM : "+v"(a5) : "v"(x) : "vcc"); \
      asm volatile(ASM : "+v"(a6) : "v"(x) : "vcc"); asm volatile(ASM : "+v"(a7) : "v"(x) : "vcc"); \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;      \
  }

SIMPLE_KERNEL(k_add_u32, "v_add_u32 %0, %1, %0")
SIMPLE_KERNEL(k_add_co_u32, "v_add_co_u32 %0, vcc, %1, %0")
SIMPLE_KERNEL(k_addc_co_u32, "v_addc_co_u32 %0, vcc, %1, %0, vcc")
SIMPLE_KERNEL(k_mul_lo_u32, "v_mul_lo_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mul_hi_u32, "v_mul_hi_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mad_u32_u24, "v_mad_u32_u24 %0, %1, %0, %1")
SIMPLE_KERNEL(k_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %1, %0")
SIMPLE_KERNEL(k_add3_u32, "v_add3_u32 %0, %1, %0, %1")
SIMPLE_KERNEL(k_and_b32, "v_and_b32 %0, %1, %0")
SIMPLE_KERNEL(k_lshlrev_b32, "v_lshlrev_b32 %0, 1, %0")
SIMPLE_KERNEL(k_alignbit_b32, "v_alignbit_b32 %0, %1, %0, 28")
SIMPLE_KERNEL(k_bfe_u32, "v_bfe_u32 %0, %0, 0, 28")

// 64-bit-operand instructions of the radix-2^28 column carries (r06): the 64-bit shift and the
// 64-bit add-with-shift the compiler uses to merge a column's accumulators
#define WIDE_KERNEL(NAME, ASM)                                                                \
  __global__ void NAME(uint64_t* out, uint32_t seed) {                                       \
    uint64_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,     \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint64_t x = seed * 3ull + threadIdx.x;                                                  \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(ASM : "+v"(a0) : "v"(x)); asm volatile(ASM : "+v"(a1) : "v"(x));          \
      asm volatile(ASM : "+v"(a2) : "v"(x)); asm volatile(ASM : "+v"(a3) : "v"(x));          \
      asm volatile(ASM : "+v"(a4) : "v"(x)); asm volatile(ASM : "+v"(a5) : "v"(x));          \
      asm volatile(ASM : "+v"(a6) : "v"(x)); asm volatile(ASM : "+v"(a7) : "v"(x));          \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;      \
  }
WIDE_KERNEL(k_lshrrev_b64, "v_lshrrev_b64 %0, 28, %0")
WIDE_KERNEL(k_lshl_add_u64, "v_lshl_add_u64 %0, %1, 0, %0")

__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
  double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  double x = 1.0000001, y = 1e-9;
  for (int i = 0; i < ITERS; ++i) {
#define S(k) asm volatile("v_fma_f64 %0, %1, %0, %2" : "+v"(a##k) : "v"(x), "v"(y));
    REP8(S)
#undef S
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ void k_pk_fma_f32(uint64_t* out, uint32_t seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a0 = {(float)seed, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f2 x = {1.0000001f, 1.0000001f}, y = {1e-9f, 1e-9f};
  for (int i = 0; i < ITERS; ++i) {
#define S(k) asm volatile("v_pk_fma_f32 %0, %1, %0, %2" : "+v"(a##k) : "v"(x), "v"(y));
    REP8(S)
#undef S
  }
  f2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(s.x + s.y);
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8, threads = 256;  // 8 waves per SIMD... 32 waves/CU
  uint64_t* out;
  CHECK(hipMalloc(&out, sizeof(uint64_t) * blocks * threads));
  struct { const char* name; kfn f; } ks[] = {
      {"v_add_u32", k_add_u32},         {"v_add_co_u32", k_add_co_u32},   {"v_addc_co_u32", k_addc_co_u32},
      {"v_add3_u32", k_add3_u32},       {"v_mul_lo_u32", k_mul_lo_u32},   {"v_mul_hi_u32", k_mul_hi_u32},
      {"v_mad_u64_u32", k_mad_u64},     {"v_mad_u32_u24", k_mad_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24},
      {"v_fma_f64", k_fma_f64},         {"v_pk_fma_f32", k_pk_fma_f32},
      {"v_and_b32", k_and_b32},         {"v_lshlrev_b32", k_lshlrev_b32}, {"v_alignbit_b32", k_alignbit_b32},
      {"v_bfe_u32", k_bfe_u32},         {"v_lshrrev_b64", k_lshrrev_b64}, {"v_lshl_add_u64", k_lshl_add_u64},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"rates\": [\n", prop.name, cus, prop.clockRate);
  double add_ns = 0;
  for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
    hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(threads), 0, 0, out, 1u);  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)rep);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    double wave_instr = (double)blocks * (threads / 64) * ITERS * 8;
    double per_simd = wave_instr / (cus * 4.0);
    double ns_per = best * 1e6 / per_simd;          // ns per wave-instruction per SIMD
    double lane_ops = wave_instr * 64 / (best * 1e-3);  // chip lane-ops per second
    if (i == 0) add_ns = ns_per;
    printf("  {\"instr\": \"%s\", \"ms\": %.3f, \"ns_per_wave_instr_per_simd\": %.4f, \"rel_to_add\": %.2f, \"chip_lane_ops_per_s\": %.4e}%s\n",
           ks[i].name, best, ns_per, ns_per / add_ns, lane_ops, i + 1 < sizeof(ks) / sizeof(ks[0]) ? "," : "");
  }
  printf("]}\n");
  return 0;
}
