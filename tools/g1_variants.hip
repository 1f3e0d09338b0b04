// Key-validation kernel experiments (tools/, not product): time variants of the decode +
// G1-membership kernel on 2^20 keys made by libmbls's SkToPk kernel, and check that every
// variant returns the product kernel's statuses and decoded points bit for bit.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I lambda_ethereum_consensus_amd/csrc \
//          tools/g1_variants.hip -L lambda_ethereum_consensus_amd/lib -lmbls -o tools/g1v
//   run:   tools/g1v [variant ...]   (no argument: all)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/mbls.h"
#include "mbls_curve.hpp"

using namespace mbls;

namespace {

__device__ __forceinline__ void load_key(const uint8_t* pks, uint32_t i, uint32_t (&w)[12]) {
  const uint4* q = reinterpret_cast<const uint4*>(pks + (size_t)i * 48);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const uint4 v = q[j];
    w[4 * j] = __builtin_bswap32(v.x);
    w[4 * j + 1] = __builtin_bswap32(v.y);
    w[4 * j + 2] = __builtin_bswap32(v.z);
    w[4 * j + 3] = __builtin_bswap32(v.w);
  }
}

__device__ __forceinline__ void store_out(uint32_t* xy, uint32_t n, uint32_t i, const aff<fp>& a) {
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    xy[(size_t)d * n + i] = a.x.v[d];
    xy[(size_t)(NL + d) * n + i] = a.y.v[d];
  }
}

// final comparison of the membership test (as g1_in_subgroup)
__device__ __forceinline__ bool g1_check(const aff<fp>& p, const jac1& q) {
  const fp zz = fp_sqr(q.z);
  const fp bx = fp_mul(fp_from(k::BETA), p.x);
  const fp ex = fp_mul(bx, zz);
  const fp ey = fp_mul(p.y, fp_mul(zz, q.z));
  int32_t d[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)q.x.v[i] - (int32_t)ex.v[i] + lazy::P4.v[i];
  const bool okx = fp_is_zero(fp_shrink(fp_carry(d)));
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (int32_t)q.y.v[i] + (int32_t)ey.v[i];
  const bool oky = fp_is_zero(fp_shrink(fp_carry(d)));
  return okx && oky && !fp_is_zero(q.z);
}

// unified ladder: one doubling body for both [|x|] passes; additions by add-2007-bl against a
// base whose (zz, zzz) are 1 on the first pass
__device__ __forceinline__ bool g1_in_subgroup_unified(const aff<fp>& p) {
  const fp one = fp_from(k::ONE);
  jac1 r = {p.x, p.y, one};
  jac1_base qb = {p.x, p.y, one, one, one};
#pragma unroll 1
  for (int it = 0; it < 126; ++it) {
    const int b = 62 - (it >= 63 ? it - 63 : it);
    r = jac_dbl(r);
    if ((k::X_ABS >> b) & 1ull) r = jac_add(r, qb);
    if (it == 62) qb = jac_base(r);
  }
  return g1_check(p, r);
}

// unified doubling body, madd on pass 1 and add on pass 2
__device__ __forceinline__ bool g1_in_subgroup_unified2(const aff<fp>& p) {
  const fp one = fp_from(k::ONE);
  jac1 r = {p.x, p.y, one};
  jac1_base qb = {p.x, p.y, one, one, one};
#pragma unroll 1
  for (int it = 0; it < 126; ++it) {
    const int b = 62 - (it >= 63 ? it - 63 : it);
    r = jac_dbl(r);
    if ((k::X_ABS >> b) & 1ull) {
      if (it < 63)
        r = jac_madd(r, {qb.x, qb.y});
      else
        r = jac_add(r, qb);
    }
    if (it == 62) qb = jac_base(r);
  }
  return g1_check(p, r);
}

template <int V>
__device__ __forceinline__ void decode_body(const uint8_t* __restrict__ pks, uint32_t n, int32_t* __restrict__ st,
                                            uint32_t* __restrict__ xy) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[12];
  load_key(pks, i, w);
  aff<fp> a;
  a.x = fp_zero();
  a.y = fp_zero();
  int32_t s = g1_uncompress(a, w);
  if (V == 0) {
    if (s == DEC_OK && !g1_in_subgroup(a)) s = DEC_NOT_IN_GROUP;
  } else if (V == 1) {
    if (s == DEC_OK && !g1_in_subgroup_unified(a)) s = DEC_NOT_IN_GROUP;
  } else if (V == 2) {
    if (s == DEC_OK && !g1_in_subgroup_unified2(a)) s = DEC_NOT_IN_GROUP;
  }  // V == 3: decompress only
  st[i] = s;
  store_out(xy, n, i, a);
}

}  // namespace

__global__ __launch_bounds__(256, 2) void k_v0(const uint8_t* pks, uint32_t n, int32_t* st, uint32_t* xy) {
  decode_body<0>(pks, n, st, xy);
}
__global__ __launch_bounds__(256, 2) void k_v1(const uint8_t* pks, uint32_t n, int32_t* st, uint32_t* xy) {
  decode_body<1>(pks, n, st, xy);
}
__global__ __launch_bounds__(256, 2) void k_v2(const uint8_t* pks, uint32_t n, int32_t* st, uint32_t* xy) {
  decode_body<2>(pks, n, st, xy);
}
__global__ __launch_bounds__(256, 2) void k_v3(const uint8_t* pks, uint32_t n, int32_t* st, uint32_t* xy) {
  decode_body<3>(pks, n, st, xy);
}

typedef void (*kfn)(const uint8_t*, uint32_t, int32_t*, uint32_t*);

int main(int argc, char** argv) {
  const uint32_t n = 1u << 20;
  struct V {
    const char* name;
    kfn f;
  } vs[] = {{"v0_product", k_v0}, {"v1_unified_add", k_v1}, {"v2_unified_madd_add", k_v2}, {"v3_decompress_only", k_v3}};
  if (mbls_init(0) != 0) {
    fprintf(stderr, "mbls_init failed\n");
    return 1;
  }
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
  // every 97th key: flip a low x bit (almost always off-curve or off-subgroup) for parity
  {
    std::vector<uint8_t> pk(48 * (size_t)n);
    mbls_dev_memcpy_d2h(pk.data(), d_pk, pk.size());
    for (uint32_t i = 0; i < n; i += 97) pk[48 * (size_t)i + 47] ^= 1;
    mbls_dev_memcpy_h2d(d_pk, pk.data(), pk.size());
  }
  int32_t* st;
  uint32_t* xy;
  hipMalloc(&st, 4 * (size_t)n);
  hipMalloc(&xy, 4 * 28 * (size_t)n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<int32_t> ref_st(n), hs(n);
  std::vector<uint32_t> ref_xy(28 * (size_t)n), hxy(28 * (size_t)n);
  int reps = 3;
  for (int a = 1; a < argc; ++a)
    if (!strcmp(argv[a], "--reps1")) reps = 1;
  for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); ++v) {
    bool want = argc <= 1;
    for (int a = 1; a < argc; ++a) want |= std::string(vs[v].name).find(argv[a]) != std::string::npos;
    if (!want && v != 0) continue;
    hipLaunchKernelGGL(vs[v].f, dim3((n + 255) / 256), dim3(256), 0, 0, d_pk, n, st, xy);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(vs[v].f, dim3((n + 255) / 256), dim3(256), 0, 0, d_pk, n, st, xy);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    hipMemcpy(hs.data(), st, 4 * (size_t)n, hipMemcpyDeviceToHost);
    hipMemcpy(hxy.data(), xy, 4 * 28 * (size_t)n, hipMemcpyDeviceToHost);
    long ok = 0, bad = 0;
    for (uint32_t i = 0; i < n; ++i) ok += (hs[i] == 0);
    if (v == 0) {
      ref_st = hs;
      ref_xy = hxy;
    } else if (v != 3) {
      for (uint32_t i = 0; i < n; ++i) bad += hs[i] != ref_st[i];
      for (size_t i = 0; i < hxy.size(); ++i) bad += hxy[i] != ref_xy[i];
    }
    printf("{\"variant\": \"%s\", \"keys\": %u, \"ms\": %.3f, \"valid\": %ld, \"mismatch\": %ld}\n", vs[v].name, n,
           best, ok, bad);
    fflush(stdout);
  }
  return 0;
}
