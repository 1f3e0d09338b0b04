// mbls_k_ssz.hip — SSZ signing roots on gfx950: the step before the
// verification path, producing the 32-byte messages the BLS kernels consume.
//
// Replaces, batched and device-resident:
//   Misc.compute_signing_root/2 (lib/lambda_ethereum_consensus/state_transition/misc.ex:243-260)
//     = hash_tree_root(SigningData{object_root, domain}) = SHA-256(object_root || domain)
//   Ssz.hash_tree_root/1 (lib/ssz.ex:51-55 -> ssz_nif) for fixed-size containers whose fields
//     are already 32-byte leaves (merkleize: pad the leaf count to a power of two with zero
//     chunks, hash pairs up to the root), and for AttestationData, whose root feeds
//     predicates.ex:120 (is_valid_indexed_attestation) for every attestation.
// One lane per object; SHA-256 words are big-endian reads of the chunk bytes.  Integer ALU
// work (~20 compressions per attestation), no MFMA, HBM traffic 128 + 32 (+ 32) bytes each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mbls_kernels.h"

namespace {

__device__ __constant__ uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// K[i] + W[i] of the constant second block of every 64-byte message (0x80, zeros, bit
// length 512): its schedule never changes, so it is folded into the round constants once
struct PadKW {
  uint32_t v[64];
  constexpr PadKW() : v() {
    constexpr uint32_t k[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t w[64] = {};
    w[0] = 0x80000000u;
    w[15] = 512u;
    for (int i = 16; i < 64; ++i) {
      const uint32_t a = w[i - 15], b = w[i - 2];
      const uint32_t s0 = ((a >> 7) | (a << 25)) ^ ((a >> 18) | (a << 14)) ^ (a >> 3);
      const uint32_t s1 = ((b >> 17) | (b << 15)) ^ ((b >> 19) | (b << 13)) ^ (b >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    for (int i = 0; i < 64; ++i) v[i] = k[i] + w[i];
  }
};
__device__ __constant__ PadKW PAD_KW = PadKW();

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

__device__ __forceinline__ void round_step(uint32_t (&s)[8], uint32_t kw) {
  const uint32_t S1 = rotr(s[4], 6) ^ rotr(s[4], 11) ^ rotr(s[4], 25);
  const uint32_t ch = (s[4] & s[5]) ^ (~s[4] & s[6]);
  const uint32_t t1 = s[7] + S1 + ch + kw;
  const uint32_t S0 = rotr(s[0], 2) ^ rotr(s[0], 13) ^ rotr(s[0], 22);
  const uint32_t mj = (s[0] & s[1]) ^ (s[0] & s[2]) ^ (s[1] & s[2]);
  s[7] = s[6];
  s[6] = s[5];
  s[5] = s[4];
  s[4] = s[3] + t1;
  s[3] = s[2];
  s[2] = s[1];
  s[1] = s[0];
  s[0] = t1 + S0 + mj;
}

// out = SHA-256(l || r) for 32-byte l, r (8 big-endian words each): two compressions, the
// second over the constant padding block
__device__ __forceinline__ void hash64(const uint32_t (&l)[8], const uint32_t (&r)[8], uint32_t (&out)[8]) {
  constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                              0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = l[i];
    w[8 + i] = r[i];
  }
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = IV[i];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t a = w[(i - 15) & 15], b = w[(i - 2) & 15];
      wi = w[i & 15] = w[i & 15] + (rotr(a, 7) ^ rotr(a, 18) ^ (a >> 3)) + w[(i - 7) & 15] +
                       (rotr(b, 17) ^ rotr(b, 19) ^ (b >> 10));
    }
    round_step(s, K256[i] + wi);
  }
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = s[i] = s[i] + IV[i];
#pragma unroll
  for (int i = 0; i < 64; ++i) round_step(s, PAD_KW.v[i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = s[i] + m[i];
}

// 32 chunk bytes at p (16-byte aligned) -> 8 big-endian words
__device__ __forceinline__ void load_chunk(const uint8_t* p, uint32_t (&w)[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  const uint32_t le[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = __builtin_bswap32(le[i]);
}
__device__ __forceinline__ void store_chunk(uint8_t* p, const uint32_t (&w)[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(__builtin_bswap32(w[0]), __builtin_bswap32(w[1]), __builtin_bswap32(w[2]),
                    __builtin_bswap32(w[3]));
  q[1] = make_uint4(__builtin_bswap32(w[4]), __builtin_bswap32(w[5]), __builtin_bswap32(w[6]),
                    __builtin_bswap32(w[7]));
}
// SSZ leaf of a uint64 (little-endian bytes, zero padded), as big-endian words
__device__ __forceinline__ void u64_chunk(uint32_t lo, uint32_t hi, uint32_t (&w)[8]) {
  w[0] = __builtin_bswap32(lo);
  w[1] = __builtin_bswap32(hi);
#pragma unroll
  for (int i = 2; i < 8; ++i) w[i] = 0;
}
__device__ __forceinline__ void zero_chunk(uint32_t (&w)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = 0;
}

constexpr int popcount_c(int v) { return v ? (v & 1) + popcount_c(v >> 1) : 0; }
constexpr int ctz_c(int v) { return (v & 1) ? 0 : 1 + ctz_c(v >> 1); }

// merge the top N stack entries pairwise, the top one at depth D
template <int D, int N>
__device__ __forceinline__ void merge_n(uint32_t (&stk)[5][8]) {
  if constexpr (N > 0) {
    hash64(stk[D - 1], stk[D], stk[D - 1]);
    merge_n<D - 1, N - 1>(stk);
  }
}
// SSZ merkleization of P (a power of two) leaves, of which the first `leaves` come from
// `chunks` and the rest are zero chunks, with a stack of one node per level: leaf I lands at
// depth popcount(I), then ctz(I + 1) merges -- all indices fixed at compile time
template <int I, int P>
__device__ __forceinline__ void merkle_leaf(const uint8_t* chunks, uint32_t leaves, uint32_t (&stk)[5][8]) {
  if constexpr (I < P) {
    constexpr int depth = popcount_c(I);
    if ((uint32_t)I < leaves)
      load_chunk(chunks + 32 * I, stk[depth]);
    else
      zero_chunk(stk[depth]);
    merge_n<depth, ctz_c(I + 1)>(stk);
    merkle_leaf<I + 1, P>(chunks, leaves, stk);
  }
}
template <int P>
__device__ __forceinline__ void merkleize(const uint8_t* chunks, uint32_t leaves, uint32_t (&root)[8]) {
  uint32_t stk[5][8];
  merkle_leaf<0, P>(chunks, leaves, stk);
#pragma unroll
  for (int j = 0; j < 8; ++j) root[j] = stk[0][j];
}

}  // namespace

// hash_tree_root of n fixed-size containers of `leaves` 32-byte leaves each (P = the leaf count
// padded to a power of two, P <= 16); chunks: n x leaves x 32 bytes
template <int P>
__global__ __launch_bounds__(256) void mbls_k_htr_chunks(const uint8_t* __restrict__ chunks, uint32_t leaves,
                                                         uint32_t n, uint8_t* __restrict__ out32) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t root[8];
  merkleize<P>(chunks + (size_t)i * leaves * 32, leaves, root);
  store_chunk(out32 + (size_t)i * 32, root);
}

// compute_signing_root(object_root, domain) = hash_tree_root(SigningData) = H(root || domain);
// domain_stride 0 = one domain for all objects, 32 = one per object
extern "C" __global__ __launch_bounds__(256) void mbls_k_signing_roots(const uint8_t* __restrict__ roots32,
                                                                      const uint8_t* __restrict__ domains32,
                                                                      uint32_t domain_stride, uint32_t n,
                                                                      uint8_t* __restrict__ out32) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t r[8], d[8], h[8];
  load_chunk(roots32 + (size_t)i * 32, r);
  load_chunk(domains32 + (size_t)i * domain_stride, d);
  hash64(r, d, h);
  store_chunk(out32 + (size_t)i * 32, h);
}

// AttestationData (phase0 SSZ, 128 bytes: slot u64 | index u64 | beacon_block_root |
// source {epoch u64, root} | target {epoch u64, root}) -> compute_signing_root(data, domain)
// (predicates.ex:118-121).  Leaves: slot, index, root, H(source), H(target), 3 zero chunks.
extern "C" __global__ __launch_bounds__(256) void mbls_k_attestation_signing_roots(
    const uint8_t* __restrict__ data128, const uint8_t* __restrict__ domains32, uint32_t domain_stride, uint32_t n,
    uint8_t* __restrict__ out32) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* q = reinterpret_cast<const uint4*>(data128 + (size_t)i * 128);
  uint32_t b[32];
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    const uint4 t = q[v];
    b[4 * v] = t.x;
    b[4 * v + 1] = t.y;
    b[4 * v + 2] = t.z;
    b[4 * v + 3] = t.w;
  }
  // little-endian dwords of the record: 0-1 slot, 2-3 index, 4-11 block root, 12-13 source
  // epoch, 14-21 source root, 22-23 target epoch, 24-31 target root
  uint32_t l0[8], l1[8], l2[8], e[8], rt[8], l3[8], l4[8];
  u64_chunk(b[0], b[1], l0);
  u64_chunk(b[2], b[3], l1);
#pragma unroll
  for (int j = 0; j < 8; ++j) l2[j] = __builtin_bswap32(b[4 + j]);
  u64_chunk(b[12], b[13], e);
#pragma unroll
  for (int j = 0; j < 8; ++j) rt[j] = __builtin_bswap32(b[14 + j]);
  hash64(e, rt, l3);  // hash_tree_root(source Checkpoint)
  u64_chunk(b[22], b[23], e);
#pragma unroll
  for (int j = 0; j < 8; ++j) rt[j] = __builtin_bswap32(b[24 + j]);
  hash64(e, rt, l4);  // hash_tree_root(target Checkpoint)
  uint32_t a[8], c[8], z[8], z1[8];
  hash64(l0, l1, a);
  hash64(l2, l3, c);
  uint32_t m0[8];
  hash64(a, c, m0);
  zero_chunk(z);
  hash64(l4, z, a);
  hash64(z, z, z1);  // zero-subtree root of two chunks
  hash64(a, z1, c);
  uint32_t root[8], d[8], sr[8];
  hash64(m0, c, root);
  load_chunk(domains32 + (size_t)i * domain_stride, d);
  hash64(root, d, sr);
  store_chunk(out32 + (size_t)i * 32, sr);
}

namespace mbls_launch {
hipError_t htr_chunks(const uint8_t* chunks, uint32_t leaves, uint32_t n, uint8_t* out32, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const dim3 g((n + 255) / 256), b(256);
  if (leaves <= 1)
    hipLaunchKernelGGL(mbls_k_htr_chunks<1>, g, b, 0, s, chunks, leaves, n, out32);
  else if (leaves <= 2)
    hipLaunchKernelGGL(mbls_k_htr_chunks<2>, g, b, 0, s, chunks, leaves, n, out32);
  else if (leaves <= 4)
    hipLaunchKernelGGL(mbls_k_htr_chunks<4>, g, b, 0, s, chunks, leaves, n, out32);
  else if (leaves <= 8)
    hipLaunchKernelGGL(mbls_k_htr_chunks<8>, g, b, 0, s, chunks, leaves, n, out32);
  else
    hipLaunchKernelGGL(mbls_k_htr_chunks<16>, g, b, 0, s, chunks, leaves, n, out32);
  return hipGetLastError();
}
hipError_t signing_roots(const uint8_t* roots32, const uint8_t* domains32, uint32_t domain_stride, uint32_t n,
                         uint8_t* out32, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mbls_k_signing_roots, dim3((n + 255) / 256), dim3(256), 0, s, roots32, domains32, domain_stride,
                     n, out32);
  return hipGetLastError();
}
hipError_t attestation_signing_roots(const uint8_t* data128, const uint8_t* domains32, uint32_t domain_stride,
                                     uint32_t n, uint8_t* out32, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_SSZ_ROOTS, s);
  hipLaunchKernelGGL(mbls_k_attestation_signing_roots, dim3((n + 255) / 256), dim3(256), 0, s, data128, domains32,
                     domain_stride, n, out32);
  return hipGetLastError();
}
}  // namespace mbls_launch
