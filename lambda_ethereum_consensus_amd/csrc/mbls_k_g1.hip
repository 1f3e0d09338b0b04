// mbls_k_g1.hip — G1 kernels: pubkey decode + key_validate, per-set aggregation, compression.
//
// These carry ~96% of a cold 512-key fast_aggregate_verify, so the Fp
// multiply is inlined here (no MBLS_FP_OUTLINE).  Replaces, per key, lighthouse
// `PublicKey::deserialize` -> blst `key_validate` (native/bls_nif/src/lib.rs:70-75,92-96,
// 110-114,129-134) and the `AggregatePublicKey::aggregate` sum (lib.rs:136-139 and inside
// blst fast_aggregate_verify).
//
// Layouts (HBM): pubkeys are the packed 48-byte ZCash encodings; decoded points are SoA,
// digit-major: xy[d * n + i], d = 0..13 x digits, 14..27 y digits (Montgomery, radix 2^28),
// so every digit load/store of a wave is one coalesced 256-byte transaction.
#include "mbls_curve.hpp"
#include "mbls_kernels.h"

#include <cstdlib>

#define MBLS_AGG_LANES_DEFAULT 32u
#define MBLS_AGG_LANES_TAB_DEFAULT 16u

using namespace mbls;

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void load_be48(const uint8_t* p, uint32_t (&w)[12]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);  // 48*i is 16-byte aligned
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const uint4 v = q[j];
    w[4 * j + 0] = bswap32(v.x);
    w[4 * j + 1] = bswap32(v.y);
    w[4 * j + 2] = bswap32(v.z);
    w[4 * j + 3] = bswap32(v.w);
  }
}

__device__ __forceinline__ void store_fp_soa(uint32_t* base, size_t n, size_t i, int d0, const fp& a) {
#pragma unroll
  for (int d = 0; d < NL; ++d) base[(size_t)(d0 + d) * n + i] = a.v[d];
}
__device__ __forceinline__ fp load_fp_soa(const uint32_t* base, size_t n, size_t i, int d0) {
  fp a;
#pragma unroll
  for (int d = 0; d < NL; ++d) a.v[d] = base[(size_t)(d0 + d) * n + i];
  return a;
}

__device__ __forceinline__ proj<fp> shfl_xor_pt(const proj<fp>& p, int m) {
  proj<fp> r;
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    r.x.v[d] = __shfl_xor(p.x.v[d], m);
    r.y.v[d] = __shfl_xor(p.y.v[d], m);
    r.z.v[d] = __shfl_xor(p.z.v[d], m);
  }
  return r;
}

// ----- The per-set key sums' group law with lazy sums (r04): RCB Algorithms 8 / 7 (as
// pt_add_affine_t / pt_add_t) with every sum, difference and 3b' = 12 multiple lazily bounded
// (mbls_lazy.hpp) and each output coordinate, a sum of two products in both formulas, reduced
// ONCE (fp_mul2): 5 + 3 x 1.5 reductions instead of 11 for the mixed addition, and one-shot
// carries instead of normalized additions.  The outputs are normalized (< 2p).
template <int A, int B, int C, int D>
__device__ __forceinline__ nz mul2(const lz<A>& a, const lz<B>& b, const lz<C>& c, const lz<D>& d) {
  static_assert(A * B + C * D <= 2400, "Montgomery input bound");
  return {fp_mul2(a.v, b.v, c.v, d.v)};
}
// P + Q, Q affine (a table row or a decoded key; not the identity)
__device__ __forceinline__ proj<fp> g1_add_affine_lz(const proj<fp>& p, const aff<fp>& q) {
  const nz X1{p.x}, Y1{p.y}, Z1{p.z}, x2{q.x}, y2{q.y};
  const nz t0 = mul(X1, x2), t1 = mul(Y1, y2);
  const lz<10> t3 = mul(x2 + y2, X1 + Y1) - (t0 + t1);
  const lz<4> t4 = mul(y2, Z1) + Y1;
  const lz<4> y3a = mul(x2, Z1) + X1;
  const lz<6> x3a = smul<3>(t0);
  const lz<24> t2 = smul<12>(Z1);  // 3b' Z1
  const lz<26> z3a = t1 + t2;
  const lz<34> t1m = t1 - t2;
  const lz<48> y3b = smul<12>(y3a);
  return {mul2(t3, t1m, t4, neg(y3b)).v, mul2(t1m, z3a, y3b, x3a).v, mul2(z3a, t4, x3a, t3).v};
}
// P + Q, both projective (the butterfly of the per-set sums)
__device__ __forceinline__ proj<fp> g1_add_lz(const proj<fp>& p, const proj<fp>& q) {
  const nz X1{p.x}, Y1{p.y}, Z1{p.z}, X2{q.x}, Y2{q.y}, Z2{q.z};
  const nz t0 = mul(X1, X2), t1 = mul(Y1, Y2), t2 = mul(Z1, Z2);
  const lz<10> t3 = mul(X1 + Y1, X2 + Y2) - (t0 + t1);
  const lz<10> t4 = mul(Y1 + Z1, Y2 + Z2) - (t1 + t2);
  const lz<10> y3a = mul(X1 + Z1, X2 + Z2) - (t0 + t2);
  const lz<6> x3a = smul<3>(t0);
  const lz<24> t2b = smul<12>(t2);  // 3b' Z1 Z2
  const lz<26> z3a = t1 + t2b;
  const lz<34> t1m = t1 - t2b;
  const lz<120> y3b = smul<12>(y3a);
  return {mul2(t3, t1m, t4, neg(y3b)).v, mul2(y3b, x3a, t1m, z3a).v, mul2(z3a, t4, x3a, t3).v};
}

}  // namespace

// One lane per key: ZCash decode (flags, x < p, sqrt of x^3 + 4, sign) and G1 membership.
// st[i]: MBLS_DEC_* code; xy: affine point (valid only when st[i] == MBLS_DEC_OK).
// pre (optional): host-detected per-key status (e.g. MBLS_DEC_PK_LENGTH) that replaces decoding.
// Launch bounds ask for 2 waves/SIMD: measured 25.6 ms vs 28.2 ms per 2^20 keys at 1 wave
// (tools/decode_variants.hip, profiles/r01_decode_variants.txt) despite a small spill.
// MBLS_KEY_BLOCK: threads per block of the key grid (no LDS, no barrier, so any multiple of 64).
#define MBLS_KEY_BLOCK 256
namespace {
__device__ __forceinline__ void decode_validate_one(const uint8_t* __restrict__ pks, uint32_t n, uint32_t i,
                                                    const int32_t* __restrict__ pre, int32_t* __restrict__ st,
                                                    uint32_t* __restrict__ xy) {
  if (pre && pre[i] != MBLS_DEC_OK) {
    st[i] = pre[i];
    return;
  }
  uint32_t w[12];
  load_be48(pks + (size_t)i * 48, w);
  aff<fp> a;
  a.x = fp_zero();
  a.y = fp_zero();
  int32_t s = g1_uncompress(a, w);
  if (s == DEC_OK && !g1_in_subgroup(a)) s = DEC_NOT_IN_GROUP;
  st[i] = s;
  store_fp_soa(xy, n, i, 0, a.x);
  store_fp_soa(xy, n, i, NL, a.y);
}
}  // namespace

extern "C" __global__ __launch_bounds__(MBLS_KEY_BLOCK, 2) void mbls_k_g1_decode_validate(const uint8_t* __restrict__ pks,
                                                                           uint32_t n, const int32_t* __restrict__ pre,
                                                                           int32_t* __restrict__ st,
                                                                           uint32_t* __restrict__ xy) {
  if (MBLS_KEY_PRIO) __builtin_amdgcn_s_setprio(MBLS_KEY_PRIO);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  decode_validate_one(pks, n, i, pre, st, xy);
}

// (Split into a decompression grid and a membership grid, r04 A/B: the shorter waves did not
// shrink the pipeline's last wave round -- 85.5-85.6k vs 86.5-86.8k sets/s at 20 steps, key grids
// 22.6 vs 22.0 ms, profiles/r04_ab1_lg6_waves_key_split.txt -- so the fused kernel stays.)

// Per-set key sums: a group of L lanes per set (L = 64, 32, 16 or 8; 64 / L sets per wave) sums
// the set's decoded keys (RCB complete mixed additions, lane-strided), butterfly-reduces across
// the group, records the FIRST failing key's code (reference error precedence: keys are
// deserialised in list order, lib.rs:92-96), and emits the PROJECTIVE sum (X, Y, Z) as set_xy
// rows 0..41: the pairing evaluates its lines at (X : Y : Z) directly (a line scaled by Z is
// killed by the final exponentiation), so the per-set inversion of an affine conversion is left
// to the one consumer that needs bytes (mbls_k_g1_compress_sets, one lane per set).
// set_st: MBLS_DEC_OK, a key's MBLS_DEC_* error, MBLS_AGG_INFINITY or MBLS_AGG_EMPTY.
// Why groups narrower than a wave: a set's sum costs (keys / L) mixed additions plus log2(L)
// butterfly additions per wave, and the butterfly's additions run on every lane of the wave, so
// at L = 64 a 512-key set costs 14 addition times per set (8 + 6, a third of them wasted), at
// L = 16 four sets share a wave's 36 (9 per set).  Pipelined batches fill the GPU and pay for
// SIMD time (the warm epoch's table gather slowed 0.9 -> 3.1 ms beside the lane-group G2 waves,
// r03 trace); a latency-bound batch (a mainnet block's 129 sets) pays for the chain length and
// keeps L = 64 (mbls_launch::agg_lanes).
namespace {
// packed wire keys, decoded into the SoA rows of mbls_k_g1_decode_validate
struct KeysSoA {
  const int32_t* st;
  const uint32_t* xy;
  uint32_t n;
  __device__ __forceinline__ int32_t status(uint32_t j) const { return st[j]; }
  __device__ __forceinline__ int32_t load(uint32_t j, aff<fp>& a) const {
    a = {load_fp_soa(xy, n, j, 0), load_fp_soa(xy, n, j, NL)};
    return st[j];
  }
};
// validator pubkey table rows addressed through an index list (rows are 128-byte AoS
// records, seven dwordx4 loads per key: a random gather touches one 128 B line pair per key)
struct KeysTable {
  const int32_t* st;
  const uint32_t* rows;
  uint32_t n_tab;
  const uint32_t* idx;
  __device__ __forceinline__ int32_t status(uint32_t j) const {
    const uint32_t r = idx[j];
    return r < n_tab ? st[r] : MBLS_DEC_UNKNOWN_INDEX;
  }
  // a row past the table (unknown index) reads row 0 instead; its status decides the set
  __device__ __forceinline__ int32_t load(uint32_t j, aff<fp>& a) const {
    const uint32_t r0 = idx[j];
    const bool in = r0 < n_tab;
    const uint4* q = reinterpret_cast<const uint4*>(rows + (size_t)(in ? r0 : 0u) * 32);
    uint32_t w[28];
#pragma unroll
    for (int v = 0; v < 7; ++v) {
      const uint4 t = q[v];
      w[4 * v] = t.x;
      w[4 * v + 1] = t.y;
      w[4 * v + 2] = t.z;
      w[4 * v + 3] = t.w;
    }
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      a.x.v[d] = w[d];
      a.y.v[d] = w[NL + d];
    }
    return in ? st[r0] : MBLS_DEC_UNKNOWN_INDEX;
  }
};

// Keys j in [lo, hi) of `src` summed by the L lanes of this lane's group (L a power of two,
// groups aligned in the wave); `live`: the group has a set (the tail groups of the last wave
// run the butterfly on identities and store nothing).  The next key's loads are issued before
// the current key's addition, so the gather's memory latency hides under the arithmetic.
template <class Src>
__device__ __forceinline__ void aggregate_set(const Src& src, uint32_t lanes, uint32_t lo, uint32_t hi, uint32_t s,
                                              bool live, uint32_t n_sets, int32_t* __restrict__ set_st,
                                              uint32_t* __restrict__ set_xy) {
  const uint32_t sub = threadIdx.x & (lanes - 1);
  uint32_t first_bad = 0xffffffffu;
  proj<fp> acc = pt_identity<fp>();
  uint32_t j = lo + sub;
  aff<fp> q;
  int32_t ks = DEC_OK;
  if (j < hi) ks = src.load(j, q);
#pragma unroll 1
  for (; j < hi; j += lanes) {
    aff<fp> qn;
    int32_t ksn = DEC_OK;
    if (j + lanes < hi) ksn = src.load(j + lanes, qn);
    if (ks != DEC_OK)
      first_bad = min(first_bad, j);
    else
      acc = g1_add_affine_lz(acc, q);
    q = qn;
    ks = ksn;
  }
#pragma unroll 1
  for (uint32_t m = 1; m < lanes; m <<= 1) {  // xor partners stay inside the aligned group
    first_bad = min(first_bad, (uint32_t)__shfl_xor((int)first_bad, (int)m));
    acc = g1_add_lz(acc, shfl_xor_pt(acc, (int)m));
  }
  if (sub != 0 || !live) return;
  int32_t out = DEC_OK;
  if (hi == lo)
    out = MBLS_AGG_EMPTY;
  else if (first_bad != 0xffffffffu)
    out = src.status(first_bad);
  else if (fp_is_zero(acc.z))
    out = MBLS_AGG_INFINITY;
  set_st[s] = out;
  store_fp_soa(set_xy, n_sets, s, 0, acc.x);
  store_fp_soa(set_xy, n_sets, s, NL, acc.y);
  store_fp_soa(set_xy, n_sets, s, 2 * NL, acc.z);
}
}  // namespace

extern "C" __global__ __launch_bounds__(64) void mbls_k_g1_aggregate(const int32_t* __restrict__ key_st,
                                                                    const uint32_t* __restrict__ key_xy,
                                                                    uint32_t n_keys,
                                                                    const uint32_t* __restrict__ key_off,
                                                                    uint32_t n_sets, int32_t* __restrict__ set_st,
                                                                    uint32_t* __restrict__ set_xy, uint32_t lanes) {
  if (MBLS_KEY_PRIO) __builtin_amdgcn_s_setprio(MBLS_KEY_PRIO);
  const uint32_t s = blockIdx.x * (64u / lanes) + threadIdx.x / lanes;
  const bool live = s < n_sets;
  const uint32_t lo = live ? key_off[s] : 0u, hi = live ? key_off[s + 1] : 0u;
  aggregate_set(KeysSoA{key_st, key_xy, n_keys}, lanes, lo, hi, s, live, n_sets, set_st, set_xy);
}

// Index-addressed form over the validator pubkey table: set s sums rows
// idx[idx_off[s] .. idx_off[s+1]); a row never set or past the table is
// MBLS_DEC_UNKNOWN_INDEX, ordered with the other key errors by list position.
extern "C" __global__ __launch_bounds__(64) void mbls_k_g1_aggregate_idx(
    const int32_t* __restrict__ tab_st, const uint32_t* __restrict__ tab_aff, uint32_t n_tab,
    const uint32_t* __restrict__ idx, const uint32_t* __restrict__ idx_off, uint32_t n_sets,
    int32_t* __restrict__ set_st, uint32_t* __restrict__ set_xy, uint32_t lanes) {
  const uint32_t s = blockIdx.x * (64u / lanes) + threadIdx.x / lanes;
  const bool live = s < n_sets;
  const uint32_t lo = live ? idx_off[s] : 0u, hi = live ? idx_off[s + 1] : 0u;
  aggregate_set(KeysTable{tab_st, tab_aff, n_tab, idx}, lanes, lo, hi, s, live, n_sets, set_st, set_xy);
}

// dst[i] = src[i]: the engine's stream-ordered copies of small caller arrays (a deferred cold
// verdict's offsets / prechecks).  hipMemcpyAsync device-to-device on a busy G2 stream blocked
// the calling thread behind that stream (r04: the pipelined table path lost ~10% to it).
extern "C" __global__ __launch_bounds__(256) void mbls_k_copy_u32(uint32_t* __restrict__ dst,
                                                                 const uint32_t* __restrict__ src, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// table rows [from, to) -> "never set"
extern "C" __global__ __launch_bounds__(256) void mbls_k_pk_table_fill(int32_t* __restrict__ tab_st, uint32_t from,
                                                                      uint32_t to) {
  const uint32_t r = from + blockIdx.x * blockDim.x + threadIdx.x;
  if (r < to) tab_st[r] = MBLS_DEC_UNKNOWN_INDEX;
}

// decoded keys (SoA) -> table rows first.. (AoS, 128 B per row) with their statuses
extern "C" __global__ __launch_bounds__(256) void mbls_k_pk_table_store(const int32_t* __restrict__ st,
                                                                       const uint32_t* __restrict__ xy, uint32_t n,
                                                                       uint32_t first, int32_t* __restrict__ tab_st,
                                                                       uint32_t* __restrict__ tab_aff) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t r = (size_t)first + i;
  tab_st[r] = st[i];
  uint32_t w[32];
#pragma unroll
  for (int d = 0; d < 2 * NL; ++d) w[d] = xy[(size_t)d * n + i];
#pragma unroll
  for (int d = 2 * NL; d < 32; ++d) w[d] = 0;
  uint4* o = reinterpret_cast<uint4*>(tab_aff + r * 32);
#pragma unroll
  for (int v = 0; v < 8; ++v) o[v] = make_uint4(w[4 * v], w[4 * v + 1], w[4 * v + 2], w[4 * v + 3]);
}

// eth_aggregate_pubkeys output: affine conversion and compression of the per-set projective
// sum (identity -> 0xc0 00..), and the status mapped to the C result code.
extern "C" __global__ __launch_bounds__(256) void mbls_k_g1_compress_sets(const int32_t* __restrict__ set_st,
                                                                         const uint32_t* __restrict__ set_xy,
                                                                         uint32_t n_sets, uint8_t* __restrict__ out48,
                                                                         int32_t* __restrict__ status) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  const int32_t st = set_st[s];
  uint32_t w[12];
  const proj<fp> p = {load_fp_soa(set_xy, n_sets, s, 0), load_fp_soa(set_xy, n_sets, s, NL),
                      load_fp_soa(set_xy, n_sets, s, 2 * NL)};
  aff<fp> a;
  pt_to_affine(a, p);
  g1_compress(w, a, st == MBLS_AGG_INFINITY);
  uint4* o = reinterpret_cast<uint4*>(out48 + (size_t)s * 48);
#pragma unroll
  for (int j = 0; j < 3; ++j)
    o[j] = make_uint4(bswap32(w[4 * j]), bswap32(w[4 * j + 1]), bswap32(w[4 * j + 2]), bswap32(w[4 * j + 3]));
  int32_t code;
  if (st == DEC_OK || st == MBLS_AGG_INFINITY)
    code = 2;  // MBLS_OK
  else if (st == MBLS_AGG_EMPTY)
    code = -9;  // Empty public key vector
  else
    code = mbls_pk_code(st);
  status[s] = code;
}

// SkToPk for a batch: pk = sk * G1, compressed (one lane per key; constant-time
// double-and-always-add over 256 bits).  Key generation for benches/tests and the
// reference's interop keys; sk is 32 bytes big-endian, already range checked.
extern "C" __global__ __launch_bounds__(256) void mbls_k_sk_to_pk(const uint8_t* __restrict__ sk32, uint32_t n,
                                                                 uint8_t* __restrict__ out48) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* q = reinterpret_cast<const uint4*>(sk32 + (size_t)i * 32);
  uint32_t sk[8];
  const uint4 v0 = q[0], v1 = q[1];
  sk[0] = bswap32(v0.x); sk[1] = bswap32(v0.y); sk[2] = bswap32(v0.z); sk[3] = bswap32(v0.w);
  sk[4] = bswap32(v1.x); sk[5] = bswap32(v1.y); sk[6] = bswap32(v1.z); sk[7] = bswap32(v1.w);
  const aff<fp> g = {fp_from(k::G1X), fp_from(k::G1Y)};
  proj<fp> r = pt_identity<fp>();
#pragma unroll 1
  for (int b = 255; b >= 0; --b) {
    r = pt_dbl(r);
    const proj<fp> t = pt_add_affine(r, g);
    const bool bit = (sk[7 - (b >> 5)] >> (b & 31)) & 1u;
    r = pt_select(bit, t, r);
  }
  aff<fp> a;
  const bool fin = pt_to_affine(a, r);
  uint32_t w[12];
  g1_compress(w, a, !fin);
  uint4* o = reinterpret_cast<uint4*>(out48 + (size_t)i * 48);
#pragma unroll
  for (int j = 0; j < 3; ++j)
    o[j] = make_uint4(bswap32(w[4 * j]), bswap32(w[4 * j + 1]), bswap32(w[4 * j + 2]), bswap32(w[4 * j + 3]));
}

// per-key decode status -> C result code (0 valid, < 0 error)
extern "C" __global__ __launch_bounds__(256) void mbls_k_map_pk_status(const int32_t* __restrict__ st, uint32_t n,
                                                                      int32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = st[i] == MBLS_DEC_OK ? 0 : mbls_pk_code(st[i]);
}

// ----- host launch wrappers ---------------------------------------------------------------
namespace mbls_launch {
hipError_t copy_u32(uint32_t* dst, const uint32_t* src, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mbls_k_copy_u32, dim3((n + 255) / 256), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}
hipError_t g1_decode_validate(const uint8_t* pks, uint32_t n, const int32_t* pre, int32_t* st, uint32_t* xy,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G1_DECODE, s);
  hipLaunchKernelGGL(mbls_k_g1_decode_validate, dim3((n + MBLS_KEY_BLOCK - 1) / MBLS_KEY_BLOCK), dim3(MBLS_KEY_BLOCK), 0, s,
                     pks, n, pre, st, xy);
  return hipGetLastError();
}
// Lanes per set of the per-set key sums (see mbls_k_g1_aggregate): 64 for latency-bound
// batches, narrower groups for batches that fill the GPU.  MBLS_AGG_LANES / MBLS_AGG_LANES_IDX
// (8, 16, 32 or 64) force the cold / table form.
static uint32_t agg_lanes(uint32_t n_sets, bool table) {
  static const uint32_t env_cold = [] {
    const char* v = std::getenv("MBLS_AGG_LANES");
    return v ? (uint32_t)std::strtoul(v, nullptr, 10) : 0u;
  }();
  static const uint32_t env_tab = [] {
    const char* v = std::getenv("MBLS_AGG_LANES_IDX");
    return v ? (uint32_t)std::strtoul(v, nullptr, 10) : 0u;
  }();
  const uint32_t e = table ? env_tab : env_cold;
  if (e == 8 || e == 16 || e == 32 || e == 64) return e;
  return n_sets >= 2048 ? (table ? MBLS_AGG_LANES_TAB_DEFAULT : MBLS_AGG_LANES_DEFAULT) : 64u;
}
hipError_t g1_aggregate(const int32_t* key_st, const uint32_t* key_xy, uint32_t n_keys, const uint32_t* key_off,
                        uint32_t n_sets, int32_t* set_st, uint32_t* set_xy, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G1_AGGREGATE, s);
  const uint32_t lanes = agg_lanes(n_sets, false), per = 64u / lanes;
  hipLaunchKernelGGL(mbls_k_g1_aggregate, dim3((n_sets + per - 1) / per), dim3(64), 0, s, key_st, key_xy, n_keys,
                     key_off, n_sets, set_st, set_xy, lanes);
  return hipGetLastError();
}
hipError_t g1_aggregate_idx(const int32_t* tab_st, const uint32_t* tab_aff, uint32_t n_tab, const uint32_t* idx,
                            const uint32_t* idx_off, uint32_t n_sets, int32_t* set_st, uint32_t* set_xy,
                            hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G1_AGGREGATE_IDX, s);
  const uint32_t lanes = agg_lanes(n_sets, true), per = 64u / lanes;
  hipLaunchKernelGGL(mbls_k_g1_aggregate_idx, dim3((n_sets + per - 1) / per), dim3(64), 0, s, tab_st, tab_aff, n_tab,
                     idx, idx_off, n_sets, set_st, set_xy, lanes);
  return hipGetLastError();
}
hipError_t pk_table_fill(int32_t* tab_st, uint32_t from, uint32_t to, hipStream_t s) {
  if (to <= from) return hipSuccess;
  hipLaunchKernelGGL(mbls_k_pk_table_fill, dim3((to - from + 255) / 256), dim3(256), 0, s, tab_st, from, to);
  return hipGetLastError();
}
hipError_t pk_table_store(const int32_t* st, const uint32_t* xy, uint32_t n, uint32_t first, int32_t* tab_st,
                          uint32_t* tab_aff, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_PK_TABLE_STORE, s);
  hipLaunchKernelGGL(mbls_k_pk_table_store, dim3((n + 255) / 256), dim3(256), 0, s, st, xy, n, first, tab_st,
                     tab_aff);
  return hipGetLastError();
}
hipError_t g1_compress_sets(const int32_t* set_st, const uint32_t* set_xy, uint32_t n_sets, uint8_t* out48,
                            int32_t* status, hipStream_t s) {
  if (n_sets == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_G1_COMPRESS, s);
  hipLaunchKernelGGL(mbls_k_g1_compress_sets, dim3((n_sets + 255) / 256), dim3(256), 0, s, set_st, set_xy, n_sets,
                     out48, status);
  return hipGetLastError();
}
hipError_t sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* out48, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mbls_k_sk_to_pk, dim3((n + 255) / 256), dim3(256), 0, s, sk32, n, out48);
  return hipGetLastError();
}
hipError_t map_pk_status(const int32_t* st, uint32_t n, int32_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  mbls_prof::Scope prof_(mbls_prof::K_MAP_PK_STATUS, s);
  hipLaunchKernelGGL(mbls_k_map_pk_status, dim3((n + 255) / 256), dim3(256), 0, s, st, n, out);
  return hipGetLastError();
}
}  // namespace mbls_launch
