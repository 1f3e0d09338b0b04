// mbls_pairing_lg.hpp — the pairing on 8-lane groups: one set per group, lane k of the group
// owns the Fp2 coefficient of w^k of every Fp12 value (k < 6; lanes 6 and 7 hold zero).
//
// Why: the per-set pairing chain of a fast_aggregate_verify batch is latency bound (a batch
// of 2,048 sets is only 32 waves), and one wave issues at most one VALU instruction per
// 4 cycles, so the chain's latency is its per-lane instruction count.  Spreading each Fp12
// operation over 6 lanes cuts that count ~4x (measured r01: single-lane verdict 13.75 M VALU
// instructions per lane, 34 ms): an Fp12 product is 6 Fp2 products per lane
// instead of 18, a cyclotomic squaring 2 Fp2 squarings instead of 9, a Miller doubling step
// two rounds of lane-parallel Fp2 products.  Coefficients move between lanes with
// ds_bpermute (no LDS allocation, no barrier: a group never leaves its own wave).
//
// The results are the same field elements as the single-lane routines of mbls_pairing.hpp
// (same formulas, same projective representatives of T), up to the weak-reduction
// representative of each coefficient, so the two are tested against each other and the
// verdicts against the oracle.  Replaces blst's miller_loop_n / final_exp behind lighthouse
// fast_aggregate_verify (native/bls_nif/src/lib.rs:99,118); re-derived.
//
// Contract: every kernel using this header runs 64-thread blocks and keeps all 8 lanes of a
// group active through every call (branches must be group uniform).
#pragma once
#include "mbls_h2c.hpp"
#include "mbls_lazy.hpp"
#include "mbls_pairing.hpp"

namespace mbls {
namespace lg {

// MBLS_LG_GROUP = 6 (a translation unit of its own, mbls_k_lg6.hip): the same routines on
// 6-lane groups, ten sets per wave (lanes 60..63 a tail group whose results are discarded)
// instead of eight with lanes 6 and 7 idle -- the same per-lane instruction stream for 25% more
// sets per wave.  There the "pad lane" reads (coefficient index 6) go through coefz(), and the
// Miller steps take P affine (Z_P = 1) so that a doubling step's second round has six products.
#ifndef MBLS_LG_GROUP
#define MBLS_LG_GROUP 8
#endif
static_assert(MBLS_LG_GROUP == 8 || MBLS_LG_GROUP == 6, "lane-group size");
#if MBLS_LG_GROUP == 8
__device__ __forceinline__ int gk() { return (int)(threadIdx.x & 7u); }      // coefficient index
__device__ __forceinline__ int gbase() { return (int)(threadIdx.x & 56u); }  // first lane of the group
#else
__device__ __forceinline__ int gk() {
  const int l = (int)threadIdx.x;
  return l < 60 ? l % 6 : l - 60;
}
__device__ __forceinline__ int gbase() { return (int)threadIdx.x - gk(); }
#endif

__device__ __forceinline__ uint32_t pull(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ fp pull(const fp& a, int src) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = pull(a.v[i], src);
  return r;
}
__device__ __forceinline__ fp2 pull(const fp2& a, int src) { return {pull(a.c0, src), pull(a.c1, src)}; }

// coefficient of w^k from its lane (8-lane groups: k = 6 reads the pad lane, zero; 6-lane
// groups: k < 6 only -- the sites whose k can be 6 for a live lane use coefz)
__device__ __forceinline__ fp2 coef(const fp2& c, int k) { return pull(c, gbase() + k); }
#if MBLS_LG_GROUP == 8
__device__ __forceinline__ fp2 coefz(const fp2& c, int k) { return coef(c, k); }
__device__ __forceinline__ fp2 pad_zero(const fp2& c) { return fp2_select(gk() < 6, c, fp2_zero()); }
#else
__device__ __forceinline__ fp2 coefz(const fp2& c, int k) {
  return fp2_select(k < 6, pull(c, gbase() + (k < 6 ? k : 0)), fp2_zero());
}
__device__ __forceinline__ fp2 pad_zero(const fp2& c) { return c; }
#endif

// a / 2 for a < 2p (normalized): add p when odd, then shift; result < 2p
MBLS_HD fp fp_half(const fp& a) {
  const uint32_t odd = a.v[0] & 1u;
  uint32_t t[NL];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t x = a.v[i] + (odd ? k::P_RAW[i] : 0u) + c;
    c = x >> 28;
    t[i] = x & M28;
  }
  t[NL - 1] |= c << 28;
  fp r;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) r.v[i] = (t[i] >> 1) | ((t[i + 1] & 1u) << 27);
  r.v[NL - 1] = t[NL - 1] >> 1;
  return r;
}
MBLS_HD fp2 fp2_half(const fp2& a) { return {fp_half(a.c0), fp_half(a.c1)}; }

// select among lane-dependent Fp2 values by k (k >= 5 -> a5; pick7: k >= 6 -> a6)
__device__ __forceinline__ fp2 pick6(int k, const fp2& a0, const fp2& a1, const fp2& a2, const fp2& a3,
                                     const fp2& a4, const fp2& a5) {
  fp2 r = fp2_select(k == 4, a4, a5);
  r = fp2_select(k == 3, a3, r);
  r = fp2_select(k == 2, a2, r);
  r = fp2_select(k == 1, a1, r);
  return fp2_select(k == 0, a0, r);
}

__device__ __forceinline__ fp2 pick7(int k, const fp2& a0, const fp2& a1, const fp2& a2, const fp2& a3,
                                     const fp2& a4, const fp2& a5, const fp2& a6) {
  return fp2_select(k >= 6, a6, pick6(k, a0, a1, a2, a3, a4, a5));
}

// Call boundary of the Fp12 products (x12_mul / _sqr / _cyc_sqr / _mul_line) and of the
// Miller steps: inlined into their callers by default, so their fp2 / point arguments and the
// running T stay in registers instead of going through scratch (a by-reference or > 32-dword
// argument list is passed in memory, and an outlined callee saves the callee-saved VGPRs it
// uses).  Measured r01 (profiles/r01_pipeline_experiments.txt, 3 runs each): warm epoch
// 346-360k -> 376-377k sets/s, deposit AV 112-116k -> 117-118k; cold and one mainnet block
// unchanged.  Inlining only one of the two families gains less (x12) or loses (steps).
#define MBLS_X12_FN __device__ __forceinline__
#define MBLS_STEP_FN __device__ __forceinline__
// the lane-group G2 doubling / addition (membership ladder, cofactor clearing): inlined too
// (warm epoch 378k / 381k -> 403k / 396k sets/s, r01; the points stay in registers)
#define MBLS_G2STEP_FN __device__ __forceinline__

// ----- Fp12 in lanes ---------------------------------------------------------------------
__device__ __forceinline__ fp2 x12_one() { return gk() == 0 ? fp2_one() : fp2_zero(); }

// p^6 Frobenius: odd powers of w change sign
__device__ __forceinline__ fp2 x12_conj(const fp2& c) { return fp2_select(gk() & 1, fp2_neg(c), c); }

// (r05) the cyclotomic squaring's and the line product's coefficient pulls, the trio steps'
// round exchanges and the line broadcasts through LDS too (xs::put2 / get2 below) instead of
// ds_bpermute: warm epoch at 100 steps 1.08-1.11M -> 1.14-1.15M sets/s, the 6-lane verdict
// 5.47-5.50 -> 5.26-5.27 ms per 2,048 sets in the pipeline (profiles/r05_ab_lg6_lds_pulls.txt)
#if MBLS_LG_GROUP == 6
// ----- Operand staging through LDS (6-lane groups): an Fp12 product's term t of lane k is
// f_i g_j' with g_j' = g_j or xi g_j, and the complex product needs g_j'.c0, g_j'.c1 and
// -g_j'.c1.  Pulled through ds_bpermute (one register, the same for every lane) each lane had to
// form xi g_j and the negation itself, per term (~220 instructions, a quarter of a term).  Here
// every lane writes its own coefficient's variants ONCE per product into LDS and each term reads
// the variant it needs by address (20 ds_read per term).  One wave per workgroup: a slot is
// 14 dwords per lane, stored as three rows of 64 x 16 B and one of 64 x 8 B (a wave's read of one
// row is one conflict-free sweep); 10 slots = 35 KiB per wave, 140 KiB for the four waves a CU
// holds at one wave per SIMD.
namespace xs {
constexpr int kSlots = 10;
__device__ __forceinline__ uint4* lo() {
  __shared__ uint4 b[kSlots * 3 * 64];
  return b;
}
__device__ __forceinline__ uint2* hi() {
  __shared__ uint2 b[kSlots * 64];
  return b;
}
// write -> read (and read -> next write) ordering across the lanes of the one wave.  Every
// kernel that uses xs:: is launched with ONE 64-lane wave per workgroup (__launch_bounds__(64),
// grids of 64-thread blocks in the mbls_launch wrappers), so this barrier only orders the wave's
// own LDS accesses: s_barrier is a scalar instruction the wave executes whatever its EXEC mask,
// and with one wave in the workgroup it completes at once.  That is what makes it valid inside
// the group-divergent branches of the 6-lane verdicts and mbls_k_av6.hip's grouped steps (ADVICE
// r05), where lanes of other groups are masked off; a multi-wave workgroup would break it.
__device__ __forceinline__ void sync() { __syncthreads(); }
__device__ __forceinline__ void put(int slot, const fp& a) {
  const int l = (int)threadIdx.x;
  uint4* L = lo() + slot * 192 + l;
  L[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  L[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
  L[128] = make_uint4(a.v[8], a.v[9], a.v[10], a.v[11]);
  hi()[slot * 64 + l] = make_uint2(a.v[12], a.v[13]);
}
__device__ __forceinline__ fp get(int slot, int src) {  // slot and src may differ per lane
  const uint4* L = lo() + slot * 192 + src;
  const uint4 x = L[0], y = L[64], z = L[128];
  const uint2 w = hi()[slot * 64 + src];
  fp r;
  r.v[0] = x.x; r.v[1] = x.y; r.v[2] = x.z; r.v[3] = x.w;
  r.v[4] = y.x; r.v[5] = y.y; r.v[6] = y.z; r.v[7] = y.w;
  r.v[8] = z.x; r.v[9] = z.y; r.v[10] = z.z; r.v[11] = z.w;
  r.v[12] = w.x; r.v[13] = w.y;
  return r;
}
// slots 2..7: the second operand's variants g.c0, g.c1, -g.c1 and (xi g).c0, (xi g).c1,
// -(xi g).c1 (bounds 2p, 2p, 4p, 6p, 4p, 8p; digits < 2^28 + 16)
__device__ __forceinline__ void put_b(const fp2& g) {
  const nz g0{g.c0}, g1{g.c1};
  const lz<4> xg1 = g0 + g1;
  put(2, g.c0);
  put(3, g.c1);
  put(4, neg(g1).v);
  put(5, (g0 - g1).v);
  put(6, xg1.v);
  put(7, neg(xg1).v);
}
// re += a0 b0' + a1 (-b1'), im += a0 b1' + a1 b0' with b' = the variant at slot v of lane sb:
// sum < 2 a 8p per component per term
__device__ __forceinline__ void term(fpcols& re, fpcols& im, const fp& a0, const fp& a1, int v, int sb) {
  const fp b0 = get(v, sb), b1 = get(v + 1, sb), nb1 = get(v + 2, sb);
  cols_mad(re, a0, b0);
  cols_mad(re, a1, nb1);
  cols_mad(im, a0, b1);
  cols_mad(im, a1, b0);
}
// (r05) bulk exchanges through the same slots: a lane's Fp2 written once
// (slots s, s + 1: 8 ds_write), another lane's read by address (8 ds_read) -- instead of 28
// ds_bpermute per Fp2 pulled.  Lane indices are masked to the wave (the tail group's pulls
// past lane 63 read some other lane's value, as ds_bpermute's wrap did; its results are
// discarded).
__device__ __forceinline__ void put2(int s, const fp2& c) {
  put(s, c.c0);
  put(s + 1, c.c1);
}
__device__ __forceinline__ fp2 get2(int s, int src) { return {get(s, src & 63), get(s + 1, src & 63)}; }
}  // namespace xs

// h = f g: h_k = sum_j f_{k-j} g_j, xi for the wrapped terms; six terms (f < 2p: sum < 6 x 2 x 2p
// x 8p = 192 p^2), one reduction per component
MBLS_X12_FN fp2 x12_mul(const fp2& f, const fp2& g) {
  xs::sync();  // the previous product's reads are done
  xs::put(0, f.c0);
  xs::put(1, f.c1);
  xs::put_b(g);
  xs::sync();
  const int k = gk() < 6 ? gk() : 0, base = gbase();
  fpcols re, im;
  cols_zero(re);
  cols_zero(im);
#pragma unroll 1
  for (int j = 0; j < 6; ++j) {
    const bool wrap = j > k;
    const int sa = (base + (wrap ? k - j + 6 : k - j)) & 63;
    xs::term(re, im, xs::get(0, sa), xs::get(1, sa), wrap ? 5 : 2, (base + j) & 63);
  }
  return fp2_cols_redc(re, im);
}

// h = f^2, the symmetric schoolbook of x12_sqr below, the weight 2 as a staged first-operand
// variant 2f (slots 8, 9; sum < 4 x 2 x 4p x 8p = 256 p^2); the (6, 6) terms are skipped
MBLS_X12_FN fp2 x12_sqr(const fp2& f) {
  constexpr uint32_t TI[4] = {0x66000000u, 0x66111121u, 0x66224332u, 0x66656463u};
  constexpr uint32_t TJ[4] = {0x66543210u, 0x66432155u, 0x66325544u, 0x66656463u};
  constexpr uint32_t XI[4] = {0x00u, 0x03u, 0x0fu, 0x15u};
  constexpr uint32_t W2[4] = {0x3eu, 0x3bu, 0x2fu, 0x00u};
  const nz2 fn = nrm(f);
  const lz2<4> f2 = smul<2>(fn);
  xs::sync();
  xs::put(0, f.c0);
  xs::put(1, f.c1);
  xs::put(8, f2.v.c0);
  xs::put(9, f2.v.c1);
  xs::put_b(f);
  xs::sync();
  const int k = gk(), base = gbase();
  fpcols re, im;
  cols_zero(re);
  cols_zero(im);
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    const int i = (TI[t] >> (4 * k)) & 15, j = (TJ[t] >> (4 * k)) & 15;
    if (i < 6) {  // (6, 6): a zero term
      const int sa = (base + i) & 63, va = ((W2[t] >> k) & 1u) ? 8 : 0;
      xs::term(re, im, xs::get(va, sa), xs::get(va + 1, sa), ((XI[t] >> k) & 1u) ? 5 : 2, (base + j) & 63);
    }
  }
  return fp2_cols_redc(re, im);
}
#else
// h = f g: h_k = sum_j f_{k-j} g_j, with xi for the wrapped terms (w^6 = xi).  The lane's six
// Fp2 products are summed unreduced and reduced once per component (lazy reduction:
// 24 + 2 Montgomery-size passes instead of 6 x 3 x 2).
MBLS_X12_FN fp2 x12_mul(const fp2& f, const fp2& g) {
  const int k = gk() < 6 ? gk() : 0;
  fpcols re, im;
  cols_zero(re);
  cols_zero(im);
#pragma unroll 1
  for (int j = 0; j < 6; ++j) {
    const bool wrap = j > k;
    const int i = wrap ? k - j + 6 : k - j;
    cols_mad2(re, im, nrm(coef(f, i)), nrm(coef(g, j)), wrap);
  }
  return pad_zero(fp2_cols_redc(re, im));
}

// h = f^2 by the symmetric schoolbook: at most 4 products per lane.  Term t of lane k is
// f_i f_j (weight 2 when i != j), times xi when i + j >= 6; (6, 6) reads the pad lane = 0.
MBLS_X12_FN fp2 x12_sqr(const fp2& f) {
  // nibble k of the constants = index for lane k (lanes 6, 7 use the pad lane)
  constexpr uint32_t TI[4] = {0x66000000u, 0x66111121u, 0x66224332u, 0x66656463u};
  constexpr uint32_t TJ[4] = {0x66543210u, 0x66432155u, 0x66325544u, 0x66656463u};
  constexpr uint32_t XI[4] = {0x00u, 0x03u, 0x0fu, 0x15u};  // bit k: term wraps (x xi)
  constexpr uint32_t W2[4] = {0x3eu, 0x3bu, 0x2fu, 0x00u};  // bit k: weight 2
  const int k = gk();
  fpcols re, im;
  cols_zero(re);
  cols_zero(im);
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    const int i = (TI[t] >> (4 * k)) & 15, j = (TJ[t] >> (4 * k)) & 15;
    const nz2 fi = nrm(coefz(f, i));
    const lz2<4> a = sel((W2[t] >> k) & 1u, smul<2>(fi), widen<4>(fi));  // weight 2: 2 f_i, lazy
    cols_mad2(re, im, a, nrm(coefz(f, j)), (XI[t] >> k) & 1u);
  }
  return pad_zero(fp2_cols_redc(re, im));
}
#endif

// Granger–Scott cyclotomic squaring (as fp12_cyclotomic_sqr): the Fp4 pairs are
// (w^0, w^3), (w^1, w^4), (w^2, w^5).  Even lanes need a^2 + xi b^2 of one pair, odd lanes
// 2ab of another (lane 1: xi 2ab); both are two Fp2 squarings per lane: (a, b) or (a + b, a - b).
//
// Each component is ONE three-product sum with one reduction (fp_muln_inl), the signs and the
// xi of lane 1 folded into the operands:
//   even lanes  a^2 + xi b^2 = ((a0+a1)(a0-a1) + (b0+b1)(b0-b1) + 2b0 (-b1))
//                            + (2a0 a1 + (b0+b1)(b0-b1) + 2b0 b1) u
//   odd lanes   2aB = (2a0 B0 + 2a1 (-B1)) + (2a0 B1 + 2a1 B0) u,  B = b, or xi b = (b0 - b1, b0 + b1)
//                     on lane 1 (so xi 2ab needs no multiplication by xi afterwards)
// and the output 3c -+ 2f is ONE digit pass 3c + 2g with g = f (odd lanes) or 4p - f (even).
// The operand selection happens before the arithmetic (one lazy op per operand instead of
// every lane computing both parities' operands), and the second operands of the products -- only
// they may carry digits up to 2^30 (fp_muln_inl) -- skip the one-shot carry (r04: cyclotomic
// squaring ~35% of the 6-lane verdict's instructions).
MBLS_X12_FN fp2 x12_cyc_sqr(const fp2& f) {
  const int k = gk();
  constexpr uint32_t SA = 0x66120120u;  // nibble k: lane of a
  constexpr uint32_t SB = 0x66453453u;  // nibble k: lane of b
#if MBLS_LG_GROUP == 6
  xs::sync();  // the previous reader of the slots is done
  xs::put2(0, f);
  xs::sync();
  const fp2 av = xs::get2(0, gbase() + ((SA >> (4 * k)) & 15)), bv = xs::get2(0, gbase() + ((SB >> (4 * k)) & 15));
#else
  const fp2 av = coef(f, (SA >> (4 * k)) & 15), bv = coef(f, (SB >> (4 * k)) & 15);
#endif
  const bool odd = k & 1, x1 = k == 1;
  const fp &a0 = av.c0, &a1 = av.c1, &b0 = bv.c0, &b1 = bv.c1;  // normalized: < 2p, digits < 2^28
  constexpr pbig_t K4 = PKB<4>::v, K8 = PKB<8>::v;  // raised 4p / 8p: a + K - b never borrows
  // first operands (digits must be < 2^28 + 16: one-shot carry)
  fp A0r, A1, A2, A0i;
  // second operands (digits < 2^30, no carry): the raw digit-wise sums / differences
  fp Q0, Q1, Q2, S0, S1, S2;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    A0r.v[i] = a0.v[i] + (odd ? a0.v[i] : a1.v[i]);         // 2a0 | a0 + a1          < 4p
    A1.v[i] = (odd ? a1.v[i] : b0.v[i]) + (odd ? a1.v[i] : b1.v[i]);  // 2a1 | b0 + b1  < 4p
    A2.v[i] = odd ? 0u : b0.v[i] << 1;                      // 0 | 2b0                < 4p
    A0i.v[i] = a0.v[i] << 1;                                // 2a0                    < 4p
    const uint32_t db = b0.v[i] + K4.v[i] - b1.v[i];        // b0 - b1                < 6p, < 2^30
    const uint32_t sb = b0.v[i] + b1.v[i];                  // b0 + b1                < 4p, < 2^29
    const uint32_t B0 = x1 ? db : b0.v[i], B1 = x1 ? sb : b1.v[i];
    Q0.v[i] = odd ? B0 : a0.v[i] + K4.v[i] - a1.v[i];       // B0 | a0 - a1           < 6p
    Q1.v[i] = odd ? K8.v[i] - B1 : db;                      // -B1 | b0 - b1          < 8p
    Q2.v[i] = odd ? 0u : K4.v[i] - b1.v[i];                 // 0 | -b1                < 4p
    S0.v[i] = odd ? B1 : a1.v[i];                           // B1 | a1                < 4p
    S1.v[i] = odd ? B0 : db;                                // B0 | b0 - b1           < 6p
    S2.v[i] = odd ? 0u : b1.v[i];                           // 0 | b1                 < 2p
  }
  // bounds (x p^2): even re 4*6 + 4*6 + 4*4, odd re 4*6 + 4*8; even im 4*2 + 4*6 + 4*2, odd im
  // 4*4 + 4*6 -- all < 2400, so each sum reduces to < 2p
  const fp P[3] = {fp_cn(A0r), fp_cn(A1), fp_cn(A2)};
  const fp Q[3] = {Q0, Q1, Q2};
  const fp R[3] = {fp_cn(A0i), P[1], P[2]};
  const fp S[3] = {S0, S1, S2};
  const fp c[2] = {fp_muln_inl<3>(P, Q), fp_muln_inl<3>(R, S)};
  // 3c + 2g, g = f (odd) or 4p - f (even): digits < 3 * 2^28 + 2 * 2^30 < 2^32, value < 14p
  fp2 out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const fp& fh = h ? f.c1 : f.c0;
    fp t;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const uint32_t g = odd ? fh.v[i] : K4.v[i] - fh.v[i];
      t.v[i] = 3u * c[h].v[i] + 2u * g;
    }
    (h ? out.c1 : out.c0) = reduce(lz<14>{fp_cn(t)}).v;
  }
  return pad_zero(out);
}

// f * (l0 + l2 w^2 + l3 w^3): three Fp2 products per lane
MBLS_X12_FN fp2 x12_mul_line(const fp2& f, const fp2& l0, const fp2& l2, const fp2& l3) {
  const int k = gk() < 6 ? gk() : 0;
#if MBLS_LG_GROUP == 6
  xs::sync();
  xs::put2(0, f);
  xs::sync();
  const fp2 f2 = xs::get2(0, gbase() + (k >= 2 ? k - 2 : k + 4)), f3 = xs::get2(0, gbase() + (k >= 3 ? k - 3 : k + 3));
#else
  const fp2 f2 = coef(f, k >= 2 ? k - 2 : k + 4), f3 = coef(f, k >= 3 ? k - 3 : k + 3);
#endif
  fpcols re, im;
  cols_zero(re);
  cols_zero(im);
  cols_mad2(re, im, nrm(f), nrm(l0), false);
  cols_mad2(re, im, nrm(f2), nrm(l2), k < 2);
  cols_mad2(re, im, nrm(f3), nrm(l3), k < 3);
  return pad_zero(fp2_cols_redc(re, im));
}

// Frobenius maps: coefficient of w^k -> conj^e(c) * gamma_e[k]
#define MBLS_GL(e, kk) fp2_from(k::FROB##e##_##kk##_C0, k::FROB##e##_##kk##_C1)
__device__ __noinline__ fp2 x12_frob(const fp2& f) {
  const fp2 g = pick6(gk(), fp2_one(), MBLS_GL(1, 1), MBLS_GL(1, 2), MBLS_GL(1, 3), MBLS_GL(1, 4), MBLS_GL(1, 5));
  return pad_zero(fp2_mul(fp2_conj(f), g));
}
__device__ __noinline__ fp2 x12_frob2(const fp2& f) {
  const fp2 g = pick6(gk(), fp2_one(), MBLS_GL(2, 1), MBLS_GL(2, 2), MBLS_GL(2, 3), MBLS_GL(2, 4), MBLS_GL(2, 5));
  return pad_zero(fp2_mul(f, g));
}
#undef MBLS_GL

// whole Fp12 in every lane of the group, and back
__device__ __forceinline__ fp12 x12_gather(const fp2& c) {
  return {{coef(c, 0), coef(c, 2), coef(c, 4)}, {coef(c, 1), coef(c, 3), coef(c, 5)}};
}
__device__ __forceinline__ fp2 x12_own(const fp12& f) {
  return pad_zero(pick6(gk(), f.c0.c0, f.c1.c0, f.c0.c1, f.c1.c1, f.c0.c2, f.c1.c2));
}

// inverse through the tower, lane parallel except for the one Fp inversion:
//   f = c0 + c1 w (c0 = lanes 0,2,4, c1 = lanes 1,3,5 as Fp6 = Fp2[v]),
//   t = c0^2 - v c1^2, t^-1 = adj(t) / N(t), f^-1 = (c0 t^-1) - (c1 t^-1) w.
// Each Fp6 square / adjugate coefficient has the shape xi^e1 x^2 + s xi^e2 y z, one lane each.
__device__ __forceinline__ fp2 xi_if(bool c, const fp2& a) { return fp2_select(c, fp2_mul_xi(a), a); }
__device__ __noinline__ fp2 x12_inv(const fp2& f) {
  const int k = gk();
  // t = c0^2 - v c1^2: lanes 0..2 A_j = (c0^2)_j, lanes 3..5 the matching (v c1^2) coefficient
  constexpr uint32_t SX = 0x66513240u, SY = 0x66131002u, SZ = 0x66355424u;  // nibble k: source lane
  const fp2 x = coef(f, (SX >> (4 * k)) & 15), y = coef(f, (SY >> (4 * k)) & 15), z = coef(f, (SZ >> (4 * k)) & 15);
  const fp2 xx = fp2_mul(x, x), yz2 = fp2_dbl(fp2_mul(y, z));
  fp2 a = fp2_add(xi_if(k == 1 || k == 5, xx), xi_if(k == 0 || k == 4, yz2));
  a = xi_if(k == 3, a);
  const fp2 t = fp2_sub(a, coef(a, k < 3 ? k + 3 : 6));  // lanes 0..2: t_j
  // adjugate C_j = xi^e1 x^2 - xi^e2 y z over t (lanes 0..2), and N(t) = t0 C0 + xi (t2 C1 + t1 C2)
  constexpr uint32_t TX = 0x66666120u, TY = 0x66666001u, TZ = 0x66666212u;
  const fp2 tx = coef(t, (TX >> (4 * k)) & 15), ty = coef(t, (TY >> (4 * k)) & 15), tz = coef(t, (TZ >> (4 * k)) & 15);
  const fp2 cj = fp2_sub(xi_if(k == 1, fp2_mul(tx, tx)), xi_if(k == 0, fp2_mul(ty, tz)));
  const fp2 pj = fp2_mul(coef(t, k == 1 ? 2 : k == 2 ? 1 : (k == 0 ? 0 : 6)), cj);  // t0 C0 | t2 C1 | t1 C2
  const fp2 nt = fp2_add(coef(pj, 0), fp2_mul_xi(fp2_add(coef(pj, 1), coef(pj, 2))));
  // N^-1 in Fp2 (every lane, one Fp inversion)
  const fp ni = fp_inv(fp2_norm(nt));
  const fp2 nti = {fp_mul(nt.c0, ni), fp_neg(fp_mul(nt.c1, ni))};
  const fp2 u = fp2_mul(cj, nti);  // lanes 0..2: (t^-1)_j
  const fp2 u0 = coef(u, 0), u1 = coef(u, 1), u2 = coef(u, 2);
  // lane k = 2j + h: coefficient j of c_h t^-1 (negated for h = 1)
  const int h = k & 1, j = k >> 1;
  const fp2 x0 = coef(f, h), x1 = coef(f, 2 + h), x2 = coef(f, 4 + h);
  // (xy)_0 = x0 u0 + xi (x1 u2 + x2 u1); (xy)_1 = x0 u1 + x1 u0 + xi x2 u2; (xy)_2 = x0 u2 + x1 u1 + x2 u0
  const fp2 p0 = fp2_mul(x0, j == 0 ? u0 : j == 1 ? u1 : u2);
  const fp2 p1 = fp2_mul(x1, j == 0 ? u2 : j == 1 ? u0 : u1);
  const fp2 p2 = fp2_mul(x2, j == 0 ? u1 : j == 1 ? u2 : u0);
  const fp2 r = fp2_add(p0, fp2_add(xi_if(j == 0, p1), xi_if(j <= 1, p2)));
  return pad_zero(fp2_select(h, fp2_neg(r), r));
}

// group verdict: f == 1
__device__ __forceinline__ bool x12_is_one(const fp2& f) {
  const int k = gk();
  const fp2 want = k == 0 ? fp2_one() : fp2_zero();
  const bool ok = fp2_eq(f, want);
  const uint64_t m = __ballot(ok);
  constexpr uint64_t all = (1ull << MBLS_LG_GROUP) - 1;
  return ((m >> gbase()) & all) == all;
}

__device__ __noinline__ fp2 x12_pow_xabs(const fp2& g) {
  fp2 r = g;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = x12_cyc_sqr(r);
    if ((k::X_ABS >> b) & 1ull) r = x12_mul(r, g);
  }
  return r;
}
__device__ __forceinline__ fp2 x12_pow_x(const fp2& g) { return x12_conj(x12_pow_xabs(g)); }

// final exponentiation, same schedule as mbls_pairing.hpp final_exp (cube of the reduced pairing)
__device__ __noinline__ fp2 x12_final_exp(const fp2& f) {
  fp2 t = x12_mul(x12_conj(f), x12_inv(f));
  t = x12_mul(x12_frob2(t), t);
  fp2 a = x12_mul(x12_pow_x(t), x12_conj(t));
  a = x12_mul(x12_pow_x(a), x12_conj(a));
  const fp2 b = x12_mul(x12_pow_x(a), x12_frob(a));
  fp2 c = x12_pow_x(x12_pow_x(b));
  c = x12_mul(x12_mul(c, x12_frob2(b)), x12_conj(b));
  const fp2 t3 = x12_mul(x12_cyc_sqr(t), t);
  return x12_mul(c, t3);
}

// ----- Miller loop: T (projective, M-type twist) is held redundantly by every lane; the
// products of one step are spread over the lanes in rounds and gathered back. -----------
struct line_lg {
  fp2 l0, l2, l3;  // f *= l0 + l2 w^2 + l3 w^3 (already evaluated at P)
};

// G1 point of the pairing in projective form (X : Y : Z): a line evaluated there is Z times
// its value at the affine point, and Fp factors vanish in the final exponentiation.
struct pt_lg {
  fp2 x, y, z;  // (X, 0), (Y, 0), (Z, 0): Fp2 operands of the lane-uniform products
};
__device__ __forceinline__ pt_lg pt_lg_from(const proj<fp>& p) {
  return {{p.x, fp_zero()}, {p.y, fp_zero()}, {p.z, fp_zero()}};
}

// The running point T of the lane-group Miller loops and G2 ladders, lazily reduced: each
// coordinate < 8p (mbls_lazy.hpp).  The steps below form every sum / difference lazily and
// reduce only the 3b' multiples (whose x12 growth would otherwise exceed the product bounds).
struct tlz {
  lz2<8> x, y, z;
};
__device__ __forceinline__ tlz tlz_from(const proj<fp2>& p) { return {{p.x}, {p.y}, {p.z}}; }
__device__ __forceinline__ tlz tlz_from(const aff<fp2>& q) { return {{q.x}, {q.y}, {fp2_one()}}; }
__device__ __forceinline__ proj<fp2> tlz_reduce(const tlz& t) {
  return {reduce(t.x).v, reduce(t.y).v, reduce(t.z).v};
}

template <int A>
__device__ __forceinline__ lz2<A> lcoef(const lz2<A>& c, int k) {
  return {coef(c.v, k)};
}
// pick6 / pick7 over lazy values: the result's bound is the largest candidate's
template <int A0, int A1, int A2, int A3, int A4, int A5>
__device__ __forceinline__ auto lpick6(int k, const lz2<A0>& a0, const lz2<A1>& a1, const lz2<A2>& a2,
                                       const lz2<A3>& a3, const lz2<A4>& a4, const lz2<A5>& a5) {
  constexpr int m01 = A0 > A1 ? A0 : A1, m23 = A2 > A3 ? A2 : A3, m45 = A4 > A5 ? A4 : A5;
  constexpr int m = m01 > m23 ? (m01 > m45 ? m01 : m45) : (m23 > m45 ? m23 : m45);
  return lz2<m>{pick6(k, a0.v, a1.v, a2.v, a3.v, a4.v, a5.v)};
}
template <int A0, int A1, int A2, int A3, int A4, int A5, int A6>
__device__ __forceinline__ auto lpick7(int k, const lz2<A0>& a0, const lz2<A1>& a1, const lz2<A2>& a2,
                                       const lz2<A3>& a3, const lz2<A4>& a4, const lz2<A5>& a5, const lz2<A6>& a6) {
  const auto r6 = lpick6(k, a0, a1, a2, a3, a4, a5);
  constexpr int m = decltype(r6)::bound > A6 ? decltype(r6)::bound : A6;
  return lz2<m>{fp2_select(k >= 6, a6.v, r6.v)};
}

// tangent line at T (c0 = Y^2 - 3b' Z^2, c2 = -3X^2, c3 = 2YZ, as miller_dbl) evaluated at
// P = (X_P : Y_P : Z_P) as c0 Z_P + c2 X_P w^2 + c3 Y_P w^3, and T <- 2T by RCB Algorithm 9
// (as pt_dbl_t)
MBLS_STEP_FN line_lg dbl_step_lg(tlz& t, const pt_lg& p) {
  const int k = gk();
  // round 1: lane 0 Y^2, 1 Z^2, 2 YZ, 3 X^2, 4 XY
  const nz2 r1 = mul(lpick6(k, t.y, t.z, t.y, t.x, t.x, t.x), lpick6(k, t.y, t.z, t.z, t.x, t.y, t.y));
  const nz2 yy = lcoef(r1, 0), zz = lcoef(r1, 1), yz = lcoef(r1, 2), xx = lcoef(r1, 3), xy = lcoef(r1, 4);
  const lz2<8> c2 = neg(smul<3>(xx));
  const lz2<4> c3 = smul<2>(yz);
  const nz2 t2 = reduce(mul_b3(zz));      // 3b' Z^2
  const lz2<16> z8 = smul<8>(yy);          // 8 Y^2
  const lz2<10> t0m = yy - smul<3>(t2);    // Y^2 - 9b' Z^2
  const lz2<4> y3s = yy + t2;
  const lz2<6> c0 = yy - t2;
  // round 2: lane 0 t2 z8, 1 YZ z8, 2 t0m (Y^2 + t2), 3 t0m XY, 4 c2 X_P, 5 c3 Y_P, 6 c0 Z_P
  // (6-lane groups: P is affine, and c0 Z_P = c0 needs no product)
  line_lg l;
#if MBLS_LG_GROUP == 8
  const nz2 r2 = mul(lpick7(k, t2, yz, t0m, t0m, c2, c3, c0),
                     lpick7(k, z8, z8, y3s, xy, nrm(p.x), nrm(p.y), nrm(p.z)));
  l.l0 = coef(r2.v, 6);
#else
  const nz2 r2 = mul(lpick6(k, t2, yz, t0m, t0m, c2, c3), lpick6(k, z8, z8, y3s, xy, nrm(p.x), nrm(p.y)));
  l.l0 = reduce(c0).v;
#endif
  l.l2 = coef(r2.v, 4);
  l.l3 = coef(r2.v, 5);
  t.x = widen<8>(smul<2>(lcoef(r2, 3)));
  t.y = widen<8>(lcoef(r2, 0) + lcoef(r2, 2));
  t.z = widen<8>(lcoef(r2, 1));
  return l;
}

// chord through T and affine Q (as miller_add: theta = Y - y_Q Z, kappa = X - x_Q Z,
// c0 = theta x_Q - kappa y_Q, c2 = -theta, c3 = kappa) evaluated at P = (X_P : Y_P : Z_P)
// (qz = (x_Q Z_P, y_Q Z_P) gives c0 Z_P), and T <- T + Q by RCB Algorithm 8 (as
// pt_add_affine_t)
MBLS_STEP_FN line_lg add_step_lg(tlz& t, const aff<fp2>& q, const aff<fp2>& qz, const pt_lg& p) {
  const int k = gk();
  const nz2 qx = nrm(q.x), qy = nrm(q.y);
  // round 1: lane 0 X xQ, 1 Y yQ, 2 (xQ + yQ)(X + Y), 3 yQ Z, 4 xQ Z
  const lz2<4> sq = qx + qy;
  const lz2<16> st = t.x + t.y;
  const nz2 r1 = mul(lpick6(k, t.x, t.y, sq, qy, qx, qx), lpick6(k, qx, qy, st, t.z, t.z, t.z));
  const nz2 t0 = lcoef(r1, 0), t1 = lcoef(r1, 1), yqz = lcoef(r1, 3), xqz = lcoef(r1, 4);
  const lz2<12> theta = t.y - yqz, kappa = t.x - xqz;
  const lz2<10> t3 = lcoef(r1, 2) - (t0 + t1);
  const lz2<10> t4 = yqz + t.y;
  const nz2 y3b = reduce(mul_b3(xqz + t.x));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2 = reduce(mul_b3(t.z));
  const lz2<4> z3a = t1 + t2;
  const lz2<6> t1m = t1 - t2;
  // round 2: lane 0 t4 y3b, 1 t3 t1m, 2 y3b t03, 3 t1m z3a, 4 t03 t3, 5 z3a t4
  const nz2 r2 = mul(lpick6(k, t4, t3, y3b, t1m, t03, z3a), lpick6(k, y3b, t1m, t03, z3a, t3, t4));
  // round 3: lane 0 theta xQ Z_P, 1 kappa yQ Z_P, 2 theta X_P, 3 kappa Y_P
  const nz2 r3 = mul(lpick6(k, theta, kappa, theta, kappa, theta, theta),
                     lpick6(k, nrm(qz.x), nrm(qz.y), nrm(p.x), nrm(p.y), nrm(p.x), nrm(p.x)));
  t.x = widen<8>(lcoef(r2, 1) - lcoef(r2, 0));
  t.y = widen<8>(lcoef(r2, 3) + lcoef(r2, 2));
  t.z = widen<8>(lcoef(r2, 5) + lcoef(r2, 4));
  line_lg l;
  l.l0 = fp2_sub(coef(r3.v, 0), coef(r3.v, 1));
  l.l2 = fp2_neg(coef(r3.v, 2));
  l.l3 = coef(r3.v, 3);
  return l;
}

// f_{|x|,Q}(P) conjugated (x < 0), as miller_loop_1 up to Fp factors (P projective)
__device__ __noinline__ fp2 miller_lg(const proj<fp>& pp, const aff<fp2>& q) {
  const pt_lg p = pt_lg_from(pp);
  const aff<fp2> qz = {fp2_mul_fp(q.x, pp.z), fp2_mul_fp(q.y, pp.z)};
  tlz t = tlz_from(q);
  fp2 f = x12_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = x12_sqr(f);
    line_lg l = dbl_step_lg(t, p);
    f = x12_mul_line(f, l.l0, l.l2, l.l3);
    if ((k::X_ABS >> b) & 1ull) {
      l = add_step_lg(t, q, qz, p);
      f = x12_mul_line(f, l.l0, l.l2, l.l3);
    }
  }
  return x12_conj(f);
}

// product of two Miller loops sharing the squarings (as miller_loop_2): f_{|x|,Q1}(P1) *
// f_{|x|,Q2}(P2), conjugated; the second pair only when use2 (group uniform)
__device__ __noinline__ fp2 miller2_lg(const proj<fp>& pp1, const aff<fp2>& q1, const proj<fp>& pp2,
                                       const aff<fp2>& q2, bool use2) {
  const pt_lg p1 = pt_lg_from(pp1), p2 = pt_lg_from(pp2);
  const aff<fp2> qz1 = {fp2_mul_fp(q1.x, pp1.z), fp2_mul_fp(q1.y, pp1.z)};
  const aff<fp2> qz2 = {fp2_mul_fp(q2.x, pp2.z), fp2_mul_fp(q2.y, pp2.z)};
  tlz t1 = tlz_from(q1), t2 = tlz_from(q2);
  fp2 f = x12_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = x12_sqr(f);
    line_lg l = dbl_step_lg(t1, p1);
    f = x12_mul_line(f, l.l0, l.l2, l.l3);
    if (use2) {
      l = dbl_step_lg(t2, p2);
      f = x12_mul_line(f, l.l0, l.l2, l.l3);
    }
    if ((k::X_ABS >> b) & 1ull) {
      l = add_step_lg(t1, q1, qz1, p1);
      f = x12_mul_line(f, l.l0, l.l2, l.l3);
      if (use2) {
        l = add_step_lg(t2, q2, qz2, p2);
        f = x12_mul_line(f, l.l0, l.l2, l.l3);
      }
    }
  }
  return x12_conj(f);
}

#if MBLS_LG_GROUP == 6
// ----- Both pairs' Miller steps at once on 6-lane groups ("trios"): lanes 0..2 of a group hold
// the first pair's T, Q and P, lanes 3..5 the second pair's, and each trio runs its own pair's
// step, the products in rounds of three.  A doubling's 5 + 6 products take 2 + 2 rounds of three
// where the two one-pair steps take 1 + 1 rounds of six each: the same four products per lane
// and the same latency.  But the sums, multiples and reductions between the rounds, which every
// lane forms redundantly, are now formed for one pair per lane instead of both, the candidate
// picks are over three values instead of six, and each lane carries one T instead of two.  The
// two lines are then broadcast to the whole group for the Fp12 line products.  P is affine
// (Z_P = 1), as for every 6-lane step.
__device__ __forceinline__ int tk() {  // index within the trio
  const int k = gk();
  return k < 3 ? k : k - 3;
}
__device__ __forceinline__ int tbase() { return gbase() + (gk() < 3 ? 0 : 3); }  // first lane of the trio
template <int A>
__device__ __forceinline__ lz2<A> tcoef(const lz2<A>& c, int i) {
  return {pull(c.v, tbase() + i)};
}
template <int A0, int A1, int A2>
__device__ __forceinline__ auto lpick3(int k, const lz2<A0>& a0, const lz2<A1>& a1, const lz2<A2>& a2) {
  constexpr int m01 = A0 > A1 ? A0 : A1;
  constexpr int m = m01 > A2 ? m01 : A2;
  return lz2<m>{fp2_select(k == 0, a0.v, fp2_select(k == 1, a1.v, a2.v))};
}
__device__ __forceinline__ line_lg pull(const line_lg& l, int src) {
  return {pull(l.l0, src), pull(l.l2, src), pull(l.l3, src)};
}
// the rounds' products and the lines exchanged through LDS (xs slots 2..7) instead of
// ds_bpermute: a product is written once and the trio's (or group's) lanes read what they need
__device__ __forceinline__ void tput(const nz2& a, const nz2& b) {
  xs::sync();
  xs::put2(2, a.v);
  xs::put2(4, b.v);
  xs::sync();
}
__device__ __forceinline__ nz2 tgeta(int i) { return {xs::get2(2, tbase() + i)}; }
__device__ __forceinline__ nz2 tgetb(int i) { return {xs::get2(4, tbase() + i)}; }
__device__ __forceinline__ void lput(const line_lg& l) {
  xs::sync();
  xs::put2(2, l.l0);
  xs::put2(4, l.l2);
  xs::put2(6, l.l3);
  xs::sync();
}
// slots 2..7 stay valid across x12_mul_line (it uses slots 0, 1 only)
__device__ __forceinline__ line_lg lget(int src) { return {xs::get2(2, src), xs::get2(4, src), xs::get2(6, src)}; }

// dbl_step_lg on a trio (same formulas and bounds)
MBLS_STEP_FN line_lg dbl_step_trio(tlz& t, const pt_lg& p) {
  const int k = tk();
  // round 1a: lane 0 Y^2, 1 Z^2, 2 YZ;  1b: lane 0 X^2, 1 XY (lane 2 repeats XY)
  const nz2 r1a = mul(lpick3(k, t.y, t.z, t.y), lpick3(k, t.y, t.z, t.z));
  const nz2 r1b = mul(t.x, lpick3(k, t.x, t.y, t.y));
  tput(r1a, r1b);
  const nz2 yy = tgeta(0), zz = tgeta(1), yz = tgeta(2), xx = tgetb(0), xy = tgetb(1);
  const lz2<8> c2 = neg(smul<3>(xx));
  const lz2<4> c3 = smul<2>(yz);
  const nz2 t2 = reduce(mul_b3(zz));      // 3b' Z^2
  const lz2<16> z8 = smul<8>(yy);          // 8 Y^2
  const lz2<10> t0m = yy - smul<3>(t2);    // Y^2 - 9b' Z^2
  const lz2<4> y3s = yy + t2;
  const lz2<6> c0 = yy - t2;
  // round 2a: lane 0 t2 z8, 1 YZ z8, 2 t0m (Y^2 + t2);  2b: lane 0 t0m XY, 1 c2 X_P, 2 c3 Y_P
  const nz2 r2a = mul(lpick3(k, t2, yz, t0m), lpick3(k, z8, z8, y3s));
  const nz2 r2b = mul(lpick3(k, t0m, c2, c3), lpick3(k, xy, nrm(p.x), nrm(p.y)));
  line_lg l;
  l.l0 = reduce(c0).v;
  tput(r2a, r2b);
  l.l2 = tgetb(1).v;
  l.l3 = tgetb(2).v;
  t.x = widen<8>(smul<2>(tgetb(0)));
  t.y = widen<8>(tgeta(0) + tgeta(2));
  t.z = widen<8>(tgeta(1));
  return l;
}

// add_step_lg on a trio (same formulas and bounds; P affine, so qz = Q)
MBLS_STEP_FN line_lg add_step_trio(tlz& t, const aff<fp2>& q, const pt_lg& p) {
  const int k = tk();
  const nz2 qx = nrm(q.x), qy = nrm(q.y);
  // round 1a: lane 0 X xQ, 1 Y yQ, 2 (xQ + yQ)(X + Y);  1b: lane 0 yQ Z, 1 xQ Z
  const lz2<4> sq = qx + qy;
  const lz2<16> st = t.x + t.y;
  const nz2 r1a = mul(lpick3(k, t.x, t.y, sq), lpick3(k, qx, qy, st));
  const nz2 r1b = mul(lpick3(k, qy, qx, qx), t.z);
  tput(r1a, r1b);
  const nz2 t0 = tgeta(0), t1 = tgeta(1), yqz = tgetb(0), xqz = tgetb(1);
  const lz2<12> theta = t.y - yqz, kappa = t.x - xqz;
  const lz2<10> t3 = tgeta(2) - (t0 + t1);
  const lz2<10> t4 = yqz + t.y;
  const nz2 y3b = reduce(mul_b3(xqz + t.x));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2 = reduce(mul_b3(t.z));
  const lz2<4> z3a = t1 + t2;
  const lz2<6> t1m = t1 - t2;
  // round 2a: lane 0 t4 y3b, 1 t3 t1m, 2 y3b t03;  2b: lane 0 t1m z3a, 1 t03 t3, 2 z3a t4
  const nz2 r2a = mul(lpick3(k, t4, t3, y3b), lpick3(k, y3b, t1m, t03));
  const nz2 r2b = mul(lpick3(k, t1m, t03, z3a), lpick3(k, z3a, t3, t4));
  // round 3a: lane 0 theta xQ, 1 kappa yQ, 2 theta X_P;  3b: kappa Y_P (every lane)
  const nz2 r3a = mul(lpick3(k, theta, kappa, theta), lpick3(k, qx, qy, nrm(p.x)));
  const nz2 r3b = mul(kappa, nrm(p.y));
  line_lg l;
  tput(r2a, r2b);
  t.x = widen<8>(tgeta(1) - tgeta(0));
  t.y = widen<8>(tgetb(0) + tgeta(2));
  t.z = widen<8>(tgetb(2) + tgetb(1));
  tput(r3a, r3b);
  l.l0 = fp2_sub(tgeta(0).v, tgeta(1).v);
  l.l2 = fp2_neg(tgeta(2).v);
  l.l3 = r3b.v;
  return l;
}

// miller2_lg with the steps on trios: this lane's pair is (p, q) -- lanes 0..2 the first pair's,
// lanes 3..5 the second's, P affine -- the second pair's lines only when use2.  (r05: inlining
// it into the 6-lane verdict with the pairs selected there grew the kernel's frame 2,244 ->
// 2,608 bytes with 336 spilled registers instead of 14, so the verdict keeps the outlined call.)
__device__ __forceinline__ fp2 miller2_trio_sel(const aff<fp>& pa, const aff<fp2>& q, bool use2) {
  const pt_lg p = {{pa.x, fp_zero()}, {pa.y, fp_zero()}, {fp_one(), fp_zero()}};
  tlz t = tlz_from(q);
  const int g0 = gbase(), g1 = gbase() + 3;
  fp2 f = x12_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = x12_sqr(f);
    line_lg l = dbl_step_trio(t, p);
    lput(l);
    line_lg m = lget(g0);
    f = x12_mul_line(f, m.l0, m.l2, m.l3);
    if (use2) {
      m = lget(g1);
      f = x12_mul_line(f, m.l0, m.l2, m.l3);
    }
    if ((k::X_ABS >> b) & 1ull) {
      l = add_step_trio(t, q, p);
      lput(l);
      m = lget(g0);
      f = x12_mul_line(f, m.l0, m.l2, m.l3);
      if (use2) {
        m = lget(g1);
        f = x12_mul_line(f, m.l0, m.l2, m.l3);
      }
    }
  }
  return x12_conj(f);
}
// (its call from the 6-lane verdict: miller2_trio_lane in mbls_k_lg6.hip)
#endif

// ----- G2 group law on lane groups (hash_to_G2's cofactor clearing, the psi test's [x] Q):
// every lane holds the point (lazy, tlz), the products of a step are spread over the lanes in
// rounds, as in the Miller steps.
__device__ __forceinline__ proj<fp2> pull(const proj<fp2>& p, int src) {
  return {pull(p.x, src), pull(p.y, src), pull(p.z, src)};
}

// RCB Algorithm 9 (as pt_dbl_t): two rounds of 4 products
#if MBLS_LG_GROUP == 8
// 8-lane groups (r04): the doubling's rounds have four products, so lane k computes component
// (k & 1) of product k >> 1 -- two Fp products and one reduction (fp_mul2) instead of a whole
// Fp2 product per lane, the round's results gathered back component-wise.  Same formulas and
// bounds as below; the second operand's component pair is selected per lane before the product.
template <int A, int C>
__device__ __forceinline__ nz mulc(const lz2<A>& a, const lz2<C>& b, int h) {
  static_assert(C < 32 && A * (C + 32) <= 2400, "Fp2 product bound");
  fp nb1;
#pragma unroll
  for (int i = 0; i < NL; ++i) nb1.v[i] = PKB<32>::v.v[i] - b.v.c1.v[i];  // digits < 2^30
  // h = 0: a0 b0 + a1 (32p - b1);  h = 1: a0 b1 + a1 b0
  return {fp_mul2(a.v.c0, fp_select(h, b.v.c1, b.v.c0), a.v.c1, fp_select(h, b.v.c0, nb1))};
}
__device__ __forceinline__ nz2 cpull(const nz& v, int prod) {
  return {{pull(v.v, gbase() + 2 * prod), pull(v.v, gbase() + 2 * prod + 1)}};
}
template <int A0, int A1, int A2, int A3>
__device__ __forceinline__ auto lpick4(int p, const lz2<A0>& a0, const lz2<A1>& a1, const lz2<A2>& a2,
                                       const lz2<A3>& a3) {
  constexpr int m01 = A0 > A1 ? A0 : A1, m23 = A2 > A3 ? A2 : A3;
  constexpr int m = m01 > m23 ? m01 : m23;
  return lz2<m>{fp2_select(p == 0, a0.v, fp2_select(p == 1, a1.v, fp2_select(p == 2, a2.v, a3.v)))};
}
MBLS_G2STEP_FN tlz g2_dbl_lg(const tlz& t) {
  const int k = gk(), p = k >> 1, h = k & 1;
  // round 1: products Y^2, Z^2, YZ, XY
  const nz r1 = mulc(lpick4(p, t.y, t.z, t.y, t.x), lpick4(p, t.y, t.z, t.z, t.y), h);
  const nz2 yy = cpull(r1, 0), zz = cpull(r1, 1), yz = cpull(r1, 2), xy = cpull(r1, 3);
  const nz2 t2 = reduce(mul_b3(zz));
  const lz2<16> z8 = smul<8>(yy);
  const lz2<10> t0m = yy - smul<3>(t2);
  const lz2<4> y3s = yy + t2;
  // round 2: t2 z8, YZ z8, t0m (Y^2 + t2), t0m XY
  const nz r2 = mulc(lpick4(p, t2, yz, t0m, t0m), lpick4(p, z8, z8, y3s, xy), h);
  return {widen<8>(smul<2>(cpull(r2, 3))), widen<8>(cpull(r2, 0) + cpull(r2, 2)), widen<8>(cpull(r2, 1))};
}
#else
MBLS_G2STEP_FN tlz g2_dbl_lg(const tlz& t) {
  const int k = gk();
  const nz2 r1 = mul(lpick6(k, t.y, t.z, t.y, t.x, t.x, t.x), lpick6(k, t.y, t.z, t.z, t.y, t.y, t.y));
  const nz2 yy = lcoef(r1, 0), zz = lcoef(r1, 1), yz = lcoef(r1, 2), xy = lcoef(r1, 3);
  const nz2 t2 = reduce(mul_b3(zz));
  const lz2<16> z8 = smul<8>(yy);
  const lz2<10> t0m = yy - smul<3>(t2);
  const lz2<4> y3s = yy + t2;
  const nz2 r2 = mul(lpick6(k, t2, yz, t0m, t0m, t2, t2), lpick6(k, z8, z8, y3s, xy, z8, z8));
  return {widen<8>(smul<2>(lcoef(r2, 3))), widen<8>(lcoef(r2, 0) + lcoef(r2, 2)), widen<8>(lcoef(r2, 1))};
}
#endif

// RCB Algorithm 7 (as pt_add_t): two rounds of 6 products
MBLS_G2STEP_FN tlz g2_add_lg(const tlz& p, const tlz& q) {
  const int k = gk();
  const nz2 r1 = mul(lpick6(k, widen<16>(p.x), widen<16>(p.y), widen<16>(p.z), p.x + p.y, p.y + p.z, p.x + p.z),
                     lpick6(k, widen<16>(q.x), widen<16>(q.y), widen<16>(q.z), q.x + q.y, q.y + q.z, q.x + q.z));
  const nz2 t0 = lcoef(r1, 0), t1 = lcoef(r1, 1), t2 = lcoef(r1, 2);
  const lz2<10> t3 = lcoef(r1, 3) - (t0 + t1);
  const lz2<10> t4 = lcoef(r1, 4) - (t1 + t2);
  const nz2 y3 = reduce(mul_b3(lcoef(r1, 5) - (t0 + t2)));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2b = reduce(mul_b3(t2));
  const lz2<4> z3 = t1 + t2b;
  const lz2<6> t1m = t1 - t2b;
  const nz2 r2 = mul(lpick6(k, t4, t3, y3, t1m, t03, z3), lpick6(k, y3, t1m, t03, z3, t3, t4));
  return {widen<8>(lcoef(r2, 1) - lcoef(r2, 0)), widen<8>(lcoef(r2, 3) + lcoef(r2, 2)),
          widen<8>(lcoef(r2, 5) + lcoef(r2, 4))};
}

// [x] q (x < 0), as pt_mul_x = -[|x|] q; q normalized, the result normalized
__device__ __noinline__ proj<fp2> g2_mul_x_lg(const proj<fp2>& q) {
  const tlz ql = tlz_from(q);
  tlz r = ql;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = g2_dbl_lg(r);
    if ((k::X_ABS >> b) & 1ull) r = g2_add_lg(r, ql);
  }
  return pt_neg(tlz_reduce(r));
}

// h_eff clearing via psi (as clear_cofactor_g2)
__device__ __noinline__ proj<fp2> clear_cofactor_g2_lg(const proj<fp2>& P) {
  const proj<fp2> t1 = g2_mul_x_lg(P);
  proj<fp2> t2 = g2_psi(P);
  proj<fp2> t3 = g2_psi(g2_psi(tlz_reduce(g2_dbl_lg(tlz_from(P)))));
  tlz u3 = g2_add_lg(tlz_from(t3), tlz_from(pt_neg(t2)));
  t2 = g2_mul_x_lg(tlz_reduce(g2_add_lg(tlz_from(t1), tlz_from(t2))));
  u3 = g2_add_lg(u3, tlz_from(t2));
  u3 = g2_add_lg(u3, tlz_from(pt_neg(t1)));
  return tlz_reduce(g2_add_lg(u3, tlz_from(pt_neg(P))));
}

// hash_to_G2 for one 32-byte message per group (as hash_to_g2_msg32): lanes 0..3 map u0,
// lanes 4..7 map u1 (6-lane groups: 0..2 and 3..5; the two SSWU maps run side by side), the
// sum's cofactor clearing runs in lane-parallel rounds.  Every lane returns H(m).
__device__ __noinline__ proj<fp2> hash_to_g2_lg(const uint32_t (&msg)[8]) {
  uint32_t ub[64];
  expand_message_xmd_msg32(ub, msg);
  const int k = gk();
  constexpr int half = MBLS_LG_GROUP / 2;  // lanes [0, half) map u0, [half, group) map u1
  const fp2 u = k < half ? fp2{fp_from_64_bytes(ub + 0), fp_from_64_bytes(ub + 16)}
                         : fp2{fp_from_64_bytes(ub + 32), fp_from_64_bytes(ub + 48)};
  const proj<fp2> q = iso3_map(map_to_curve_sswu(u));
  const proj<fp2> p = tlz_reduce(g2_add_lg(tlz_from(pull(q, gbase())), tlz_from(pull(q, gbase() + half))));
  return clear_cofactor_g2_lg(p);
}


// ----- 16-lane groups (r02): one Fp component per lane --------------------------------------
// Lane c = 2k + h of a 16-lane group holds component h (0: c0, 1: c1) of the coefficient of w^k
// (k < 6; lanes 12..15 hold zero).  The per-set pairing chain of a latency-bound batch is as
// long as its per-lane instruction count, and here an Fp12 product costs 12 Fp products + 1
// reduction per lane (8-lane form: 24 + 2), a cyclotomic squaring 3 + 1 (6 + 2), a sparse
// line product 6 + 1 (12 + 2), for the same number of ds_bpermute dwords.  The Miller steps
// (T and the line, lane-uniform results), the inversion and the Frobenius maps stay 8-lane
// code, which the two halves of a 16-lane group run in duplicate (gk() / gbase() address the
// half); values cross between the forms with ds_bpermute.  Same field elements as the 8-lane
// and one-lane routines (same formulas, same operand bounds per column accumulator).
__device__ __forceinline__ int hc() { return (int)(threadIdx.x & 15u); }     // component lane
__device__ __forceinline__ int hbase() { return (int)(threadIdx.x & 48u); }  // first lane of the group

__device__ __forceinline__ fp pad16(const fp& v) { return fp_select(hc() < 12, v, fp_zero()); }

// the 8-lane value (the same in both halves) -> this lane's component: lane (k, h) reads lane k
// of half h, which offers its c_h
__device__ __forceinline__ fp x16_from8(const fp2& f) {
  const int c = hc();
  const fp x = fp_select(threadIdx.x & 8u, f.c1, f.c0);
  return pull(x, hbase() + 8 * (c & 1) + (c >> 1));
}
// this lane's component -> the 8-lane value in both halves (pad lanes 6, 7 read zero lanes)
__device__ __forceinline__ fp2 x16_to8(const fp& v) {
  const int k = gk();
  return {pull(v, hbase() + 2 * k), pull(v, hbase() + 2 * k + 1)};
}
__device__ __forceinline__ fp x16_one() { return hc() == 0 ? fp_one() : fp_zero(); }
// p^6 Frobenius: odd powers of w change sign
__device__ __forceinline__ fp x16_conj(const fp& v) { return pad16(fp_select((hc() >> 1) & 1, fp_neg(v), v)); }

// one component of cols_mad2's lazy Fp2 product sum (h = 0: real, 1: imaginary part):
//   real  a0 x0 + a1 (-x1),  imaginary  a0 x1 + a1 x0,  (x0, x1) = b or b xi = (b0 - b1, b0 + b1)
// Per accumulator the same products and operand bounds as cols_mad2's re / im.
template <int A>
__device__ __forceinline__ void cols_mad1(fpcols& acc, const lz<A>& a0, const lz<A>& a1, const nz& b0, const nz& b1,
                                          bool xi, bool h) {
  static_assert(6 * 2 * 8 * A <= 2400, "lazy column sum bound");
  const lz<4> s = b0 + b1;
  const lz<6> d = b0 - b1;
  const fp x0 = fp_select(xi, d.v, b0.v), x1 = fp_select(xi, s.v, b1.v);
  cols_mad(acc, a0.v, fp_select(h, x1, x0));
  cols_mad(acc, a1.v, fp_select(h, x0, neg(lz<4>{x1}).v));
}
// both components of coefficient i
__device__ __forceinline__ nz x16_c(const fp& f, int i, int h) { return nrm(pull(f, hbase() + 2 * i + h)); }

// ----- Operand staging through LDS for the 16-lane products (as xs:: for 6-lane groups): lane
// (j, h) writes, once per product, its own component and -- with its partner's component pulled
// once -- its share of coefficient j's second-operand variants:
//   h = 0: b0, (xi b).c0 = b0 - b1, -b1          h = 1: b1, (xi b).c1 = b0 + b1, -(xi b).c1
// (bounds 2p, 6p, 4p | 2p, 4p, 8p), and a term of lane (k, h) reads its two products' operands
// by address: real  a0 x0 + a1 (-x1),  imaginary  a0 x1 + a1 x0  (x = b or xi b).  Slots: 0 the
// component, 1 twice it (squaring), 2..4 the variants; 5 x 56 B per lane, 17.5 KiB per wave.
namespace xs16 {
constexpr int kSlots = 5;
__device__ __forceinline__ uint4* lo() {
  __shared__ uint4 b[kSlots * 3 * 64];
  return b;
}
__device__ __forceinline__ uint2* hi() {
  __shared__ uint2 b[kSlots * 64];
  return b;
}
__device__ __forceinline__ void sync() { __syncthreads(); }
__device__ __forceinline__ void put(int slot, const fp& a) {
  const int l = (int)threadIdx.x;
  uint4* L = lo() + slot * 192 + l;
  L[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  L[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
  L[128] = make_uint4(a.v[8], a.v[9], a.v[10], a.v[11]);
  hi()[slot * 64 + l] = make_uint2(a.v[12], a.v[13]);
}
__device__ __forceinline__ fp get(int slot, int src) {
  const uint4* L = lo() + slot * 192 + src;
  const uint4 x = L[0], y = L[64], z = L[128];
  const uint2 w = hi()[slot * 64 + src];
  fp r;
  r.v[0] = x.x; r.v[1] = x.y; r.v[2] = x.z; r.v[3] = x.w;
  r.v[4] = y.x; r.v[5] = y.y; r.v[6] = y.z; r.v[7] = y.w;
  r.v[8] = z.x; r.v[9] = z.y; r.v[10] = z.z; r.v[11] = z.w;
  r.v[12] = w.x; r.v[13] = w.y;
  return r;
}
// slots 2..4 from this lane's component v of a normalized value (pad lanes hold 0)
__device__ __forceinline__ void put_b(const fp& v) {
  const bool h = hc() & 1;
  const nz mine{v}, other{pull(v, (int)(threadIdx.x ^ 1u))};
  const lz<6> d = (h ? other : mine) - (h ? mine : other);  // b0 - b1
  const lz<4> sm = mine + other;                            // b0 + b1
  put(2, v);
  put(3, h ? sm.v : d.v);
  put(4, h ? neg(sm).v : neg(other).v);
}
// acc += a0 first + a1 second for lane (k, h) and coefficient j (xi: the wrapped term)
__device__ __forceinline__ void term(fpcols& acc, int sa, int va, int j, bool xi) {
  const int h = hc() & 1, base = hbase(), v = xi ? 3 : 2;
  const fp a0 = get(va, base + sa), a1 = get(va, base + sa + 1);
  const fp first = get(v, base + 2 * j + h);
  const fp second = h ? get(v, base + 2 * j) : get(4, base + 2 * j + (xi ? 1 : 0));
  cols_mad(acc, a0, first);
  cols_mad(acc, a1, second);
}
}  // namespace xs16

// h = f g (as x12_mul): six terms, sum < 6 x 2 x 2p x 8p
MBLS_X12_FN fp x16_mul(const fp& f, const fp& g) {
  xs16::sync();
  xs16::put(0, f);
  xs16::put_b(g);
  xs16::sync();
  const int c = hc();
  const int k = (c >> 1) < 6 ? (c >> 1) : 0;
  fpcols acc;
  cols_zero(acc);
#pragma unroll 1
  for (int j = 0; j < 6; ++j) {
    const bool wrap = j > k;
    const int i = wrap ? k - j + 6 : k - j;
    xs16::term(acc, 2 * i, 0, j, wrap);
  }
  return pad16(cols_redc(acc));
}

// h = f^2 (as x12_sqr, same term tables): the weight 2 as the staged first-operand variant 2f
// (slot 1; sum < 4 x 2 x 4p x 8p); the (6, 6) terms are skipped
MBLS_X12_FN fp x16_sqr(const fp& f) {
  constexpr uint32_t TI[4] = {0x66000000u, 0x66111121u, 0x66224332u, 0x66656463u};
  constexpr uint32_t TJ[4] = {0x66543210u, 0x66432155u, 0x66325544u, 0x66656463u};
  constexpr uint32_t XI[4] = {0x00u, 0x03u, 0x0fu, 0x15u};
  constexpr uint32_t W2[4] = {0x3eu, 0x3bu, 0x2fu, 0x00u};
  xs16::sync();
  xs16::put(0, f);
  xs16::put(1, smul<2>(nrm(f)).v);
  xs16::put_b(f);
  xs16::sync();
  const int k = hc() >> 1;
  fpcols acc;
  cols_zero(acc);
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    const int i = (TI[t] >> (4 * k)) & 15, j = (TJ[t] >> (4 * k)) & 15;
    if (i < 6) xs16::term(acc, 2 * i, ((W2[t] >> k) & 1u) ? 1 : 0, j, (XI[t] >> k) & 1u);
  }
  return pad16(cols_redc(acc));
}

// Granger-Scott cyclotomic squaring (as x12_cyc_sqr): this lane's component h of coefficient k
// is ONE three-product sum with one reduction, its operands selected per lane before the
// arithmetic (x12_cyc_sqr's P . Q for h = 0, R . S for h = 1, lane 1's xi folded into the second
// operands, so no partner exchange after the product), and the output 3c -+ 2f in one pass
// (r04: the previous form built every candidate operand and fixed lane 1 with a pull afterwards)
MBLS_X12_FN fp x16_cyc_sqr(const fp& f) {
  const int c = hc(), k = c >> 1;
  const bool h = c & 1, odd = k & 1, x1 = k == 1;
  constexpr uint32_t SA = 0x66120120u;
  constexpr uint32_t SB = 0x66453453u;
  const int ia = (SA >> (4 * k)) & 15, ib = (SB >> (4 * k)) & 15;
  const fp a0 = x16_c(f, ia, 0).v, a1 = x16_c(f, ia, 1).v, b0 = x16_c(f, ib, 0).v, b1 = x16_c(f, ib, 1).v;
  constexpr pbig_t K4 = PKB<4>::v, K8 = PKB<8>::v;
  fp X0, X1, X2, Y0, Y1, Y2;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    X0.v[i] = a0.v[i] + ((h || odd) ? a0.v[i] : a1.v[i]);               // 2a0 | a0 + a1          < 4p
    X1.v[i] = (odd ? a1.v[i] : b0.v[i]) + (odd ? a1.v[i] : b1.v[i]);    // 2a1 | b0 + b1          < 4p
    X2.v[i] = odd ? 0u : b0.v[i] << 1;                                  // 0 | 2b0                < 4p
    const uint32_t db = b0.v[i] + K4.v[i] - b1.v[i];                    // b0 - b1                < 6p
    const uint32_t sb = b0.v[i] + b1.v[i];                              // b0 + b1                < 4p
    const uint32_t B0 = x1 ? db : b0.v[i], B1 = x1 ? sb : b1.v[i];
    Y0.v[i] = h ? (odd ? B1 : a1.v[i]) : (odd ? B0 : a0.v[i] + K4.v[i] - a1.v[i]);
    Y1.v[i] = h ? (odd ? B0 : db) : (odd ? K8.v[i] - B1 : db);
    Y2.v[i] = odd ? 0u : (h ? b1.v[i] : K4.v[i] - b1.v[i]);
  }
  const fp X[3] = {fp_cn(X0), fp_cn(X1), fp_cn(X2)};
  const fp Y[3] = {Y0, Y1, Y2};
  const fp cv = fp_muln_inl<3>(X, Y);
  // 3c + 2g, g = f (odd) or 4p - f (even): digits < 3 * 2^28 + 2 * 2^30 < 2^32, value < 14p
  fp t;
#pragma unroll
  for (int i = 0; i < NL; ++i) t.v[i] = 3u * cv.v[i] + 2u * (odd ? f.v[i] : K4.v[i] - f.v[i]);
  return pad16(reduce(lz<14>{fp_cn(t)}).v);
}

// f * (l0 + l2 w^2 + l3 w^3) (as x12_mul_line; the line is the same in every lane)
MBLS_X12_FN fp x16_mul_line(const fp& f, const fp2& l0, const fp2& l2, const fp2& l3) {
  const int c = hc(), h = c & 1;
  const int k = (c >> 1) < 6 ? (c >> 1) : 0;
  const int i2 = k >= 2 ? k - 2 : k + 4, i3 = k >= 3 ? k - 3 : k + 3;
  fpcols acc;
  cols_zero(acc);
  cols_mad1(acc, x16_c(f, k, 0), x16_c(f, k, 1), nrm(l0.c0), nrm(l0.c1), false, h);
  cols_mad1(acc, x16_c(f, i2, 0), x16_c(f, i2, 1), nrm(l2.c0), nrm(l2.c1), k < 2, h);
  cols_mad1(acc, x16_c(f, i3, 0), x16_c(f, i3, 1), nrm(l3.c0), nrm(l3.c1), k < 3, h);
  return pad16(cols_redc(acc));
}

// group verdict: f == 1
__device__ __forceinline__ bool x16_is_one(const fp& v) {
  const bool ok = fp_eq(v, x16_one());
  const uint64_t m = __ballot(ok);
  return ((m >> hbase()) & 0xffffull) == 0xffffull;
}

__device__ __noinline__ fp x16_pow_xabs(const fp& g) {
  fp r = g;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    r = x16_cyc_sqr(r);
    if ((k::X_ABS >> b) & 1ull) r = x16_mul(r, g);
  }
  return r;
}
__device__ __forceinline__ fp x16_pow_x(const fp& g) { return x16_conj(x16_pow_xabs(g)); }

// final exponentiation, x12_final_exp's schedule; inversion and Frobenius maps in the 8-lane form
__device__ __noinline__ fp x16_final_exp(const fp& f) {
  fp t = x16_mul(x16_conj(f), x16_from8(x12_inv(x16_to8(f))));
  t = x16_mul(x16_from8(x12_frob2(x16_to8(t))), t);
  fp a = x16_mul(x16_pow_x(t), x16_conj(t));
  a = x16_mul(x16_pow_x(a), x16_conj(a));
  const fp b = x16_mul(x16_pow_x(a), x16_from8(x12_frob(x16_to8(a))));
  fp c = x16_pow_x(x16_pow_x(b));
  c = x16_mul(x16_mul(c, x16_from8(x12_frob2(x16_to8(b)))), x16_conj(b));
  const fp t3 = x16_mul(x16_cyc_sqr(t), t);
  return x16_mul(c, t3);
}

// Miller steps on 16-lane groups: each round's Fp2 products (one per 8-lane lane k in
// dbl_step_lg / add_step_lg) split by component, lane (k, h) computing component h of product k
// with one reduction (as mul(lz2, lz2): (a0 b0 + a1 (32p - b1)) + (a0 b1 + a1 b0) u)
template <int A, int C>
__device__ __forceinline__ fp mul16(const lz2<A>& a, const lz2<C>& b, int h) {
  static_assert(C < 32 && A * (C + 32) <= 2400, "Fp2 product bound");
  fp nb1;
#pragma unroll
  for (int i = 0; i < NL; ++i) nb1.v[i] = PKB<32>::v.v[i] - b.v.c1.v[i];  // digits < 2^30
  return fp_mul2(a.v.c0, fp_select(h, b.v.c1, b.v.c0), a.v.c1, fp_select(h, b.v.c0, nb1));
}
// product idx of a round, as an Fp2 in every lane
__device__ __forceinline__ nz2 lcoef16(const fp& v, int idx) {
  return nrm(fp2{pull(v, hbase() + 2 * idx), pull(v, hbase() + 2 * idx + 1)});
}
// dbl_step_lg with the rounds split by component
MBLS_STEP_FN line_lg dbl_step16(tlz& t, const pt_lg& p) {
  const int k = hc() >> 1, h = hc() & 1;
  const fp r1 = mul16(lpick6(k, t.y, t.z, t.y, t.x, t.x, t.x), lpick6(k, t.y, t.z, t.z, t.x, t.y, t.y), h);
  const nz2 yy = lcoef16(r1, 0), zz = lcoef16(r1, 1), yz = lcoef16(r1, 2), xx = lcoef16(r1, 3), xy = lcoef16(r1, 4);
  const lz2<8> c2 = neg(smul<3>(xx));
  const lz2<4> c3 = smul<2>(yz);
  const nz2 t2 = reduce(mul_b3(zz));
  const lz2<16> z8 = smul<8>(yy);
  const lz2<10> t0m = yy - smul<3>(t2);
  const lz2<4> y3s = yy + t2;
  const lz2<6> c0 = yy - t2;
  const fp r2 = mul16(lpick7(k, t2, yz, t0m, t0m, c2, c3, c0), lpick7(k, z8, z8, y3s, xy, nrm(p.x), nrm(p.y), nrm(p.z)), h);
  line_lg l;
  l.l0 = lcoef16(r2, 6).v;
  l.l2 = lcoef16(r2, 4).v;
  l.l3 = lcoef16(r2, 5).v;
  t.x = widen<8>(smul<2>(lcoef16(r2, 3)));
  t.y = widen<8>(lcoef16(r2, 0) + lcoef16(r2, 2));
  t.z = widen<8>(lcoef16(r2, 1));
  return l;
}
// add_step_lg with the rounds split by component
MBLS_STEP_FN line_lg add_step16(tlz& t, const aff<fp2>& q, const aff<fp2>& qz, const pt_lg& p) {
  const int k = hc() >> 1, h = hc() & 1;
  const nz2 qx = nrm(q.x), qy = nrm(q.y);
  const lz2<4> sq = qx + qy;
  const lz2<16> st = t.x + t.y;
  const fp r1 = mul16(lpick6(k, t.x, t.y, sq, qy, qx, qx), lpick6(k, qx, qy, st, t.z, t.z, t.z), h);
  const nz2 t0 = lcoef16(r1, 0), t1 = lcoef16(r1, 1), yqz = lcoef16(r1, 3), xqz = lcoef16(r1, 4);
  const lz2<12> theta = t.y - yqz, kappa = t.x - xqz;
  const lz2<10> t3 = lcoef16(r1, 2) - (t0 + t1);
  const lz2<10> t4 = yqz + t.y;
  const nz2 y3b = reduce(mul_b3(xqz + t.x));
  const lz2<6> t03 = smul<3>(t0);
  const nz2 t2 = reduce(mul_b3(t.z));
  const lz2<4> z3a = t1 + t2;
  const lz2<6> t1m = t1 - t2;
  const fp r2 = mul16(lpick6(k, t4, t3, y3b, t1m, t03, z3a), lpick6(k, y3b, t1m, t03, z3a, t3, t4), h);
  const fp r3 = mul16(lpick6(k, theta, kappa, theta, kappa, theta, theta),
                      lpick6(k, nrm(qz.x), nrm(qz.y), nrm(p.x), nrm(p.y), nrm(p.x), nrm(p.x)), h);
  t.x = widen<8>(lcoef16(r2, 1) - lcoef16(r2, 0));
  t.y = widen<8>(lcoef16(r2, 3) + lcoef16(r2, 2));
  t.z = widen<8>(lcoef16(r2, 5) + lcoef16(r2, 4));
  line_lg l;
  l.l0 = fp2_sub(lcoef16(r3, 0).v, lcoef16(r3, 1).v);
  l.l2 = fp2_neg(lcoef16(r3, 2).v);
  l.l3 = lcoef16(r3, 3).v;
  return l;
}

// Miller loops (as miller_lg / miller2_lg): T, the lines and f in the 16-lane form
__device__ __noinline__ fp miller16(const proj<fp>& pp, const aff<fp2>& q) {
  const pt_lg p = pt_lg_from(pp);
  const aff<fp2> qz = {fp2_mul_fp(q.x, pp.z), fp2_mul_fp(q.y, pp.z)};
  tlz t = tlz_from(q);
  fp f = x16_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = x16_sqr(f);
    line_lg l = dbl_step16(t, p);
    f = x16_mul_line(f, l.l0, l.l2, l.l3);
    if ((k::X_ABS >> b) & 1ull) {
      l = add_step16(t, q, qz, p);
      f = x16_mul_line(f, l.l0, l.l2, l.l3);
    }
  }
  return x16_conj(f);
}
__device__ __noinline__ fp miller2_16(const proj<fp>& pp1, const aff<fp2>& q1, const proj<fp>& pp2, const aff<fp2>& q2,
                                      bool use2) {
  const pt_lg p1 = pt_lg_from(pp1), p2 = pt_lg_from(pp2);
  const aff<fp2> qz1 = {fp2_mul_fp(q1.x, pp1.z), fp2_mul_fp(q1.y, pp1.z)};
  const aff<fp2> qz2 = {fp2_mul_fp(q2.x, pp2.z), fp2_mul_fp(q2.y, pp2.z)};
  tlz t1 = tlz_from(q1), t2 = tlz_from(q2);
  fp f = x16_one();
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = x16_sqr(f);
    line_lg l = dbl_step16(t1, p1);
    f = x16_mul_line(f, l.l0, l.l2, l.l3);
    if (use2) {
      l = dbl_step16(t2, p2);
      f = x16_mul_line(f, l.l0, l.l2, l.l3);
    }
    if ((k::X_ABS >> b) & 1ull) {
      l = add_step16(t1, q1, qz1, p1);
      f = x16_mul_line(f, l.l0, l.l2, l.l3);
      if (use2) {
        l = add_step16(t2, q2, qz2, p2);
        f = x16_mul_line(f, l.l0, l.l2, l.l3);
      }
    }
  }
  return x16_conj(f);
}

}  // namespace lg
}  // namespace mbls
