// fp64_mont.hip -- one measured attempt at the field product on the FP64 FMA pipe (VERDICT r04
// next #6; tools/, not product).
//
// profiles/r01_isa_rates.json: v_fma_f64 issues at 3.30e13 lane-ops/s on MI355X, v_mad_u64_u32 at
// 3.20e13.  An FMA's 53-bit significand carries a 48 x 48-bit product exactly when split in two,
// against 28 x 28 bits of a radix-2^28 mad.  This is an exact Montgomery product on that pipe:
//   * p and the operands in 8 signed digits of radix B = 2^48 (doubles holding integers), R = 2^384;
//   * a product x y (|x|, |y| < 2^49) split exactly as h = fma(x, y, C) - C (C = 3 * 2^99: the sum's
//     ulp is 2^48, so h is x y rounded to a multiple of B) and l = fma(x, y, -h) = x y - h, |l| <= 2^47;
//     column sums accumulate the h (exact: multiples of B below 2^100) and the l separately;
//   * Montgomery reduction digit by digit with a BALANCED digit m = x p' mods B (the l part of
//     v p', no floor needed) and the carry (v + m p_0) / B, exact because v + m p_0 is a multiple of
//     B below 2^97 (one rounding of an exactly representable value);
//   * inputs < 2p, output < 2p (R > 4p), as the radix-2^28 product it is compared with.
// 64 + 64 products x 5 FP64 operations + ~100 for digits and carries: ~740 operations per product
// against the radix-2^28 product's 392 mads + ~110.  The host build (-DFP64_HOST, std::fma) checks
// the arithmetic bit-exactly against Python integers; the device build measures Fp-mul/s in
// tools/fp_rates.hip's harness (4 dependent chains per lane, 16 waves per CU) for comparison with
// profiles/r01_fp_rates_radix28.json (6.88e10).
//
// host check:  g++ -O2 -mfma -DFP64_HOST -x c++ tools/fp64_mont.hip -o /tmp/fp64h && /tmp/fp64h
//              (200,000 products of operands in [0, 2p) incl. 0, 1, p - 1, 2p - 1: result in (-2p, 2p),
//              2,000 of them checked congruent to a b R^-1 mod p with 128-bit-limb integers)
// device:      hipcc --offload-arch=gfx950 -O3 -o tools/fp64_mont tools/fp64_mont.hip
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#ifdef FP64_HOST
#define FD inline
#define FMA(a, b, c) std::fma((a), (b), (c))
#else
#include <hip/hip_runtime.h>
#define FD __device__ __forceinline__
#define FMA(a, b, c) __fma_rn((a), (b), (c))
#endif

namespace f64 {
constexpr int L = 8;                       // digits
constexpr double B = 281474976710656.0;    // 2^48
constexpr double IB = 1.0 / B;             // 2^-48 (exact)
constexpr double C = 3.0 * 633825300114114700748351602688.0;  // 3 * 2^99: ulp of [2^100, 2^101) is 2^48
constexpr double CR = 6755399441055744.0;  // 1.5 * 2^52: rounds a |v| < 2^51 to an integer
// p in balanced radix-2^48 digits and p' = -p^-1 mod 2^48 (balanced), filled by init_consts
struct Consts {
  double p[L];
  double pinv;
};

struct fe {
  double d[L];
};

// h + l = x y exactly, h a multiple of B (|x y| < 2^99)
FD void split(double x, double y, double& h, double& l) {
  h = FMA(x, y, C) - C;
  l = FMA(x, y, -h);
}

FD fe mont_mul(const fe& a, const fe& b, const Consts& k) {
  // column k: lo[k] (sum of l parts, |.| < 2^52) and hi[k] (sum of h parts of weight B^k: exact
  // multiples of B below 2^100)
  double lo[2 * L], hi[2 * L];
#pragma unroll
  for (int i = 0; i < 2 * L; ++i) lo[i] = hi[i] = 0.0;
#pragma unroll
  for (int i = 0; i < L; ++i)
#pragma unroll
    for (int j = 0; j < L; ++j) {
      double h, l;
      split(a.d[i], b.d[j], h, l);
      lo[i + j] += l;
      hi[i + j] += h;
    }
  // reduction: digit i of the running value v_i = lo[i] + carry (the carry holds column i-1's
  // h parts / B and the exact quotient of the previous step)
  double carry = 0.0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const double v = lo[i] + carry;                   // |v| < 2^53, exact
    const double vr = FMA(-(FMA(v, IB, CR) - CR), B, v);  // v mods B (|vr| <= 2^47): m depends on it only
    double mh, m;
    split(vr, k.pinv, mh, m);         // m = v p' mods B (balanced, |m| <= 2^47)
    carry = FMA(m, k.p[0], v) * IB;   // (v + m p_0) / B: exact (a multiple of B below 2^96)
    carry = FMA(hi[i], IB, carry);    // column i's h parts belong to column i + 1
#pragma unroll
    for (int j = 1; j < L; ++j) {
      double h, l;
      split(m, k.p[j], h, l);
      lo[i + j] += l;
      hi[i + j] += h;
    }
  }
  // columns L .. 2L-1: normalise into balanced digits
  fe r;
#pragma unroll
  for (int i = L; i < 2 * L; ++i) {
    const double v = lo[i] + carry;            // |v| < 2^53
    const double q = FMA(v, IB, CR) - CR;      // round(v / B)
    r.d[i - L] = FMA(-q, B, v);                // v - q B, |.| <= 2^47
    carry = FMA(hi[i], IB, q);
  }
  r.d[L - 1] = FMA(carry, B, r.d[L - 1]);  // top digit keeps the last carry (|value| < 2p)
  return r;
}
}  // namespace f64

#ifdef FP64_HOST
// ---------------------------------------------------------------- host exactness check ---
#include <random>
#include <string>
#include <vector>
typedef unsigned __int128 u128;
// tiny big-integer helpers on 8 x 64-bit words (little endian), enough for p, R and products
struct big {
  uint64_t w[13] = {};
};
static const char* P_HEX =
    "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab";
static big from_hex(const char* h) {
  big r;
  const int n = (int)strlen(h);
  for (int i = 0; i < n; ++i) {
    const char c = h[n - 1 - i];
    const uint64_t v = c <= '9' ? c - '0' : c - 'a' + 10;
    r.w[i / 16] |= v << (4 * (i % 16));
  }
  return r;
}
static int cmp(const big& a, const big& b) {
  for (int i = 12; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
static big sub(const big& a, const big& b) {
  big r;
  uint64_t br = 0;
  for (int i = 0; i < 13; ++i) {
    const u128 t = (u128)a.w[i] - b.w[i] - br;
    r.w[i] = (uint64_t)t;
    br = (uint64_t)(t >> 127);
  }
  return r;
}
static big add(const big& a, const big& b) {
  big r;
  uint64_t c = 0;
  for (int i = 0; i < 13; ++i) {
    const u128 t = (u128)a.w[i] + b.w[i] + c;
    r.w[i] = (uint64_t)t;
    c = (uint64_t)(t >> 64);
  }
  return r;
}
static big mul(const big& a, const big& b) {
  big r;
  for (int i = 0; i < 7; ++i) {
    uint64_t c = 0;
    for (int j = 0; j + i < 13 && j < 7; ++j) {
      const u128 t = (u128)a.w[i] * b.w[j] + r.w[i + j] + c;
      r.w[i + j] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
  }
  return r;
}
static big shr48(const big& a) {
  big r;
  for (int i = 0; i < 13; ++i) r.w[i] = (a.w[i] >> 48) | (i + 1 < 13 ? a.w[i + 1] << 16 : 0);
  return r;
}
// balanced digits of a (0 <= a < 2^384) <-> integer value of balanced digits (may be negative:
// then returned as value + 2^416 wrap; callers only convert non-negative values)
static f64::fe to_fe(big a) {
  f64::fe r;
  for (int i = 0; i < f64::L; ++i) {
    int64_t d = (int64_t)(a.w[0] & ((1ull << 48) - 1));
    a = shr48(a);
    if (d >= (1ll << 47) && i < f64::L - 1) {
      d -= (1ll << 48);
      big one;
      one.w[0] = 1;
      a = add(a, one);
    }
    r.d[i] = (double)d;
  }
  return r;
}
// value of balanced digits as (negative?, magnitude)
static big from_fe(const f64::fe& x, bool& negative) {
  big pos, neg;
  for (int i = f64::L - 1; i >= 0; --i) {
    big b48;
    b48.w[0] = 1ull << 48;
    pos = mul(pos, b48);
    neg = mul(neg, b48);
    const double d = x.d[i];
    big t;
    t.w[0] = (uint64_t)std::fabs(d);
    if (d >= 0)
      pos = add(pos, t);
    else
      neg = add(neg, t);
  }
  negative = cmp(pos, neg) < 0;
  return negative ? sub(neg, pos) : sub(pos, neg);
}
int main() {
  const big p = from_hex(P_HEX);
  // p' = -p^-1 mod 2^48 by Newton iteration on 64 bits
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - p.w[0] * inv;
  int64_t pinv = (int64_t)((0 - inv) & ((1ull << 48) - 1));
  if (pinv >= (1ll << 47)) pinv -= 1ll << 48;
  f64::Consts k;
  const f64::fe pf = to_fe(p);
  for (int i = 0; i < f64::L; ++i) k.p[i] = pf.d[i];
  k.pinv = (double)pinv;
  big two_p = add(p, p);
  std::mt19937_64 rng(7);
  int bad = 0;
  const int N = 200000;
  for (int t = 0; t < N; ++t) {
    big a, b;
    for (int i = 0; i < 6; ++i) a.w[i] = rng(), b.w[i] = rng();
    a.w[5] &= (1ull << 62) - 1;  // < 2^382
    b.w[5] &= (1ull << 62) - 1;
    while (cmp(a, two_p) >= 0) a = sub(a, p);
    while (cmp(b, two_p) >= 0) b = sub(b, p);
    if (t < 8) {  // edge operands: 0, 1, 2p - 1, p - 1
      const big one = [] { big o; o.w[0] = 1; return o; }();
      const big e[4] = {big(), one, sub(two_p, one), sub(p, one)};
      a = e[t % 4];
      b = e[(t / 4 + t) % 4];
    }
    const f64::fe r = f64::mont_mul(to_fe(a), to_fe(b), k);
    bool negative = false;
    big got = from_fe(r, negative);
    // reference: a b R^-1 mod p, checked as got R == a b (mod p) and 0 <= got < 2p
    big R;
    R.w[6] = 1;  // 2^384
    big lhs = mul(got, R), rhs = mul(a, b);
    // reduce both mod p by repeated subtraction of shifted p (slow, host check only)
    auto modp = [&](big x) {
      for (int s = 400; s >= 0; --s) {
        big ps = p;
        for (int q = 0; q < s; ++q) ps = add(ps, ps);
        if (ps.w[12]) continue;
        while (cmp(x, ps) >= 0) x = sub(x, ps);
      }
      return x;
    };
    const bool in_range = cmp(got, two_p) < 0;  // |result| < 2p: a valid input of the next product
    bool congruent = true;
    if (t < 2000 || t % 1000 == 0) {
      const big l = modp(lhs), rr = modp(rhs);
      congruent = negative ? (cmp(l, big()) == 0 ? cmp(rr, big()) == 0 : cmp(add(l, rr), p) == 0) : cmp(l, rr) == 0;
    }
    if (!in_range || !congruent) {
      if (bad < 5) std::fprintf(stderr, "case %d: in_range %d congruent %d negative %d\n", t, in_range, congruent, negative);
      ++bad;
    }
  }
  std::printf("{\"host_check\": \"%s\", \"cases\": %d, \"full_congruence_checked\": 2000, \"bad\": %d}\n",
              bad ? "FAIL" : "ok", N, bad);
  return bad ? 1 : 0;
}
#else
// ---------------------------------------------------------------- device throughput --------
#define CHECK(x)                                                                                 \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      return 1;                                                                                  \
    }                                                                                            \
  } while (0)

#ifdef WAVES  // -DWAVES=2: 256 registers per lane (the default occupancy spills the column sums)
#define OCC __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
#else
#define OCC
#endif
__global__ __launch_bounds__(256) OCC void k_chain(double* out, const double* in, int n, int iters, f64::Consts k) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  f64::fe x0, x1, x2, x3, y;
#pragma unroll
  for (int i = 0; i < f64::L; ++i) {
    x0.d[i] = in[i * n + g];
    y.d[i] = in[(i + f64::L) * n + g];
  }
  x1 = y;
  x2 = x0;
  x2.d[0] += 1.0;
  x3 = y;
  x3.d[0] += 1.0;
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
    x0 = f64::mont_mul(x0, y, k);
    x1 = f64::mont_mul(x1, y, k);
    x2 = f64::mont_mul(x2, y, k);
    x3 = f64::mont_mul(x3, y, k);
  }
#pragma unroll
  for (int i = 0; i < f64::L; ++i) out[i * n + g] = x0.d[i] + x1.d[i] + x2.d[i] + x3.d[i];
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int n = prop.multiProcessorCount * 256 * 4;  // 16 waves per CU, as tools/fp_rates.hip
  const int iters = 256;
  // p's balanced digits and p' (the host check derives them; the values are fixed)
  f64::Consts k;
  {
    // computed here the same way as the host check (integers < 2^64 per 48-bit digit)
    const uint64_t w[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                           0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
    __int128 carry = 0;
    for (int i = 0; i < 8; ++i) {
      // bits [48 i, 48 i + 48) of p
      const int b = 48 * i, q = b / 64, r = b % 64;
      unsigned __int128 v = (unsigned __int128)(q < 6 ? w[q] : 0) >> r;
      if (r > 16 && q + 1 < 6) v |= (unsigned __int128)w[q + 1] << (64 - r);
      __int128 d = (__int128)(uint64_t)(v & ((1ull << 48) - 1)) + carry;
      carry = 0;
      if (d >= ((__int128)1 << 47) && i < 7) {
        d -= (__int128)1 << 48;
        carry = 1;
      }
      k.p[i] = (double)(int64_t)d;
    }
    uint64_t inv = 1;
    for (int i = 0; i < 7; ++i) inv *= 2 - w[0] * inv;
    int64_t pinv = (int64_t)((0 - inv) & ((1ull << 48) - 1));
    if (pinv >= (1ll << 47)) pinv -= 1ll << 48;
    k.pinv = (double)pinv;
  }
  double *in, *out;
  CHECK(hipMalloc(&in, sizeof(double) * n * 16));
  CHECK(hipMalloc(&out, sizeof(double) * n * 8));
  double* h = (double*)malloc(sizeof(double) * n * 16);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n * 16; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const int limb = (i / n) % 8;
    int64_t d = (int64_t)(s & ((1ull << 47) - 1)) - (1ll << 46);  // balanced digits
    if (limb == 7) d = (int64_t)(s & ((1ull << 40) - 1));          // value < 2^376 < p
    h[i] = (double)d;
  }
  CHECK(hipMemcpy(in, h, sizeof(double) * n * 16, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, out, in, n, 4, k);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, out, in, n, iters, k);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double muls = (double)n * iters * 4;
#ifndef WAVES
#define WAVES 0
#endif
  printf("{\"variant\": \"fp64_fma_radix48\", \"waves_per_simd_bound\": %d, ", WAVES);
  printf("\"ms\": %.3f, \"fp_mul_per_s\": %.4e, \"vs_radix28_6.88e10\": %.3f}\n",
         best, muls / (best * 1e-3), muls / (best * 1e-3) / 6.8799e10);
  return 0;
}
#endif
