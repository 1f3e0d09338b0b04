// mbls_kernels.h — device status codes shared by the kernels and the host engine, and the
// host-side launch wrappers each kernel translation unit exports.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Static wave priorities (s_setprio) of the two kernel families that share SIMDs in a cold
// call: the latency-critical G2 / pairing chain and the throughput-bound key validation.
// Compile-time so variant builds can be compared.
#define MBLS_G2_PRIO 3
#define MBLS_KEY_PRIO 0

#include "mbls_codes.h"

// public-key decode code -> C result code (lighthouse PublicKey::deserialize errors)
__host__ __device__ inline int32_t mbls_pk_code(int32_t dec) {
  switch (dec) {
    case MBLS_DEC_BAD_ENCODING: return -1;
    case MBLS_DEC_NOT_ON_CURVE: return -2;
    case MBLS_DEC_NOT_IN_GROUP: return -3;
    case MBLS_DEC_INFINITY: return -5;  // InvalidInfinityPublicKey (checked before blst)
    case MBLS_DEC_PK_LENGTH: return -6;  // InvalidByteLength
    case MBLS_DEC_UNKNOWN_INDEX: return -12;  // UnknownValidatorIndex (pubkey table)
    default: return -1;
  }
}
__host__ __device__ inline bool mbls_is_pk_error(int32_t dec) {
  return (dec >= MBLS_DEC_BAD_ENCODING && dec <= MBLS_DEC_INFINITY) || dec == MBLS_DEC_PK_LENGTH ||
         dec == MBLS_DEC_UNKNOWN_INDEX;
}
// signature decode code -> C result code (only decode failures are errors)
__host__ __device__ inline int32_t mbls_sig_code(int32_t dec) {
  return dec == MBLS_DEC_BAD_ENCODING ? -1 : dec == MBLS_DEC_NOT_ON_CURVE ? -2 : 0;
}

// fast_aggregate_verify / verify outcome when no pairing is needed (reference precedence,
// signature decode error, first key error, host message-level outcome,
// empty key list, then the boolean rules), or MBLS_NEEDS_PAIRING.
#define MBLS_NEEDS_PAIRING (-1000)
__host__ __device__ inline int32_t mbls_fav_precheck(int32_t ss, int32_t ps, int32_t sp, uint32_t nk, int32_t eth) {
  if (ss == MBLS_DEC_BAD_ENCODING || ss == MBLS_DEC_NOT_ON_CURVE) return mbls_sig_code(ss);
  if (mbls_is_pk_error(ps)) return mbls_pk_code(ps);
  if (sp != 0) return sp;
  if (nk == 0) return (eth && ss == MBLS_DEC_INFINITY) ? 1 : 0;
  if (ss == MBLS_DEC_NONE || ps == MBLS_AGG_INFINITY || ss == MBLS_DEC_SIG_NOT_IN_G2) return 0;
  return MBLS_NEEDS_PAIRING;
}

// Per-kernel timing hooks (implemented in mbls_engine.cpp; no-ops unless mbls_prof_enable(1)).
namespace mbls_prof {
enum Kernel {
  K_G1_DECODE = 0,
  K_G1_AGGREGATE,
  K_G1_COMPRESS,
  K_MAP_PK_STATUS,
  K_G2_SIG_DECODE,
  K_HASH_TO_G2,
  K_FAV_VERDICT,
  K_AV_VERDICT,
  K_SIGN,
  K_G2_AGGREGATE,
  K_SK_TO_PK,
  K_SIG_MILLER,
  K_G1_AGGREGATE_IDX,
  K_PK_TABLE_STORE,
  K_MILLER_PAIRS,
  K_RLC,
  K_G2_PREP,
  K_SSZ_ROOTS,
  K_FAV_VERDICT_1L,    // the one-lane form of K_FAV_VERDICT (counted in both)
  K_FAV_VERDICT_LG8,   // the 8-lane form on padded 8-lane groups (MBLS_LG6=0)
  K_FAV_VERDICT_LG16,  // the 16-lane form
  K_KEY_MILLER,        // key-side Miller loop of the split latency chain
  K_FAV_VERDICT_LG6,   // the 8-lane form on 6-lane groups (the default; r05: counted apart from LG8)
  K_COUNT
};
extern bool g_on;
void begin(int kid, hipStream_t s);
void end(int kid, hipStream_t s);
struct Scope {
  int kid;
  hipStream_t s;
  Scope(int k, hipStream_t st) : kid(k), s(st) {
    if (g_on) begin(kid, s);
  }
  ~Scope() {
    if (g_on) end(kid, s);
  }
};
}  // namespace mbls_prof

namespace mbls_launch {
// mbls_k_g1.hip
hipError_t g1_decode_validate(const uint8_t* pks, uint32_t n, const int32_t* pre, int32_t* st, uint32_t* xy,
                              hipStream_t s);
hipError_t map_pk_status(const int32_t* st, uint32_t n, int32_t* out, hipStream_t s);
hipError_t sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* out48, hipStream_t s);
hipError_t g1_aggregate(const int32_t* key_st, const uint32_t* key_xy, uint32_t n_keys, const uint32_t* key_off,
                        uint32_t n_sets, int32_t* set_st, uint32_t* set_xy, hipStream_t s);
// validator pubkey table (AoS rows of 32 dwords: x digits 0..13, y digits 14..27, pad)
hipError_t pk_table_fill(int32_t* tab_st, uint32_t from, uint32_t to, hipStream_t s);
hipError_t pk_table_store(const int32_t* st, const uint32_t* xy, uint32_t n, uint32_t first, int32_t* tab_st,
                          uint32_t* tab_aff, hipStream_t s);
hipError_t g1_aggregate_idx(const int32_t* tab_st, const uint32_t* tab_aff, uint32_t n_tab, const uint32_t* idx,
                            const uint32_t* idx_off, uint32_t n_sets, int32_t* set_st, uint32_t* set_xy,
                            hipStream_t s);
hipError_t g1_compress_sets(const int32_t* set_st, const uint32_t* set_xy, uint32_t n_sets, uint8_t* out48,
                            int32_t* status, hipStream_t s);
// mbls_k_g2.hip
hipError_t g2_sig_decode(const uint8_t* sigs, uint32_t n, int32_t group_check, const int32_t* pre, int32_t* st,
                         uint32_t* xy, hipStream_t s);
hipError_t hash_to_g2(const uint8_t* msgs, uint32_t n, uint32_t* hxy, hipStream_t s);
// one-lane signature decode (group check on) + H(m) side by side in one launch
hipError_t g2_prep_1l(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                      uint32_t* sig_xy, uint32_t* hxy, hipStream_t s);
// the same outputs from the two-wave hash_to_g2 then g2_sig_decode (mbls_k_g2w.hip) on one stream
hipError_t g2_prep_split(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                         uint32_t* sig_xy, uint32_t* hxy, hipStream_t s);
hipError_t sig_miller(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sets, uint32_t* fsig, hipStream_t s);
hipError_t fav_verdict(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                       const uint32_t* sig_xy, const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets,
                       int32_t eth_variant, const int32_t* set_pre, int32_t* status, hipStream_t s);
// lane-group forms (8 lanes per set); fsig is lane-major, 8 * n_sets lanes of 28 dwords
// rlc_ok (optional): a passed random-linear-combination check; candidates then verdict 1
// without their own pairing, and the signature-side loops are skipped
hipError_t sig_miller_lg(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sets, uint32_t* fsig,
                         const int32_t* rlc_ok, hipStream_t s);
hipError_t fav_verdict_lg(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* key_off, const int32_t* sig_st,
                          const uint32_t* sig_xy, const uint32_t* fsig, const uint32_t* h_xy, uint32_t n_sets,
                          int32_t eth_variant, const int32_t* set_pre, const int32_t* rlc_ok, int32_t* status,
                          hipStream_t s, int32_t fsig_onelane);
hipError_t hash_to_g2_lg(const uint8_t* msgs, uint32_t n, uint32_t* hxy, hipStream_t s);
// Largest private (scratch) segment, bytes per lane, of the kernels of one family, from the
// loaded code objects (hipFuncGetAttributes; device must be current): the one-lane pairing
// kernels (mbls_k_pair.hip), the one-lane G2 kernels (mbls_k_g2.hip) and the lane-group
// kernels (mbls_k_lg.hip).  The engine sizes its scratch-stream pool from them.
size_t onelane_pair_private_bytes();
size_t onelane_g2_private_bytes();
size_t lane_group_private_bytes();
// signature decode (+ optional signature-side Miller values) and H(m) side by side, lane groups;
// parts: 1 the hash blocks only, 2 the signature blocks only, 3 both
hipError_t g2_prep_lg(const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n, int32_t* sig_st,
                      uint32_t* sig_xy, uint32_t* hxy, uint32_t* fsig, hipStream_t s, uint32_t parts = 3);
// the split latency chain (r03): key-side Miller values f_{|x|,H(m)}(apk) in fsig's lane layout,
// then the verdict from them and the signature-side values (precheck, product, final exp)
hipError_t key_miller_lg(const int32_t* pk_st, const uint32_t* pk_xy, const uint32_t* h_xy, uint32_t n_sets,
                         uint32_t* fpk, hipStream_t s);
hipError_t fav_final_lg(const int32_t* pk_st, const uint32_t* key_off, const int32_t* sig_st, const uint32_t* fsig,
                        const uint32_t* fpk, uint32_t n_sets, int32_t eth_variant, const int32_t* set_pre,
                        int32_t* status, hipStream_t s);
hipError_t miller_pairs(const int32_t* key_st, const uint32_t* key_xy, const uint32_t* h_xy, uint32_t n_pairs,
                        const uint32_t* key_off, uint32_t n_sets, uint32_t* fpair, hipStream_t s);
hipError_t av_verdict_lg(const int32_t* key_st, uint32_t n_pairs, const uint32_t* key_off, const int32_t* sig_st,
                         const uint32_t* fsig, const uint32_t* fpair, uint32_t n_sets, const int32_t* set_pre,
                         int32_t* status, hipStream_t s);
// random-linear-combination batch check, FAV pipeline
struct RlcBufs {
  int32_t* cand;    // n_sets: 1 = set needs a pairing (and is in the combination)
  uint32_t* p_xy;   // 42 rows x n_sets: [r_s] apk_s (projective)
  uint32_t* q_xy;   // 84 rows x n_sets: [r_s] sigma_s (projective), then partial sums
  uint32_t* q_tmp;  // 84 rows x ceil(n_sets / 64)
  uint32_t* fr;     // lane layout, 8 n_sets lanes: Miller values, then partial products
  uint32_t* fr_tmp; // lane layout, 8 ceil(n_sets / 16) lanes
  int32_t* ok;      // 1 int: the batch passed
};
hipError_t rlc_scale(const int32_t* set_st, const uint32_t* set_xy, const uint32_t* key_off, const int32_t* sig_st,
                     const uint32_t* sig_xy, uint32_t n_sets, int32_t eth, const int32_t* set_pre,
                     const uint32_t (&seed)[8], const RlcBufs& b, hipStream_t s);
hipError_t rlc_sum_g2(uint32_t* q_xy, uint32_t* q_tmp, uint32_t n, uint32_t** result, hipStream_t s);
hipError_t rlc_check(const RlcBufs& b, const uint32_t* h_xy, uint32_t n_sets, const uint32_t* q_sum,
                     hipStream_t s);
hipError_t av_verdict(const int32_t* key_st, const uint32_t* key_xy, uint32_t n_pairs, const uint32_t* key_off,
                      const int32_t* sig_st, const uint32_t* sig_xy, const uint32_t* h_xy, uint32_t n_sets,
                      const int32_t* set_pre, int32_t* status, hipStream_t s);
hipError_t sign(const uint8_t* sk32, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t s);
hipError_t g2_aggregate(const int32_t* sig_st, const uint32_t* sig_xy, uint32_t n_sigs, const uint32_t* off,
                        uint32_t n_sets, uint8_t* out96, int32_t* status, hipStream_t s);
// mbls_k_ssz.hip (SSZ signing roots)
hipError_t htr_chunks(const uint8_t* chunks, uint32_t leaves, uint32_t n, uint8_t* out32, hipStream_t s);
hipError_t signing_roots(const uint8_t* roots32, const uint8_t* domains32, uint32_t domain_stride, uint32_t n,
                         uint8_t* out32, hipStream_t s);
hipError_t attestation_signing_roots(const uint8_t* data128, const uint8_t* domains32, uint32_t domain_stride,
                                     uint32_t n, uint8_t* out32, hipStream_t s);
}  // namespace mbls_launch
