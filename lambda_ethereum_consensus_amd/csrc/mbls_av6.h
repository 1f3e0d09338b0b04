// mbls_av6.h — launch wrappers of mbls_k_av6.hip (aggregate_verify on 6-lane groups with joint
// Miller loops over groups of pairs, r05).  A header of its own, included only by the engine and
// that translation unit, so that adding these entry points rebuilds neither the other kernels nor
// the one-lane pairing unit (mbls_kernels.h is included by every kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbls_launch {
// upper bound on the groups of a batch: the size of fgrp is av_groups_bound x 8 lanes x 28 dwords
uint32_t av_groups_bound(uint32_t n_pairs, uint32_t n_sets);
// grp_off (n_sets + 1 words): the group plan; fgrp: one Fp12 per group (lane layout)
hipError_t av_pairs_lg6(const int32_t* key_st, const uint32_t* key_xy, const uint32_t* h_xy, uint32_t n_pairs,
                        const uint32_t* key_off, uint32_t n_sets, const int32_t* sig_st, const uint32_t* sig_xy,
                        uint32_t* grp_off, uint32_t* fgrp, hipStream_t s);
hipError_t av_verdict_grp_lg6(const int32_t* key_st, const uint32_t* key_off, const int32_t* sig_st,
                              const uint32_t* grp_off, const uint32_t* fgrp, uint32_t n_sets, const int32_t* set_pre,
                              int32_t* status, hipStream_t s);
}  // namespace mbls_launch
