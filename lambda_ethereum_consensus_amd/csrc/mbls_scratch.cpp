// mbls_scratch.cpp — the per-device scratch plan of libmbls: which private
// segments the runtime may keep per hardware queue, so that no assignment of the library's
// kernels to GPU_MAX_HW_QUEUES queues can exhaust the device's scratch pool.  Split from
// mbls_engine.cpp (r05); the engine applies the plan when it initialises on a device.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/mbls.h"
#include "mbls_host.hpp"
#include "mbls_scratch.h"

namespace {

// ------------------------------------------------------------------ scratch plan (r05) ----
// two runs aborted with HSA_STATUS_ERROR_OUT_OF_RESOURCES (free device
// memory 264 GB) when lane-group and one-lane preps rotated over all ten queues.  Measured
// (tools/scratch_probe.hip, profiles/r05_scratch_probe.json): the runtime keeps each queue's
// scratch sized for a full-device dispatch of the largest frame it has run (5,216 B/lane ->
// 2.74 GB per queue) out of one 32 GiB pool per device, up to a retain threshold of 24 GiB.
// Per queue in the r04 bench process: the three one-lane streams 9,428 B (4.94 GB each), five
// more G2 streams 5,232 B (2.74 GB), the engine stream 7,104 B (Sign, 3.72 GB): 32.3 of 34.4 GB
// with every queue's block live, and a queue growing 4,240 -> 5,232 B (lane-group prep, then a
// one-lane prep: what MBLS_WARM_FILL=4 and the deferral window of 2 did more often) needs a new
// contiguous 2.74 GB block while the others are busy -- the pool's remaining free space, split
// in two, held it twice over but not in one piece.  The fix bounds what any queue can keep,
// whatever runs where (concurrent callers, user streams sharing a queue): plan_scratch
// (mbls_host.hpp) picks the largest threshold with queues x threshold + one full-device use-once
// dispatch of the largest frame <= pool, and the first engine on a device sets it
// (hsa_amd_agent_set_async_scratch_limit).  Frames above it run use-once, sized to their own
// grid (2,048 sets of the one-lane verdict: 19 MB).  Use-once is not free: ~0.15 ms of queue time
// per dispatch (probe), and with a threshold below the one-lane prep's frame (a first r05 plan
// priced GPU_MAX_HW_QUEUES + 1 queues: threshold 4,400 B) every pipelined table call paid it --
// warm epoch 861-869k vs 963k-1.000M sets/s (profiles/r05_scratch_ab.txt).  With ten queues the
// plan keeps every frame up to 5,248 B (the preps, the pairs' Miller loops) and makes only Sign,
// the one-lane verdicts and aggregate_verify's two-wave H(m) (one dispatch per batch) use-once.  MBLS_SCRATCH_RETAIN=runtime leaves the runtime's
// threshold (the r04 behaviour + clamp).
extern "C" {
// every kernel of the library (host stubs; hipFuncGetAttributes reads each one's private
// segment from the loaded code object).  tests/test_scratch_plan.py checks on the CPU that this
// list covers every kernel with a private segment in libmbls's gfx950 code objects.
__global__ void mbls_k_g1_decode_validate();
__global__ void mbls_k_g1_aggregate();
__global__ void mbls_k_g1_aggregate_idx();
__global__ void mbls_k_copy_u32();
__global__ void mbls_k_pk_table_fill();
__global__ void mbls_k_pk_table_store();
__global__ void mbls_k_g1_compress_sets();
__global__ void mbls_k_sk_to_pk();
__global__ void mbls_k_map_pk_status();
__global__ void mbls_k_g2_sig_decode();
__global__ void mbls_k_hash_to_g2();
__global__ void mbls_k_g2_prep_1l();
__global__ void mbls_k_rlc_scale();
__global__ void mbls_k_rlc_sum_g2();
__global__ void mbls_k_sign();
__global__ void mbls_k_g2_aggregate();
__global__ void mbls_k_sig_miller_lg();
__global__ void mbls_k_fav_verdict_lg();
__global__ void mbls_k_fav_verdict_lg16();
__global__ void mbls_k_av_verdict_lg();
__global__ void mbls_k_hash_to_g2_lg();
__global__ void mbls_k_g2_prep_lg();
__global__ void mbls_k_g2_prep_lg16();
__global__ void mbls_k_key_miller_lg();
__global__ void mbls_k_key_miller_lg16();
__global__ void mbls_k_fav_final_lg();
__global__ void mbls_k_fav_final_lg16();
__global__ void mbls_k_rlc_miller_lg();
__global__ void mbls_k_rlc_prod_lg();
__global__ void mbls_k_rlc_final_lg();
__global__ void mbls_k_fav_verdict_lg6();
__global__ void mbls_k_av_verdict_lg6();
__global__ void mbls_k_g2_prep_lg6();
__global__ void mbls_k_key_miller_lg6();
__global__ void mbls_k_fav_final_lg6();
__global__ void mbls_k_sig_miller();
__global__ void mbls_k_fav_verdict();
__global__ void mbls_k_miller_pairs();
__global__ void mbls_k_av_verdict();
__global__ void mbls_k_signing_roots();
__global__ void mbls_k_attestation_signing_roots();
__global__ void mbls_k_av_group_plan();
__global__ void mbls_k_av_pairs_lg6();
__global__ void mbls_k_av_verdict_grp_lg6();
}
#define MBLS_SK(n) {#n, reinterpret_cast<const void*>(&n)}
struct ScratchKernel {
  const char* name;
  const void* fn;
};
const ScratchKernel kScratchKernels[] = {
    MBLS_SK(mbls_k_g1_decode_validate), MBLS_SK(mbls_k_g1_aggregate),     MBLS_SK(mbls_k_g1_aggregate_idx),
    MBLS_SK(mbls_k_copy_u32),           MBLS_SK(mbls_k_pk_table_fill),    MBLS_SK(mbls_k_pk_table_store),
    MBLS_SK(mbls_k_g1_compress_sets),   MBLS_SK(mbls_k_sk_to_pk),         MBLS_SK(mbls_k_map_pk_status),
    MBLS_SK(mbls_k_g2_sig_decode),      MBLS_SK(mbls_k_hash_to_g2),       MBLS_SK(mbls_k_g2_prep_1l),
    MBLS_SK(mbls_k_rlc_scale),          MBLS_SK(mbls_k_rlc_sum_g2),       MBLS_SK(mbls_k_sign),
    MBLS_SK(mbls_k_g2_aggregate),       MBLS_SK(mbls_k_sig_miller_lg),    MBLS_SK(mbls_k_fav_verdict_lg),
    MBLS_SK(mbls_k_fav_verdict_lg16),   MBLS_SK(mbls_k_av_verdict_lg),    MBLS_SK(mbls_k_hash_to_g2_lg),
    MBLS_SK(mbls_k_g2_prep_lg),         MBLS_SK(mbls_k_g2_prep_lg16),     MBLS_SK(mbls_k_key_miller_lg),
    MBLS_SK(mbls_k_key_miller_lg16),    MBLS_SK(mbls_k_fav_final_lg),     MBLS_SK(mbls_k_fav_final_lg16),
    MBLS_SK(mbls_k_rlc_miller_lg),      MBLS_SK(mbls_k_rlc_prod_lg),      MBLS_SK(mbls_k_rlc_final_lg),
    MBLS_SK(mbls_k_fav_verdict_lg6),    MBLS_SK(mbls_k_av_verdict_lg6),   MBLS_SK(mbls_k_g2_prep_lg6),
    MBLS_SK(mbls_k_key_miller_lg6),     MBLS_SK(mbls_k_fav_final_lg6),    MBLS_SK(mbls_k_sig_miller),
    MBLS_SK(mbls_k_fav_verdict),        MBLS_SK(mbls_k_miller_pairs),     MBLS_SK(mbls_k_av_verdict),
    MBLS_SK(mbls_k_signing_roots),      MBLS_SK(mbls_k_attestation_signing_roots), MBLS_SK(mbls_k_av_group_plan),
    MBLS_SK(mbls_k_av_pairs_lg6),       MBLS_SK(mbls_k_av_verdict_grp_lg6),
};
#undef MBLS_SK
constexpr int kNumScratchKernels = (int)(sizeof(kScratchKernels) / sizeof(kScratchKernels[0]));

struct HsaAgentFind {
  uint32_t bdf = 0, domain = 0;
  bool found = false;
  hsa_agent_t agent{};
  std::vector<hsa_agent_t> gpus;  // every GPU agent in runtime order (fallback: by ordinal)
};
hsa_status_t find_agent(hsa_agent_t a, void* p) {
  auto* f = static_cast<HsaAgentFind*>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  f->gpus.push_back(a);
  uint32_t bdf = 0, dom = 0;
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if (!f->found && bdf == f->bdf && dom == f->domain) {
    f->agent = a;
    f->found = true;
  }
  return HSA_STATUS_SUCCESS;
}

// one plan per device ordinal, applied by the first engine that initialises on it
struct ScratchState {
  std::mutex mu;
  std::vector<int> done;
  std::vector<mbls_scratch_plan_t> plans;
};
ScratchState& scratch_state() {
  static ScratchState* s = new ScratchState();  // immortal, as the registry
  return *s;
}
int queues_from_env() {
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  return q ? std::max(1, std::atoi(q)) : 4;
}
mbls_scratch_plan_t make_plan(uint64_t pool, uint64_t cur, uint32_t queues, uint32_t cus, const std::vector<uint32_t>& fr) {
  const mbls_host::ScratchPlan p =
      mbls_host::plan_scratch(pool, cur, queues, 64ull * 32ull * cus, fr.data(), (uint32_t)fr.size());
  mbls_scratch_plan_t o{};
  o.pool_bytes = pool;
  o.retain_default = cur;
  o.retain_bytes = p.retain;
  o.worst_retained = p.worst_retained;
  o.worst_use_once = p.worst_use_once;
  o.queues = queues;
  o.max_frame = p.max_frame;
  o.max_retained_frame = p.max_retained_frame;
  o.safe = p.safe ? 1 : 0;
  o.applied = 0;
  return o;
}
// Returns the plan applied to `device` (computing and setting it on first use).
mbls_scratch_plan_t apply_scratch_plan(int device, int n_cu) {
  ScratchState& S = scratch_state();
  std::lock_guard<std::mutex> g(S.mu);
  for (size_t i = 0; i < S.done.size(); ++i)
    if (S.done[i] == device) return S.plans[i];
  std::vector<uint32_t> fr;
  for (const auto& k : kScratchKernels) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k.fn) == hipSuccess && a.localSizeBytes) fr.push_back((uint32_t)a.localSizeBytes);
  }
  mbls_scratch_plan_t plan{};
  HsaAgentFind f;
  int bus = 0, dev = 0, dom = 0;
  (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device);
  (void)hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device);
  (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device);
  f.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
  f.domain = (uint32_t)dom;
  uint64_t pool = 0, cur = 0;
  if (hsa_init() == HSA_STATUS_SUCCESS) {  // (HIP initialised the runtime: a reference count)
    (void)hsa_iterate_agents(find_agent, &f);
    if (!f.found && device < (int)f.gpus.size()) {  // (PCI ids unavailable: the runtime's order)
      f.agent = f.gpus[device];
      f.found = true;
    }
    if (f.found) {
      (void)hsa_agent_get_info(f.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, &pool);
      (void)hsa_agent_get_info(f.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT, &cur);
    }
  }
  static const bool keep_runtime = [] {
    const char* v = std::getenv("MBLS_SCRATCH_RETAIN");
    return v && std::strcmp(v, "runtime") == 0;
  }();
  if (pool && cur) {
    // every hardware queue of the process: HIP maps all streams of the device -- the engine's, a
    // caller's, RCCL's -- onto at most GPU_MAX_HW_QUEUES of them
    plan = make_plan(pool, cur, (uint32_t)queues_from_env(), (uint32_t)std::max(n_cu, 1), fr);
    if (!keep_runtime && plan.safe && plan.retain_bytes < cur &&
        hsa_amd_agent_set_async_scratch_limit(f.agent, (size_t)plan.retain_bytes) == HSA_STATUS_SUCCESS)
      plan.applied = 1;
    else if (plan.retain_bytes >= cur)
      plan.applied = 1;  // the runtime's own threshold is already within the plan
    if (!plan.applied)
      std::fprintf(stderr, "libmbls: scratch retain threshold left at %.2f GB (plan %.2f GB, %s)\n", cur / 1e9,
                   plan.retain_bytes / 1e9, keep_runtime ? "MBLS_SCRATCH_RETAIN=runtime" : "not settable");
  } else {
    std::fprintf(stderr, "libmbls: device %d scratch limits unavailable; scratch plan not applied\n", device);
  }
  S.done.push_back(device);
  S.plans.push_back(plan);
  return plan;
}


}  // namespace

namespace mbls_scratch {
int hw_queues() { return queues_from_env(); }
mbls_scratch_plan_t apply(int device, int n_cu) { return apply_scratch_plan(device, n_cu); }
}  // namespace mbls_scratch

extern "C" {
int32_t mbls_scratch_plan(uint64_t pool_bytes, uint64_t retain_default, uint32_t queues, uint32_t cus,
                          const uint32_t* frames, uint32_t n_frames, mbls_scratch_plan_t* out) {
  if (!out || (n_frames && !frames) || queues == 0 || cus == 0) return MBLS_ERR_ARGUMENT;
  *out = make_plan(pool_bytes, retain_default, queues, cus, std::vector<uint32_t>(frames, frames + n_frames));
  return 0;
}
const char* mbls_scratch_kernel(int32_t i) { return i >= 0 && i < kNumScratchKernels ? kScratchKernels[i].name : nullptr; }
}  // extern "C"
