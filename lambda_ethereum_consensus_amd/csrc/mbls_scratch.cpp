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
// the one-lane verdicts and aggregate_verify's two-wave H(m) (one dispatch per batch) use-once.
// r06: the plan prices ONE full-device use-once block, but concurrent callers and pipelined calls
// can put several use-once dispatches on different queues at once: every
// such dispatch now passes the device's use-once gate (class UseOnce below), which keeps the sum
// of the live use-once blocks within pool - queues x threshold.  A plan that is not safe or not
// settable makes engine initialisation fail (MBLS_ERR_SCRATCH_PLAN) instead of running unguarded.
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
#define MBLS_SK(n) {#n, reinterpret_cast<const void*>(&n), false}
#define MBLS_SKG(n) {#n, reinterpret_cast<const void*>(&n), true}
struct ScratchKernel {
  const char* name;
  const void* fn;
  bool gated;  // every dispatch of it passes the use-once gate (the engine's use_once())
};
const ScratchKernel kScratchKernels[] = {
    MBLS_SK(mbls_k_g1_decode_validate), MBLS_SK(mbls_k_g1_aggregate),     MBLS_SK(mbls_k_g1_aggregate_idx),
    MBLS_SK(mbls_k_copy_u32),           MBLS_SK(mbls_k_pk_table_fill),    MBLS_SK(mbls_k_pk_table_store),
    MBLS_SK(mbls_k_g1_compress_sets),   MBLS_SK(mbls_k_sk_to_pk),         MBLS_SK(mbls_k_map_pk_status),
    MBLS_SK(mbls_k_g2_sig_decode),      MBLS_SKG(mbls_k_hash_to_g2),       MBLS_SK(mbls_k_g2_prep_1l),
    MBLS_SK(mbls_k_rlc_scale),          MBLS_SK(mbls_k_rlc_sum_g2),       MBLS_SKG(mbls_k_sign),
    MBLS_SK(mbls_k_g2_aggregate),       MBLS_SK(mbls_k_sig_miller_lg),    MBLS_SK(mbls_k_fav_verdict_lg),
    MBLS_SK(mbls_k_fav_verdict_lg16),   MBLS_SK(mbls_k_av_verdict_lg),    MBLS_SK(mbls_k_hash_to_g2_lg),
    MBLS_SK(mbls_k_g2_prep_lg),         MBLS_SK(mbls_k_g2_prep_lg16),     MBLS_SK(mbls_k_key_miller_lg),
    MBLS_SK(mbls_k_key_miller_lg16),    MBLS_SK(mbls_k_fav_final_lg),     MBLS_SK(mbls_k_fav_final_lg16),
    MBLS_SK(mbls_k_rlc_miller_lg),      MBLS_SK(mbls_k_rlc_prod_lg),      MBLS_SK(mbls_k_rlc_final_lg),
    MBLS_SK(mbls_k_fav_verdict_lg6),    MBLS_SK(mbls_k_av_verdict_lg6),   MBLS_SK(mbls_k_g2_prep_lg6),
    MBLS_SK(mbls_k_key_miller_lg6),     MBLS_SK(mbls_k_fav_final_lg6),    MBLS_SK(mbls_k_sig_miller),
    MBLS_SKG(mbls_k_fav_verdict),        MBLS_SK(mbls_k_miller_pairs),     MBLS_SKG(mbls_k_av_verdict),
    MBLS_SK(mbls_k_signing_roots),      MBLS_SK(mbls_k_attestation_signing_roots), MBLS_SK(mbls_k_av_group_plan),
    MBLS_SK(mbls_k_av_pairs_lg6),       MBLS_SK(mbls_k_av_verdict_grp_lg6),
};
#undef MBLS_SK
#undef MBLS_SKG
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
// The use-once gate of one device: the use-once dispatches admitted and not yet seen complete.
struct LiveDispatch {
  hipEvent_t ev;
  uint64_t bytes;
};
struct Gate {
  std::mutex mu;
  int device = -1;
  uint64_t budget = 0, retain = 0, lane_slots = 0;
  std::vector<LiveDispatch> live;  // admission order
  std::vector<hipEvent_t> spare;   // completed events for reuse
  uint64_t live_bytes = 0;
  mbls_scratch::UseOnceStats stats{0, 0, 0};
};
struct ScratchState {
  std::mutex mu;
  std::vector<int> done;
  std::vector<mbls_scratch_plan_t> plans;
  std::vector<int32_t> rcs;
  std::vector<Gate*> gates;  // immortal, one per planned device
};
ScratchState& scratch_state() {
  static ScratchState* s = new ScratchState();  // immortal, as the registry
  return *s;
}
int queues_from_env() {
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  return q ? std::max(1, std::atoi(q)) : 4;
}
mbls_scratch_plan_t make_plan(uint64_t pool, uint64_t cur, uint32_t queues, uint32_t cus, const std::vector<uint32_t>& fr,
                              const uint8_t* gated) {
  const mbls_host::ScratchPlan p =
      mbls_host::plan_scratch(pool, cur, queues, 64ull * 32ull * cus, fr.data(), gated, (uint32_t)fr.size());
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
  o.use_once_budget = pool > p.worst_retained ? pool - p.worst_retained : 0;
  return o;
}
// Computes and sets the plan of `device` on first use; returns 0 or MBLS_ERR_SCRATCH_PLAN (the
// same verdict for every later engine on the device).
int32_t apply_scratch_plan(int device, int n_cu, mbls_scratch_plan_t* out) {
  ScratchState& S = scratch_state();
  std::lock_guard<std::mutex> g(S.mu);
  for (size_t i = 0; i < S.done.size(); ++i)
    if (S.done[i] == device) {
      *out = S.plans[i];
      return S.rcs[i];
    }
  std::vector<uint32_t> fr;
  std::vector<uint8_t> gated;
  for (const auto& k : kScratchKernels) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, k.fn) == hipSuccess && a.localSizeBytes) {
      fr.push_back((uint32_t)a.localSizeBytes);
      gated.push_back(k.gated ? 1 : 0);
    }
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
  const uint32_t cus = (uint32_t)std::max(n_cu, 1);
  int32_t rc = 0;
  if (pool && cur) {
    // every hardware queue of the process: HIP maps all streams of the device -- the engine's, a
    // caller's, RCCL's -- onto at most GPU_MAX_HW_QUEUES of them
    plan = make_plan(pool, cur, (uint32_t)queues_from_env(), cus, fr, gated.data());
    if (plan.safe && plan.retain_bytes >= cur)
      plan.applied = 1;  // the runtime's own threshold is already within the plan
    else if (plan.safe &&
             hsa_amd_agent_set_async_scratch_limit(f.agent, (size_t)plan.retain_bytes) == HSA_STATUS_SUCCESS)
      plan.applied = 1;
    if (!plan.applied) {
      std::fprintf(stderr,
                   "libmbls: device %d scratch plan %s (pool %.2f GB, %u queues, largest frame %u B): engine not "
                   "initialised\n",
                   device, plan.safe ? "not settable" : "not safe", pool / 1e9, plan.queues, plan.max_frame);
      rc = MBLS_ERR_SCRATCH_PLAN;
    }
  } else {
    std::fprintf(stderr, "libmbls: device %d scratch limits unavailable: engine not initialised\n", device);
    rc = MBLS_ERR_SCRATCH_PLAN;
  }
  Gate* gt = new Gate();
  gt->device = device;
  gt->budget = plan.use_once_budget;
  if (const char* v = std::getenv("MBLS_USE_ONCE_BUDGET"))  // test knob: a tighter gate (bytes)
    gt->budget = std::min<uint64_t>(gt->budget, std::strtoull(v, nullptr, 10));
  gt->retain = plan.retain_bytes;
  gt->lane_slots = 64ull * 32ull * cus;
  S.done.push_back(device);
  S.plans.push_back(plan);
  S.rcs.push_back(rc);
  S.gates.push_back(gt);
  *out = plan;
  return rc;
}

Gate* gate_of(int device) {
  ScratchState& S = scratch_state();
  std::lock_guard<std::mutex> g(S.mu);
  for (size_t i = 0; i < S.done.size(); ++i)
    if (S.done[i] == device) return S.gates[i];
  return nullptr;
}

// host stubs of the use-once kernels, in UseOnceKernel order
const void* const kUseOnceFn[mbls_scratch::UO_COUNT] = {
    reinterpret_cast<const void*>(&mbls_k_fav_verdict), reinterpret_cast<const void*>(&mbls_k_av_verdict),
    reinterpret_cast<const void*>(&mbls_k_hash_to_g2), reinterpret_cast<const void*>(&mbls_k_sign)};

uint64_t frame_of(mbls_scratch::UseOnceKernel k) {
  static std::once_flag once;
  static uint64_t fr[mbls_scratch::UO_COUNT] = {};
  std::call_once(once, [] {
    for (int i = 0; i < mbls_scratch::UO_COUNT; ++i) {
      hipFuncAttributes a{};
      if (hipFuncGetAttributes(&a, kUseOnceFn[i]) == hipSuccess) fr[i] = a.localSizeBytes;
    }
  });
  return fr[k];
}

}  // namespace

namespace mbls_scratch {
UseOnce::UseOnce(UseOnceKernel k, uint64_t lanes, hipStream_t s) : s_(s) {
  int device = 0;
  if ((rc = hipGetDevice(&device)) != hipSuccess) return;
  Gate* gt = gate_of(device);
  const uint64_t frame = frame_of(k);
  if (!gt || frame * gt->lane_slots <= gt->retain) return;  // retained by its queue: not gated
  gate_ = gt;
  need_ = frame * std::min(lanes, gt->lane_slots);
  lk_ = std::unique_lock<std::mutex>(gt->mu);
  // forget the dispatches that completed (any order: they ran on different queues)
  size_t w = 0;
  for (size_t i = 0; i < gt->live.size(); ++i) {
    const hipError_t q = hipEventQuery(gt->live[i].ev);
    if (q == hipSuccess) {
      gt->live_bytes -= gt->live[i].bytes;
      gt->spare.push_back(gt->live[i].ev);
    } else {
      gt->live[w++] = gt->live[i];
    }
  }
  gt->live.resize(w);
  // over budget: this dispatch starts only after the oldest earlier ones finished (they stay
  // counted until their events fire: a later admission may still overlap them)
  uint64_t overlapping = gt->live_bytes;
  bool waited = false;
  for (size_t i = 0; i < gt->live.size() && overlapping + need_ > gt->budget; ++i) {
    if ((rc = hipStreamWaitEvent(s, gt->live[i].ev, 0)) != hipSuccess) return;
    overlapping -= gt->live[i].bytes;
    waited = true;
  }
  gt->stats.admitted++;
  if (waited) gt->stats.waited++;
  gt->stats.peak_live = std::max(gt->stats.peak_live, overlapping + need_);
}
hipError_t UseOnce::done(hipError_t launch_rc) {
  Gate* gt = static_cast<Gate*>(gate_);
  if (!gt || launch_rc != hipSuccess || rc != hipSuccess) return launch_rc;
  hipEvent_t ev = nullptr;
  if (!gt->spare.empty()) {
    ev = gt->spare.back();
    gt->spare.pop_back();
  } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    return hipErrorOutOfMemory;
  }
  if (hipEventRecord(ev, s_) != hipSuccess) {
    gt->spare.push_back(ev);
    return hipErrorLaunchFailure;
  }
  gt->live.push_back({ev, need_});
  gt->live_bytes += need_;
  return launch_rc;
}
UseOnce::~UseOnce() = default;
UseOnceStats use_once_stats(int device) {
  Gate* gt = gate_of(device);
  if (!gt) return {0, 0, 0};
  std::lock_guard<std::mutex> g(gt->mu);
  return gt->stats;
}
int hw_queues() { return queues_from_env(); }
int32_t apply(int device, int n_cu, mbls_scratch_plan_t* out) { return apply_scratch_plan(device, n_cu, out); }
}  // namespace mbls_scratch

extern "C" {
int32_t mbls_scratch_plan(uint64_t pool_bytes, uint64_t retain_default, uint32_t queues, uint32_t cus,
                          const uint32_t* frames, const uint8_t* gated, uint32_t n_frames, mbls_scratch_plan_t* out) {
  if (!out || (n_frames && !frames) || queues == 0 || cus == 0) return MBLS_ERR_ARGUMENT;
  *out = make_plan(pool_bytes, retain_default, queues, cus, std::vector<uint32_t>(frames, frames + n_frames), gated);
  return 0;
}
const char* mbls_scratch_kernel(int32_t i) { return i >= 0 && i < kNumScratchKernels ? kScratchKernels[i].name : nullptr; }
int32_t mbls_scratch_kernel_gated(int32_t i) {
  return i >= 0 && i < kNumScratchKernels ? (kScratchKernels[i].gated ? 1 : 0) : MBLS_ERR_ARGUMENT;
}
int32_t mbls_scratch_gate_stats(uint64_t* out3) {
  if (!out3) return MBLS_ERR_ARGUMENT;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return MBLS_ERR_DEVICE;
  const mbls_scratch::UseOnceStats st = mbls_scratch::use_once_stats(device);
  out3[0] = st.admitted;
  out3[1] = st.waited;
  out3[2] = st.peak_live;
  return 0;
}
}  // extern "C"
