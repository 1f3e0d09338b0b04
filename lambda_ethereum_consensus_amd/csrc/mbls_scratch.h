// mbls_scratch.h — internal: the per-device scratch plan (mbls_scratch.cpp), applied by the
// engine when it initialises on a device.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

#include "../../include/mbls.h"

namespace mbls_scratch {
// hardware queues per process as the launcher set them (GPU_MAX_HW_QUEUES, HIP's default 4)
int hw_queues();
// the plan applied to `device` (computed and set on first use; one per device for the process)
// (MBLS_ERR_SCRATCH_PLAN when the plan is not safe, not settable or the limits are unreadable:
// the engine then refuses to initialise)
int32_t apply(int device, int n_cu, mbls_scratch_plan_t* out);

// The kernels whose frames lie above every plan's retain threshold on MI355X (Sign, the one-lane
// verdicts, the two-wave H(m)): each dispatch of one of them takes a use-once block.
enum UseOnceKernel : int { UO_FAV_VERDICT = 0, UO_AV_VERDICT, UO_HASH_TO_G2, UO_SIGN, UO_COUNT };

// Admission of one dispatch of `k` over `lanes` lanes on stream `s` (ADVICE
// r05): the dispatch's use-once block is frame x min(lanes, 64 x 32 x CUs) bytes, and the gate
// keeps the blocks of all use-once dispatches that may be live on the device at once -- every
// queue and every caller thread -- within use_once_budget = pool - queues x retain.  When the
// new need would exceed it, `s` waits (device side, hipStreamWaitEvent) for the oldest earlier
// dispatches, which stay counted until their completion events fire; a kernel whose frame the
// device retains passes untouched.  Holds the device's gate lock from admission to done(), so
// the launch and its completion event are registered atomically.
class UseOnce {
 public:
  UseOnce(UseOnceKernel k, uint64_t lanes, hipStream_t s);
  ~UseOnce();
  hipError_t rc = hipSuccess;   // admission failed (a stream wait could not be enqueued)
  hipError_t done(hipError_t launch_rc);  // records the dispatch's completion; returns launch_rc
  UseOnce(const UseOnce&) = delete;
  UseOnce& operator=(const UseOnce&) = delete;

 private:
  void* gate_ = nullptr;
  std::unique_lock<std::mutex> lk_;
  hipStream_t s_ = nullptr;
  uint64_t need_ = 0;
};
// telemetry of the gate of `device` (tests): dispatches admitted, those that had to wait, the
// largest sum of live use-once bytes admitted
struct UseOnceStats {
  uint64_t admitted, waited, peak_live;
};
UseOnceStats use_once_stats(int device);
}  // namespace mbls_scratch
