// mbls_scratch.h — internal: the per-device scratch plan (mbls_scratch.cpp), applied by the
// engine when it initialises on a device.
#pragma once
#include "../../include/mbls.h"

namespace mbls_scratch {
// hardware queues per process as the launcher set them (GPU_MAX_HW_QUEUES, HIP's default 4)
int hw_queues();
// the plan applied to `device` (computed and set on first use; one per device for the process)
mbls_scratch_plan_t apply(int device, int n_cu);
}  // namespace mbls_scratch
