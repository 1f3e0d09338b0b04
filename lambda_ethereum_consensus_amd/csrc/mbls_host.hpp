// mbls_host.hpp — host-only helpers of the engine: packing Erlang-style binaries into
// pinned staging (with the per-element pre-status codes the device pipeline consumes) and
// the key-balanced split of a batch over engines.  No HIP dependency, so the multi-threaded
// staging and the partition are also built and run under ASan / UBSan / TSan on the CPU
// (tests/sanitize/host_sanitize.cpp, tests/test_sanitizers.py).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/mbls.h"
#include "mbls_codes.h"

namespace mbls_host {

// Host binaries (the NIF's Erlang binaries) are packed straight into a call context's pinned
// staging by up to kStageThreads threads (no engine lock held), then copied with async DMA;
// lengths known on the host become per-element pre-status codes for the device pipeline.
constexpr unsigned kStageThreads = 8;
constexpr size_t kStageGrain = size_t(1) << 15;  // elements per thread below which one thread packs

template <class F>
void par_for(size_t n, F&& f) {
  const size_t want = std::min<size_t>(kStageThreads, (n + kStageGrain - 1) / kStageGrain);
  if (want <= 1) {
    f(size_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(want - 1);
  const size_t chunk = (n + want - 1) / want;
  for (size_t t = 1; t < want; ++t) {
    const size_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) th.emplace_back([&f, lo, hi] { f(lo, hi); });
  }
  f(size_t(0), std::min(n, chunk));
  for (auto& t : th) t.join();
}

// pubkey binaries -> packed 48-byte slots + pre-status (lighthouse PublicKey::deserialize: the
// exact infinity encoding is decided on the device, other lengths are InvalidByteLength)
inline void pack_pks(const mbls_bin* b, size_t n, uint8_t* out, int32_t* pre) {
  par_for(n, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      if (b[k].len == 48 && b[k].data) {
        std::memcpy(out + 48 * k, b[k].data, 48);
        pre[k] = MBLS_DEC_OK;
      } else {
        std::memset(out + 48 * k, 0, 48);
        pre[k] = MBLS_DEC_PK_LENGTH;
      }
    }
  });
}
// signature binaries: anything but 96 bytes fails blst Signature::from_bytes (BAD_ENCODING)
inline void pack_sigs(const mbls_bin* b, size_t n, uint8_t* out, int32_t* pre) {
  par_for(n, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      if (b[k].len == 96 && b[k].data) {
        std::memcpy(out + 96 * k, b[k].data, 96);
        pre[k] = MBLS_DEC_OK;
      } else {
        std::memset(out + 96 * k, 0, 96);
        pre[k] = MBLS_DEC_BAD_ENCODING;
      }
    }
  });
}
// one message per set: a message that is not 32 bytes marks its set (set_pre) with
// MBLS_ERR_MESSAGE_LENGTH (Hash256::from_slice, lib.rs:58,98,117)
inline void pack_msgs(const mbls_bin* b, size_t n, uint8_t* out, int32_t* set_pre) {
  par_for(n, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const bool ok = b[k].len == 32 && b[k].data;
      if (ok)
        std::memcpy(out + 32 * k, b[k].data, 32);
      else
        std::memset(out + 32 * k, 0, 32);
      set_pre[k] = ok ? 0 : MBLS_ERR_MESSAGE_LENGTH;
    }
  });
}

// Cost of a set for the key-balanced split: its keys (cold key validation, ~1,560 Fp
// multiplications each, dominates a 512-key set) plus a fixed share for its G2 chain
// (signature decode, H(m), pairing: ~26k Fp multiplications ~ 16 keys).
constexpr uint64_t kSetWeight = 16;
inline uint64_t prefix_cost(const uint32_t* key_off, size_t s) {
  return key_off ? (uint64_t)(key_off[s] - key_off[0]) + kSetWeight * s : (kSetWeight + 1) * s;
}
inline void plan_shards(const uint32_t* key_off, size_t n, uint32_t parts, uint32_t* b) {
  const uint64_t total = prefix_cost(key_off, n);
  b[0] = 0;
  for (uint32_t j = 1; j < parts; ++j) {
    const uint64_t target = (total * j + parts / 2) / parts;
    size_t lo = b[j - 1], hi = n;  // first s >= b[j-1] with prefix(s) >= target
    while (lo < hi) {
      const size_t mid = lo + (hi - lo) / 2;
      if (prefix_cost(key_off, mid) < target)
        lo = mid + 1;
      else
        hi = mid;
    }
    // the boundary nearest the target (one heavy set then gets a chunk of its own)
    if (lo > b[j - 1] && target - prefix_cost(key_off, lo - 1) < prefix_cost(key_off, lo) - target) --lo;
    b[j] = (uint32_t)lo;
  }
  b[parts] = (uint32_t)n;
}

// Scratch (private segment) plan (r05, include/mbls.h mbls_scratch_plan).  Measured on MI355X
// (tools/scratch_probe.hip -> profiles/r05_scratch_probe.json): the runtime backs the scratch of
// every hardware queue of the process out of ONE pool per device (HSA_AMD_AGENT_INFO_SCRATCH_
// LIMIT_MAX = 32 GiB) and, when a dispatch's need is at most the retain threshold
// (..._SCRATCH_LIMIT_CURRENT = 24 GiB by default), keeps it assigned to the queue sized for a
// full-device dispatch whatever the grid: frame bytes per lane x 64 lanes x 32 wave slots x CUs
// (one 64-lane wave with a 5,216-byte frame took 2.74 GB; a queue that later needs a bigger
// frame gives its block back and takes a bigger one).  Needs above the threshold are "use once":
// sized to the dispatch's own grid and released after it.  With ten queues each retaining up to
// the largest frame routed to it, the pool can run out (or fragment) while every queue is busy:
// HSA_STATUS_ERROR_OUT_OF_RESOURCES, a dead queue.  The plan picks the
// largest threshold T (one of the kernels' frames, never above the runtime's default) with
//   queues x T x lane_slots  +  largest frame above T x lane_slots  <=  pool
// and T at least every frame the engine does NOT gate (`gated`, r06): a frame above T runs
// use-once, and the engine's use-once gate (mbls_scratch.h UseOnce) keeps the use-once blocks
// live at once -- on any queues, from any callers -- within pool - queues x T, which the second
// term shows holds the largest one.  So every queue retaining the largest frame it may keep AND
// every admitted use-once block together stay within the pool.  No such T (too many queues for
// the ungated frames, or one full-device frame above the pool): not safe, and the engine refuses
// to initialise rather than run unguarded.  gated == nullptr: every kernel is gated.
struct ScratchPlan {
  uint64_t retain = 0;          // threshold (bytes per queue) to run the device with
  uint64_t worst_retained = 0;  // queues x largest retained per-queue need
  uint64_t worst_use_once = 0;  // one full-device use-once dispatch of the largest frame above it
  uint32_t max_frame = 0;       // largest frame (bytes per lane) of any kernel
  uint32_t max_retained_frame = 0;
  bool safe = false;
};
inline ScratchPlan plan_scratch(uint64_t pool, uint64_t retain_default, uint32_t queues, uint64_t lane_slots,
                                const uint32_t* frames, const uint8_t* gated, uint32_t n) {
  ScratchPlan p;
  uint32_t ungated = 0;  // the threshold must keep these retained: the gate never sees them
  for (uint32_t i = 0; i < n; ++i) {
    p.max_frame = std::max(p.max_frame, frames[i]);
    if (gated && !gated[i]) ungated = std::max(ungated, frames[i]);
  }
  // candidates: 0 (nothing retained) and every frame, largest feasible wins
  bool found = false;
  uint32_t best = 0;
  for (uint32_t i = 0; i <= n; ++i) {
    const uint32_t c = i < n ? frames[i] : 0u;
    const uint64_t need = (uint64_t)c * lane_slots;
    if (c < ungated) continue;
    if (need > retain_default) continue;  // the plan only ever lowers the runtime's threshold
    const uint64_t once = p.max_frame > c ? (uint64_t)p.max_frame * lane_slots : 0;
    if ((uint64_t)queues * need + once <= pool && (!found || c > best)) {
      best = c;
      found = true;
    }
  }
  p.max_retained_frame = best;
  p.retain = (uint64_t)best * lane_slots;
  p.worst_retained = (uint64_t)queues * p.retain;
  p.worst_use_once = p.max_frame > best ? (uint64_t)p.max_frame * lane_slots : 0;
  p.safe = found;
  return p;
}

}  // namespace mbls_host
