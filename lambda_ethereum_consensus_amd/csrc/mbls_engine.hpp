// mbls_engine.hpp -- internal to libmbls: the engine state shared by the two host translation
// units of the engine -- mbls_engine.cpp (registry, lifecycle, host staging, layer 1, the C ABI)
// and mbls_pipeline.cpp (the layer-2 FAV / verify / aggregate_verify pipelines with their
// deferral and fill state machines, split out in r06).  Not installed; include/mbls.h is the API.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mbls.h"
#include "mbls_av6.h"
#include "mbls_host.hpp"
#include "mbls_kernels.h"
#include "mbls_scratch.h"

namespace mbls_launch {  // (mbls_k_g1.hip; declared here so that mbls_kernels.h, which every kernel
                         // translation unit includes, stays unchanged)
hipError_t copy_u32(uint32_t* dst, const uint32_t* src, uint32_t n, hipStream_t s);
}

namespace mbls_eng {

using namespace mbls_host;

// BLS12-381 group order r, big-endian
constexpr uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                              0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                              0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    want = want + want / 4;  // grow with slack
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Engine-owned device scratch of the layer-2 entry points that do not run the FAV pipeline
// (aggregate_verify, aggregate_pubkeys, validate_pubkeys, signature aggregation, table
// builds).  Users on different caller streams are ordered through Engine::ev_scratch.
enum Slot { S_KEY_ST, S_KEY_XY, S_SET_ST, S_SET_XY, S_SIG_ST, S_SIG_XY, S_H_XY, S_FPAIR, S_FSIG, S_GRP_OFF, S_NSLOTS };

// Per-call state of the pipelined fast_aggregate_verify path (a ring of them), so that the
// G2-side chain of call i (on a G2 stream) overlaps the key validation of calls i+1, i+2, ...
struct FavStage {
  DevBuf set_st, set_xy, sig_st, sig_xy, h_xy, fsig;
  DevBuf key_st, key_xy;  // cold keys decoded for this call (aggregated on the G2 stream)
  DevBuf rlc_cand, rlc_p, rlc_q, rlc_qtmp, rlc_fr, rlc_frtmp, rlc_ok;  // MBLS_FAV_RLC only
  // engine-owned copies of a deferred verdict's caller inputs (key counts, pre-status), made
  // on the call's G2 stream at call time: the launch that comes later reads only these
  DevBuf off_copy, pre_copy;
  DevBuf fpk;  // key-side Miller values of the split latency chain (lane layout, as fsig)
  hipEvent_t ev_g1 = nullptr, ev_done = nullptr, ev_pre = nullptr;
  bool pending = false;  // ev_done recorded and not yet known complete
  void release() {
    for (DevBuf* b : {&set_st, &set_xy, &sig_st, &sig_xy, &h_xy, &fsig, &key_st, &key_xy, &rlc_cand, &rlc_p, &rlc_q,
                      &rlc_qtmp, &rlc_fr, &rlc_frtmp, &rlc_ok, &off_copy, &pre_copy, &fpk})
      b->release();
    for (hipEvent_t* ev : {&ev_g1, &ev_pre, &ev_done}) {
      if (*ev) (void)hipEventDestroy(*ev);
      *ev = nullptr;
    }
    pending = false;
  }
};

// A layer-1 (host-binary) call's staging: pinned host buffers the binaries are packed into,
// the device copies of the inputs, the status / bytes the call returns, and the event that
// completes the call.  An engine holds kCtx of them, so that many calls are in flight.
enum HSlot { H_PKS, H_MSGS, H_SIGS, H_KPRE, H_SPRE, H_SETPRE, H_OFF, H_IDX, H_STATUS, H_BYTES, H_COUNT };
enum CSlot { C_PKS, C_MSGS, C_SIGS, C_KPRE, C_SPRE, C_SETPRE, C_OFF, C_IDX, C_STATUS, C_BYTES, C_NSLOTS };
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
};
struct CallCtx {
  HostBuf h[H_COUNT];
  DevBuf d[C_NSLOTS];
  hipEvent_t done = nullptr;
  bool busy = false;
  void release() {
    for (auto& b : h) {
      if (b.p) (void)hipHostFree(b.p);
      b.p = nullptr;
      b.cap = 0;
    }
    for (auto& b : d) b.release();
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
  }
};

struct Engine {
  std::mutex mu;  // enqueue order and engine state; never held across a GPU wait of a call
  bool ready = false;
  int want_device = -1;  // ordinal requested by mbls_init / mbls_init_devices
  int device = -1;
  hipStream_t stream = nullptr;  // default engine stream (keys, layer-1 uploads)
  // G1 side (key validation / table gather + per-set sums) of latency-critical FAV calls, off
  // the caller stream: the caller stream then holds only the caller's own work, so the next
  // call's input event does not wait for this call's keys (one mainnet block: the sync
  // aggregate's G2 chain no longer starts 2.7 ms late behind the attestations' key kernel)
  hipStream_t kstream = nullptr;  // the last G2 stream when the pool has one to spare, else `stream`
  // A second key stream (the G2 stream before kstream, same CU mask) when the pool has two to
  // spare: consecutive latency calls alternate between them, so a small call's keys (the
  // 512-key sync aggregate of a mainnet block) validate beside a large call's instead of
  // after it (r03: the sync aggregate's chain waited 3 ms behind the attestations' key grid).
  hipStream_t kstream2 = nullptr;
  int ks_rr = 0;
  int warm_rr = 0;  // pipelined table calls: G2 stream rotation over the lane-group pool + kstream2
  int n_lg = 0;                    // G2 streams the lane-group calls rotate over (key streams excluded)
  int kstream_cus = 0;             // CUs kstream's mask leaves to key kernels (0: unmasked)
  // G2-side streams (signature decode, H(m), Miller loops, verdicts), overlapped with the G1
  // pipeline on the caller stream.  One per remaining hardware queue: the per-set G2 chain
  // of a FAV call is latency bound (~3x the key-validation time of its batch), so the number
  // of calls whose chains run side by side is what bounds FAV throughput.
  static constexpr int kMaxG2 = 15;
  hipStream_t g2[kMaxG2] = {};
  int n_g2 = 0;
  hipEvent_t ev_in = nullptr, ev_aux = nullptr;
  hipEvent_t ev_join[kMaxG2 + 2] = {};  // mbls_dev_stream_wait_engine
  hipEvent_t ev_scratch = nullptr;      // last layer-2 user of buf[] (ordered across streams)
  bool scratch_used = false;
  DevBuf buf[S_NSLOTS];
  // ring of per-call FAV states, one more than the G2 streams so that every stream can hold a
  // call in flight while the caller stream validates the next batch's keys
  static constexpr int kMaxFavStages = kMaxG2 + 1;
  FavStage fav[kMaxFavStages];
  int n_fav = 0;
  int fav_parity = 0;
  int g2_rr = 0;  // next G2-side stream of the FAV pipeline
  int av_rr = 0;  // next stream triple of the pipelined aggregate_verify path (dev_av)
  // One-lane pairing kernels (Bls.verify batches, cold FAV verdicts) rotate over at most
  // kScratchStreams G2 streams: they carry ~11 KB of scratch per lane, the runtime reserves
  // scratch per hardware queue for a full-occupancy dispatch, and more than three such queues
  // at once exhausts it (HSA_STATUS_ERROR_OUT_OF_RESOURCES with 8 queues, r01).
  static constexpr int kScratchStreams = 3;  // default; MBLS_SCRATCH_STREAMS overrides
  int n_scratch = kScratchStreams;
  int scratch_rr = 0;
  int key_rr = 0;  // MBLS_KEY_STREAMS=2: which stream carries this cold call's G1 side
  hipStream_t aux() const { return g2[0]; }
  // layer-1 call contexts (pipelining): kCtx calls of this engine may be in flight at once
  static constexpr int kCtx = 3;
  CallCtx ctx[kCtx];
  std::mutex ctx_mu;
  std::condition_variable ctx_cv;
  int inflight = 0;  // layer-1 calls enqueued and not yet complete (guarded by mu)
  // validator pubkey table: validated affine keys resident in HBM,
  // AoS rows of 32 dwords, one status word per row
  struct {
    int32_t* st = nullptr;
    uint32_t* aff = nullptr;
    uint32_t n = 0, cap = 0;
  } tab;
  // RCCL communicator of the one-process-per-GPU job: only the sharded
  // pubkey-table build exchanges data; verification never does
  ncclComm_t comm = nullptr;
  int comm_rank = 0, comm_world = 1;
  bool comm_broken = false;  // an aborted collective may never finish: teardown skips the drains
  // A cold one-lane FAV call's verdict kernel, not yet launched (flush_verdict): its form is
  // chosen by what the engine sees next -- another FAV / verify call (more key work for the
  // long one-lane chain to hide behind: one lane per set) or anything else, e.g. a
  // synchronize (the caller now waits for this verdict: lane groups, ~3x lower latency).
  // A pipelined table call leaves its whole G2 side -- prep and joint verdict -- the same way
  // (r04): another call next -> the throughput prep (one lane per set); anything else -> the
  // lane-group prep, whose chain is about half as long (the chain the caller waits for at the end
  // of a pipelined run); the 6-lane joint verdict either way.
  struct {
    bool active = false;
    bool table = false;         // a table call's G2 side (prep + joint verdict)
    bool prep_onelane = false;  // table: its throughput prep is the one-lane form (not filling)
    const uint8_t* sigs = nullptr;  // table: the caller's inputs (read by the deferred prep)
    const uint8_t* msgs = nullptr;
    const int32_t* sig_pre = nullptr;
    const uint32_t* key_off = nullptr;  // table: the caller's index offsets and prechecks
    const int32_t* set_pre = nullptr;
    int stage = 0;
    hipStream_t ax = nullptr;
    bool has_pre = false;       // set_pre was given (copied into the stage's pre_copy)
    int32_t* status = nullptr;  // the caller's; must stay allocated until results are observed
    uint32_t n_sets = 0;
    int32_t eth = 0;
  } defer;
  int32_t defer_rc = 0;  // a failed deferred launch, reported by the next synchronize
  mbls_scratch_plan_t scratch{};  // the device's scratch plan (mbls_scratch.cpp)
};

// ---------------------------------------------------------------- registry (mbls_engine.cpp)
std::vector<Engine*> engines();  // every engine of the process
Engine& eng();                   // the calling thread's layer-2 engine (mbls_dev_select)
int32_t init_locked(Engine& e, int32_t device);

// Which form each FAV / verify call took (read through mbls_prof_read by name, counted while
// profiling is on): the forced-form parity tests assert that an MBLS_* knob selected the form
// for EVERY call (no knob may select a path its tests do not pin).
enum PathId {
  P_PREP_1L_TABLE,   // pipelined table call: one-lane fused prep (MBLS_WARM_PREP default)
  P_PREP_LG,         // lane-group prep (latency calls, small batches, MBLS_WARM_PREP=lg)
  P_PREP_1L_COLD,    // one-lane cold call: fused one-lane prep
  P_MILLER_SPLIT,    // signature-side Miller loop in its own kernel
  P_MILLER_JOINT,    // both Miller loops in the verdict (shared squarings)
  P_KEY_ALT,         // cold one-lane call's key side on the alternate stream (MBLS_KEY_STREAMS=2)
  P_VERIFY_KEY_ALT,  // verify call's key decode on the alternate stream (default; MBLS_KEY_STREAMS=1 off)
  P_LAT_KSTREAM2,    // latency call's key side on the second key stream (MBLS_LAT_KEY_STREAMS=1 off)
  P_WARM_FILL,       // pipelined table call during the pipeline fill: lane-group prep (MBLS_WARM_FILL)
  P_WARM_DEFER,      // pipelined table call whose G2 side (prep + joint verdict) was deferred (MBLS_DEFER_VERDICT)
  P_AV_GROUPED,      // aggregate_verify on 6-lane groups, joint Miller loops over groups of pairs (MBLS_AV_FORM=grouped)
  P_AV_ONELANE,      // aggregate_verify, the key pairs one lane per couple (default)
  P_PREP_SPLIT,      // one-lane prep as the two-wave hash + decode kernels (MBLS_PREP_SPLIT; verify default)
  P_AV_PIPELINED,    // aggregate_verify on its own FAV stage + G2 stream triple (r05 cross-call pipeline)
  P_COUNT
};
extern const char* const kPathNames[P_COUNT];
extern std::atomic<uint64_t> g_path[P_COUNT];
void path(PathId p);

#define MBLS_TRY(x)                                   \
  do {                                                \
    if ((x) != hipSuccess) return MBLS_ERR_DEVICE;    \
  } while (0)
#define MBLS_ENSURE(slot, bytes)                      \
  do {                                                \
    if (!e.buf[slot].ensure(bytes)) return MBLS_ERR_DEVICE; \
  } while (0)

inline hipStream_t pick(Engine& e, void* s) { return s ? static_cast<hipStream_t>(s) : e.stream; }

// Every dispatch of a kernel whose frame lies above the device's retain threshold goes through
// the device's use-once gate (mbls_scratch.h): `launch` runs with the gate held.
template <class F>
hipError_t use_once(mbls_scratch::UseOnceKernel k, uint64_t n, hipStream_t s, F&& launch) {
  mbls_scratch::UseOnce g(k, (n + 63) / 64 * 64, s);
  if (g.rc != hipSuccess) return g.rc;
  return g.done(launch());
}


enum : int { PREP_VERIFY = 1, PREP_COLD = 2, PREP_TABLE = 4 };
hipError_t launch_prep_1l(int kind, const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n,
                          int32_t* sig_st, uint32_t* sig_xy, uint32_t* hxy, hipStream_t s);

// ------------------------------------------- the layer-2 pipelines (mbls_pipeline.cpp) ----
int32_t flush_verdict(Engine& e, bool more);

// The engine lock.  Taking it first launches a deferred verdict (flush_verdict), in its
// latency form unless the holder is about to enqueue more FAV / verify work (`more`); a failed
// launch is kept in e.defer_rc for the next synchronize.
struct EngineLock {
  std::lock_guard<std::mutex> g;
  explicit EngineLock(Engine& e, bool more = false) : g(e.mu) { (void)flush_verdict(e, more); }
};


int32_t scratch_begin(Engine& e, hipStream_t st);
int32_t scratch_end(Engine& e, hipStream_t st);
uint32_t hash_lg_max();
bool defer_ok();

// Where a FAV call's keys come from: packed wire encodings (cold: decode + KeyValidate every
// key, as the reference NIF does) or rows of the validator pubkey table (warm).
struct G1Src {
  const uint8_t* pks = nullptr;  // cold: n_keys x 48 B, sets by key_off
  const int32_t* key_pre = nullptr;
  const uint32_t* idx = nullptr;  // warm: table rows, sets by key_off
};

int32_t dev_fav(Engine& e, const G1Src& src, const uint32_t* key_off, uint32_t n_keys, const uint8_t* msgs,
                const uint8_t* sigs, uint32_t n_sets, int32_t flags, const int32_t* sig_pre, const int32_t* set_pre,
                int32_t* status, hipStream_t st, hipEvent_t* done = nullptr, bool latency = false,
                hipStream_t* tail = nullptr, bool may_defer = false);
int32_t dev_verify(Engine& e, const uint8_t* pks, const uint8_t* msgs, const uint8_t* sigs, uint32_t n_sets,
                   const int32_t* key_pre, const int32_t* sig_pre, const int32_t* set_pre, int32_t* status,
                   hipStream_t st, hipEvent_t* done = nullptr, hipStream_t* tail = nullptr);
int32_t dev_av(Engine& e, const uint8_t* pks, const uint8_t* msgs, const uint32_t* key_off, uint32_t n_pairs,
               const uint8_t* sigs, uint32_t n_sets, const int32_t* key_pre, const int32_t* sig_pre,
               const int32_t* set_pre, int32_t* status, hipStream_t st, bool join);
int32_t dev_agg_pks(Engine& e, const uint8_t* pks, const uint32_t* key_off, uint32_t n_keys, uint32_t n_sets,
                    const int32_t* key_pre, uint8_t* out48, int32_t* status, hipStream_t st);

}  // namespace mbls_eng
