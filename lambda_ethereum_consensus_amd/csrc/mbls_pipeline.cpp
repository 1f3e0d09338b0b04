// mbls_pipeline.cpp -- the layer-2 pipelines of libmbls (split from mbls_engine.cpp, r06):
// fast_aggregate_verify (cold keys or the validator table), Bls.verify batches and
// aggregate_verify, each enqueued over the engine's key and G2 streams with a ring of per-call
// stages, and the state machines that decide a call's forms when the engine sees what follows:
// the deferred verdict / G2 side (Engine::defer, flush_verdict) and the pipelined table path's
// fill.  DESIGN.md §3 "Which form where"; the callers (layer 1 and the mbls_dev_* entries) are
// in mbls_engine.cpp.
#include "mbls_engine.hpp"

namespace mbls_eng {

// The one-lane G2 prep (signature decode + H(m)): one fused launch at one wave per SIMD, or
// the two-wave hash and decode kernels back to back.  MBLS_PREP_SPLIT is a mask of the call
// kinds that split (1 verify batches, 2 cold FAV, 4 table FAV); default 1.  Measured r05
// (profiles/r05_ab_prep_split.txt): gossip 1.44M -> 1.48-1.50M verify/s (throughput-bound: the
// two-wave waves share SIMDs), the cold epoch even, the pipelined table epoch -33% (its calls
// are bound by the G2 chain's latency, which the shared SIMDs lengthen).
hipError_t launch_prep_1l(int kind, const uint8_t* sigs, const int32_t* sig_pre, const uint8_t* msgs, uint32_t n,
                          int32_t* sig_st, uint32_t* sig_xy, uint32_t* hxy, hipStream_t s) {
  static const int split = [] {
    const char* v = std::getenv("MBLS_PREP_SPLIT");
    return v ? std::atoi(v) : int(PREP_VERIFY);
  }();
  if (split & kind) path(P_PREP_SPLIT);
  if (!(split & kind)) return mbls_launch::g2_prep_1l(sigs, sig_pre, msgs, n, sig_st, sig_xy, hxy, s);
  return use_once(mbls_scratch::UO_HASH_TO_G2, n, s, [&] {
    return mbls_launch::g2_prep_split(sigs, sig_pre, msgs, n, sig_st, sig_xy, hxy, s);
  });
}

// Launch the deferred verdict of the last cold FAV call (Engine::defer): one lane per set when
// more FAV / verify work follows (`more`), else the lane-group form (the call is the last in
// flight and its caller is about to wait: measured, cold epoch at 20 steps, the one-lane tail
// of the last call was ~40 ms of drain).  A deferred table call: its prep in the one-lane form
// when more work follows (the lane-group form while the pipeline fills), else in the lane-group
// form, then its 6-lane joint verdict.  Caller holds e.mu.
int32_t flush_verdict(Engine& e, bool more) {
  if (!e.defer.active) return 0;
  const auto d = e.defer;
  e.defer.active = false;
  FavStage& f = e.fav[d.stage];
  // a cold call's key_off / set_pre were copied into the stage when the call was enqueued; a
  // table call's are read where the caller left them, like its signatures and messages
  const uint32_t* key_off = d.table ? d.key_off : f.off_copy.as<uint32_t>();
  const int32_t* set_pre = d.table ? d.set_pre : d.has_pre ? f.pre_copy.as<int32_t>() : nullptr;
  hipError_t rc = hipSetDevice(e.device);
  if (rc == hipSuccess && d.table) {
    const bool onelane = more && d.prep_onelane;
    path(onelane ? P_PREP_1L_TABLE : P_PREP_LG);
    rc = onelane ? launch_prep_1l(PREP_TABLE, d.sigs, d.sig_pre, d.msgs, d.n_sets, f.sig_st.as<int32_t>(),
                                f.sig_xy.as<uint32_t>(), f.h_xy.as<uint32_t>(), d.ax)
                 : mbls_launch::g2_prep_lg(d.sigs, d.sig_pre, d.msgs, d.n_sets, f.sig_st.as<int32_t>(),
                                           f.sig_xy.as<uint32_t>(), f.h_xy.as<uint32_t>(), nullptr, d.ax);
    if (rc == hipSuccess) rc = hipStreamWaitEvent(d.ax, f.ev_g1, 0);  // the per-set key sums
    // (the 6-lane joint verdict either way: the 16-lane joint form is hardly shorter -- 4.9 vs
    // 5.5 ms per 2,048 sets -- for 2.2x the SIMD time, r04)
    if (rc == hipSuccess)
      rc = mbls_launch::fav_verdict_lg(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), key_off,
                                       f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), nullptr, f.h_xy.as<uint32_t>(),
                                       d.n_sets, d.eth, set_pre, nullptr, d.status, d.ax, /*fsig_onelane=*/0);
  } else if (rc == hipSuccess)
    rc = more ? use_once(mbls_scratch::UO_FAV_VERDICT, d.n_sets, d.ax,
                         [&] {
                           return mbls_launch::fav_verdict(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), key_off,
                                                           f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(),
                                                           f.fsig.as<uint32_t>(), f.h_xy.as<uint32_t>(), d.n_sets,
                                                           d.eth, set_pre, d.status, d.ax);
                         })
              : mbls_launch::fav_verdict_lg(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), key_off,
                                            f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), f.fsig.as<uint32_t>(),
                                            f.h_xy.as<uint32_t>(), d.n_sets, d.eth, set_pre, nullptr, d.status,
                                            d.ax, /*fsig_onelane=*/1);
  if (rc == hipSuccess) rc = hipEventRecord(f.ev_done, d.ax);
  if (rc != hipSuccess) {
    e.defer_rc = MBLS_ERR_DEVICE;
    return MBLS_ERR_DEVICE;
  }
  return 0;
}

// Layer-2 users of the engine scratch buf[] on possibly different caller streams: each waits
// for the previous user's work and marks its own end.
int32_t scratch_begin(Engine& e, hipStream_t st) {
  if (e.scratch_used) MBLS_TRY(hipStreamWaitEvent(st, e.ev_scratch, 0));
  return 0;
}
int32_t scratch_end(Engine& e, hipStream_t st) {
  MBLS_TRY(hipEventRecord(e.ev_scratch, st));
  e.scratch_used = true;
  return 0;
}
// ---------------------------------------------------------------- layer 2 internals ----

// Above this many messages per call, hash_to_G2 always runs one lane per message (enough
// waves to fill the GPU).  MBLS_HASH_LG_MAX overrides.
uint32_t hash_lg_max() {
  static const uint32_t v = [] {
    const char* s = std::getenv("MBLS_HASH_LG_MAX");
    return s ? (uint32_t)std::strtoul(s, nullptr, 10) : 8192u;
  }();
  return v;
}

// MBLS_DEFER_VERDICT=0 launches every verdict right away (the r01 behaviour; Engine::defer)
bool defer_ok() {
  static const bool on = [] {
    const char* v = std::getenv("MBLS_DEFER_VERDICT");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  return on;
}

// fast_aggregate_verify pipeline.  Each call runs on two streams:
//   st : key decode + validation (the dominant, throughput-bound kernel) or the table gather,
//        per-set aggregation
//   g2 : signature decode + G2 membership, H(m), signature-side Miller loop (no key input),
//        then -- once the aggregate keys exist -- key-side Miller loop x signature-side value,
//        final exponentiation, verdict (optionally the RLC batch check first).
// g2 rotates over the engine's G2 streams (one per remaining hardware queue), so the
// latency-bound per-set chains of that many calls run side by side on the SIMDs the key
// waves leave.  Per-call buffers live in a ring of FavStages; reuse of a stage waits for its
// previous verdict (ev_done).  `done` (optional) receives the event that completes this
// call's status, `tail` the stream it is recorded on (a layer-1 call appends its status
// download there, so the caller stream is not held behind this call's verdict).
int32_t dev_fav(Engine& e, const G1Src& src, const uint32_t* key_off, uint32_t n_keys, const uint8_t* msgs,
                const uint8_t* sigs, uint32_t n_sets, int32_t flags, const int32_t* sig_pre, const int32_t* set_pre,
                int32_t* status, hipStream_t st, hipEvent_t* done, bool latency,
                hipStream_t* tail, bool may_defer) {
  const int32_t eth = flags & MBLS_FAV_ETH;
  const bool rlc = (flags & MBLS_FAV_RLC) != 0;
  // The G2 chain is the critical path for table keys, or for few enough cold keys that their
  // validation is short: then signature decode (+ its Miller loop) and H(m) run side by side
  // on lane groups in one launch (mbls_k_g2_prep_lg).  Behind a long key validation the
  // one-lane forms cost fewer instructions and hide anyway.  Measured r01: warm epoch
  // 198k -> 255k sets/s with the lane-group hash, cold epoch 75k -> 72k (so not there).
  // A synchronous host call with nothing else in flight (`latency`) waits for its own
  // verdicts: its G2 chain is critical too.
  // MBLS_G2_CRITICAL_KEYS moves the cold-key threshold (tests force the one-lane path with 0).
  static const uint32_t critical_keys = [] {
    const char* v = std::getenv("MBLS_G2_CRITICAL_KEYS");
    return v ? (uint32_t)std::strtoul(v, nullptr, 10) : (1u << 18);
  }();
  const bool g2_critical = (latency || src.idx != nullptr || n_keys <= critical_keys) && n_sets <= hash_lg_max();
  // Table (warm) calls decode the signatures and hash the messages one lane per set, both in one
  // launch (mbls_k_g2_prep_1l: 64 waves per 2,048 sets instead of 512 lane-group waves that each
  // run the square roots 8x redundantly), keeping the lane-group verdict.  A pipelined warm epoch
  // is bound by SIMD time (the lane-group prep was ~60% of it) and by the G2 streams' time per
  // call.  Measured r03 (20 steps, profiles/r03_warm_prep_ab.txt): 610k -> 756k sets/s, cold
  // epoch unchanged.  MBLS_WARM_PREP=lg restores the lane-group prep (g2_prep_lg).
  static const bool warm_onelane_prep = [] {
    const char* v = std::getenv("MBLS_WARM_PREP");
    return !(v && std::strcmp(v, "lg") == 0);
  }();
  // (throughput batches only: a small table batch -- a block's committees -- is latency bound,
  // and its lane-group prep is ~2x shorter than the one-lane H(m))
  const bool warm_pipelined = src.idx != nullptr && !latency && n_sets > 1024;
  // Pipeline fill (r04): while fewer than MBLS_WARM_FILL earlier calls are still in flight the
  // SIMDs are mostly idle (a one-lane prep is 64 waves per 2,048 sets for ~6 ms), so such a call
  // takes the lane-group prep: about half the latency for more SIMD time, which is free there.
  // 0 turns it off.  Default 1: thresholds 1 and 2 measured the same (979k vs 977-982k, A/B 8),
  // and lane-group preps in flight on several queues at once have hit the runtime's scratch
  // limit (HSA_STATUS_ERROR_OUT_OF_RESOURCES with 4, A/B 18; a deferral window of 2, A/B 11), so
  // at most one fill prep and the one tail prep of a run ever use that form.
  static const int warm_fill = [] {
    const char* v = std::getenv("MBLS_WARM_FILL");
    return v ? std::max(0, std::atoi(v)) : 1;
  }();
  bool filling = false;
  if (warm_onelane_prep && warm_pipelined && warm_fill > 0) {
    int busy = 0;
    for (int i = 0; i < e.n_fav && busy < warm_fill; ++i)
      if (e.fav[i].pending && hipEventQuery(e.fav[i].ev_done) == hipErrorNotReady) ++busy;
    filling = busy < warm_fill;
    if (filling) path(P_WARM_FILL);
  }
  const bool prep_onelane = warm_onelane_prep && warm_pipelined && !filling;
  // Verdict behind a long key validation (cold, not critical, exact): one lane per set, the
  // signature-side Miller loop in its own kernel ahead of the key wait.  A lane group holds a
  // SIMD's registers for 8x the lanes (and issues 2.3x the instructions) while the key waves
  // are what bounds the step; the one-lane chain is long but the calls' chains overlap on the
  // G2 streams.  Measured r01 (epoch step, 4 queues): lane groups 76.6k, one lane 84.5k sets/s.
  // MBLS_FAV_VERDICT=lg keeps lane groups.
  static const bool one_lane_ok = [] {
    const char* v = std::getenv("MBLS_FAV_VERDICT");
    return !(v && std::strcmp(v, "lg") == 0);
  }();
  const bool one_lane = one_lane_ok && !g2_critical && !rlc;
  const int stage = e.fav_parity;
  FavStage& f = e.fav[stage];
  e.fav_parity = (e.fav_parity + 1) % e.n_fav;
  hipStream_t ax;
  if (one_lane) {
    ax = e.g2[e.scratch_rr];
    e.scratch_rr = (e.scratch_rr + 1) % e.n_scratch;
  } else if (warm_onelane_prep && warm_pipelined && e.kstream2) {  // (filling or not: one rotation)
    // pipelined table calls also rotate over the second latency key stream (idle outside cold
    // latency calls): their chain (one-lane prep, lane-group verdict) holds a stream ~14 ms per
    // 2,048-set call, so the number of streams bounds the warm epoch's rate
    ax = e.warm_rr < e.n_lg ? e.g2[e.warm_rr] : e.kstream2;
    e.warm_rr = (e.warm_rr + 1) % (e.n_lg + 1);
  } else {
    ax = e.g2[e.g2_rr];
    e.g2_rr = (e.g2_rr + 1) % e.n_lg;
  }
  if (tail) *tail = ax;
  if (!f.set_st.ensure(sizeof(int32_t) * n_sets) || !f.set_xy.ensure(sizeof(uint32_t) * 42 * n_sets) ||
      !f.sig_st.ensure(sizeof(int32_t) * n_sets) || !f.sig_xy.ensure(sizeof(uint32_t) * 56 * n_sets) ||
      !f.h_xy.ensure(sizeof(uint32_t) * 56 * n_sets) || !f.fsig.ensure(sizeof(uint32_t) * 28 * 8 * n_sets))
    return MBLS_ERR_DEVICE;
  // G1 side on the caller stream: the table gather + per-set sums (warm), or the cold key
  // validation alone -- each call decodes into its stage's own key buffers and the per-set
  // aggregation runs on the G2 stream, so the caller stream runs the key kernels of
  // consecutive calls back to back (no aggregation bubble between them).
  MBLS_TRY(hipEventRecord(e.ev_in, st));
  // (a masked kstream only while the key grid fits one round of its CUs at 2 waves per SIMD:
  // a bigger grid would pay a partial extra round for the reserved CUs)
  const bool ks_fits = e.kstream_cus == 0 || (uint64_t)(n_keys + 63) / 64 <= (uint64_t)e.kstream_cus * 8;
  if (g2_critical && !rlc && e.kstream != st && ks_fits) {  // G1 side on the engine's key stream
    st = e.kstream;
    // (cold keys only: a table gather is short, and the warm epoch's 2,048-set calls gained
    // nothing from the second stream, r03)
    if (e.kstream2 && !src.idx && (e.ks_rr ^= 1)) {
      st = e.kstream2;
      path(P_LAT_KSTREAM2);
    }
    MBLS_TRY(hipStreamWaitEvent(st, e.ev_in, 0));
  }
  if (f.pending) MBLS_TRY(hipStreamWaitEvent(st, f.ev_done, 0));
  // MBLS_MILLER=split|joint forces where the signature-side Miller loop runs (read once)
  static const int miller_env = [] {
    const char* v = std::getenv("MBLS_MILLER");
    return !v ? -1 : std::strcmp(v, "split") == 0 ? 1 : 0;
  }();
  const bool split = miller_env >= 0 ? miller_env == 1 : src.idx == nullptr;
  if (!one_lane) path(split ? P_MILLER_SPLIT : P_MILLER_JOINT);  // (one-lane calls always split)
  // A pipelined table call (layer 2) leaves its whole G2 side to the engine (Engine::defer,
  // flush_verdict): the gather runs now, the prep and the joint verdict when the engine sees what
  // follows.  Their inputs are the caller's (the documented lifetime: every path that may
  // overwrite or free them launches pending work first).
  if (may_defer && defer_ok() && warm_pipelined && !split && !rlc) {
    MBLS_TRY(mbls_launch::g1_aggregate_idx(e.tab.st, e.tab.aff, e.tab.n, src.idx, key_off, n_sets,
                                           f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), st));
    MBLS_TRY(hipEventRecord(f.ev_g1, st));
    MBLS_TRY(hipStreamWaitEvent(ax, e.ev_in, 0));
    if (f.pending) MBLS_TRY(hipStreamWaitEvent(ax, f.ev_done, 0));
    f.pending = true;
    e.defer.active = true;
    e.defer.table = true;
    e.defer.key_off = key_off;
    e.defer.set_pre = set_pre;
    e.defer.prep_onelane = prep_onelane;
    e.defer.sigs = sigs;
    e.defer.msgs = msgs;
    e.defer.sig_pre = sig_pre;
    e.defer.stage = stage;
    e.defer.ax = ax;
    e.defer.has_pre = set_pre != nullptr;
    e.defer.status = status;
    e.defer.n_sets = n_sets;
    e.defer.eth = eth;
    path(P_WARM_DEFER);
    return 0;
  }
  // A latency-critical call enqueues its G2 prep (signature decode + check + signature-side
  // Miller loop, H(m); lane groups, a whole SIMD per wave) BEFORE its key kernel: enqueued
  // after it, the prep waves wait until the key waves have left whole SIMDs free (one mainnet
  // block: the 1,024 key waves sit one per SIMD for ~1.9 ms).
  bool prep_done = false;
  // The latency chain split in three (r03, mbls_k_lg.hip): a cold latency-critical call runs
  // H(m) and then, once its key sums exist, the key-side Miller loop on a second lane-group
  // stream (hx), beside the signature chain (decode + check + signature-side Miller loop) on ax;
  // a final kernel on ax multiplies the two Miller values and exponentiates.  The key-side loop
  // no longer waits for the longer of the two prep chains.  MBLS_LAT_SPLIT=0: the fused prep
  // and one verdict kernel (r02).
  static const bool lat_split_ok = [] {
    const char* v = std::getenv("MBLS_LAT_SPLIT");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  hipStream_t hx = nullptr;
  if (lat_split_ok && g2_critical && !rlc && !src.idx && split && e.n_lg > 1) {
    hx = e.g2[e.g2_rr];
    if (hx == ax) {
      e.g2_rr = (e.g2_rr + 1) % e.n_lg;
      hx = e.g2[e.g2_rr];
    }
    e.g2_rr = (e.g2_rr + 1) % e.n_lg;
    if (!f.fpk.ensure(sizeof(uint32_t) * 28 * 8 * n_sets)) return MBLS_ERR_DEVICE;
  }
  if (g2_critical && !rlc && !prep_onelane) {
    path(P_PREP_LG);
    MBLS_TRY(hipStreamWaitEvent(ax, e.ev_in, 0));
    if (f.pending) MBLS_TRY(hipStreamWaitEvent(ax, f.ev_done, 0));
    if (hx) {
      MBLS_TRY(hipStreamWaitEvent(hx, e.ev_in, 0));
      if (f.pending) MBLS_TRY(hipStreamWaitEvent(hx, f.ev_done, 0));
      MBLS_TRY(mbls_launch::g2_prep_lg(sigs, sig_pre, msgs, n_sets, f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(),
                                       f.h_xy.as<uint32_t>(), f.fsig.as<uint32_t>(), ax, /*parts=*/2));
      MBLS_TRY(mbls_launch::g2_prep_lg(sigs, sig_pre, msgs, n_sets, f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(),
                                       f.h_xy.as<uint32_t>(), nullptr, hx, /*parts=*/1));
    } else {
      MBLS_TRY(mbls_launch::g2_prep_lg(sigs, sig_pre, msgs, n_sets, f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(),
                                       f.h_xy.as<uint32_t>(), split ? f.fsig.as<uint32_t>() : nullptr, ax));
    }
    prep_done = true;
  }
  // (the per-set sums stay on the key stream, right behind the key grid: on their own stream,
  // r03, the next key grid started at once but the queued one-lane G2 waves, which need whole
  // SIMDs, starved -- 82.3k vs 87.7k sets/s, profiles/r03_warm_prep_ab.txt)
  // MBLS_KEY_STREAMS=2: cold one-lane calls alternate their G1 side (key validation + per-set
  // sums) between the caller stream and the first G2 stream outside the scratch pool (idle in
  // this mode), so one call's key grid can fill the tail of the previous call's.  Off by
  // default: measured r01 (epoch, 2 x 50 steps) 80.0k vs 84.5k sets/s -- two key grids side by
  // side delay both calls' key sums and the one-lane verdict chains behind them.
  static const int key_streams = [] {
    const char* v = std::getenv("MBLS_KEY_STREAMS");
    return v ? std::max(1, std::min(2, std::atoi(v))) : 1;
  }();
  if (key_streams > 1 && one_lane && !src.idx && e.n_g2 > e.n_scratch) {
    e.key_rr ^= 1;
    if (e.key_rr) {
      path(P_KEY_ALT);
      hipStream_t kx = e.g2[e.n_scratch];
      MBLS_TRY(hipStreamWaitEvent(kx, e.ev_in, 0));
      if (f.pending) MBLS_TRY(hipStreamWaitEvent(kx, f.ev_done, 0));
      st = kx;
    }
  }
  if (src.idx) {
    MBLS_TRY(mbls_launch::g1_aggregate_idx(e.tab.st, e.tab.aff, e.tab.n, src.idx, key_off, n_sets,
                                           f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), st));
  } else {
    if (!f.key_st.ensure(sizeof(int32_t) * (size_t)std::max(n_keys, 1u)) ||
        !f.key_xy.ensure(sizeof(uint32_t) * 28 * (size_t)std::max(n_keys, 1u)))
      return MBLS_ERR_DEVICE;
    // (a persistent key grid taking 64-key chunks from an atomic counter was measured r03 and
    // removed: 86.8-87.4k vs 85.5-87.9k sets/s, its chunks are whole waves like the dispatcher's)
    MBLS_TRY(mbls_launch::g1_decode_validate(src.pks, n_keys, src.key_pre, f.key_st.as<int32_t>(),
                                             f.key_xy.as<uint32_t>(), st));
    MBLS_TRY(mbls_launch::g1_aggregate(f.key_st.as<int32_t>(), f.key_xy.as<uint32_t>(), n_keys, key_off, n_sets,
                                       f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), st));
  }
  MBLS_TRY(hipEventRecord(f.ev_g1, st));
  // G2 side: after the caller's inputs and after this stage's previous verdict
  MBLS_TRY(hipStreamWaitEvent(ax, e.ev_in, 0));
  if (f.pending) MBLS_TRY(hipStreamWaitEvent(ax, f.ev_done, 0));
  // join with the G1 side (once, before the first kernel that reads the per-set key sums)
  bool joined = false;
  auto g1_join = [&]() -> int32_t {
    if (joined) return 0;
    joined = true;
    MBLS_TRY(hipStreamWaitEvent(ax, f.ev_g1, 0));
    return 0;
  };
  // Cold keys (a long G1 side): the signature-side Miller loop runs ahead of the key wait,
  // leaving a short tail.  Table keys (a short gather): both loops in one 2-pair loop after the
  // gather (shared squarings, fewer instructions).  Measured r01 (epoch step): cold split
  // 74.9k vs joint 68.9k sets/s; warm joint 198k vs split 188k.  MBLS_MILLER=split|joint.
  bool fsig_done = false;
  if (prep_done) {
    fsig_done = true;
  } else {
    // (one-lane calls keep their signature decode + H(m) on the call's own G2 stream: on the
    // streams outside the scratch pool, r02, they lost -- 79.7-81.2k vs 86.2k sets/s,
    // profiles/r02_knob_sweep.txt)
    const hipStream_t px = ax;
    if (g2_critical && !prep_onelane) {
      path(P_PREP_LG);
      MBLS_TRY(
          mbls_launch::g2_sig_decode(sigs, n_sets, 1, sig_pre, f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), px));
      MBLS_TRY(mbls_launch::hash_to_g2_lg(msgs, n_sets, f.h_xy.as<uint32_t>(), px));
    } else {  // both one-lane chains side by side in one launch (mbls_k_g2_prep_1l)
      path(prep_onelane ? P_PREP_1L_TABLE : P_PREP_1L_COLD);
      MBLS_TRY(launch_prep_1l(prep_onelane ? PREP_TABLE : PREP_COLD, sigs, sig_pre, msgs, n_sets,
                            f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), f.h_xy.as<uint32_t>(), px));
    }
  }
  const int32_t* rlc_ok = nullptr;
  if (rlc) {
    // one combined pairing check over the batch; the per-set kernels below then only run
    // (on device, reading the flag) if it failed
    mbls_launch::RlcBufs b;
    const uint32_t nq = (n_sets + 63) / 64, nf = (n_sets + 16) / 16;
    if (!f.rlc_cand.ensure(sizeof(int32_t) * n_sets) || !f.rlc_p.ensure(sizeof(uint32_t) * 42 * n_sets) ||
        !f.rlc_q.ensure(sizeof(uint32_t) * 84 * n_sets) || !f.rlc_qtmp.ensure(sizeof(uint32_t) * 84 * nq) ||
        !f.rlc_fr.ensure(sizeof(uint32_t) * 28 * 8 * (n_sets + 1)) || !f.rlc_frtmp.ensure(sizeof(uint32_t) * 28 * 8 * nf) ||
        !f.rlc_ok.ensure(sizeof(int32_t)))
      return MBLS_ERR_DEVICE;
    b.cand = f.rlc_cand.as<int32_t>();
    b.p_xy = f.rlc_p.as<uint32_t>();
    b.q_xy = f.rlc_q.as<uint32_t>();
    b.q_tmp = f.rlc_qtmp.as<uint32_t>();
    b.fr = f.rlc_fr.as<uint32_t>();
    b.fr_tmp = f.rlc_frtmp.as<uint32_t>();
    b.ok = f.rlc_ok.as<int32_t>();
    uint32_t seed[8];
    std::random_device rd;  // per-call secret: the scalars must not be predictable
    for (uint32_t& w : seed) w = rd();
    if (int32_t r = g1_join()) return r;
    MBLS_TRY(mbls_launch::rlc_scale(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), key_off, f.sig_st.as<int32_t>(),
                                    f.sig_xy.as<uint32_t>(), n_sets, eth, set_pre, seed, b, ax));
    uint32_t* q_sum = nullptr;
    MBLS_TRY(mbls_launch::rlc_sum_g2(b.q_xy, b.q_tmp, n_sets, &q_sum, ax));
    MBLS_TRY(mbls_launch::rlc_check(b, f.h_xy.as<uint32_t>(), n_sets, q_sum, ax));
    rlc_ok = b.ok;
  }
  if (one_lane) {
    MBLS_TRY(mbls_launch::sig_miller(f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), n_sets, f.fsig.as<uint32_t>(),
                                     ax));
    if (int32_t r = g1_join()) return r;
    f.pending = true;
    // Only a layer-2 call (may_defer) leaves its verdict to the engine: its results are
    // observed through synchronize / join / copy, which launch it.  A layer-1 call enqueues its
    // status download on `ax` right after this and waits for it, so its verdict launches now
    // (a deferred host-batch verdict was downloaded before it had run).
    if (may_defer && defer_ok()) {
      // the later launch must not read caller memory that may be gone or rewritten by then
      if (!f.off_copy.ensure(sizeof(uint32_t) * ((size_t)n_sets + 1)) ||
          (set_pre && !f.pre_copy.ensure(sizeof(int32_t) * (size_t)n_sets)))
        return MBLS_ERR_DEVICE;
      MBLS_TRY(mbls_launch::copy_u32(f.off_copy.as<uint32_t>(), key_off, n_sets + 1, ax));
      if (set_pre)
        MBLS_TRY(mbls_launch::copy_u32(f.pre_copy.as<uint32_t>(), reinterpret_cast<const uint32_t*>(set_pre), n_sets,
                                       ax));
      e.defer.active = true;
      e.defer.table = false;
      e.defer.stage = stage;
      e.defer.ax = ax;
      e.defer.has_pre = set_pre != nullptr;
      e.defer.status = status;
      e.defer.n_sets = n_sets;
      e.defer.eth = eth;
      return 0;
    }
    MBLS_TRY(use_once(mbls_scratch::UO_FAV_VERDICT, n_sets, ax, [&] {
      return mbls_launch::fav_verdict(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), key_off, f.sig_st.as<int32_t>(),
                                      f.sig_xy.as<uint32_t>(), f.fsig.as<uint32_t>(), f.h_xy.as<uint32_t>(), n_sets,
                                      eth, set_pre, status, ax);
    }));
    MBLS_TRY(hipEventRecord(f.ev_done, ax));
    if (done) *done = f.ev_done;
    return 0;
  }
  if (hx) {  // split latency chain: key-side Miller loop on hx after H(m) and the key sums
    MBLS_TRY(hipStreamWaitEvent(hx, f.ev_g1, 0));
    MBLS_TRY(mbls_launch::key_miller_lg(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), f.h_xy.as<uint32_t>(), n_sets,
                                        f.fpk.as<uint32_t>(), hx));
    MBLS_TRY(hipEventRecord(f.ev_pre, hx));
    MBLS_TRY(hipStreamWaitEvent(ax, f.ev_pre, 0));
    MBLS_TRY(mbls_launch::fav_final_lg(f.set_st.as<int32_t>(), key_off, f.sig_st.as<int32_t>(), f.fsig.as<uint32_t>(),
                                       f.fpk.as<uint32_t>(), n_sets, eth, set_pre, status, ax));
    MBLS_TRY(hipEventRecord(f.ev_done, ax));
    f.pending = true;
    if (done) *done = f.ev_done;
    return 0;
  }
  if (split && !fsig_done)
    MBLS_TRY(mbls_launch::sig_miller_lg(f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), n_sets,
                                        f.fsig.as<uint32_t>(), rlc_ok, ax));
  if (int32_t r = g1_join()) return r;
  MBLS_TRY(mbls_launch::fav_verdict_lg(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), key_off,
                                       f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(),
                                       split ? f.fsig.as<uint32_t>() : nullptr, f.h_xy.as<uint32_t>(), n_sets, eth,
                                       set_pre, rlc_ok, status, ax, 0));
  MBLS_TRY(hipEventRecord(f.ev_done, ax));
  f.pending = true;
  if (done) *done = f.ev_done;
  return 0;
}

// Bls.verify batches, pipelined across calls like dev_fav: the keys are decoded on the caller
// stream into the call's stage, the signature decode, H(m) and the one-lane verdict (a
// 2-pair Miller loop with shared squarings per set: these batches are large, so one lane per
// set fills the GPU) run on the call's G2 stream, so consecutive calls overlap.
int32_t dev_verify(Engine& e, const uint8_t* pks, const uint8_t* msgs, const uint8_t* sigs, uint32_t n_sets,
                   const int32_t* key_pre, const int32_t* sig_pre, const int32_t* set_pre, int32_t* status,
                   hipStream_t st, hipEvent_t* done, hipStream_t* tail) {
  FavStage& f = e.fav[e.fav_parity];
  e.fav_parity = (e.fav_parity + 1) % e.n_fav;
  hipStream_t ax = e.g2[e.scratch_rr];
  e.scratch_rr = (e.scratch_rr + 1) % e.n_scratch;
  if (tail) *tail = ax;
  if (!f.set_st.ensure(sizeof(int32_t) * n_sets) || !f.set_xy.ensure(sizeof(uint32_t) * 42 * n_sets) ||
      !f.sig_st.ensure(sizeof(int32_t) * n_sets) || !f.sig_xy.ensure(sizeof(uint32_t) * 56 * n_sets) ||
      !f.h_xy.ensure(sizeof(uint32_t) * 56 * n_sets))
    return MBLS_ERR_DEVICE;
  MBLS_TRY(hipEventRecord(e.ev_in, st));
  // Consecutive calls alternate their key decode between the caller stream and the first G2
  // stream outside the scratch pool, so one call's 1,024 key waves fill the tail of the
  // previous call's.  Measured r01 (gossip, 2 x 50 steps): 893k vs 881k verify/s; the same
  // alternation loses on the cold FAV epoch (80k vs 84.5k), where it stays off.
  // MBLS_KEY_STREAMS=1 turns it off here, =2 turns it on in dev_fav too.
  hipStream_t ks = st;
  static const bool key2 = [] {
    const char* v = std::getenv("MBLS_KEY_STREAMS");
    return !v || std::atoi(v) >= 2;
  }();
  if (key2 && e.n_g2 > e.n_scratch && (e.key_rr ^= 1)) {
    path(P_VERIFY_KEY_ALT);
    ks = e.g2[e.n_scratch];
    MBLS_TRY(hipStreamWaitEvent(ks, e.ev_in, 0));
  }
  if (f.pending) MBLS_TRY(hipStreamWaitEvent(ks, f.ev_done, 0));
  MBLS_TRY(mbls_launch::g1_decode_validate(pks, n_sets, key_pre, f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), ks));
  MBLS_TRY(hipEventRecord(f.ev_g1, ks));
  MBLS_TRY(hipStreamWaitEvent(ax, e.ev_in, 0));
  if (f.pending) MBLS_TRY(hipStreamWaitEvent(ax, f.ev_done, 0));
  MBLS_TRY(launch_prep_1l(PREP_VERIFY, sigs, sig_pre, msgs, n_sets, f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(),
                        f.h_xy.as<uint32_t>(), ax));
  MBLS_TRY(hipStreamWaitEvent(ax, f.ev_g1, 0));
  // The verdict (a 2-pair Miller loop with shared squarings + final exponentiation per set) on
  // lane groups -- 6-lane groups for throughput batches, 16-lane for <= 1,024 sets -- or one lane
  // per set (MBLS_VERIFY_VERDICT=1l, the r03 form).  r04: since the trio Miller steps and the
  // LDS-staged Fp12 products the 6-lane joint verdict costs less SIMD time per set than the
  // one-lane one (0.53 vs 0.61 SIMD-ms), which bounds the gossip stream.
  static const bool verify_onelane = [] {
    const char* v = std::getenv("MBLS_VERIFY_VERDICT");
    return v && std::strcmp(v, "1l") == 0;
  }();
  if (verify_onelane)
    MBLS_TRY(use_once(mbls_scratch::UO_FAV_VERDICT, n_sets, ax, [&] {
      return mbls_launch::fav_verdict(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), nullptr, f.sig_st.as<int32_t>(),
                                      f.sig_xy.as<uint32_t>(), nullptr, f.h_xy.as<uint32_t>(), n_sets, 0, set_pre,
                                      status, ax);
    }));
  else
    MBLS_TRY(mbls_launch::fav_verdict_lg(f.set_st.as<int32_t>(), f.set_xy.as<uint32_t>(), nullptr,
                                         f.sig_st.as<int32_t>(), f.sig_xy.as<uint32_t>(), nullptr,
                                         f.h_xy.as<uint32_t>(), n_sets, 0, set_pre, nullptr, status, ax, 0));
  MBLS_TRY(hipEventRecord(f.ev_done, ax));
  f.pending = true;
  if (done) *done = f.ev_done;
  return 0;
}

// aggregate_verify batches.  The three inputs decode side by side: keys on the caller stream,
// H(m) (the longest: one lane per message) on the first G2 stream, the signatures -- and, in the
// default form, their Miller loops -- on the second (r04 ran the signature decode and H(m) one
// after the other on one stream and the signature-side Miller loop after the key pairs').
// Default: the key pairs' Miller loops one lane per pair couple (mbls_k_miller_pairs, shared
// squarings per couple), then per set the product with the signature-side value and the final
// exponentiation on a 6-lane group.  MBLS_AV_FORM=grouped (r05, csrc/mbls_k_av6.hip): a set's
// pairs, the signature pair first, in groups of four, one joint Miller loop per group on a 6-lane
// group; its frames are 588 B against 5,248 B, but it costs 23% more SIMD time per pair (r05:
// 48.8 vs 38.0 ms per 16,384 x 16 batch, profiles/r05_deposit_forms.txt): lane groups spread an
// Fp12 squaring or line product over six lanes at ~1.5x the one-lane arithmetic, which pays for
// latency-bound batches, not for this throughput-bound one.
//
// Pipelined (r05, the default form with >= 3 G2 streams): a call takes a stage of the FAV ring
// (its own buffers) and a triple of G2 streams -- keys then the signatures' decode + Miller loop
// on one, H(m) on the second, the pairs' Miller loops and the verdict on the third -- and forks
// from `st` only for the caller's inputs, so call i+1's keys and H(m) run beside call i's
// pairs and verdict; before, every call forked from `st` behind the previous call's verdict and
// the chip idled in each kernel's tail (deposit: the step equalled the sum of the kernels'
// alone-times).  `join` (layer 1: the status is downloaded on `st` next) orders the verdict
// before `st`'s later work; a layer-2 call leaves it to the engine's synchronize / join / copy,
// as a deferred FAV verdict.
int32_t dev_av(Engine& e, const uint8_t* pks, const uint8_t* msgs, const uint32_t* key_off, uint32_t n_pairs,
               const uint8_t* sigs, uint32_t n_sets, const int32_t* key_pre, const int32_t* sig_pre,
               const int32_t* set_pre, int32_t* status, hipStream_t st, bool join) {
  static const bool grouped = [] {
    const char* v = std::getenv("MBLS_AV_FORM");
    return v && std::strcmp(v, "grouped") == 0;
  }();
  if (!grouped && e.n_g2 >= 3) {
    path(P_AV_ONELANE);
    path(P_AV_PIPELINED);
    const size_t np = std::max(n_pairs, 1u);
    FavStage& f = e.fav[e.fav_parity];
    e.fav_parity = (e.fav_parity + 1) % e.n_fav;
    const int r = e.av_rr;
    e.av_rr = (e.av_rr + 1) % std::max(1, e.n_g2 / 3);
    const hipStream_t ks = e.g2[3 * r], hs = e.g2[3 * r + 1], ds = e.g2[3 * r + 2];
    if (!f.key_st.ensure(sizeof(int32_t) * np) || !f.key_xy.ensure(sizeof(uint32_t) * 28 * np) ||
        !f.sig_st.ensure(sizeof(int32_t) * n_sets) || !f.sig_xy.ensure(sizeof(uint32_t) * 56 * n_sets) ||
        !f.h_xy.ensure(sizeof(uint32_t) * 56 * np) || !f.fpk.ensure(sizeof(uint32_t) * 28 * 8 * np) ||
        !f.fsig.ensure(sizeof(uint32_t) * 28 * 8 * (size_t)n_sets))
      return MBLS_ERR_DEVICE;
    auto* key_st = f.key_st.as<int32_t>();
    auto* key_xy = f.key_xy.as<uint32_t>();
    auto* sig_st = f.sig_st.as<int32_t>();
    auto* sig_xy = f.sig_xy.as<uint32_t>();
    auto* h_xy = f.h_xy.as<uint32_t>();
    auto* fsig = f.fsig.as<uint32_t>();
    auto* fpair = f.fpk.as<uint32_t>();
    MBLS_TRY(hipEventRecord(e.ev_in, st));  // the caller's inputs
    for (hipStream_t s : {ks, hs}) {
      MBLS_TRY(hipStreamWaitEvent(s, e.ev_in, 0));
      if (f.pending) MBLS_TRY(hipStreamWaitEvent(s, f.ev_done, 0));  // the stage's previous user
    }
    MBLS_TRY(use_once(mbls_scratch::UO_HASH_TO_G2, n_pairs, hs,
                      [&] { return mbls_launch::hash_to_g2(msgs, n_pairs, h_xy, hs); }));
    MBLS_TRY(hipEventRecord(f.ev_pre, hs));
    MBLS_TRY(mbls_launch::g1_decode_validate(pks, n_pairs, key_pre, key_st, key_xy, ks));
    MBLS_TRY(mbls_launch::g2_sig_decode(sigs, n_sets, 1, sig_pre, sig_st, sig_xy, ks));
    MBLS_TRY(mbls_launch::sig_miller_lg(sig_st, sig_xy, n_sets, fsig, nullptr, ks));
    MBLS_TRY(hipEventRecord(f.ev_g1, ks));
    MBLS_TRY(hipStreamWaitEvent(ds, f.ev_g1, 0));
    MBLS_TRY(hipStreamWaitEvent(ds, f.ev_pre, 0));
    MBLS_TRY(mbls_launch::miller_pairs(key_st, key_xy, h_xy, n_pairs, key_off, n_sets, fpair, ds));
    MBLS_TRY(mbls_launch::av_verdict_lg(key_st, n_pairs, key_off, sig_st, fsig, fpair, n_sets, set_pre, status, ds));
    MBLS_TRY(hipEventRecord(f.ev_done, ds));
    f.pending = true;
    if (join) MBLS_TRY(hipStreamWaitEvent(st, f.ev_done, 0));
    return 0;
  }
  const size_t np = std::max(n_pairs, 1u);
  const size_t n_grp = mbls_launch::av_groups_bound(n_pairs, n_sets);
  MBLS_ENSURE(S_KEY_ST, sizeof(int32_t) * np);
  MBLS_ENSURE(S_KEY_XY, sizeof(uint32_t) * 28 * np);
  MBLS_ENSURE(S_SIG_ST, sizeof(int32_t) * (size_t)n_sets);
  MBLS_ENSURE(S_SIG_XY, sizeof(uint32_t) * 56 * (size_t)n_sets);
  MBLS_ENSURE(S_H_XY, sizeof(uint32_t) * 56 * np);
  MBLS_ENSURE(S_FPAIR, sizeof(uint32_t) * 28 * 8 * (grouped ? n_grp : np));
  if (!grouped) MBLS_ENSURE(S_FSIG, sizeof(uint32_t) * 28 * 8 * (size_t)n_sets);
  if (grouped) MBLS_ENSURE(S_GRP_OFF, sizeof(uint32_t) * ((size_t)n_sets + 1));
  auto* key_st = e.buf[S_KEY_ST].as<int32_t>();
  auto* key_xy = e.buf[S_KEY_XY].as<uint32_t>();
  auto* sig_st = e.buf[S_SIG_ST].as<int32_t>();
  auto* sig_xy = e.buf[S_SIG_XY].as<uint32_t>();
  auto* h_xy = e.buf[S_H_XY].as<uint32_t>();
  auto* fsig = e.buf[S_FSIG].as<uint32_t>();
  if (int32_t r = scratch_begin(e, st)) return r;
  path(grouped ? P_AV_GROUPED : P_AV_ONELANE);
  // fork: H(m) on g2[0], the signatures on g2[1] (when the pool has a second stream), keys here
  const hipStream_t hs = e.g2[0], ss = e.n_g2 > 1 ? e.g2[1] : e.g2[0];
  MBLS_TRY(hipEventRecord(e.ev_in, st));
  MBLS_TRY(hipStreamWaitEvent(hs, e.ev_in, 0));
  if (ss != hs) MBLS_TRY(hipStreamWaitEvent(ss, e.ev_in, 0));
  MBLS_TRY(use_once(mbls_scratch::UO_HASH_TO_G2, n_pairs, hs,
                      [&] { return mbls_launch::hash_to_g2(msgs, n_pairs, h_xy, hs); }));
  MBLS_TRY(mbls_launch::g2_sig_decode(sigs, n_sets, 1, sig_pre, sig_st, sig_xy, ss));
  if (!grouped) MBLS_TRY(mbls_launch::sig_miller_lg(sig_st, sig_xy, n_sets, fsig, nullptr, ss));
  MBLS_TRY(mbls_launch::g1_decode_validate(pks, n_pairs, key_pre, key_st, key_xy, st));
  MBLS_TRY(hipEventRecord(e.ev_aux, hs));
  MBLS_TRY(hipStreamWaitEvent(st, e.ev_aux, 0));
  if (ss != hs) {
    MBLS_TRY(hipEventRecord(e.ev_join[0], ss));
    MBLS_TRY(hipStreamWaitEvent(st, e.ev_join[0], 0));
  }
  if (grouped) {
    MBLS_TRY(mbls_launch::av_pairs_lg6(key_st, key_xy, h_xy, n_pairs, key_off, n_sets, sig_st, sig_xy,
                                       e.buf[S_GRP_OFF].as<uint32_t>(), e.buf[S_FPAIR].as<uint32_t>(), st));
    MBLS_TRY(mbls_launch::av_verdict_grp_lg6(key_st, key_off, sig_st, e.buf[S_GRP_OFF].as<uint32_t>(),
                                             e.buf[S_FPAIR].as<uint32_t>(), n_sets, set_pre, status, st));
  } else {
    // pairs in parallel (one lane per couple), then per set: product of its pair values with the
    // signature-side value and the final exponentiation on a 6-lane group
    MBLS_TRY(mbls_launch::miller_pairs(key_st, key_xy, h_xy, n_pairs, key_off, n_sets, e.buf[S_FPAIR].as<uint32_t>(),
                                       st));
    MBLS_TRY(mbls_launch::av_verdict_lg(key_st, n_pairs, key_off, sig_st, fsig, e.buf[S_FPAIR].as<uint32_t>(),
                                        n_sets, set_pre, status, st));
  }
  return scratch_end(e, st);
}

int32_t dev_agg_pks(Engine& e, const uint8_t* pks, const uint32_t* key_off, uint32_t n_keys, uint32_t n_sets,
                    const int32_t* key_pre, uint8_t* out48, int32_t* status, hipStream_t st) {
  MBLS_ENSURE(S_KEY_ST, sizeof(int32_t) * (size_t)std::max(n_keys, 1u));
  MBLS_ENSURE(S_KEY_XY, sizeof(uint32_t) * 28 * (size_t)std::max(n_keys, 1u));
  MBLS_ENSURE(S_SET_ST, sizeof(int32_t) * (size_t)n_sets);
  MBLS_ENSURE(S_SET_XY, sizeof(uint32_t) * 42 * (size_t)n_sets);
  auto* key_st = e.buf[S_KEY_ST].as<int32_t>();
  auto* key_xy = e.buf[S_KEY_XY].as<uint32_t>();
  auto* set_st = e.buf[S_SET_ST].as<int32_t>();
  auto* set_xy = e.buf[S_SET_XY].as<uint32_t>();
  if (int32_t r = scratch_begin(e, st)) return r;
  MBLS_TRY(mbls_launch::g1_decode_validate(pks, n_keys, key_pre, key_st, key_xy, st));
  MBLS_TRY(mbls_launch::g1_aggregate(key_st, key_xy, n_keys, key_off, n_sets, set_st, set_xy, st));
  MBLS_TRY(mbls_launch::g1_compress_sets(set_st, set_xy, n_sets, out48, status, st));
  return scratch_end(e, st);
}

}  // namespace mbls_eng
