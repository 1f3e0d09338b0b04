// mbls_engine.cpp — host side of libmbls.so: the C ABI of include/mbls.h.
//
// Layer 1 (mbls_bls_*) restates the reference NIF native/bls_nif/src/lib.rs call by call:
// argument checks that depend only on binary lengths are decided here and threaded into
// the device pipeline as per-element "pre-status" codes, so the reference's precedence
// (signature decode -> keys in list order -> message -> boolean rules) is resolved on the
// device exactly once.  Layer 2 (mbls_dev_*) enqueues the HIP kernels on a caller stream.
//
// Engines: one per GPU of the process (mbls_init_devices; mbls_init = one GPU).  A layer-1
// batch is split into contiguous chunks of sets balanced by key count (mbls_plan_shards) and
// each engine verifies its chunk on its own host thread, streams and pinned staging
// (sets are independent, no exchange).  Layer-1 calls are pipelined: each
// takes one of the engine's call contexts (pinned staging + device inputs + a completion
// event), packs its binaries without the engine lock, holds the lock only to enqueue, and
// waits for its own verdicts outside it, so call i+1's staging and key validation overlap
// call i's G2 chain.
//
// There is no CPU arithmetic here: every decode, subgroup check, hash, pairing and
// aggregation runs in the kernels of mbls_k_g1.hip / mbls_k_g2.hip / mbls_k_lg.hip, and a
// missing or failing GPU surfaces as MBLS_ERR_DEVICE.
#include "mbls_engine.hpp"

using namespace mbls_eng;

namespace mbls_eng {

// Hardware queues per process, read as the launcher set them: HIP maps each stream to one of
// GPU_MAX_HW_QUEUES hardware queues (HIP's default 4) and kernels of streams that share a queue
// serialise, so the engine creates one G2 stream per queue beyond the caller's.  The library
// never changes the process environment; bench.py, the tests and smoke() export
// GPU_MAX_HW_QUEUES=10 before the first HIP call (two latency key streams + seven lane-group
// streams; r03 A/B profiles/r03_hw_queues_ab.txt: 8 / 10 / 12 queues -> one mainnet block
// pipelined 157 / 218 / 222 blocks/s, cold epoch 88.2k / 88.1k / 85.0k sets/s).
int g2_streams() {
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  const int n = q ? std::atoi(q) : 4;
  return std::min(std::max(n, 2), Engine::kMaxG2 + 1) - 1;
}

// ---------------------------------------------------------------- engine registry -------
// Immortal (never destroyed): a call that still holds an Engine& must never see it freed, and
// no static destructor may touch engine state after the HIP runtime began to unload (r02: exit
// under rocprofv3 crashed in __cxa_finalize).  Engines replaced by mbls_init_devices are kept
// in `retired`, torn down but not freed; process exit tears engines down from an atexit hook
// registered after the HIP runtime initialised, so it runs before the runtime's own teardown.
struct Registry {
  std::mutex mu;
  std::vector<std::unique_ptr<Engine>> engines;
  std::vector<std::unique_ptr<Engine>> retired;
  std::atomic<uint32_t> rr{0};  // round-robin engine pick for calls too small to split
};
Registry& reg() {
  static Registry* r = new Registry();
  return *r;
}
thread_local int tl_slot = 0;  // mbls_dev_select: the engine layer-2 calls of this thread use

// the engines of the process (engine 0 is created on first use for device 0 / mbls_init's)
std::vector<Engine*> engines() {
  Registry& R = reg();
  std::lock_guard<std::mutex> g(R.mu);
  if (R.engines.empty()) R.engines.emplace_back(new Engine());
  std::vector<Engine*> out;
  out.reserve(R.engines.size());
  for (auto& e : R.engines) out.push_back(e.get());
  return out;
}
// the engine of the calling thread's layer-2 calls
Engine& eng() {
  Registry& R = reg();
  std::lock_guard<std::mutex> g(R.mu);
  if (R.engines.empty()) R.engines.emplace_back(new Engine());
  const int s = (tl_slot >= 0 && tl_slot < (int)R.engines.size()) ? tl_slot : 0;
  return *R.engines[s];
}

void exit_teardown();
// Process exit: release the engines' streams, events and memory while the HIP runtime is
// still whole.  Registered after the runtime's first call, so it runs before the runtime's own
// exit-time teardown (r02: leaving them to it crashed in __cxa_finalize under rocprofv3).
void register_exit_teardown() {
  static std::once_flag once;
  std::call_once(once, [] { std::atexit(exit_teardown); });
}

int32_t init_locked(Engine& e, int32_t device) {
  // an aborted collective may sit on the engine stream forever: every later call fails loudly
  // instead of queueing behind it, until mbls_shutdown abandons those streams (teardown_locked)
  if (e.comm_broken) return MBLS_ERR_DEVICE;
  if (e.ready) return hipSetDevice(e.device) == hipSuccess ? 0 : MBLS_ERR_DEVICE;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MBLS_ERR_DEVICE;
  if (device < 0) device = e.want_device < 0 ? 0 : e.want_device;
  if (device >= n) return MBLS_ERR_ARGUMENT;
  if (hipSetDevice(device) != hipSuccess) return MBLS_ERR_DEVICE;
  int n_cu = 0;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
  // no kernel runs on a device whose scratch plan is not in force
  if (int32_t r = mbls_scratch::apply(device, n_cu, &e.scratch)) return r;
  if (hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking) != hipSuccess) return MBLS_ERR_DEVICE;
  e.n_g2 = g2_streams();
  {
    const char* v = std::getenv("MBLS_SCRATCH_STREAMS");
    e.n_scratch = std::max(1, std::min(e.n_g2, v ? std::atoi(v) : Engine::kScratchStreams));
  }
  // Every stream at normal priority: high-priority G2 streams dispatch their chains ahead of the
  // key-validation grid (signature decode 26.8 -> 4.3 ms) but two verdicts then run beside the
  // keys at once and the epoch step slows 27.4 -> 29.0 ms (measured r01; a high-priority stream
  // for the cold per-set sums, r03: 87.9k vs 88.1k sets/s, no gain).  Both experiments removed.
  // no stream of its own for kstream: every stream beyond the hardware queues would share a
  // queue with another and serialise against it (a ninth stream on 8 queues: cold epoch
  // 87k -> 68k sets/s)
  const bool spare = e.n_g2 > e.n_scratch + 1;
  static const bool one_kstream = [] {  // MBLS_LAT_KEY_STREAMS=1: a single latency key stream (r02)
    const char* v = std::getenv("MBLS_LAT_KEY_STREAMS");
    return v && std::atoi(v) == 1;
  }();
  const bool spare2 = spare && e.n_g2 > e.n_scratch + 2 && !one_kstream;
  // kstream leaves the last kKeyCuReserve CUs to the G2 streams: a latency call's lane-group
  // prep needs whole SIMDs, and an unmasked key grid of one mainnet block (1,024 waves) puts one
  // wave on every SIMD for ~1.9 ms.  Measured r02 (block latency): unmasked 10.54, 16 CUs 10.54,
  // 32 CUs 9.69, 48 CUs 9.81, 64 CUs 10.51 ms; re-checked r03 with the split chain (32: 6.43 ms,
  // 16 / 64 / unmasked 7.24-7.26 ms, profiles/r03_cu_reserve_ab.txt)
  constexpr int kKeyCuReserve = 32;
  std::vector<uint32_t> m_ks;
  if (spare && n_cu > 4 * kKeyCuReserve) {
    m_ks.assign((n_cu + 31) / 32, 0u);
    for (int c = 0; c < n_cu - kKeyCuReserve; ++c) m_ks[c / 32] |= 1u << (c % 32);
    e.kstream_cus = n_cu - kKeyCuReserve;
  }
  for (int i = 0; i < e.n_g2; ++i) {
    hipError_t rc;
    if ((i == e.n_g2 - 1 || (spare2 && i == e.n_g2 - 2)) && !m_ks.empty())
      rc = hipExtStreamCreateWithCUMask(&e.g2[i], (uint32_t)m_ks.size(), m_ks.data());
    else
      rc = hipStreamCreateWithFlags(&e.g2[i], hipStreamNonBlocking);
    if (rc != hipSuccess) return MBLS_ERR_DEVICE;
  }
  e.kstream = spare ? e.g2[e.n_g2 - 1] : e.stream;
  e.kstream2 = spare2 ? e.g2[e.n_g2 - 2] : nullptr;
  e.n_lg = spare2 ? e.n_g2 - 2 : spare ? e.n_g2 - 1 : e.n_g2;
  e.n_fav = e.n_g2 + 1;
  const unsigned noT = hipEventDisableTiming;
  if (hipEventCreateWithFlags(&e.ev_in, noT) != hipSuccess) return MBLS_ERR_DEVICE;
  if (hipEventCreateWithFlags(&e.ev_aux, noT) != hipSuccess) return MBLS_ERR_DEVICE;
  if (hipEventCreateWithFlags(&e.ev_scratch, noT) != hipSuccess) return MBLS_ERR_DEVICE;
  for (int i = 0; i <= e.n_g2 + 1; ++i)
    if (hipEventCreateWithFlags(&e.ev_join[i], noT) != hipSuccess) return MBLS_ERR_DEVICE;
  for (auto& f : e.fav) {
    if (hipEventCreateWithFlags(&f.ev_g1, noT) != hipSuccess) return MBLS_ERR_DEVICE;
    if (hipEventCreateWithFlags(&f.ev_pre, noT) != hipSuccess) return MBLS_ERR_DEVICE;
    if (hipEventCreateWithFlags(&f.ev_done, noT) != hipSuccess) return MBLS_ERR_DEVICE;
  }
  // a call's completion is waited on by its (BEAM dirty scheduler / Python) thread: block in
  // the driver instead of spinning a host core
  for (auto& c : e.ctx)
    if (hipEventCreateWithFlags(&c.done, noT | hipEventBlockingSync) != hipSuccess) return MBLS_ERR_DEVICE;
  e.scratch_used = false;
  e.inflight = 0;
  e.device = device;
  e.ready = true;
  register_exit_teardown();
  return 0;
}

const char* const kPathNames[P_COUNT] = {"path_prep_1l_table", "path_prep_lg",     "path_prep_1l_cold",
                                         "path_miller_split",  "path_miller_joint", "path_key_alt",
                                         "path_verify_key_alt", "path_lat_kstream2", "path_warm_fill",
                                         "path_warm_defer",    "path_av_grouped",   "path_av_onelane",
                                         "path_prep_split",    "path_av_pipelined"};
std::atomic<uint64_t> g_path[P_COUNT];
void path(PathId p) {
  if (mbls_prof::g_on) g_path[p].fetch_add(1, std::memory_order_relaxed);
}



int32_t flush_verdict(Engine& e, bool more);
void teardown_locked(Engine& e, bool at_exit = false) {
  if (!e.ready) return;
  if (at_exit)
    e.defer.active = false;  // nobody will observe it
  else
    (void)flush_verdict(e, false);
  (void)hipSetDevice(e.device);
  if (e.comm_broken) {
    // the streams may hold an aborted collective that never completes: abandon them (no drain,
    // no destroy) together with the memory the collective may still write (the table), and
    // start over with a fresh engine on the next call
    e.comm = nullptr;
    e.comm_rank = 0;
    e.comm_world = 1;
    e.comm_broken = false;
    e.stream = e.kstream = e.kstream2 = nullptr;
    for (int i = 0; i < e.n_g2; ++i) e.g2[i] = nullptr;
    e.n_g2 = 0;
    e.tab.st = nullptr;
    e.tab.aff = nullptr;
    e.tab.n = e.tab.cap = 0;
    for (auto& f : e.fav) f.pending = false;
    e.ready = false;
    return;
  }
  (void)hipStreamSynchronize(e.stream);
  for (int i = 0; i < e.n_g2; ++i) (void)hipStreamSynchronize(e.g2[i]);
  // at exit the communicator is left to RCCL (a destroy can wait on peers that are gone)
  if (e.comm && !at_exit) (void)ncclCommDestroy(e.comm);
  e.comm = nullptr;
  e.comm_rank = 0;
  e.comm_world = 1;
  for (auto& b : e.buf) b.release();
  for (auto& c : e.ctx) c.release();
  for (hipEvent_t* ev : {&e.ev_in, &e.ev_aux, &e.ev_scratch}) {
    if (*ev) (void)hipEventDestroy(*ev);
    *ev = nullptr;
  }
  for (auto& ev : e.ev_join) {
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
  }
  (void)hipStreamDestroy(e.stream);
  e.stream = nullptr;
  e.kstream = nullptr;
  e.kstream2 = nullptr;
  e.ks_rr = 0;
  e.warm_rr = 0;
  e.kstream_cus = 0;
  for (int i = 0; i < e.n_g2; ++i) (void)hipStreamDestroy(e.g2[i]);
  for (auto& f : e.fav) f.release();
  e.n_g2 = 0;
  e.g2_rr = e.scratch_rr = e.key_rr = e.fav_parity = 0;
  if (e.tab.st) (void)hipFree(e.tab.st);
  if (e.tab.aff) (void)hipFree(e.tab.aff);
  e.tab.st = nullptr;
  e.tab.aff = nullptr;
  e.tab.n = e.tab.cap = 0;
  e.ready = false;
}

void exit_teardown() {
  Registry& R = reg();
  std::unique_lock<std::mutex> g(R.mu, std::try_to_lock);
  if (!g.owns_lock()) return;  // a thread is inside the registry: leave everything as it is
  for (auto& e : R.engines) {
    std::unique_lock<std::mutex> ge(e->mu, std::try_to_lock);
    if (ge.owns_lock()) teardown_locked(*e, /*at_exit=*/true);
  }
}


// ---------------------------------------------------------------- host staging ---------
// Packing and the batch split: mbls_host.hpp.  The pinned buffers belong to a call context.
template <class T>
T* pinned(CallCtx& c, HSlot slot, size_t n) {
  HostBuf& b = c.h[slot];
  const size_t bytes = std::max<size_t>(sizeof(T) * n, 64);
  if (bytes > b.cap) {
    const size_t want = std::max(bytes, b.cap * 2);
    if (b.p) (void)hipHostFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    if (hipHostMalloc(&b.p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
    b.cap = want;
  }
  return static_cast<T*>(b.p);
}

// Holds one of an engine's call contexts for the duration of a layer-1 call (waits while all
// are busy) and initialises the engine (the calling thread's current device = the engine's).
struct Lease {
  Engine& e;
  CallCtx* c = nullptr;
  int32_t rc = 0;
  bool enqueued = false;  // counted in e.inflight until the lease ends
  explicit Lease(Engine& en) : e(en) {
    {
      EngineLock g(e);
      rc = init_locked(e, -1);
    }
    if (rc) return;
    std::unique_lock<std::mutex> lk(e.ctx_mu);
    e.ctx_cv.wait(lk, [&] {
      for (auto& x : e.ctx)
        if (!x.busy) return true;
      return false;
    });
    for (auto& x : e.ctx)
      if (!x.busy) {
        x.busy = true;
        c = &x;
        break;
      }
  }
  ~Lease() {
    if (enqueued) {
      EngineLock g(e);
      --e.inflight;
    }
    if (!c) return;
    std::lock_guard<std::mutex> lk(e.ctx_mu);
    c->busy = false;
    e.ctx_cv.notify_one();
  }
  // async H2D of n T's from pinned slot h into the context's device slot d (engine stream;
  // engine lock held by the caller)
  template <class T>
  int32_t up(CSlot d, HSlot h, size_t n, const T** dptr) {
    if (n == 0) {
      *dptr = nullptr;
      return 0;
    }
    if (!c->d[d].ensure(sizeof(T) * n)) return MBLS_ERR_DEVICE;
    MBLS_TRY(hipMemcpyAsync(c->d[d].p, c->h[h].p, sizeof(T) * n, hipMemcpyHostToDevice, e.stream));
    *dptr = c->d[d].as<T>();
    return 0;
  }
  template <class T>
  T* dev(CSlot d, size_t n) {
    return c->d[d].ensure(sizeof(T) * std::max<size_t>(n, 1)) ? c->d[d].as<T>() : nullptr;
  }
  // enqueue the download of `bytes` from device slot d into pinned slot h on `tail` (engine
  // lock held by the caller)
  int32_t down(HSlot h, CSlot d, size_t bytes, hipStream_t tail) {
    if (bytes) MBLS_TRY(hipMemcpyAsync(c->h[h].p, c->d[d].p, bytes, hipMemcpyDeviceToHost, tail));
    return 0;
  }
  // the call's completion event, after everything it enqueued on `tail`
  int32_t record(hipStream_t tail) {
    MBLS_TRY(hipEventRecord(c->done, tail));
    ++e.inflight;
    enqueued = true;
    return 0;
  }
  // a failed enqueue: let whatever was issued drain before the context is reused
  int32_t fail(int32_t r) {
    // kernels of this call may already sit on the key stream and the G2 streams, reading the
    // context's device inputs: all of them drain before the context can be reused
    (void)hipStreamSynchronize(e.stream);
    for (int i = 0; i < e.n_g2; ++i) (void)hipStreamSynchronize(e.g2[i]);
    return r;
  }
  // wait (engine lock NOT held) for this call's completion event
  int32_t wait() { return hipEventSynchronize(c->done) == hipSuccess ? 0 : MBLS_ERR_DEVICE; }
};

size_t first_bad_len(const mbls_bin* a, size_t n, size_t want) {
  for (size_t i = 0; i < n; ++i)
    if (a[i].len != want) return a[i].len;
  return 0;
}

// ------------------------------------------------------------- multi-engine dispatch ----
// below this cost a call goes whole to one engine (the split's host threads are not free)
constexpr uint64_t kMinShardCost = uint64_t(1) << 15;

// Runs fn(engine, lo, hi) over contiguous, cost-balanced chunks of sets [0, n), one chunk per
// engine, each on its own host thread (the caller's thread takes chunk 0).  Calls too small
// to split go whole to one engine, round robin, so concurrent small callers spread over GPUs.
template <class F>
int32_t run_sharded(const uint32_t* key_off, size_t n, F&& fn) {
  const std::vector<Engine*> es = engines();
  const size_t ne = es.size();
  if (ne == 1) return fn(*es[0], size_t(0), n);
  if (prefix_cost(key_off, n) < kMinShardCost) {
    Engine& e = *es[reg().rr.fetch_add(1, std::memory_order_relaxed) % ne];
    return fn(e, size_t(0), n);
  }
  std::vector<uint32_t> b(ne + 1);
  plan_shards(key_off, n, (uint32_t)ne, b.data());
  std::vector<int32_t> rc(ne, 0);
  std::vector<std::thread> th;
  for (size_t j = 1; j < ne; ++j)
    if (b[j] < b[j + 1]) th.emplace_back([&, j] { rc[j] = fn(*es[j], (size_t)b[j], (size_t)b[j + 1]); });
  if (b[0] < b[1]) rc[0] = fn(*es[0], (size_t)b[0], (size_t)b[1]);
  for (auto& t : th) t.join();
  for (int32_t r : rc)
    if (r) return r;
  return 0;
}
// one engine for a single-output call (round robin over the process's engines)
Engine& pick_engine() {
  const std::vector<Engine*> es = engines();
  return *es[es.size() == 1 ? 0 : reg().rr.fetch_add(1, std::memory_order_relaxed) % es.size()];
}

// ---------------------------------------------------------------- layer-1 per engine ----
// n sets of (eth_)fast_aggregate_verify on engine e; key_off is the caller's array (set i's
// keys are public_keys[key_off[i] .. key_off[i+1]-1], key_off[0] need not be 0).
int32_t fav_batch_on(Engine& e, const mbls_bin* public_keys, const uint32_t* key_off, const mbls_bin* messages,
                     const mbls_bin* signatures, size_t n, int32_t flags, int32_t* results, size_t* err_got) {
  const uint32_t k0 = key_off[0], n_keys = key_off[n] - k0;
  Lease L(e);
  if (L.rc) return L.rc;
  CallCtx& c = *L.c;
  auto* hp = pinned<uint8_t>(c, H_PKS, 48 * (size_t)n_keys);
  auto* hkp = pinned<int32_t>(c, H_KPRE, n_keys);
  auto* hs = pinned<uint8_t>(c, H_SIGS, 96 * n);
  auto* hsp = pinned<int32_t>(c, H_SPRE, n);
  auto* hm = pinned<uint8_t>(c, H_MSGS, 32 * n);
  auto* hsetp = pinned<int32_t>(c, H_SETPRE, n);
  auto* ho = pinned<uint32_t>(c, H_OFF, n + 1);
  auto* hst = pinned<int32_t>(c, H_STATUS, n);
  if (!hp || !hkp || !hs || !hsp || !hm || !hsetp || !ho || !hst) return MBLS_ERR_DEVICE;
  pack_pks(public_keys + k0, n_keys, hp, hkp);
  pack_sigs(signatures, n, hs, hsp);
  pack_msgs(messages, n, hm, hsetp);
  for (size_t i = 0; i <= n; ++i) ho[i] = key_off[i] - k0;
  {
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    const uint8_t *d_pks, *d_msgs, *d_sigs;
    const int32_t *d_kpre, *d_spre, *d_setpre;
    const uint32_t* d_off;
    int32_t* d_st = L.dev<int32_t>(C_STATUS, n);
    if (!d_st) return MBLS_ERR_DEVICE;
    int32_t r = L.up(C_PKS, H_PKS, 48 * (size_t)n_keys, &d_pks);
    if (!r) r = L.up(C_KPRE, H_KPRE, n_keys, &d_kpre);
    if (!r) r = L.up(C_SIGS, H_SIGS, 96 * n, &d_sigs);
    if (!r) r = L.up(C_SPRE, H_SPRE, n, &d_spre);
    if (!r) r = L.up(C_MSGS, H_MSGS, 32 * n, &d_msgs);
    if (!r) r = L.up(C_SETPRE, H_SETPRE, n, &d_setpre);
    if (!r) r = L.up(C_OFF, H_OFF, n + 1, &d_off);
    if (r) return L.fail(r);
    G1Src src;
    src.pks = d_pks;
    src.key_pre = d_kpre;
    hipStream_t tail = e.stream;
    r = dev_fav(e, src, d_off, n_keys, d_msgs, d_sigs, (uint32_t)n, flags, d_spre, d_setpre, d_st, e.stream, nullptr,
                e.inflight == 0, &tail);
    if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t) * n, tail);
    if (!r) r = L.record(tail);
    if (r) return L.fail(r);
  }
  if (int32_t r = L.wait()) return r;
  std::memcpy(results, hst, sizeof(int32_t) * n);
  if (err_got)
    for (size_t i = 0; i < n; ++i)
      err_got[i] = results[i] == MBLS_ERR_PUBKEY_LENGTH
                       ? first_bad_len(public_keys + key_off[i], key_off[i + 1] - key_off[i], 48)
                   : results[i] == MBLS_ERR_MESSAGE_LENGTH ? messages[i].len
                                                           : 0;
  return 0;
}

int32_t verify_batch_on(Engine& e, const mbls_bin* public_keys, const mbls_bin* messages, const mbls_bin* signatures,
                        size_t n, int32_t* results, size_t* err_got) {
  Lease L(e);
  if (L.rc) return L.rc;
  CallCtx& c = *L.c;
  auto* hp = pinned<uint8_t>(c, H_PKS, 48 * n);
  auto* hkp = pinned<int32_t>(c, H_KPRE, n);
  auto* hs = pinned<uint8_t>(c, H_SIGS, 96 * n);
  auto* hsp = pinned<int32_t>(c, H_SPRE, n);
  auto* hm = pinned<uint8_t>(c, H_MSGS, 32 * n);
  auto* hsetp = pinned<int32_t>(c, H_SETPRE, n);
  auto* hst = pinned<int32_t>(c, H_STATUS, n);
  if (!hp || !hkp || !hs || !hsp || !hm || !hsetp || !hst) return MBLS_ERR_DEVICE;
  pack_pks(public_keys, n, hp, hkp);
  pack_sigs(signatures, n, hs, hsp);
  pack_msgs(messages, n, hm, hsetp);
  {
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    const uint8_t *d_pks, *d_msgs, *d_sigs;
    const int32_t *d_kpre, *d_spre, *d_setpre;
    int32_t* d_st = L.dev<int32_t>(C_STATUS, n);
    if (!d_st) return MBLS_ERR_DEVICE;
    int32_t r = L.up(C_PKS, H_PKS, 48 * n, &d_pks);
    if (!r) r = L.up(C_KPRE, H_KPRE, n, &d_kpre);
    if (!r) r = L.up(C_SIGS, H_SIGS, 96 * n, &d_sigs);
    if (!r) r = L.up(C_SPRE, H_SPRE, n, &d_spre);
    if (!r) r = L.up(C_MSGS, H_MSGS, 32 * n, &d_msgs);
    if (!r) r = L.up(C_SETPRE, H_SETPRE, n, &d_setpre);
    if (r) return L.fail(r);
    hipStream_t tail = e.stream;
    r = dev_verify(e, d_pks, d_msgs, d_sigs, (uint32_t)n, d_kpre, d_spre, d_setpre, d_st, e.stream, nullptr, &tail);
    if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t) * n, tail);
    if (!r) r = L.record(tail);
    if (r) return L.fail(r);
  }
  if (int32_t r = L.wait()) return r;
  std::memcpy(results, hst, sizeof(int32_t) * n);
  if (err_got)
    for (size_t i = 0; i < n; ++i)
      err_got[i] = results[i] == MBLS_ERR_PUBKEY_LENGTH    ? public_keys[i].len
                   : results[i] == MBLS_ERR_MESSAGE_LENGTH ? messages[i].len
                                                           : 0;
  return 0;
}

int32_t av_batch_on(Engine& e, const mbls_bin* public_keys, const uint32_t* key_off, const mbls_bin* messages,
                    const uint32_t* msg_off, const mbls_bin* signatures, size_t n, int32_t* results,
                    size_t* err_got) {
  const uint32_t k0 = key_off[0], n_pairs = key_off[n] - k0;
  Lease L(e);
  if (L.rc) return L.rc;
  CallCtx& c = *L.c;
  auto* set_pre = pinned<int32_t>(c, H_SETPRE, n);
  auto* h_msgs = pinned<uint8_t>(c, H_MSGS, 32 * (size_t)n_pairs);
  auto* hp = pinned<uint8_t>(c, H_PKS, 48 * (size_t)n_pairs);
  auto* hkp = pinned<int32_t>(c, H_KPRE, n_pairs);
  auto* hs = pinned<uint8_t>(c, H_SIGS, 96 * n);
  auto* hsp = pinned<int32_t>(c, H_SPRE, n);
  auto* ho = pinned<uint32_t>(c, H_OFF, n + 1);
  auto* hst = pinned<int32_t>(c, H_STATUS, n);
  if (!set_pre || !h_msgs || !hp || !hkp || !hs || !hsp || !ho || !hst) return MBLS_ERR_DEVICE;
  std::vector<size_t> bad_msg_len(n, 0);
  // per set: Hash256::from_slice on every message happens after key decoding (lib.rs:76-79),
  // then msgs.len() != pubkeys.len() is {:ok, false}; a passing set gets one message per key
  // slot, others zero slots
  par_for(n, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const uint32_t nk = key_off[i + 1] - key_off[i], nm = msg_off[i + 1] - msg_off[i];
      int32_t pre = 0;
      for (uint32_t j = 0; j < nm; ++j)
        if (messages[msg_off[i] + j].len != 32 || !messages[msg_off[i] + j].data) {
          pre = MBLS_ERR_MESSAGE_LENGTH;
          bad_msg_len[i] = messages[msg_off[i] + j].len;
          break;
        }
      if (pre == 0 && nm != nk) pre = MBLS_SET_FALSE;
      set_pre[i] = pre;
      uint8_t* dst = h_msgs + 32 * (size_t)(key_off[i] - k0);
      for (uint32_t j = 0; j < nk; ++j) {
        if (pre == 0)
          std::memcpy(dst + 32 * j, messages[msg_off[i] + j].data, 32);
        else
          std::memset(dst + 32 * j, 0, 32);
      }
    }
  });
  pack_pks(public_keys + k0, n_pairs, hp, hkp);
  pack_sigs(signatures, n, hs, hsp);
  for (size_t i = 0; i <= n; ++i) ho[i] = key_off[i] - k0;
  {
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    const uint8_t *d_pks, *d_msgs, *d_sigs;
    const int32_t *d_kpre, *d_spre, *d_setpre;
    const uint32_t* d_off;
    int32_t* d_st = L.dev<int32_t>(C_STATUS, n);
    if (!d_st) return MBLS_ERR_DEVICE;
    int32_t r = L.up(C_PKS, H_PKS, 48 * (size_t)n_pairs, &d_pks);
    if (!r) r = L.up(C_KPRE, H_KPRE, n_pairs, &d_kpre);
    if (!r) r = L.up(C_SIGS, H_SIGS, 96 * n, &d_sigs);
    if (!r) r = L.up(C_SPRE, H_SPRE, n, &d_spre);
    if (!r) r = L.up(C_MSGS, H_MSGS, 32 * (size_t)n_pairs, &d_msgs);
    if (!r) r = L.up(C_SETPRE, H_SETPRE, n, &d_setpre);
    if (!r) r = L.up(C_OFF, H_OFF, n + 1, &d_off);
    if (r) return L.fail(r);
    r = dev_av(e, d_pks, d_msgs, d_off, n_pairs, d_sigs, (uint32_t)n, d_kpre, d_spre, d_setpre, d_st, e.stream,
               /*join=*/true);
    if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t) * n, e.stream);
    if (!r) r = L.record(e.stream);
    if (r) return L.fail(r);
  }
  if (int32_t r = L.wait()) return r;
  std::memcpy(results, hst, sizeof(int32_t) * n);
  if (err_got)
    for (size_t i = 0; i < n; ++i)
      err_got[i] = results[i] == MBLS_ERR_PUBKEY_LENGTH
                       ? first_bad_len(public_keys + key_off[i], key_off[i + 1] - key_off[i], 48)
                   : results[i] == MBLS_ERR_MESSAGE_LENGTH ? bad_msg_len[i]
                                                           : 0;
  return 0;
}

int32_t fav_indexed_on(Engine& e, const uint32_t* idx, const uint32_t* idx_off, const mbls_bin* messages,
                       const mbls_bin* signatures, size_t n, int32_t flags, int32_t* results, size_t* err_got) {
  const uint32_t k0 = idx_off[0], n_idx = idx_off[n] - k0;
  Lease L(e);
  if (L.rc) return L.rc;
  CallCtx& c = *L.c;
  auto* hs = pinned<uint8_t>(c, H_SIGS, 96 * n);
  auto* hsp = pinned<int32_t>(c, H_SPRE, n);
  auto* hm = pinned<uint8_t>(c, H_MSGS, 32 * n);
  auto* hsetp = pinned<int32_t>(c, H_SETPRE, n);
  auto* ho = pinned<uint32_t>(c, H_OFF, n + 1);
  auto* hi = pinned<uint32_t>(c, H_IDX, n_idx);
  auto* hst = pinned<int32_t>(c, H_STATUS, n);
  if (!hs || !hsp || !hm || !hsetp || !ho || !hi || !hst) return MBLS_ERR_DEVICE;
  pack_sigs(signatures, n, hs, hsp);
  pack_msgs(messages, n, hm, hsetp);
  for (size_t i = 0; i <= n; ++i) ho[i] = idx_off[i] - k0;
  if (n_idx) std::memcpy(hi, idx + k0, sizeof(uint32_t) * n_idx);
  {
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    const uint8_t *d_msgs, *d_sigs;
    const int32_t *d_spre, *d_setpre;
    const uint32_t *d_off, *d_idx;
    int32_t* d_st = L.dev<int32_t>(C_STATUS, n);
    if (!d_st) return MBLS_ERR_DEVICE;
    int32_t r = L.up(C_SIGS, H_SIGS, 96 * n, &d_sigs);
    if (!r) r = L.up(C_SPRE, H_SPRE, n, &d_spre);
    if (!r) r = L.up(C_MSGS, H_MSGS, 32 * n, &d_msgs);
    if (!r) r = L.up(C_SETPRE, H_SETPRE, n, &d_setpre);
    if (!r) r = L.up(C_OFF, H_OFF, n + 1, &d_off);
    if (!r) r = L.up(C_IDX, H_IDX, n_idx, &d_idx);
    if (r) return L.fail(r);
    G1Src src;
    src.idx = d_idx ? d_idx : d_off;  // n_idx == 0: never read
    hipStream_t tail = e.stream;
    r = dev_fav(e, src, d_off, n_idx, d_msgs, d_sigs, (uint32_t)n, flags, d_spre, d_setpre, d_st, e.stream, nullptr,
                e.inflight == 0, &tail);
    if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t) * n, tail);
    if (!r) r = L.record(tail);
    if (r) return L.fail(r);
  }
  if (int32_t r = L.wait()) return r;
  std::memcpy(results, hst, sizeof(int32_t) * n);
  if (err_got)
    for (size_t i = 0; i < n; ++i) err_got[i] = results[i] == MBLS_ERR_MESSAGE_LENGTH ? messages[i].len : 0;
  return 0;
}

// ---------------------------------------------------------------- kernel timing --------
struct ProfRec {
  int kid;
  hipEvent_t a, b;
};
struct Prof {
  std::mutex mu;
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> pool;
  double total_ms[mbls_prof::K_COUNT] = {};
  uint64_t count[mbls_prof::K_COUNT] = {};
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  void resolve() {
    for (auto& r : pending) {
      if (!r.b) continue;
      float ms = 0.f;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
        total_ms[r.kid] += ms;
        count[r.kid] += 1;
      }
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pending.clear();
  }
};
Prof& prof() {
  static Prof* p = new Prof();  // immortal, as the registry
  return *p;
}
const char* const kKernelNames[mbls_prof::K_COUNT] = {
    "g1_decode_validate", "g1_aggregate", "g1_compress_sets", "map_pk_status", "g2_sig_decode",
    "hash_to_g2",         "fav_verdict",  "av_verdict",       "sign",          "g2_aggregate",
    "sk_to_pk",           "sig_miller",   "g1_aggregate_idx", "pk_table_store", "miller_pairs", "rlc", "g2_prep", "ssz_roots",
    "fav_verdict_1l",     "fav_verdict_lg8", "fav_verdict_lg16", "key_miller",    "fav_verdict_lg6"};

}  // namespace mbls_eng

namespace mbls_prof {
bool g_on = false;
void begin(int kid, hipStream_t s) {
  Prof& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  ProfRec r{kid, p.get(), nullptr};
  (void)hipEventRecord(r.a, s);
  p.pending.push_back(r);
}
void end(int kid, hipStream_t s) {
  Prof& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  for (auto it = p.pending.rbegin(); it != p.pending.rend(); ++it)
    if (it->kid == kid && !it->b) {
      it->b = p.get();
      (void)hipEventRecord(it->b, s);
      break;
    }
}
}  // namespace mbls_prof

// ---------------------------------------------------------- batch telemetry -----------
// Per-operation counters behind mbls_stats_read (include/mbls.h): calls, sets, keys, error
// returns and wall time inside the call, relaxed atomics.  An API entry that calls another
// (mbls_bls_verify -> mbls_bls_verify_batch) counts once, as the outer operation.
namespace {
struct OpCounters {
  std::atomic<uint64_t> calls{0}, sets{0}, keys{0}, errors{0}, ns{0};
};
OpCounters g_ops[MBLS_OP_COUNT];
thread_local int tl_op_depth = 0;
template <class F>
int32_t counted(int op, uint64_t sets, uint64_t keys, F&& body) {
  struct Depth {
    Depth() { ++tl_op_depth; }
    ~Depth() { --tl_op_depth; }
  };
  if (tl_op_depth > 0) {
    Depth d;
    return body();
  }
  const auto t0 = std::chrono::steady_clock::now();
  int32_t r;
  {
    Depth d;
    r = body();
  }
  const uint64_t ns =
      (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  OpCounters& c = g_ops[op];
  c.calls.fetch_add(1, std::memory_order_relaxed);
  c.sets.fetch_add(sets, std::memory_order_relaxed);
  c.keys.fetch_add(keys, std::memory_order_relaxed);
  if (r < 0) c.errors.fetch_add(1, std::memory_order_relaxed);
  c.ns.fetch_add(ns, std::memory_order_relaxed);
  return r;
}
// keys (or pairs) of a batch from its offsets, 0 when absent or malformed (the call itself
// rejects those), read before the call runs
uint64_t off_span(const uint32_t* off, uint32_t n) { return n && off && off[n] >= off[0] ? off[n] - off[0] : 0; }
const char* const kOpNames[MBLS_OP_COUNT] = {"verify",        "fast_aggregate_verify", "eth_fast_aggregate_verify",
                                             "aggregate_verify", "eth_aggregate_pubkeys", "aggregate",
                                             "sign",          "key_validate",          "signing_roots"};
}  // namespace

// ============================================================== C ABI ===================
extern "C" {

int32_t mbls_prof_enable(int32_t on) {
  mbls_prof::g_on = on != 0;
  return 0;
}
int32_t mbls_prof_reset(void) {
  Prof& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  p.resolve();
  for (int i = 0; i < mbls_prof::K_COUNT; ++i) {
    p.total_ms[i] = 0;
    p.count[i] = 0;
  }
  for (auto& c : g_path) c = 0;
  return 0;
}
int32_t mbls_prof_read(const char* kernel, double* total_ms, uint64_t* launches) {
  Prof& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  p.resolve();
  for (int i = 0; i < mbls_prof::K_COUNT; ++i)
    if (kernel && std::strcmp(kernel, kKernelNames[i]) == 0) {
      if (total_ms) *total_ms = p.total_ms[i];
      if (launches) *launches = p.count[i];
      return 0;
    }
  for (int i = 0; i < P_COUNT; ++i)  // path counters: calls that took the form, no time
    if (kernel && std::strcmp(kernel, kPathNames[i]) == 0) {
      if (total_ms) *total_ms = 0;
      if (launches) *launches = g_path[i].load();
      return 0;
    }
  return MBLS_ERR_ARGUMENT;
}

// ------------------------------------------------------------------ telemetry ----------
const char* mbls_op_name(int32_t op) { return op >= 0 && op < MBLS_OP_COUNT ? kOpNames[op] : nullptr; }
int32_t mbls_stats_read(mbls_op_stats* out, int32_t n, int32_t reset) {
  if (!out || n < 0) return MBLS_ERR_ARGUMENT;
  const int32_t m = std::min<int32_t>(n, MBLS_OP_COUNT);
  for (int32_t i = 0; i < m; ++i) {
    OpCounters& c = g_ops[i];
    if (reset) {
      out[i] = {c.calls.exchange(0), c.sets.exchange(0), c.keys.exchange(0), c.errors.exchange(0), c.ns.exchange(0)};
    } else {
      out[i] = {c.calls.load(), c.sets.load(), c.keys.load(), c.errors.load(), c.ns.load()};
    }
  }
  // (reset clears only the entries copied out: a caller built against a smaller
  // MBLS_OP_COUNT keeps the newer operations' counts for callers that read them)
  return m;
}

// ------------------------------------------------------------------ lifecycle ----------
int32_t mbls_init(int32_t device) {
  {
    Registry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    if (R.engines.empty()) R.engines.emplace_back(new Engine());
    if (!R.engines[0]->ready) R.engines[0]->want_device = device;
  }
  Engine& e = *engines()[0];
  EngineLock g(e);
  return init_locked(e, device);
}

int32_t mbls_init_devices(const int32_t* devices, uint32_t n) {
  if (!devices || n == 0 || n > 64) return MBLS_ERR_ARGUMENT;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return MBLS_ERR_DEVICE;
  for (uint32_t i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= count) return MBLS_ERR_ARGUMENT;
  Registry& R = reg();
  {
    std::lock_guard<std::mutex> g(R.mu);
    bool any_ready = false;
    for (auto& e : R.engines) any_ready |= e->ready;
    if (any_ready) {  // idempotent for the same list, an error otherwise
      bool same = R.engines.size() == n;
      for (uint32_t i = 0; same && i < n; ++i) same = R.engines[i]->device == devices[i];
      return same ? 0 : MBLS_ERR_ARGUMENT;
    }
    // replaced engines are torn down (none is ready) and kept, never freed: a thread that
    // still holds one must not touch freed memory
    for (auto& e : R.engines) R.retired.push_back(std::move(e));
    R.engines.clear();
    for (uint32_t i = 0; i < n; ++i) {
      R.engines.emplace_back(new Engine());
      R.engines.back()->want_device = devices[i];
    }
  }
  for (Engine* e : engines()) {
    std::lock_guard<std::mutex> g(e->mu);
    if (int32_t r = init_locked(*e, e->want_device)) return r;
  }
  return 0;
}

int32_t mbls_engine_count(void) { return (int32_t)engines().size(); }

int32_t mbls_dev_select(int32_t engine) {
  if (engine < 0 || engine >= (int32_t)engines().size()) return MBLS_ERR_ARGUMENT;
  tl_slot = engine;
  Engine& e = eng();
  EngineLock g(e);
  return init_locked(e, -1);
}

int32_t mbls_plan_shards(const uint32_t* key_off, size_t n_sets, uint32_t parts, uint32_t* bounds) {
  if (!bounds || parts == 0 || n_sets > UINT32_MAX) return MBLS_ERR_ARGUMENT;
  if (key_off)
    for (size_t i = 0; i < n_sets; ++i)
      if (key_off[i + 1] < key_off[i]) return MBLS_ERR_ARGUMENT;
  plan_shards(key_off, n_sets, parts, bounds);
  return 0;
}

int32_t mbls_scratch_info(mbls_scratch_plan_t* out) {
  if (!out) return MBLS_ERR_ARGUMENT;
  Engine& e = eng();
  EngineLock g(e);
  if (!e.ready) return MBLS_ERR_DEVICE;
  *out = e.scratch;
  return 0;
}
int32_t mbls_debug_fail_deferred(int32_t engine, int32_t code) {
  const std::vector<Engine*> es = engines();
  if (engine < 0 || engine >= (int32_t)es.size() || code >= 0) return MBLS_ERR_ARGUMENT;
  EngineLock g(*es[engine]);
  es[engine]->defer_rc = code;
  return 0;
}

// Tears every engine down in place (streams, events, buffers, table, communicator); the
// Engine objects stay allocated, so a thread that still holds one sees an engine that is not
// ready (it re-initialises on its next call) instead of freed memory.  Must not race with
// calls in flight (include/mbls.h).
void mbls_shutdown(void) {
  Registry& R = reg();
  std::lock_guard<std::mutex> g(R.mu);
  for (auto& e : R.engines) {
    std::lock_guard<std::mutex> ge(e->mu);
    teardown_locked(*e);
  }
  tl_slot = 0;
}

const char* mbls_version(void) { return "mbls 0.2.0 (gfx950, radix-2^28 Montgomery, multi-device)"; }

// ------------------------------------------------- device memory / stream plumbing -----
int32_t mbls_dev_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
void* mbls_dev_malloc(size_t bytes) {
  Engine& e = eng();
  {
    EngineLock g(e);
    if (init_locked(e, -1)) return nullptr;
  }
  void* p = nullptr;
  if (hipMalloc(&p, std::max<size_t>(bytes, 1)) != hipSuccess) return nullptr;
  return p;
}
int32_t mbls_dev_synchronize(void* stream);
// Every engine of the process (memory handed to engine j by another thread, or
// before an mbls_dev_select switch, may still be read by engine j's streams): each engine's
// pending deferred verdict is launched (its latency form) and all its streams drain.  Returns 0
// when every stream drained, else MBLS_ERR_DEVICE (the memory may still be in use).  The CALLING
// thread's engine's failed deferred launch is reported separately through *deferred (0 if none)
// and consumed, as its synchronize would, only once the drain completed; another engine's stays
// for that engine's own synchronize (one engine's failure must not fail every copy
// and free of the process until a thread that may be gone synchronizes it).  The two are kept
// apart because a failed deferred launch is itself recorded as MBLS_ERR_DEVICE.
int32_t drain_all_engines(int32_t* deferred) {
  Engine& me = eng();
  *deferred = 0;
  for (Engine* e : engines()) {
    hipStream_t ss[Engine::kMaxG2 + 1];
    int n = 0, dev = -1;
    {
      EngineLock g(*e);
      if (!e->ready) continue;
      dev = e->device;
      ss[n++] = e->stream;
      for (int i = 0; i < e->n_g2; ++i) ss[n++] = e->g2[i];
    }
    if (hipSetDevice(dev) != hipSuccess) return MBLS_ERR_DEVICE;
    for (int i = 0; i < n; ++i)
      if (hipStreamSynchronize(ss[i]) != hipSuccess) return MBLS_ERR_DEVICE;
  }
  // back to the calling thread's engine's device for whatever it does next
  if (me.ready && hipSetDevice(me.device) != hipSuccess) return MBLS_ERR_DEVICE;
  EngineLock g(me);
  *deferred = me.defer_rc;
  me.defer_rc = 0;
  return 0;
}
// Freeing or overwriting device memory an engine may still read: every engine drains first
// (drain_all_engines), so memory handed to an earlier call can be reused or released as soon as
// these return.  The free / copy happens whenever every stream drained; a deferred-launch error
// of the caller's engine is returned after it (the free / copy has still taken effect).
int32_t mbls_dev_free(void* p) {
  int32_t deferred = 0;
  if (drain_all_engines(&deferred)) return MBLS_ERR_DEVICE;  // a stream did not drain
  const bool ok = hipFree(p) == hipSuccess;
  return deferred ? deferred : ok ? 0 : MBLS_ERR_DEVICE;
}
int32_t mbls_dev_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  int32_t deferred = 0;
  if (drain_all_engines(&deferred)) return MBLS_ERR_DEVICE;
  const bool ok = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  return deferred ? deferred : ok ? 0 : MBLS_ERR_DEVICE;
}
int32_t mbls_dev_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  Engine& me = eng();
  {
    EngineLock g(me, /*more=*/true);
    if (int32_t r = init_locked(me, -1)) return r;
  }
  const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : me.stream;
  for (Engine* e : engines()) {
    EngineLock g(*e, /*more=*/e == &me);
    if (!e->ready) continue;
    if (hipSetDevice(e->device) != hipSuccess) return MBLS_ERR_DEVICE;
    hipStream_t src_s[Engine::kMaxG2 + 1];
    src_s[0] = e->stream;
    for (int i = 0; i < e->n_g2; ++i) src_s[i + 1] = e->g2[i];
    for (int i = 0; i <= e->n_g2; ++i) {
      if (src_s[i] == s) continue;
      MBLS_TRY(hipEventRecord(e->ev_join[i], src_s[i]));
      MBLS_TRY(hipStreamWaitEvent(s, e->ev_join[i], 0));
    }
  }
  MBLS_TRY(hipSetDevice(me.device));
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : MBLS_ERR_DEVICE;
}
int32_t mbls_dev_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  // the engines' streams are non-blocking: a plain hipMemcpy does not wait for them, so the
  // results written there (status words) are completed first -- on EVERY engine, as for the
  // uploads (a thread that selected engine 1 may read a status buffer engine 0's
  // deferred verdict writes)
  int32_t deferred = 0;
  if (drain_all_engines(&deferred)) return MBLS_ERR_DEVICE;
  if (deferred) return deferred;
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : MBLS_ERR_DEVICE;
}
void* mbls_dev_stream_create(void) {
  Engine& e = eng();
  {
    EngineLock g(e);
    if (init_locked(e, -1)) return nullptr;
  }
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  return s;
}
int32_t mbls_dev_stream_destroy(void* stream) {
  return hipStreamDestroy(static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : MBLS_ERR_DEVICE;
}
void* mbls_dev_event_create(void) {
  hipEvent_t ev = nullptr;
  if (hipEventCreate(&ev) != hipSuccess) return nullptr;
  return ev;
}
int32_t mbls_dev_event_destroy(void* event) {
  return hipEventDestroy(static_cast<hipEvent_t>(event)) == hipSuccess ? 0 : MBLS_ERR_DEVICE;
}
int32_t mbls_dev_event_record(void* event, void* stream) {
  Engine& e = eng();
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e.stream;
  return hipEventRecord(static_cast<hipEvent_t>(event), s) == hipSuccess ? 0 : MBLS_ERR_DEVICE;
}
float mbls_dev_event_elapsed_ms(void* start, void* stop) {
  float ms = -1.f;
  if (hipEventSynchronize(static_cast<hipEvent_t>(stop)) != hipSuccess) return -1.f;
  if (hipEventElapsedTime(&ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)) != hipSuccess)
    return -1.f;
  return ms;
}

// Wait for all work the engine enqueued on `stream` and on its own streams.
int32_t mbls_dev_synchronize(void* stream) {
  Engine& e = eng();
  hipStream_t s = nullptr, own = nullptr;
  int n_g2 = 0;
  hipStream_t g2[Engine::kMaxG2];
  {
    EngineLock g(e);
    if (!e.ready) return 0;
    MBLS_TRY(hipSetDevice(e.device));
    if (e.defer_rc) {
      const int32_t r = e.defer_rc;
      e.defer_rc = 0;
      return r;
    }
    s = pick(e, stream);
    own = e.stream;
    n_g2 = e.n_g2;
    for (int i = 0; i < n_g2; ++i) g2[i] = e.g2[i];
  }
  MBLS_TRY(hipStreamSynchronize(s));
  if (s != own) MBLS_TRY(hipStreamSynchronize(own));
  for (int i = 0; i < n_g2; ++i) MBLS_TRY(hipStreamSynchronize(g2[i]));
  return 0;
}

// Make `stream` wait (device side) for everything the engine has enqueued so far on its own
// streams, so an event a caller records on `stream` afterwards completes with those calls.
int32_t mbls_dev_stream_wait_engine(void* stream) {
  Engine& e = eng();
  EngineLock g(e);
  if (int32_t r = init_locked(e, -1)) return r;
  hipStream_t s = pick(e, stream);
  hipStream_t src[Engine::kMaxG2 + 2];
  src[0] = e.stream;
  for (int i = 0; i < e.n_g2; ++i) src[i + 1] = e.g2[i];
  for (int i = 0; i <= e.n_g2; ++i) {
    if (src[i] == s) continue;
    MBLS_TRY(hipEventRecord(e.ev_join[i], src[i]));
    MBLS_TRY(hipStreamWaitEvent(s, e.ev_join[i], 0));
  }
  return 0;
}

// ----------------------------------------------------------------- layer 2 -------------
int32_t mbls_dev_fast_aggregate_verify(const uint8_t* pks48, const uint32_t* key_off, uint32_t n_keys,
                                       const uint8_t* msgs32, const uint8_t* sigs96, uint32_t n_sets,
                                       int32_t eth_variant, int32_t* status, void* stream) {
  return counted((eth_variant & MBLS_FAV_ETH) ? MBLS_OP_ETH_FAST_AGGREGATE_VERIFY : MBLS_OP_FAST_AGGREGATE_VERIFY, n_sets, n_keys, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!key_off || !msgs32 || !sigs96 || !status || (n_keys && !pks48)) return MBLS_ERR_ARGUMENT;
    G1Src src;
    src.pks = pks48;
    return dev_fav(e, src, key_off, n_keys, msgs32, sigs96, n_sets, eth_variant, nullptr, nullptr, status,
                   pick(e, stream), nullptr, false, nullptr, /*may_defer=*/true);
  });
}

int32_t mbls_dev_verify(const uint8_t* pks48, const uint8_t* msgs32, const uint8_t* sigs96, uint32_t n_sets,
                        int32_t* status, void* stream) {
  return counted(MBLS_OP_VERIFY, n_sets, n_sets, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!pks48 || !msgs32 || !sigs96 || !status) return MBLS_ERR_ARGUMENT;
    return dev_verify(e, pks48, msgs32, sigs96, n_sets, nullptr, nullptr, nullptr, status, pick(e, stream));
  });
}

int32_t mbls_dev_aggregate_verify(const uint8_t* pks48, const uint8_t* msgs32, const uint32_t* key_off,
                                  uint32_t n_pairs, const uint8_t* sigs96, uint32_t n_sets, int32_t* status,
                                  void* stream) {
  return counted(MBLS_OP_AGGREGATE_VERIFY, n_sets, n_pairs, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!key_off || !sigs96 || !status || (n_pairs && (!pks48 || !msgs32))) return MBLS_ERR_ARGUMENT;
    return dev_av(e, pks48, msgs32, key_off, n_pairs, sigs96, n_sets, nullptr, nullptr, nullptr, status,
                  pick(e, stream), /*join=*/false);
  });
}

int32_t mbls_dev_aggregate_pubkeys(const uint8_t* pks48, const uint32_t* key_off, uint32_t n_keys, uint32_t n_sets,
                                   uint8_t* out48, int32_t* status, void* stream) {
  return counted(MBLS_OP_ETH_AGGREGATE_PUBKEYS, n_sets, n_keys, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!key_off || !out48 || !status || (n_keys && !pks48)) return MBLS_ERR_ARGUMENT;
    return dev_agg_pks(e, pks48, key_off, n_keys, n_sets, nullptr, out48, status, pick(e, stream));
  });
}

int32_t mbls_dev_validate_pubkeys(const uint8_t* pks48, uint32_t n_keys, int32_t* status, void* stream) {
  return counted(MBLS_OP_KEY_VALIDATE, n_keys, n_keys, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_keys == 0) return 0;
    if (!pks48 || !status) return MBLS_ERR_ARGUMENT;
    MBLS_ENSURE(S_KEY_ST, sizeof(int32_t) * (size_t)n_keys);
    MBLS_ENSURE(S_KEY_XY, sizeof(uint32_t) * 28 * (size_t)n_keys);
    hipStream_t st = pick(e, stream);
    if (int32_t r = scratch_begin(e, st)) return r;
    MBLS_TRY(mbls_launch::g1_decode_validate(pks48, n_keys, nullptr, e.buf[S_KEY_ST].as<int32_t>(),
                                             e.buf[S_KEY_XY].as<uint32_t>(), st));
    MBLS_TRY(mbls_launch::map_pk_status(e.buf[S_KEY_ST].as<int32_t>(), n_keys, status, st));
    return scratch_end(e, st);
  });
}

int32_t mbls_dev_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* out48, void* stream) {
  return counted(MBLS_OP_SIGN, n, 0, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!sk32 || !out48) return MBLS_ERR_ARGUMENT;
    MBLS_TRY(mbls_launch::sk_to_pk(sk32, n, out48, pick(e, stream)));
    return 0;
  });
}

int32_t mbls_dev_sign(const uint8_t* sk32, const uint8_t* msgs32, uint32_t n, uint8_t* out96, void* stream) {
  return counted(MBLS_OP_SIGN, n, 0, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!sk32 || !msgs32 || !out96) return MBLS_ERR_ARGUMENT;
    const hipStream_t ss = pick(e, stream);
    MBLS_TRY(use_once(mbls_scratch::UO_SIGN, n, ss, [&] { return mbls_launch::sign(sk32, msgs32, n, out96, ss); }));
    return 0;
  });
}

// Bls.aggregate for n_sets sets of device-resident signatures (set i = sigs off[i]..off[i+1])
int32_t mbls_dev_aggregate_signatures(const uint8_t* sigs96, const uint32_t* off, uint32_t n_sigs, uint32_t n_sets,
                                      uint8_t* out96, int32_t* status, void* stream) {
  return counted(MBLS_OP_AGGREGATE, n_sets, 0, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!off || !out96 || !status || (n_sigs && !sigs96)) return MBLS_ERR_ARGUMENT;
    MBLS_ENSURE(S_SIG_ST, sizeof(int32_t) * (size_t)std::max(n_sigs, 1u));
    MBLS_ENSURE(S_SIG_XY, sizeof(uint32_t) * 56 * (size_t)std::max(n_sigs, 1u));
    hipStream_t st = pick(e, stream);
    if (int32_t r = scratch_begin(e, st)) return r;
    MBLS_TRY(mbls_launch::g2_sig_decode(sigs96, n_sigs, 0, nullptr, e.buf[S_SIG_ST].as<int32_t>(),
                                        e.buf[S_SIG_XY].as<uint32_t>(), st));
    MBLS_TRY(mbls_launch::g2_aggregate(e.buf[S_SIG_ST].as<int32_t>(), e.buf[S_SIG_XY].as<uint32_t>(), n_sigs, off,
                                       n_sets, out96, status, st));
    return scratch_end(e, st);
  });
}

// ---------------------------------------------------------- SSZ signing roots ----------
int32_t mbls_dev_hash_tree_root_chunks(const uint8_t* chunks32, uint32_t leaves, uint32_t n, uint8_t* out32,
                                       void* stream) {
  return counted(MBLS_OP_SIGNING_ROOTS, n, 0, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!chunks32 || !out32 || leaves == 0 || leaves > 16) return MBLS_ERR_ARGUMENT;
    MBLS_TRY(mbls_launch::htr_chunks(chunks32, leaves, n, out32, pick(e, stream)));
    return 0;
  });
}
int32_t mbls_dev_signing_roots(const uint8_t* object_roots32, const uint8_t* domains32, uint32_t domain_stride,
                               uint32_t n, uint8_t* out32, void* stream) {
  return counted(MBLS_OP_SIGNING_ROOTS, n, 0, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!object_roots32 || !domains32 || !out32 || (domain_stride != 0 && domain_stride != 32))
      return MBLS_ERR_ARGUMENT;
    MBLS_TRY(mbls_launch::signing_roots(object_roots32, domains32, domain_stride, n, out32, pick(e, stream)));
    return 0;
  });
}
int32_t mbls_dev_attestation_data_signing_roots(const uint8_t* data128, const uint8_t* domains32,
                                                uint32_t domain_stride, uint32_t n, uint8_t* out32, void* stream) {
  return counted(MBLS_OP_SIGNING_ROOTS, n, 0, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!data128 || !domains32 || !out32 || (domain_stride != 0 && domain_stride != 32)) return MBLS_ERR_ARGUMENT;
    MBLS_TRY(mbls_launch::attestation_signing_roots(data128, domains32, domain_stride, n, out32, pick(e, stream)));
    return 0;
  });
}

extern "C++" {
namespace {
// host-buffer form: inputs through a call context's pinned staging, roots back through it;
// `launch` enqueues the kernel on the engine stream
template <class Launch>
int32_t ssz_host(const uint8_t* a, size_t a_bytes, const uint8_t* b, size_t b_bytes, size_t n, uint8_t* out32,
                 Launch&& launch) {
  Engine& e = pick_engine();
  Lease L(e);
  if (L.rc) return L.rc;
  auto* ha = pinned<uint8_t>(*L.c, H_PKS, a_bytes);
  auto* hb = pinned<uint8_t>(*L.c, H_MSGS, b_bytes);
  auto* ho = pinned<uint8_t>(*L.c, H_BYTES, 32 * n);
  if (!ha || !hb || !ho) return MBLS_ERR_DEVICE;
  par_for(a_bytes / 32, [&](size_t lo, size_t hi) { std::memcpy(ha + 32 * lo, a + 32 * lo, 32 * (hi - lo)); });
  if (b_bytes) std::memcpy(hb, b, b_bytes);
  {
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    const uint8_t *da, *db = nullptr;
    uint8_t* dout = L.dev<uint8_t>(C_BYTES, 32 * n);
    if (!dout) return MBLS_ERR_DEVICE;
    int32_t r = L.up(C_PKS, H_PKS, a_bytes, &da);
    if (!r && b_bytes) r = L.up(C_MSGS, H_MSGS, b_bytes, &db);
    if (!r && launch(e, da, db, dout) != hipSuccess) r = MBLS_ERR_DEVICE;
    if (!r) r = L.down(H_BYTES, C_BYTES, 32 * n, e.stream);
    if (!r) r = L.record(e.stream);
    if (r) return L.fail(r);
  }
  if (int32_t r = L.wait()) return r;
  std::memcpy(out32, ho, 32 * n);
  return 0;
}
}  // namespace
}  // extern "C++"

int32_t mbls_hash_tree_root_chunks(const uint8_t* chunks32, uint32_t leaves, size_t n, uint8_t* out32) {
  return counted(MBLS_OP_SIGNING_ROOTS, n, 0, [&]() -> int32_t {
    if (n == 0) return 0;
    if (!chunks32 || !out32 || leaves == 0 || leaves > 16 || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    return ssz_host(chunks32, 32 * (size_t)leaves * n, nullptr, 0, n, out32,
                    [&](Engine& e, const uint8_t* da, const uint8_t*, uint8_t* o) {
                      return mbls_launch::htr_chunks(da, leaves, (uint32_t)n, o, e.stream);
                    });
  });
}
int32_t mbls_signing_roots(const uint8_t* object_roots32, const uint8_t* domains32, uint32_t domain_stride, size_t n,
                           uint8_t* out32) {
  return counted(MBLS_OP_SIGNING_ROOTS, n, 0, [&]() -> int32_t {
    if (n == 0) return 0;
    if (!object_roots32 || !domains32 || !out32 || (domain_stride != 0 && domain_stride != 32) || n > UINT32_MAX)
      return MBLS_ERR_ARGUMENT;
    return ssz_host(object_roots32, 32 * n, domains32, domain_stride ? 32 * n : 32, n, out32,
                    [&](Engine& e, const uint8_t* da, const uint8_t* db, uint8_t* o) {
                      return mbls_launch::signing_roots(da, db, domain_stride, (uint32_t)n, o, e.stream);
                    });
  });
}
int32_t mbls_attestation_data_signing_roots(const uint8_t* data128, const uint8_t* domains32,
                                            uint32_t domain_stride, size_t n, uint8_t* out32) {
  return counted(MBLS_OP_SIGNING_ROOTS, n, 0, [&]() -> int32_t {
    if (n == 0) return 0;
    if (!data128 || !domains32 || !out32 || (domain_stride != 0 && domain_stride != 32) || n > UINT32_MAX)
      return MBLS_ERR_ARGUMENT;
    return ssz_host(data128, 128 * n, domains32, domain_stride ? 32 * n : 32, n, out32,
                    [&](Engine& e, const uint8_t* da, const uint8_t* db, uint8_t* o) {
                      return mbls_launch::attestation_signing_roots(da, db, domain_stride, (uint32_t)n, o, e.stream);
                    });
  });
}

// ------------------------------------------------------- validator pubkey table --------
namespace {
// wait for every stream the engine enqueues on (table updates are setup operations and must
// not race with in-flight calls that read the table or the key scratch); layer-2 users of the
// scratch on caller streams are waited for through their last recorded scratch event
int32_t quiesce(Engine& e) {
  MBLS_TRY(hipStreamSynchronize(e.stream));
  for (int i = 0; i < e.n_g2; ++i) MBLS_TRY(hipStreamSynchronize(e.g2[i]));
  if (e.scratch_used) MBLS_TRY(hipEventSynchronize(e.ev_scratch));
  return 0;
}
int32_t table_reserve(Engine& e, uint32_t need) {
  if (need <= e.tab.cap) return 0;
  const uint32_t cap = std::max<uint32_t>(need, e.tab.cap + e.tab.cap / 2);
  int32_t* st = nullptr;
  uint32_t* aff = nullptr;
  if (hipMalloc(&st, sizeof(int32_t) * (size_t)cap) != hipSuccess) return MBLS_ERR_DEVICE;
  if (hipMalloc(&aff, sizeof(uint32_t) * 32 * (size_t)cap) != hipSuccess) {
    (void)hipFree(st);
    return MBLS_ERR_DEVICE;
  }
  if (e.tab.n) {
    MBLS_TRY(hipMemcpyAsync(st, e.tab.st, sizeof(int32_t) * e.tab.n, hipMemcpyDeviceToDevice, e.stream));
    MBLS_TRY(hipMemcpyAsync(aff, e.tab.aff, sizeof(uint32_t) * 32 * (size_t)e.tab.n, hipMemcpyDeviceToDevice,
                            e.stream));
  }
  MBLS_TRY(mbls_launch::pk_table_fill(st, e.tab.n, cap, e.stream));
  MBLS_TRY(hipStreamSynchronize(e.stream));
  if (e.tab.st) (void)hipFree(e.tab.st);
  if (e.tab.aff) (void)hipFree(e.tab.aff);
  e.tab.st = st;
  e.tab.aff = aff;
  e.tab.cap = cap;
  return 0;
}
int32_t table_set_locked(Engine& e, uint32_t first, const uint8_t* d_pks, uint32_t n, int32_t* d_status) {
  if ((uint64_t)first + n > 0xffffffffull) return MBLS_ERR_ARGUMENT;
  if (int32_t r = quiesce(e)) return r;
  if (int32_t r = table_reserve(e, first + n)) return r;
  MBLS_ENSURE(S_KEY_ST, sizeof(int32_t) * (size_t)n);
  MBLS_ENSURE(S_KEY_XY, sizeof(uint32_t) * 28 * (size_t)n);
  auto* key_st = e.buf[S_KEY_ST].as<int32_t>();
  auto* key_xy = e.buf[S_KEY_XY].as<uint32_t>();
  MBLS_TRY(mbls_launch::g1_decode_validate(d_pks, n, nullptr, key_st, key_xy, e.stream));
  MBLS_TRY(mbls_launch::pk_table_store(key_st, key_xy, n, first, e.tab.st, e.tab.aff, e.stream));
  if (d_status) MBLS_TRY(mbls_launch::map_pk_status(key_st, n, d_status, e.stream));
  MBLS_TRY(hipStreamSynchronize(e.stream));
  e.tab.n = std::max(e.tab.n, first + n);
  return 0;
}
// host keys -> rows first.. of engine e's table (status: host, optional)
int32_t table_set_host(Engine& e, uint32_t first, const uint8_t* pks48, uint32_t n, int32_t* status) {
  Lease L(e);
  if (L.rc) return L.rc;
  auto* hp = pinned<uint8_t>(*L.c, H_PKS, 48 * (size_t)n);
  auto* hst = pinned<int32_t>(*L.c, H_STATUS, n);
  if (!hp || !hst) return MBLS_ERR_DEVICE;
  par_for(n, [&](size_t lo, size_t hi) { std::memcpy(hp + 48 * lo, pks48 + 48 * lo, 48 * (hi - lo)); });
  EngineLock g(e);
  if (int32_t r = init_locked(e, -1)) return r;
  const uint8_t* d_pks;
  int32_t* d_st = status ? L.dev<int32_t>(C_STATUS, n) : nullptr;
  if (status && !d_st) return MBLS_ERR_DEVICE;
  if (int32_t r = L.up(C_PKS, H_PKS, 48 * (size_t)n, &d_pks)) return L.fail(r);
  if (int32_t r = table_set_locked(e, first, d_pks, n, d_st)) return L.fail(r);
  if (status) {
    MBLS_TRY(hipMemcpy(hst, d_st, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    std::memcpy(status, hst, sizeof(int32_t) * n);
  }
  return 0;
}
}  // namespace

int32_t mbls_dev_pk_table_set(uint32_t first, const uint8_t* pks48, uint32_t n, int32_t* status, void* stream) {
  return counted(MBLS_OP_KEY_VALIDATE, n, n, [&]() -> int32_t {
    (void)stream;  // synchronous: runs on the engine stream after quiescing the engine
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!pks48) return MBLS_ERR_ARGUMENT;
    return table_set_locked(e, first, pks48, n, status);
  });
}

// host keys: every engine of the process gets the rows (each GPU validates them; a table
// replicated by RCCL is mbls_dev_pk_table_set_sharded's job in the one-process-per-GPU model)
int32_t mbls_pk_table_set(uint32_t first, const uint8_t* pks48, uint32_t n, int32_t* status) {
  return counted(MBLS_OP_KEY_VALIDATE, n, n, [&]() -> int32_t {
    if (n == 0) return 0;
    if (!pks48) return MBLS_ERR_ARGUMENT;
    const std::vector<Engine*> es = engines();
    std::vector<int32_t> rc(es.size(), 0);
    std::vector<std::thread> th;
    for (size_t j = 1; j < es.size(); ++j)
      th.emplace_back([&, j] { rc[j] = table_set_host(*es[j], first, pks48, n, nullptr); });
    rc[0] = table_set_host(*es[0], first, pks48, n, status);
    for (auto& t : th) t.join();
    for (int32_t r : rc)
      if (r) return r;
    return 0;
  });
}

// ---------------------------------------------- multi-GPU table build ----
static_assert(sizeof(ncclUniqueId) == MBLS_COMM_ID_BYTES, "RCCL unique id size");

int32_t mbls_comm_unique_id(uint8_t* out) {
  if (!out) return MBLS_ERR_ARGUMENT;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return MBLS_ERR_DEVICE;
  std::memcpy(out, &id, sizeof id);
  return 0;
}

// The communicator is non-blocking (config.blocking = 0): init and the table's all-gather are
// polled against a deadline (MBLS_COMM_TIMEOUT_MS, default 120 s), and a rank that never shows up
// or a collective that never completes aborts the communicator and returns MBLS_ERR_DEVICE
// instead of hanging the caller (a BEAM node, a bench rank) forever.
static int comm_timeout_ms() {
  static const int v = [] {
    const char* t = std::getenv("MBLS_COMM_TIMEOUT_MS");
    const int ms = t ? std::atoi(t) : 120000;
    return ms > 0 ? ms : 120000;
  }();
  return v;
}
// Poll the communicator's async state until it leaves ncclInProgress (or the deadline passes).
// `enqueued`: collectives of this communicator may already sit on the engine stream (ADVICE r04:
// an abort after ncclGroupEnd must mark the engine's streams unusable, as the poll below does).
static int32_t comm_wait(Engine& e, std::chrono::steady_clock::time_point deadline, const char* what,
                         bool enqueued = false) {
  for (;;) {
    ncclResult_t st = ncclSuccess;
    if (ncclCommGetAsyncError(e.comm, &st) != ncclSuccess) st = ncclSystemError;
    if (st == ncclSuccess) return 0;
    if (st != ncclInProgress || std::chrono::steady_clock::now() > deadline) {
      std::fprintf(stderr, "libmbls: RCCL %s %s; communicator aborted\n", what,
                   st == ncclInProgress ? "timed out" : ncclGetErrorString(st));
      (void)ncclCommAbort(e.comm);
      e.comm = nullptr;
      e.comm_rank = 0;
      e.comm_world = 1;
      if (enqueued) e.comm_broken = true;
      return MBLS_ERR_DEVICE;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

int32_t mbls_comm_init(const uint8_t* id_bytes, int32_t rank, int32_t world) {
  if (!id_bytes || world < 1 || rank < 0 || rank >= world) return MBLS_ERR_ARGUMENT;
  Engine& e = eng();
  EngineLock g(e);
  if (int32_t r = init_locked(e, -1)) return r;
  if (e.comm) {
    (void)ncclCommDestroy(e.comm);
    e.comm = nullptr;
  }
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof id);
  MBLS_TRY(hipSetDevice(e.device));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(comm_timeout_ms());
  const ncclResult_t rc = ncclCommInitRankConfig(&e.comm, world, id, rank, &cfg);
  if ((rc != ncclSuccess && rc != ncclInProgress) || !e.comm) {
    std::fprintf(stderr, "libmbls: ncclCommInitRankConfig: %s\n", ncclGetErrorString(rc));
    if (e.comm) (void)ncclCommAbort(e.comm);
    e.comm = nullptr;
    return MBLS_ERR_DEVICE;
  }
  if (int32_t r = comm_wait(e, deadline, "communicator init")) return r;
  e.comm_rank = rank;
  e.comm_world = world;
  return 0;
}

int32_t mbls_comm_destroy(void) {
  Engine& e = eng();
  EngineLock g(e);
  if (e.comm) (void)ncclCommDestroy(e.comm);
  e.comm = nullptr;
  e.comm_rank = 0;
  e.comm_world = 1;
  return 0;
}

// Every rank holds the same n wire keys (the validator registry); rank k decodes and
// KeyValidates rows [k*shard, (k+1)*shard) into its table, then one in-place all-gather of the
// 128-byte rows (and one of the status words) replicates the table on every GPU.
int32_t mbls_dev_pk_table_set_sharded(const uint8_t* pks48, uint32_t n, int32_t* status, void* stream) {
  return counted(MBLS_OP_KEY_VALIDATE, n, n, [&]() -> int32_t {
    (void)stream;  // synchronous, on the engine stream
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n == 0) return 0;
    if (!pks48) return MBLS_ERR_ARGUMENT;
    if (!e.comm) return table_set_locked(e, 0, pks48, n, status);  // one GPU: the local build
    const uint32_t world = (uint32_t)e.comm_world, rank = (uint32_t)e.comm_rank;
    const uint32_t shard = (n + world - 1) / world;
    const uint64_t padded = (uint64_t)shard * world;
    if (padded > 0xffffffffull) return MBLS_ERR_ARGUMENT;
    const uint32_t lo = std::min<uint32_t>(n, rank * shard), hi = std::min<uint32_t>(n, lo + shard);
    if (int32_t r = quiesce(e)) return r;
    if (int32_t r = table_reserve(e, (uint32_t)padded)) return r;
    if (hi > lo)
      if (int32_t r = table_set_locked(e, lo, pks48 + 48 * (size_t)lo, hi - lo, nullptr)) return r;
    // this rank's padding rows (past n) read as unknown on every rank after the gather
    MBLS_TRY(mbls_launch::pk_table_fill(e.tab.st, std::max(hi, rank * shard), (rank + 1) * shard, e.stream));
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(comm_timeout_ms());
    auto enq_ok = [](ncclResult_t r) { return r == ncclSuccess || r == ncclInProgress; };
    if (!enq_ok(ncclGroupStart())) return MBLS_ERR_DEVICE;
    const bool ok =
        enq_ok(ncclAllGather(e.tab.aff + (size_t)rank * shard * 32, e.tab.aff, (size_t)shard * 32, ncclUint32, e.comm,
                             e.stream)) &&
        enq_ok(ncclAllGather(e.tab.st + (size_t)rank * shard, e.tab.st, shard, ncclInt32, e.comm, e.stream));
    if (!enq_ok(ncclGroupEnd()) || !ok) {
      // part of the group may be enqueued: nothing may wait on e.stream behind it
      (void)ncclCommAbort(e.comm);
      e.comm = nullptr;
      e.comm_rank = 0;
      e.comm_world = 1;
      e.comm_broken = true;
      return MBLS_ERR_DEVICE;
    }
    if (int32_t r = comm_wait(e, deadline, "all-gather enqueue", /*enqueued=*/true)) return r;
    if (status) MBLS_TRY(mbls_launch::map_pk_status(e.tab.st, n, status, e.stream));
    // the gather completes on the device: poll the stream against the same deadline
    for (;;) {
      const hipError_t q = hipStreamQuery(e.stream);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return MBLS_ERR_DEVICE;
      if (std::chrono::steady_clock::now() > deadline) {
        std::fprintf(stderr, "libmbls: RCCL table all-gather timed out; communicator aborted\n");
        (void)ncclCommAbort(e.comm);
        e.comm = nullptr;
        e.comm_rank = 0;
        e.comm_world = 1;
        e.comm_broken = true;  // a collective may still sit on e.stream: exit must not wait for it
        return MBLS_ERR_DEVICE;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    e.tab.n = std::max(e.tab.n, n);
    return 0;
  });
}

uint32_t mbls_pk_table_size(void) {
  Engine& e = eng();
  EngineLock g(e);
  return e.tab.n;
}

int32_t mbls_pk_table_clear(void) {
  for (Engine* ep : engines()) {
    Engine& e = *ep;
    EngineLock g(e);
    if (!e.ready || !e.tab.cap) continue;
    MBLS_TRY(hipSetDevice(e.device));
    if (int32_t r = quiesce(e)) return r;
    MBLS_TRY(mbls_launch::pk_table_fill(e.tab.st, 0, e.tab.cap, e.stream));
    MBLS_TRY(hipStreamSynchronize(e.stream));
    e.tab.n = 0;
  }
  return 0;
}

int32_t mbls_dev_fast_aggregate_verify_indexed(const uint32_t* idx, const uint32_t* idx_off, uint32_t n_idx,
                                               const uint8_t* msgs32, const uint8_t* sigs96, uint32_t n_sets,
                                               int32_t eth_variant, int32_t* status, void* stream) {
  return counted((eth_variant & MBLS_FAV_ETH) ? MBLS_OP_ETH_FAST_AGGREGATE_VERIFY : MBLS_OP_FAST_AGGREGATE_VERIFY, n_sets, n_idx, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e, /*more=*/true);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!idx_off || !msgs32 || !sigs96 || !status || (n_idx && !idx)) return MBLS_ERR_ARGUMENT;
    if (!e.tab.st && (int32_t)table_reserve(e, 1)) return MBLS_ERR_DEVICE;  // empty table: every row unknown
    G1Src src;
    src.idx = idx ? idx : reinterpret_cast<const uint32_t*>(idx_off);  // n_idx == 0: never read
    return dev_fav(e, src, idx_off, n_idx, msgs32, sigs96, n_sets, eth_variant, nullptr, nullptr, status,
                   pick(e, stream), nullptr, false, nullptr, /*may_defer=*/true);
  });
}

int32_t mbls_dev_aggregate_pubkeys_indexed(const uint32_t* idx, const uint32_t* idx_off, uint32_t n_idx,
                                           uint32_t n_sets, uint8_t* out48, int32_t* status, void* stream) {
  return counted(MBLS_OP_ETH_AGGREGATE_PUBKEYS, n_sets, n_idx, [&]() -> int32_t {
    Engine& e = eng();
    EngineLock g(e);
    if (int32_t r = init_locked(e, -1)) return r;
    if (n_sets == 0) return 0;
    if (!idx_off || !out48 || !status || (n_idx && !idx)) return MBLS_ERR_ARGUMENT;
    if (!e.tab.st && (int32_t)table_reserve(e, 1)) return MBLS_ERR_DEVICE;
    MBLS_ENSURE(S_SET_ST, sizeof(int32_t) * (size_t)n_sets);
    MBLS_ENSURE(S_SET_XY, sizeof(uint32_t) * 42 * (size_t)n_sets);
    hipStream_t st = pick(e, stream);
    auto* set_st = e.buf[S_SET_ST].as<int32_t>();
    auto* set_xy = e.buf[S_SET_XY].as<uint32_t>();
    if (int32_t r = scratch_begin(e, st)) return r;
    MBLS_TRY(mbls_launch::g1_aggregate_idx(e.tab.st, e.tab.aff, e.tab.n, idx ? idx : idx_off, idx_off, n_sets, set_st,
                                           set_xy, st));
    MBLS_TRY(mbls_launch::g1_compress_sets(set_st, set_xy, n_sets, out48, status, st));
    return scratch_end(e, st);
  });
}

// eth_aggregate_pubkeys over table rows, host buffers (the sync committee of
// accessors.ex:14-20 given as validator indices)
int32_t mbls_eth_aggregate_pubkeys_indexed(const uint32_t* idx, size_t n, uint8_t out48[48]) {
  return counted(MBLS_OP_ETH_AGGREGATE_PUBKEYS, 1, n, [&]() -> int32_t {
    if (n == 0) return MBLS_ERR_EMPTY_PUBKEYS;  // lib.rs:127
    if (!idx || !out48 || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    Engine& e = pick_engine();
    Lease L(e);
    if (L.rc) return L.rc;
    auto* hi = pinned<uint32_t>(*L.c, H_IDX, n);
    auto* ho = pinned<uint32_t>(*L.c, H_OFF, 2);
    auto* hst = pinned<int32_t>(*L.c, H_STATUS, 1);
    auto* hb = pinned<uint8_t>(*L.c, H_BYTES, 48);
    if (!hi || !ho || !hst || !hb) return MBLS_ERR_DEVICE;
    std::memcpy(hi, idx, sizeof(uint32_t) * n);
    ho[0] = 0;
    ho[1] = (uint32_t)n;
    {
      EngineLock g(e);
      if (int32_t r = init_locked(e, -1)) return r;
      if (!e.tab.st && (int32_t)table_reserve(e, 1)) return MBLS_ERR_DEVICE;
      const uint32_t *d_idx, *d_off;
      int32_t* d_st = L.dev<int32_t>(C_STATUS, 1);
      uint8_t* d_out = L.dev<uint8_t>(C_BYTES, 48);
      if (!d_st || !d_out || !e.buf[S_SET_ST].ensure(sizeof(int32_t)) ||
          !e.buf[S_SET_XY].ensure(sizeof(uint32_t) * 42))
        return MBLS_ERR_DEVICE;
      int32_t r = L.up(C_IDX, H_IDX, n, &d_idx);
      if (!r) r = L.up(C_OFF, H_OFF, 2, &d_off);
      if (!r) r = scratch_begin(e, e.stream);
      if (!r && mbls_launch::g1_aggregate_idx(e.tab.st, e.tab.aff, e.tab.n, d_idx, d_off, 1,
                                              e.buf[S_SET_ST].as<int32_t>(), e.buf[S_SET_XY].as<uint32_t>(),
                                              e.stream) != hipSuccess)
        r = MBLS_ERR_DEVICE;
      if (!r && mbls_launch::g1_compress_sets(e.buf[S_SET_ST].as<int32_t>(), e.buf[S_SET_XY].as<uint32_t>(), 1, d_out,
                                              d_st, e.stream) != hipSuccess)
        r = MBLS_ERR_DEVICE;
      if (!r) r = scratch_end(e, e.stream);
      if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t), e.stream);
      if (!r) r = L.down(H_BYTES, C_BYTES, 48, e.stream);
      if (!r) r = L.record(e.stream);
      if (r) return L.fail(r);
    }
    if (int32_t r = L.wait()) return r;
    std::memcpy(out48, hb, 48);
    return hst[0];
  });
}

int32_t mbls_fast_aggregate_verify_indexed_batch(const uint32_t* idx, const uint32_t* idx_off,
                                                 const mbls_bin* messages, const mbls_bin* signatures, size_t n,
                                                 int32_t eth_variant, int32_t* results, size_t* err_got) {
  return counted((eth_variant & MBLS_FAV_ETH) ? MBLS_OP_ETH_FAST_AGGREGATE_VERIFY : MBLS_OP_FAST_AGGREGATE_VERIFY, n, off_span(idx_off, n), [&]() -> int32_t {
    if (n == 0) return 0;
    if (!idx_off || !messages || !signatures || !results || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    if (idx_off[n] - idx_off[0] && !idx) return MBLS_ERR_ARGUMENT;
    for (size_t i = 0; i < n; ++i)
      if (idx_off[i + 1] < idx_off[i]) return MBLS_ERR_ARGUMENT;
    // an engine whose table was never built still answers (every row unknown)
    for (Engine* ep : engines()) {
      Engine& e = *ep;
      EngineLock g(e);
      if (int32_t r = init_locked(e, -1)) return r;
      if (!e.tab.st && (int32_t)table_reserve(e, 1)) return MBLS_ERR_DEVICE;
    }
    return run_sharded(idx_off, n, [&](Engine& e, size_t lo, size_t hi) {
      return fav_indexed_on(e, idx, idx_off + lo, messages + lo, signatures + lo, hi - lo, eth_variant, results + lo,
                            err_got ? err_got + lo : nullptr);
    });
  });
}

// ----------------------------------------------------------------- layer 1 -------------
int32_t mbls_bls_verify_batch(const mbls_bin* public_keys, const mbls_bin* messages, const mbls_bin* signatures,
                              size_t n, int32_t* results, size_t* err_got) {
  return counted(MBLS_OP_VERIFY, n, n, [&]() -> int32_t {
    if (n == 0) return 0;
    if (!public_keys || !messages || !signatures || !results || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    return run_sharded(nullptr, n, [&](Engine& e, size_t lo, size_t hi) {
      return verify_batch_on(e, public_keys + lo, messages + lo, signatures + lo, hi - lo, results + lo,
                             err_got ? err_got + lo : nullptr);
    });
  });
}

int32_t mbls_bls_fast_aggregate_verify_batch(const mbls_bin* public_keys, const uint32_t* key_off,
                                             const mbls_bin* messages, const mbls_bin* signatures, size_t n,
                                             int32_t eth_variant, int32_t* results, size_t* err_got) {
  return counted((eth_variant & MBLS_FAV_ETH) ? MBLS_OP_ETH_FAST_AGGREGATE_VERIFY : MBLS_OP_FAST_AGGREGATE_VERIFY, n, off_span(key_off, n), [&]() -> int32_t {
    if (n == 0) return 0;
    if (!key_off || !messages || !signatures || !results || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    if (key_off[n] - key_off[0] && !public_keys) return MBLS_ERR_ARGUMENT;
    for (size_t i = 0; i < n; ++i)
      if (key_off[i + 1] < key_off[i]) return MBLS_ERR_ARGUMENT;
    return run_sharded(key_off, n, [&](Engine& e, size_t lo, size_t hi) {
      return fav_batch_on(e, public_keys, key_off + lo, messages + lo, signatures + lo, hi - lo, eth_variant,
                          results + lo, err_got ? err_got + lo : nullptr);
    });
  });
}

int32_t mbls_bls_aggregate_verify_batch(const mbls_bin* public_keys, const uint32_t* key_off,
                                        const mbls_bin* messages, const uint32_t* msg_off,
                                        const mbls_bin* signatures, size_t n, int32_t* results, size_t* err_got) {
  return counted(MBLS_OP_AGGREGATE_VERIFY, n, off_span(key_off, n), [&]() -> int32_t {
    if (n == 0) return 0;
    if (!key_off || !msg_off || !signatures || !results || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    if ((key_off[n] - key_off[0] && !public_keys) || (msg_off[n] - msg_off[0] && !messages)) return MBLS_ERR_ARGUMENT;
    for (size_t i = 0; i < n; ++i)
      if (key_off[i + 1] < key_off[i] || msg_off[i + 1] < msg_off[i]) return MBLS_ERR_ARGUMENT;
    return run_sharded(key_off, n, [&](Engine& e, size_t lo, size_t hi) {
      return av_batch_on(e, public_keys, key_off + lo, messages, msg_off + lo, signatures + lo, hi - lo, results + lo,
                         err_got ? err_got + lo : nullptr);
    });
  });
}

int32_t mbls_bls_verify(mbls_bin public_key, mbls_bin message, mbls_bin signature, size_t* err_got) {
  return counted(MBLS_OP_VERIFY, 1, 1, [&]() -> int32_t {
    int32_t r = 0;
    size_t got = 0;
    const int32_t rc = mbls_bls_verify_batch(&public_key, &message, &signature, 1, &r, &got);
    if (err_got) *err_got = got;
    return rc ? rc : r;
  });
}

int32_t mbls_bls_fast_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, mbls_bin message,
                                       mbls_bin signature, size_t* err_got) {
  return counted(MBLS_OP_FAST_AGGREGATE_VERIFY, 1, n_keys, [&]() -> int32_t {
    const uint32_t off[2] = {0, (uint32_t)n_keys};
    int32_t r = 0;
    size_t got = 0;
    const int32_t rc = mbls_bls_fast_aggregate_verify_batch(public_keys, off, &message, &signature, 1, 0, &r, &got);
    if (err_got) *err_got = got;
    return rc ? rc : r;
  });
}

int32_t mbls_bls_eth_fast_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, mbls_bin message,
                                           mbls_bin signature, size_t* err_got) {
  return counted(MBLS_OP_ETH_FAST_AGGREGATE_VERIFY, 1, n_keys, [&]() -> int32_t {
    const uint32_t off[2] = {0, (uint32_t)n_keys};
    int32_t r = 0;
    size_t got = 0;
    const int32_t rc = mbls_bls_fast_aggregate_verify_batch(public_keys, off, &message, &signature, 1, 1, &r, &got);
    if (err_got) *err_got = got;
    return rc ? rc : r;
  });
}

int32_t mbls_bls_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, const mbls_bin* messages,
                                  size_t n_messages, mbls_bin signature, size_t* err_got) {
  return counted(MBLS_OP_AGGREGATE_VERIFY, 1, n_keys, [&]() -> int32_t {
    const uint32_t koff[2] = {0, (uint32_t)n_keys};
    const uint32_t moff[2] = {0, (uint32_t)n_messages};
    int32_t r = 0;
    size_t got = 0;
    const int32_t rc = mbls_bls_aggregate_verify_batch(public_keys, koff, messages, moff, &signature, 1, &r, &got);
    if (err_got) *err_got = got;
    return rc ? rc : r;
  });
}

int32_t mbls_bls_eth_aggregate_pubkeys(const mbls_bin* public_keys, size_t n, uint8_t out48[48], size_t* err_got) {
  return counted(MBLS_OP_ETH_AGGREGATE_PUBKEYS, 1, n, [&]() -> int32_t {
    if (err_got) *err_got = 0;
    if (n == 0) return MBLS_ERR_EMPTY_PUBKEYS;  // lib.rs:127
    if (!public_keys || !out48 || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    Engine& e = pick_engine();
    Lease L(e);
    if (L.rc) return L.rc;
    auto* hp = pinned<uint8_t>(*L.c, H_PKS, 48 * n);
    auto* hkp = pinned<int32_t>(*L.c, H_KPRE, n);
    auto* ho = pinned<uint32_t>(*L.c, H_OFF, 2);
    auto* hst = pinned<int32_t>(*L.c, H_STATUS, 1);
    auto* hb = pinned<uint8_t>(*L.c, H_BYTES, 48);
    if (!hp || !hkp || !ho || !hst || !hb) return MBLS_ERR_DEVICE;
    pack_pks(public_keys, n, hp, hkp);
    ho[0] = 0;
    ho[1] = (uint32_t)n;
    {
      EngineLock g(e);
      if (int32_t r = init_locked(e, -1)) return r;
      const uint8_t* d_pks;
      const int32_t* d_kpre;
      const uint32_t* d_off;
      int32_t* d_st = L.dev<int32_t>(C_STATUS, 1);
      uint8_t* d_out = L.dev<uint8_t>(C_BYTES, 48);
      if (!d_st || !d_out) return MBLS_ERR_DEVICE;
      int32_t r = L.up(C_PKS, H_PKS, 48 * n, &d_pks);
      if (!r) r = L.up(C_KPRE, H_KPRE, n, &d_kpre);
      if (!r) r = L.up(C_OFF, H_OFF, 2, &d_off);
      if (!r) r = dev_agg_pks(e, d_pks, d_off, (uint32_t)n, 1, d_kpre, d_out, d_st, e.stream);
      if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t), e.stream);
      if (!r) r = L.down(H_BYTES, C_BYTES, 48, e.stream);
      if (!r) r = L.record(e.stream);
      if (r) return L.fail(r);
    }
    if (int32_t r = L.wait()) return r;
    std::memcpy(out48, hb, 48);
    const int32_t st = hst[0];
    if (st == MBLS_ERR_PUBKEY_LENGTH && err_got) *err_got = first_bad_len(public_keys, n, 48);
    return st;
  });
}

int32_t mbls_bls_aggregate(const mbls_bin* signatures, size_t n, uint8_t out96[96], size_t* err_got) {
  return counted(MBLS_OP_AGGREGATE, 1, 0, [&]() -> int32_t {
    if (err_got) *err_got = 0;
    if (n == 0) return MBLS_ERR_EMPTY_SIGNATURES;  // lib.rs:34
    if (!signatures || !out96 || n > UINT32_MAX) return MBLS_ERR_ARGUMENT;
    Engine& e = pick_engine();
    Lease L(e);
    if (L.rc) return L.rc;
    auto* hs = pinned<uint8_t>(*L.c, H_SIGS, 96 * n);
    auto* hsp = pinned<int32_t>(*L.c, H_SPRE, n);
    auto* ho = pinned<uint32_t>(*L.c, H_OFF, 2);
    auto* hst = pinned<int32_t>(*L.c, H_STATUS, 1);
    auto* hb = pinned<uint8_t>(*L.c, H_BYTES, 96);
    if (!hs || !hsp || !ho || !hst || !hb) return MBLS_ERR_DEVICE;
    pack_sigs(signatures, n, hs, hsp);
    ho[0] = 0;
    ho[1] = (uint32_t)n;
    {
      EngineLock g(e);
      if (int32_t r = init_locked(e, -1)) return r;
      const uint8_t* d_sigs;
      const int32_t* d_spre;
      const uint32_t* d_off;
      int32_t* d_st = L.dev<int32_t>(C_STATUS, 1);
      uint8_t* d_out = L.dev<uint8_t>(C_BYTES, 96);
      if (!d_st || !d_out) return MBLS_ERR_DEVICE;
      if (!e.buf[S_SIG_ST].ensure(sizeof(int32_t) * n) || !e.buf[S_SIG_XY].ensure(sizeof(uint32_t) * 56 * n))
        return MBLS_ERR_DEVICE;
      int32_t r = L.up(C_SIGS, H_SIGS, 96 * n, &d_sigs);
      if (!r) r = L.up(C_SPRE, H_SPRE, n, &d_spre);
      if (!r) r = L.up(C_OFF, H_OFF, 2, &d_off);
      if (!r) r = scratch_begin(e, e.stream);
      if (!r && mbls_launch::g2_sig_decode(d_sigs, (uint32_t)n, 0, d_spre, e.buf[S_SIG_ST].as<int32_t>(),
                                           e.buf[S_SIG_XY].as<uint32_t>(), e.stream) != hipSuccess)
        r = MBLS_ERR_DEVICE;
      if (!r && mbls_launch::g2_aggregate(e.buf[S_SIG_ST].as<int32_t>(), e.buf[S_SIG_XY].as<uint32_t>(), (uint32_t)n,
                                          d_off, 1, d_out, d_st, e.stream) != hipSuccess)
        r = MBLS_ERR_DEVICE;
      if (!r) r = scratch_end(e, e.stream);
      if (!r) r = L.down(H_STATUS, C_STATUS, sizeof(int32_t), e.stream);
      if (!r) r = L.down(H_BYTES, C_BYTES, 96, e.stream);
      if (!r) r = L.record(e.stream);
      if (r) return L.fail(r);
    }
    if (int32_t r = L.wait()) return r;
    std::memcpy(out96, hb, 96);
    return hst[0];
  });
}

int32_t mbls_bls_sign(mbls_bin private_key, mbls_bin message, uint8_t out96[96], size_t* err_got) {
  return counted(MBLS_OP_SIGN, 1, 0, [&]() -> int32_t {
    if (err_got) *err_got = 0;
    if (!out96) return MBLS_ERR_ARGUMENT;
    // lighthouse SecretKey::deserialize (lib.rs:20): length, all-zero, then blst sk < r
    if (private_key.len != 32 || !private_key.data) {
      if (err_got) *err_got = private_key.len;
      return MBLS_ERR_SECRET_KEY_LENGTH;
    }
    bool zero = true;
    for (int i = 0; i < 32; ++i) zero &= private_key.data[i] == 0;
    if (zero) return MBLS_ERR_ZERO_SECRET_KEY;
    if (std::memcmp(private_key.data, R_BE, 32) >= 0) return MBLS_ERR_BAD_ENCODING;
    if (message.len != 32 || !message.data) {  // Hash256::from_slice (lib.rs:25)
      if (err_got) *err_got = message.len;
      return MBLS_ERR_MESSAGE_LENGTH;
    }
    Engine& e = pick_engine();
    Lease L(e);
    if (L.rc) return L.rc;
    auto* hk = pinned<uint8_t>(*L.c, H_PKS, 32);
    auto* hm = pinned<uint8_t>(*L.c, H_MSGS, 32);
    auto* hb = pinned<uint8_t>(*L.c, H_BYTES, 96);
    if (!hk || !hm || !hb) return MBLS_ERR_DEVICE;
    std::memcpy(hk, private_key.data, 32);
    std::memcpy(hm, message.data, 32);
    {
      EngineLock g(e);
      if (int32_t r = init_locked(e, -1)) return r;
      const uint8_t *d_sk, *d_m;
      uint8_t* d_out = L.dev<uint8_t>(C_BYTES, 96);
      if (!d_out) return MBLS_ERR_DEVICE;
      int32_t r = L.up(C_PKS, H_PKS, 32, &d_sk);
      if (!r) r = L.up(C_MSGS, H_MSGS, 32, &d_m);
      if (!r && use_once(mbls_scratch::UO_SIGN, 1, e.stream,
                         [&] { return mbls_launch::sign(d_sk, d_m, 1, d_out, e.stream); }) != hipSuccess)
        r = MBLS_ERR_DEVICE;
      if (!r) r = L.down(H_BYTES, C_BYTES, 96, e.stream);
      if (!r) r = L.record(e.stream);
      if (r) return L.fail(r);
    }
    if (int32_t r = L.wait()) return r;
    std::memcpy(out96, hb, 96);
    std::memset(hk, 0, 32);  // the secret key's staging copy does not outlive the call
    return MBLS_OK;
  });
}

}  // extern "C"
