// mbls_queue.cpp — the batching queue of SURVEY.md §8f-1, in the engine.
//
// The reference verifies one signature set per NIF call: gossip attestations one at a time
// (gossip_consumer.ex:15-18, Broadway concurrency 1), the state transition per operation
// (operations.ex:52,367,470, predicates.ex:128).  A GPU needs thousands of sets per launch, so
// concurrent single-set callers (BEAM dirty schedulers calling the NIF, Python threads) are
// coalesced here: each call enqueues a request that borrows the caller's buffers and blocks;
// worker threads flush the pending requests as *_batch device submissions when `max_sets` are
// pending or `max_wait_us` after the oldest arrived, then wake every caller with exactly the
// result the per-call API returns for its set.  Two workers by default (MBLS_QUEUE_WORKERS):
// the engine pipelines layer-1 calls, so batch i+1's staging and key validation overlap
// batch i's G2 chain.  Bls.* and its callers stay
// unchanged; the NIF shim routes through the queue when it is running.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mbls.h"

namespace {

enum Kind { K_VERIFY = 0, K_FAV = 1, K_ETH_FAV = 2, K_NKINDS };

struct Request {
  Kind kind;
  const mbls_bin* pks;  // FAV: n_keys keys; verify: one key
  size_t n_keys;
  mbls_bin msg, sig;
  int32_t result = 0;
  size_t got = 0;
  bool done = false;
};

struct Queue {
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<Request*> pending;
  std::vector<std::thread> workers;
  bool running = false, stopping = false;
  uint32_t max_sets = 4096;
  std::chrono::microseconds max_wait{500};
  std::chrono::steady_clock::time_point oldest;
  uint64_t batches = 0, sets = 0;
};

Queue& q() {
  static Queue s;
  return s;
}

// one device submission per kind present in `batch`
void flush(std::vector<Request*>& batch) {
  for (int k = 0; k < K_NKINDS; ++k) {
    std::vector<Request*> rs;
    for (Request* r : batch)
      if (r->kind == k) rs.push_back(r);
    if (rs.empty()) continue;
    const size_t n = rs.size();
    std::vector<mbls_bin> msgs(n), sigs(n), keys;
    std::vector<uint32_t> off(n + 1, 0);
    for (size_t i = 0; i < n; ++i) {
      msgs[i] = rs[i]->msg;
      sigs[i] = rs[i]->sig;
      for (size_t j = 0; j < rs[i]->n_keys; ++j) keys.push_back(rs[i]->pks[j]);
      off[i + 1] = (uint32_t)keys.size();
    }
    std::vector<int32_t> res(n, 0);
    std::vector<size_t> got(n, 0);
    int32_t rc;
    const mbls_bin* kp = keys.empty() ? nullptr : keys.data();
    if (k == K_VERIFY)
      rc = mbls_bls_verify_batch(kp, msgs.data(), sigs.data(), n, res.data(), got.data());
    else
      rc = mbls_bls_fast_aggregate_verify_batch(kp, off.data(), msgs.data(), sigs.data(), n, k == K_ETH_FAV ? 1 : 0,
                                                res.data(), got.data());
    for (size_t i = 0; i < n; ++i) {
      rs[i]->result = rc ? rc : res[i];
      rs[i]->got = rc ? 0 : got[i];
    }
  }
}

void worker_main() {
  Queue& Q = q();
  std::unique_lock<std::mutex> lk(Q.mu);
  for (;;) {
    Q.cv_work.wait(lk, [&] { return Q.stopping || !Q.pending.empty(); });
    if (Q.pending.empty()) {
      if (Q.stopping) return;
      continue;  // another worker took the batch
    }
    // wait for a full batch or the deadline of the oldest request
    const auto deadline = Q.oldest + Q.max_wait;
    Q.cv_work.wait_until(lk, deadline, [&] { return Q.stopping || Q.pending.size() >= Q.max_sets; });
    if (Q.pending.empty()) continue;  // another worker flushed it meanwhile
    std::vector<Request*> batch;
    while (!Q.pending.empty() && batch.size() < Q.max_sets) {
      batch.push_back(Q.pending.front());
      Q.pending.pop_front();
    }
    if (!Q.pending.empty()) {
      Q.oldest = std::chrono::steady_clock::now();
      Q.cv_work.notify_one();  // an idle worker takes the remainder while this batch runs
    }
    lk.unlock();
    flush(batch);
    lk.lock();
    Q.batches += 1;
    Q.sets += batch.size();
    for (Request* r : batch) r->done = true;
    Q.cv_done.notify_all();
  }
}

int32_t submit(Request& r) {
  Queue& Q = q();
  std::unique_lock<std::mutex> lk(Q.mu);
  if (!Q.running || Q.stopping) return MBLS_ERR_ARGUMENT;  // queue not started
  if (Q.pending.empty()) Q.oldest = std::chrono::steady_clock::now();
  Q.pending.push_back(&r);
  if (Q.pending.size() >= Q.max_sets || Q.pending.size() == 1) Q.cv_work.notify_one();
  Q.cv_done.wait(lk, [&] { return r.done; });
  return r.result;
}

}  // namespace

extern "C" {

int32_t mbls_queue_start(uint32_t max_sets, uint32_t max_wait_us) {
  Queue& Q = q();
  std::lock_guard<std::mutex> g(Q.mu);
  if (Q.running) return 0;
  Q.max_sets = max_sets ? max_sets : 4096;
  Q.max_wait = std::chrono::microseconds(max_wait_us);
  Q.stopping = false;
  Q.batches = Q.sets = 0;
  const char* w = std::getenv("MBLS_QUEUE_WORKERS");
  const int n_workers = w ? std::max(1, std::min(8, std::atoi(w))) : 2;
  for (int i = 0; i < n_workers; ++i) Q.workers.emplace_back(worker_main);
  Q.running = true;
  return 0;
}

int32_t mbls_queue_stop(void) {
  Queue& Q = q();
  {
    std::lock_guard<std::mutex> g(Q.mu);
    if (!Q.running) return 0;
    Q.stopping = true;
  }
  Q.cv_work.notify_all();
  for (auto& t : Q.workers) t.join();
  Q.workers.clear();
  std::lock_guard<std::mutex> g(Q.mu);
  Q.running = false;
  Q.stopping = false;
  return 0;
}

int32_t mbls_queue_running(void) {
  Queue& Q = q();
  std::lock_guard<std::mutex> g(Q.mu);
  return Q.running && !Q.stopping;
}

int32_t mbls_queue_stats(uint64_t* batches, uint64_t* sets) {
  Queue& Q = q();
  std::lock_guard<std::mutex> g(Q.mu);
  if (batches) *batches = Q.batches;
  if (sets) *sets = Q.sets;
  return 0;
}

int32_t mbls_queue_verify(mbls_bin public_key, mbls_bin message, mbls_bin signature, size_t* err_got) {
  Request r{K_VERIFY, &public_key, 1, message, signature};
  const int32_t rc = submit(r);
  if (err_got) *err_got = r.got;
  return rc;
}

int32_t mbls_queue_fast_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, mbls_bin message,
                                         mbls_bin signature, int32_t eth_variant, size_t* err_got) {
  if (n_keys && !public_keys) return MBLS_ERR_ARGUMENT;
  Request r{eth_variant ? K_ETH_FAV : K_FAV, public_keys, n_keys, message, signature};
  const int32_t rc = submit(r);
  if (err_got) *err_got = r.got;
  return rc;
}

}  // extern "C"
