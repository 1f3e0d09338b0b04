// TEST-ONLY: the batching queue (csrc/mbls_queue.cpp) with its two workers under TSan or
// ASan/UBSan, over a host-only fake of the two layer-1 batch calls it flushes into (no GPU).
// The fake's verdict is a function of the request's bytes, so every caller can check that
// it got its own result back; batches must coalesce.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "mbls.h"

static std::atomic<int> g_calls{0};

static int32_t verdict(const mbls_bin* pks, size_t n, mbls_bin msg, mbls_bin sig) {
  if (msg.len != 32) return MBLS_ERR_MESSAGE_LENGTH;
  for (size_t i = 0; i < n; ++i)
    if (pks[i].len != 48) return MBLS_ERR_PUBKEY_LENGTH;
  unsigned x = sig.data[0] ^ msg.data[0];
  for (size_t i = 0; i < n; ++i) x ^= pks[i].data[0];
  return (int32_t)(x & 1u);
}

extern "C" int32_t mbls_bls_verify_batch(const mbls_bin* pks, const mbls_bin* msgs, const mbls_bin* sigs, size_t n,
                                         int32_t* results, size_t* err_got) {
  g_calls++;
  std::this_thread::sleep_for(std::chrono::microseconds(300));  // a device call in flight
  for (size_t i = 0; i < n; ++i) {
    results[i] = verdict(&pks[i], 1, msgs[i], sigs[i]);
    err_got[i] = results[i] < 0 ? 1 : 0;
  }
  return 0;
}
extern "C" int32_t mbls_bls_fast_aggregate_verify_batch(const mbls_bin* pks, const uint32_t* key_off,
                                                        const mbls_bin* msgs, const mbls_bin* sigs, size_t n,
                                                        int32_t eth, int32_t* results, size_t* err_got) {
  g_calls++;
  std::this_thread::sleep_for(std::chrono::microseconds(300));
  for (size_t i = 0; i < n; ++i) {
    const uint32_t nk = key_off[i + 1] - key_off[i];
    results[i] = nk == 0 ? (eth ? 1 : 0) : verdict(pks + key_off[i], nk, msgs[i], sigs[i]);
    err_got[i] = 0;
  }
  return 0;
}

int main() {
  if (mbls_queue_start(32, 500) != 0) return 1;
  const int T = 48, R = 25;
  std::vector<std::thread> th;
  std::atomic<int> bad{0};
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      std::vector<uint8_t> buf(96 * 8);
      for (int r = 0; r < R; ++r) {
        for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(t * 31 + r * 7 + i);
        mbls_bin pk[5];
        const size_t nk = (size_t)((t + r) % 6);
        for (size_t i = 0; i < 5; ++i) pk[i] = {buf.data() + 96 * (i + 1), 48};
        mbls_bin msg{buf.data(), (size_t)((t + r) % 17 == 0 ? 31 : 32)}, sig{buf.data() + 32, 96};
        size_t got = 0;
        int32_t rc, want;
        if (r % 3 == 0) {
          rc = mbls_queue_verify(pk[0], msg, sig, &got);
          want = verdict(pk, 1, msg, sig);
        } else {
          const int eth = r % 2;
          rc = mbls_queue_fast_aggregate_verify(pk, nk > 5 ? 5 : nk, msg, sig, eth, &got);
          want = nk == 0 ? (eth ? 1 : 0) : verdict(pk, nk > 5 ? 5 : nk, msg, sig);
        }
        if (rc != want) bad++;
      }
    });
  for (auto& x : th) x.join();
  uint64_t batches = 0, sets = 0;
  mbls_queue_stats(&batches, &sets);
  mbls_queue_stop();
  if (mbls_queue_verify(mbls_bin{nullptr, 0}, mbls_bin{nullptr, 0}, mbls_bin{nullptr, 0}, nullptr) !=
      MBLS_ERR_ARGUMENT)
    return 1;  // stopped queue refuses
  std::printf("queue OK batches=%llu sets=%llu device_calls=%d bad=%d\n", (unsigned long long)batches,
              (unsigned long long)sets, g_calls.load(), bad.load());
  return (bad == 0 && sets == (uint64_t)(T * R) && batches < sets / 2) ? 0 : 1;
}
