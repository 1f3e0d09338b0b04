// TEST-ONLY: the engine's host-side staging and batch split (csrc/mbls_host.hpp) under
// ASan/UBSan or TSan (tests/test_sanitizers.py).  par_for packs with up to 8 threads above
// 2^15 elements; several caller threads stage at once, as concurrent layer-1 calls do.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "mbls_host.hpp"

using namespace mbls_host;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL %s\n", what);
  return 1;
}

static int stage_once(unsigned seed, size_t n) {
  std::mt19937 rng(seed);
  std::vector<std::vector<uint8_t>> store(n);
  std::vector<mbls_bin> pks(n), sigs(n), msgs(n);
  for (size_t i = 0; i < n; ++i) {
    const size_t len = (rng() % 50 == 0) ? rng() % 100 : 48 + (i % 3 == 0 ? 48 : 0);
    store[i].resize(std::max<size_t>(len, 96));
    for (auto& b : store[i]) b = (uint8_t)rng();
    pks[i] = {store[i].data(), (i % 7 == 0) ? (size_t)47 : (size_t)48};
    sigs[i] = {store[i].data(), (i % 11 == 0) ? (size_t)95 : (size_t)96};
    msgs[i] = {store[i].data(), (i % 13 == 0) ? (size_t)31 : (size_t)32};
  }
  std::vector<uint8_t> pk_out(48 * n), sig_out(96 * n), msg_out(32 * n);
  std::vector<int32_t> kpre(n), spre(n), setpre(n);
  pack_pks(pks.data(), n, pk_out.data(), kpre.data());
  pack_sigs(sigs.data(), n, sig_out.data(), spre.data());
  pack_msgs(msgs.data(), n, msg_out.data(), setpre.data());
  for (size_t i = 0; i < n; ++i) {
    const bool pk_ok = i % 7 != 0, sig_ok = i % 11 != 0, msg_ok = i % 13 != 0;
    if ((kpre[i] == MBLS_DEC_OK) != pk_ok || (spre[i] == MBLS_DEC_OK) != sig_ok || (setpre[i] == 0) != msg_ok)
      return fail("pre-status");
    if (pk_ok && std::memcmp(pk_out.data() + 48 * i, store[i].data(), 48)) return fail("pk bytes");
    if (sig_ok && std::memcmp(sig_out.data() + 96 * i, store[i].data(), 96)) return fail("sig bytes");
    if (msg_ok && std::memcmp(msg_out.data() + 32 * i, store[i].data(), 32)) return fail("msg bytes");
  }
  return 0;
}

static int check_plan(std::mt19937& rng) {
  const uint32_t parts = 1 + rng() % 9;
  const size_t n = rng() % 3000;
  std::vector<uint32_t> off(n + 1, 0);
  for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + (rng() % 4 == 0 ? 0 : rng() % 2049);
  std::vector<uint32_t> b(parts + 1);
  plan_shards(n ? off.data() : nullptr, n, parts, b.data());
  if (b[0] != 0 || b[parts] != n) return fail("plan ends");
  uint64_t maxset = 0;
  for (size_t i = 0; i < n; ++i) maxset = std::max<uint64_t>(maxset, off[i + 1] - off[i] + kSetWeight);
  const uint64_t total = n ? prefix_cost(off.data(), n) : 0;
  for (uint32_t j = 0; j < parts; ++j) {
    if (b[j] > b[j + 1]) return fail("plan order");
    const uint64_t c = n ? prefix_cost(off.data(), b[j + 1]) - prefix_cost(off.data(), b[j]) : 0;
    if (c > total / parts + 2 * maxset) return fail("plan balance");
  }
  return 0;
}

int main() {
  // several callers staging concurrently, each big enough for par_for to use its threads
  std::vector<std::thread> th;
  std::vector<int> rc(4, 0);
  for (int t = 0; t < 4; ++t) th.emplace_back([&rc, t] { rc[t] = stage_once(100 + t, (size_t)100000 + 777 * t); });
  for (auto& x : th) x.join();
  for (int r : rc)
    if (r) return r;
  if (stage_once(7, 0) || stage_once(8, 1) || stage_once(9, 40000)) return 1;
  std::mt19937 rng(5);
  for (int i = 0; i < 300; ++i)
    if (check_plan(rng)) return 1;
  std::puts("host staging OK");
  return 0;
}
