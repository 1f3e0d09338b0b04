/* TEST-ONLY: both NIF shims (Elixir.Bls, Elixir.Bls.Device) under ASan/UBSan on the CPU
 * (tests/test_sanitizers.py).  The shims are compiled with nif_init renamed per module and
 * linked with the fake BEAM term model (tests/nif_stub/fake_beam.c), the real status strings
 * (csrc/mbls_status.cpp), the real batching queue (csrc/mbls_queue.cpp) and the host-only fake
 * of libmbls below, whose outcome is a function of the bytes, so every success, error, raise
 * and badarg path of the shims runs, including their list walks, mallocs and frees.
 * Prints "nif OK" and exits 0 when every call rendered as expected. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "erl_nif.h"
#include "mbls.h"

const ErlNifEntry* bls_nif_init(void);
const ErlNifEntry* dev_nif_init(void);
void fb_reset(void);
ERL_NIF_TERM fb_bin(const void* data, size_t len);
ERL_NIF_TERM fb_list(const ERL_NIF_TERM* elems, size_t n);
ERL_NIF_TERM fb_uint(unsigned long v);
size_t fb_show(ERL_NIF_TERM t, char* out, size_t cap);

/* ------------------------------------------------------------ fake libmbls -------- */
static uint32_t g_rows;
static unsigned char g_table[1024];

int32_t mbls_init(int32_t device) { return device == 0 ? 0 : MBLS_ERR_DEVICE; }
int32_t mbls_init_devices(const int32_t* d, uint32_t n) { return (n && d[0] == 0) ? 0 : MBLS_ERR_DEVICE; }

/* the fake's verdict: a 0xDE signature byte is a device fault, else the low bit of a xor */
static int32_t fake_verdict(const mbls_bin* pks, size_t n, mbls_bin msg, mbls_bin sig, size_t* got) {
  if (sig.len != 96) return MBLS_ERR_BAD_ENCODING;
  if (sig.data[0] == 0xDE) return MBLS_ERR_DEVICE;
  for (size_t i = 0; i < n; ++i)
    if (pks[i].len != 48) {
      *got = pks[i].len;
      return MBLS_ERR_PUBKEY_LENGTH;
    }
  if (msg.len != 32) {
    *got = msg.len;
    return MBLS_ERR_MESSAGE_LENGTH;
  }
  unsigned x = sig.data[1] ^ msg.data[0];
  for (size_t i = 0; i < n; ++i) x ^= pks[i].data[47];
  return (int32_t)(x & 1u);
}

int32_t mbls_bls_sign(mbls_bin sk, mbls_bin msg, uint8_t out96[96], size_t* got) {
  if (sk.len != 32) {
    *got = sk.len;
    return MBLS_ERR_SECRET_KEY_LENGTH;
  }
  if (msg.len != 32) {
    *got = msg.len;
    return MBLS_ERR_MESSAGE_LENGTH;
  }
  for (int i = 0; i < 96; ++i) out96[i] = (uint8_t)(sk.data[i % 32] ^ msg.data[(i + 5) % 32]);
  return MBLS_OK;
}
int32_t mbls_bls_aggregate(const mbls_bin* s, size_t n, uint8_t out96[96], size_t* got) {
  (void)got;
  if (!n) return MBLS_ERR_EMPTY_SIGNATURES;
  memset(out96, 0, 96);
  for (size_t i = 0; i < n; ++i) {
    if (s[i].len != 96) return MBLS_ERR_BAD_ENCODING;
    for (int j = 0; j < 96; ++j) out96[j] ^= s[i].data[j];
  }
  return MBLS_OK;
}
int32_t mbls_bls_verify(mbls_bin pk, mbls_bin msg, mbls_bin sig, size_t* got) { return fake_verdict(&pk, 1, msg, sig, got); }
int32_t mbls_bls_aggregate_verify(const mbls_bin* pks, size_t npk, const mbls_bin* msgs, size_t nm, mbls_bin sig,
                                  size_t* got) {
  if (npk != nm || !npk) return MBLS_FALSE;
  int32_t r = MBLS_TRUE;
  for (size_t i = 0; i < npk; ++i) {
    int32_t v = fake_verdict(&pks[i], 1, msgs[i], sig, got);
    if (v < 0) return v;
    r &= v;
  }
  return r;
}
int32_t mbls_bls_fast_aggregate_verify(const mbls_bin* pks, size_t n, mbls_bin msg, mbls_bin sig, size_t* got) {
  return n ? fake_verdict(pks, n, msg, sig, got) : MBLS_FALSE;
}
int32_t mbls_bls_eth_fast_aggregate_verify(const mbls_bin* pks, size_t n, mbls_bin msg, mbls_bin sig, size_t* got) {
  return n ? fake_verdict(pks, n, msg, sig, got) : MBLS_TRUE;
}
int32_t mbls_bls_eth_aggregate_pubkeys(const mbls_bin* pks, size_t n, uint8_t out48[48], size_t* got) {
  if (!n) return MBLS_ERR_EMPTY_PUBKEYS;
  memset(out48, 0, 48);
  for (size_t i = 0; i < n; ++i) {
    if (pks[i].len != 48) {
      *got = pks[i].len;
      return MBLS_ERR_PUBKEY_LENGTH;
    }
    for (int j = 0; j < 48; ++j) out48[j] ^= pks[i].data[j];
  }
  return MBLS_OK;
}
/* layer-1 batches (the queue flushes into these) */
int32_t mbls_bls_verify_batch(const mbls_bin* pks, const mbls_bin* msgs, const mbls_bin* sigs, size_t n,
                              int32_t* results, size_t* err_got) {
  for (size_t i = 0; i < n; ++i) {
    err_got[i] = 0;
    results[i] = fake_verdict(&pks[i], 1, msgs[i], sigs[i], &err_got[i]);
  }
  return 0;
}
int32_t mbls_bls_fast_aggregate_verify_batch(const mbls_bin* pks, const uint32_t* key_off, const mbls_bin* msgs,
                                             const mbls_bin* sigs, size_t n, int32_t eth, int32_t* results,
                                             size_t* err_got) {
  for (size_t i = 0; i < n; ++i) {
    const size_t k = key_off[i + 1] - key_off[i];
    err_got[i] = 0;
    results[i] = k ? fake_verdict(pks + key_off[i], k, msgs[i], sigs[i], &err_got[i]) : (eth ? MBLS_TRUE : MBLS_FALSE);
  }
  return 0;
}
int32_t mbls_pk_table_set(uint32_t first, const uint8_t* pks48, uint32_t n, int32_t* status) {
  if (first + n > sizeof g_table) return MBLS_ERR_DEVICE;
  for (uint32_t i = 0; i < n; ++i) {
    status[i] = pks48[48 * i] == 0xFF ? MBLS_ERR_NOT_ON_CURVE : 0;
    g_table[first + i] = status[i] == 0 ? pks48[48 * i + 47] : 0;
  }
  if (first + n > g_rows) g_rows = first + n;
  return 0;
}
uint32_t mbls_pk_table_size(void) { return g_rows; }
int32_t mbls_fast_aggregate_verify_indexed_batch(const uint32_t* idx, const uint32_t* off, const mbls_bin* msgs,
                                                 const mbls_bin* sigs, size_t n, int32_t eth, int32_t* res,
                                                 size_t* got) {
  for (size_t s = 0; s < n; ++s) {
    got[s] = 0;
    if (off[s + 1] == off[s]) {
      res[s] = eth ? MBLS_TRUE : MBLS_FALSE;
      continue;
    }
    if (sigs[s].len != 96) {
      res[s] = MBLS_ERR_BAD_ENCODING;
      continue;
    }
    if (sigs[s].data[0] == 0xDE) return MBLS_ERR_DEVICE;
    unsigned x = sigs[s].data[1];
    res[s] = MBLS_TRUE;
    for (uint32_t j = off[s]; j < off[s + 1]; ++j) {
      if (idx[j] >= g_rows) {
        res[s] = MBLS_ERR_UNKNOWN_INDEX;
        break;
      }
      x ^= g_table[idx[j]];
    }
    if (res[s] == MBLS_TRUE && msgs[s].len != 32) {
      got[s] = msgs[s].len;
      res[s] = MBLS_ERR_MESSAGE_LENGTH;
    }
    if (res[s] == MBLS_TRUE) res[s] = (int32_t)((x ^ msgs[s].data[0]) & 1u);
  }
  return 0;
}
int32_t mbls_eth_aggregate_pubkeys_indexed(const uint32_t* idx, size_t n, uint8_t out48[48]) {
  if (!n) return MBLS_ERR_EMPTY_PUBKEYS;
  memset(out48, 0, 48);
  for (size_t i = 0; i < n; ++i) {
    if (idx[i] >= g_rows) return MBLS_ERR_UNKNOWN_INDEX;
    out48[i % 48] ^= g_table[idx[i]];
  }
  return MBLS_OK;
}
int32_t mbls_attestation_data_signing_roots(const uint8_t* d, const uint8_t* dom, uint32_t stride, size_t n,
                                            uint8_t* out32) {
  (void)stride;
  for (size_t i = 0; i < n; ++i)
    for (int j = 0; j < 32; ++j) out32[32 * i + j] = (uint8_t)(d[128 * i + j] ^ d[128 * i + 127 - j] ^ dom[j]);
  return 0;
}
static const char* const g_op_names[MBLS_OP_COUNT] = {"verify", "fast_aggregate_verify", "eth_fast_aggregate_verify",
                                                     "aggregate_verify", "eth_aggregate_pubkeys", "aggregate",
                                                     "sign", "key_validate", "signing_roots"};
const char* mbls_op_name(int32_t op) { return op >= 0 && op < MBLS_OP_COUNT ? g_op_names[op] : NULL; }
int32_t mbls_stats_read(mbls_op_stats* out, int32_t n, int32_t reset) {
  (void)reset;
  const int32_t m = n < MBLS_OP_COUNT ? n : MBLS_OP_COUNT;
  for (int32_t i = 0; i < m; ++i) {
    out[i].calls = (uint64_t)i + 1;
    out[i].sets = 10u * (uint64_t)i;
    out[i].keys = 100u * (uint64_t)i;
    out[i].errors = 0;
    out[i].ns = 1000u * (uint64_t)i;
  }
  return m;
}

/* ------------------------------------------------------------------ driver -------- */
typedef ERL_NIF_TERM (*nif_fn)(ErlNifEnv*, int, const ERL_NIF_TERM[]);
static int g_bad;

static ERL_NIF_TERM call(const ErlNifEntry* e, const char* name, int argc, const ERL_NIF_TERM* argv) {
  for (int i = 0; i < e->num_of_funcs; ++i)
    if (!strcmp(e->funcs[i].name, name) && (int)e->funcs[i].arity == argc)
      return ((nif_fn)e->funcs[i].fptr)(NULL, argc, argv);
  fprintf(stderr, "no %s/%d\n", name, argc);
  exit(2);
}

static void expect(const ErlNifEntry* e, const char* name, int argc, const ERL_NIF_TERM* argv, const char* want) {
  char buf[1024];
  fb_show(call(e, name, argc, argv), buf, sizeof buf);
  if (strncmp(buf, want, strlen(want)) != 0) {
    fprintf(stderr, "%s: got %s want %s\n", name, buf, want);
    g_bad++;
  }
}

static ERL_NIF_TERM bin_of(int len, int fill) {
  unsigned char b[256];
  memset(b, fill, sizeof b);
  return fb_bin(b, (size_t)len);
}
static ERL_NIF_TERM list_of(int n, int len, int fill) {
  ERL_NIF_TERM t[600];
  for (int i = 0; i < n; ++i) t[i] = bin_of(len, fill);
  return fb_list(t, (size_t)n);
}

struct qarg {
  const ErlNifEntry* e;
  int id;
};
static pthread_mutex_t g_term_mu = PTHREAD_MUTEX_INITIALIZER;

static void scenario(const ErlNifEntry* bls, const ErlNifEntry* dev) {
  ERL_NIF_TERM a[3];
  /* Elixir.Bls: success, reference-visible errors, raises, badarg */
  a[0] = bin_of(32, 1), a[1] = bin_of(32, 2);
  expect(bls, "sign", 2, a, "{ok,<<3,3,3");
  a[0] = bin_of(31, 1);
  expect(bls, "sign", 2, a, "{error,<<\"InvalidSecretKeyLength { got: 31, expected: 32 }\">>}");
  a[0] = list_of(3, 96, 7);
  expect(bls, "aggregate", 1, a, "{ok,<<7,7");
  a[0] = fb_list(NULL, 0);
  expect(bls, "aggregate", 1, a, "{error,<<\"Empty signature vector\">>}");
  a[0] = bin_of(48, 1), a[1] = bin_of(32, 2), a[2] = bin_of(96, 0);
  expect(bls, "verify", 3, a, "{ok,true}");  /* 0 ^ 2 ^ 1 = 3 -> low bit 1 */
  a[2] = bin_of(96, 0xDE);
  expect(bls, "verify", 3, a, "raise:{bls_device_error,<<\"DeviceError\">>}");
  a[0] = bin_of(47, 1), a[2] = bin_of(96, 0);
  expect(bls, "verify", 3, a, "{error,<<\"InvalidByteLength { got: 47, expected: 48 }\">>}");
  a[0] = list_of(512, 48, 3), a[1] = bin_of(32, 2), a[2] = bin_of(96, 0);
  expect(bls, "fast_aggregate_verify", 3, a, "{ok,false}");  /* 512 x 3 cancels: 2 -> 0 */
  a[0] = list_of(511, 48, 3);
  expect(bls, "eth_fast_aggregate_verify", 3, a, "{ok,true}");
  a[0] = fb_list(NULL, 0);
  expect(bls, "eth_fast_aggregate_verify", 3, a, "{ok,true}");
  expect(bls, "fast_aggregate_verify", 3, a, "{ok,false}");
  a[0] = list_of(4, 48, 3), a[1] = bin_of(31, 2);
  expect(bls, "fast_aggregate_verify", 3, a, "{error,<<\"InvalidMessageLength { got: 31, expected: 32 }\">>}");
  a[0] = list_of(2, 48, 3), a[1] = list_of(2, 32, 2), a[2] = bin_of(96, 0);
  expect(bls, "aggregate_verify", 3, a, "{ok,true}");
  a[1] = bin_of(32, 2);
  expect(bls, "aggregate_verify", 3, a, "badarg");
  a[0] = list_of(512, 48, 9);
  expect(bls, "eth_aggregate_pubkeys", 1, a, "{ok,<<");
  {
    ERL_NIF_TERM mixed[2] = {bin_of(48, 1), fb_uint(5)};
    a[0] = fb_list(mixed, 2);
    expect(bls, "eth_aggregate_pubkeys", 1, a, "badarg");
  }
  /* Elixir.Bls.Device */
  {
    ERL_NIF_TERM rows[5] = {bin_of(48, 1), bin_of(48, 0xFF), bin_of(48, 2), bin_of(48, 3), bin_of(48, 4)};
    a[0] = fb_uint(0), a[1] = fb_list(rows, 5);
    expect(dev, "pk_table_set", 2, a, "{ok,[ok,{error,<<\"BlstError(BLST_POINT_NOT_ON_CURVE)\">>},ok,ok,ok]}");
    rows[2] = bin_of(47, 2);
    a[1] = fb_list(rows, 5);
    expect(dev, "pk_table_set", 2, a, "badarg");
  }
  expect(dev, "pk_table_size", 0, a, "5");
  expect(dev, "stats", 0, a, "[{verify,1,0,0,0,0},{fast_aggregate_verify,2,10,100,0,1}");
  {
    ERL_NIF_TERM ix[3] = {fb_uint(0), fb_uint(2), fb_uint(3)};
    a[0] = fb_list(ix, 3), a[1] = bin_of(32, 1), a[2] = bin_of(96, 0);
    expect(dev, "fast_aggregate_verify_indices", 3, a, "{ok,true}");  /* 1^2^3^1 = 1 */
    ix[1] = fb_uint(77);
    a[0] = fb_list(ix, 3);
    expect(dev, "eth_fast_aggregate_verify_indices", 3, a, "{error,<<\"UnknownValidatorIndex\">>}");
    a[2] = bin_of(96, 0xDE);
    expect(dev, "fast_aggregate_verify_indices", 3, a, "raise:{bls_device_error,<<\"DeviceError\">>}");
    a[0] = fb_list(NULL, 0), a[2] = bin_of(96, 0);
    expect(dev, "eth_fast_aggregate_verify_indices", 3, a, "{ok,true}");
    ix[1] = fb_uint(4);
    a[0] = fb_list(ix, 3);
    expect(dev, "eth_aggregate_pubkeys_indices", 1, a, "{ok,<<");
    a[0] = fb_list(NULL, 0);
    expect(dev, "eth_aggregate_pubkeys_indices", 1, a, "{error,<<\"Empty public key vector\">>}");
  }
  {
    unsigned char d[3 * 128];
    for (int i = 0; i < (int)sizeof d; ++i) d[i] = (unsigned char)i;
    a[0] = fb_bin(d, sizeof d), a[1] = bin_of(32, 0);
    expect(dev, "attestation_signing_roots", 2, a, "{ok,<<");
    a[0] = fb_bin(d, 127);
    expect(dev, "attestation_signing_roots", 2, a, "badarg");
  }
}

/* with the queue running, concurrent callers of the verify entries; terms are built and
 * rendered under a lock (the fake term heap is single-threaded), the NIF calls run unlocked */
static void* queue_caller(void* p) {
  struct qarg* q = (struct qarg*)p;
  for (int r = 0; r < 20; ++r) {
    ERL_NIF_TERM a[3];
    pthread_mutex_lock(&g_term_mu);
    const int n = 1 + (q->id + r) % 5;
    a[0] = list_of(n, 48, 3), a[1] = bin_of(32, 2), a[2] = bin_of(96, r & 1);
    pthread_mutex_unlock(&g_term_mu);
    ERL_NIF_TERM out = call(q->e, "fast_aggregate_verify", 3, a);
    pthread_mutex_lock(&g_term_mu);
    char buf[64];
    fb_show(out, buf, sizeof buf);
    const unsigned x = (unsigned)(r & 1) ^ 2u ^ (n & 1 ? 3u : 0u);
    if (strcmp(buf, (x & 1) ? "{ok,true}" : "{ok,false}") != 0) g_bad++;
    pthread_mutex_unlock(&g_term_mu);
  }
  return NULL;
}

int main(void) {
  const ErlNifEntry* bls = bls_nif_init();
  const ErlNifEntry* dev = dev_nif_init();
  if (bls->load(NULL, NULL, 0) != 0 || dev->load(NULL, NULL, 0) != 0) return 3;
  scenario(bls, dev);
  /* upgrade with MBLS_QUEUE: the verify entries go through the batching queue */
  setenv("MBLS_QUEUE", "8,300", 1);
  if (bls->upgrade(NULL, NULL, NULL, 0) != 0 || !mbls_queue_running()) return 4;
  scenario(bls, dev);
  pthread_t th[12];
  struct qarg qa[12];
  for (int i = 0; i < 12; ++i) {
    qa[i].e = bls, qa[i].id = i;
    pthread_create(&th[i], NULL, queue_caller, &qa[i]);
  }
  for (int i = 0; i < 12; ++i) pthread_join(th[i], NULL);
  mbls_queue_stop();
  fb_reset();
  if (g_bad) {
    fprintf(stderr, "%d mismatches\n", g_bad);
    return 1;
  }
  puts("nif OK");
  return 0;
}
