/*
 * bls_nif.c — Erlang NIF `Elixir.Bls` backed by libmbls (include/mbls.h).
 *
 * Drop-in replacement for the reference's Rustler NIF native/bls_nif/src/lib.rs: same
 * module, same seven functions and arities (lib.rs:147-158), same term shapes
 * ({:ok, true|false|binary} / {:error, binary}).  Modelled on the reference's own C NIF
 * native/libp2p_nif/libp2p.c (NIF table + ERL_NIF_INIT, :erlang.load_nif from
 * lib/libp2p/libp2p.ex:6-11).  Calls block on the GPU, so every entry is scheduled on a
 * dirty CPU scheduler (the reference runs them on a normal scheduler).
 *
 * Build (where Erlang headers exist):
 *   gcc -O2 -fPIC -shared -I$(ERLANG_INCLUDES) -I include -o priv/native/bls_nif.so \
 *       lambda_ethereum_consensus_amd/nif/bls_nif.c -L lambda_ethereum_consensus_amd/lib -lmbls
 */
#include <erl_nif.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mbls.h"

static ERL_NIF_TERM atom_ok, atom_error, atom_true, atom_false;

static ERL_NIF_TERM make_error(ErlNifEnv* env, int32_t code, size_t got) {
  char msg[192];
  size_t n = mbls_status_message(code, got, msg, sizeof msg);
  ERL_NIF_TERM bin;
  unsigned char* p = enif_make_new_binary(env, n, &bin);
  memcpy(p, msg, n);
  return enif_make_tuple2(env, atom_error, bin);
}

static ERL_NIF_TERM bool_result(ErlNifEnv* env, int32_t code, size_t got) {
  if (code == MBLS_TRUE) return enif_make_tuple2(env, atom_ok, atom_true);
  if (code == MBLS_FALSE) return enif_make_tuple2(env, atom_ok, atom_false);
  return make_error(env, code, got);
}

static ERL_NIF_TERM bytes_result(ErlNifEnv* env, int32_t code, size_t got, const uint8_t* out, size_t len) {
  if (code != MBLS_OK) return make_error(env, code, got);
  ERL_NIF_TERM bin;
  unsigned char* p = enif_make_new_binary(env, len, &bin);
  memcpy(p, out, len);
  return enif_make_tuple2(env, atom_ok, bin);
}

static int get_bin(ErlNifEnv* env, ERL_NIF_TERM t, mbls_bin* b) {
  ErlNifBinary eb;
  if (!enif_inspect_binary(env, t, &eb)) return 0;
  b->data = eb.data;
  b->len = eb.size;
  return 1;
}

/* list of binaries -> malloc'd array (caller frees); 0 on badarg */
static int get_bin_list(ErlNifEnv* env, ERL_NIF_TERM list, mbls_bin** out, size_t* n) {
  unsigned len;
  if (!enif_get_list_length(env, list, &len)) return 0;
  mbls_bin* a = (mbls_bin*)malloc(sizeof(mbls_bin) * (len ? len : 1));
  if (!a) return 0;
  ERL_NIF_TERM head, tail = list;
  for (unsigned i = 0; i < len; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !get_bin(env, head, &a[i])) {
      free(a);
      return 0;
    }
  }
  *out = a;
  *n = len;
  return 1;
}

static ERL_NIF_TERM nif_sign(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  mbls_bin sk, msg;
  if (argc != 2 || !get_bin(env, argv[0], &sk) || !get_bin(env, argv[1], &msg)) return enif_make_badarg(env);
  uint8_t out[96];
  size_t got = 0;
  int32_t rc = mbls_bls_sign(sk, msg, out, &got);
  return bytes_result(env, rc, got, out, 96);
}

static ERL_NIF_TERM nif_aggregate(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  mbls_bin* sigs;
  size_t n;
  if (argc != 1 || !get_bin_list(env, argv[0], &sigs, &n)) return enif_make_badarg(env);
  uint8_t out[96];
  size_t got = 0;
  int32_t rc = mbls_bls_aggregate(sigs, n, out, &got);
  free(sigs);
  return bytes_result(env, rc, got, out, 96);
}

static ERL_NIF_TERM nif_verify(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  mbls_bin pk, msg, sig;
  if (argc != 3 || !get_bin(env, argv[0], &pk) || !get_bin(env, argv[1], &msg) || !get_bin(env, argv[2], &sig))
    return enif_make_badarg(env);
  size_t got = 0;
  /* concurrent dirty-scheduler callers coalesce into one device batch */
  int32_t rc = mbls_queue_running() ? mbls_queue_verify(pk, msg, sig, &got) : mbls_bls_verify(pk, msg, sig, &got);
  return bool_result(env, rc, got);
}

static ERL_NIF_TERM fav_common(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[], int eth) {
  mbls_bin *pks, msg, sig;
  size_t n;
  if (argc != 3 || !get_bin_list(env, argv[0], &pks, &n)) return enif_make_badarg(env);
  if (!get_bin(env, argv[1], &msg) || !get_bin(env, argv[2], &sig)) {
    free(pks);
    return enif_make_badarg(env);
  }
  size_t got = 0;
  int32_t rc = mbls_queue_running() ? mbls_queue_fast_aggregate_verify(pks, n, msg, sig, eth, &got)
               : eth               ? mbls_bls_eth_fast_aggregate_verify(pks, n, msg, sig, &got)
                                   : mbls_bls_fast_aggregate_verify(pks, n, msg, sig, &got);
  free(pks);
  return bool_result(env, rc, got);
}
static ERL_NIF_TERM nif_fast_aggregate_verify(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  return fav_common(env, argc, argv, 0);
}
static ERL_NIF_TERM nif_eth_fast_aggregate_verify(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  return fav_common(env, argc, argv, 1);
}

static ERL_NIF_TERM nif_aggregate_verify(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  mbls_bin *pks, *msgs, sig;
  size_t npk, nmsg;
  if (argc != 3 || !get_bin_list(env, argv[0], &pks, &npk)) return enif_make_badarg(env);
  if (!get_bin_list(env, argv[1], &msgs, &nmsg)) {
    free(pks);
    return enif_make_badarg(env);
  }
  if (!get_bin(env, argv[2], &sig)) {
    free(pks);
    free(msgs);
    return enif_make_badarg(env);
  }
  size_t got = 0;
  int32_t rc = mbls_bls_aggregate_verify(pks, npk, msgs, nmsg, sig, &got);
  free(pks);
  free(msgs);
  return bool_result(env, rc, got);
}

static ERL_NIF_TERM nif_eth_aggregate_pubkeys(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  mbls_bin* pks;
  size_t n;
  if (argc != 1 || !get_bin_list(env, argv[0], &pks, &n)) return enif_make_badarg(env);
  uint8_t out[48];
  size_t got = 0;
  int32_t rc = mbls_bls_eth_aggregate_pubkeys(pks, n, out, &got);
  free(pks);
  return bytes_result(env, rc, got, out, 48);
}

/* additive: attestation_signing_roots(datas, domain) -- datas is one binary
 * of n concatenated 128-byte AttestationData SSZ encodings, domain 32 bytes; returns
 * {:ok, <<root::256, ...>>} (n x 32 bytes), the compute_signing_root of each (misc.ex:243-260) */
static ERL_NIF_TERM nif_attestation_signing_roots(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  ErlNifBinary d, dom;
  if (argc != 2 || !enif_inspect_binary(env, argv[0], &d) || !enif_inspect_binary(env, argv[1], &dom) ||
      d.size % 128 != 0 || dom.size != 32)
    return enif_make_badarg(env);
  const size_t n = d.size / 128;
  ERL_NIF_TERM bin;
  unsigned char* out = enif_make_new_binary(env, 32 * n, &bin);
  const int32_t rc = n ? mbls_attestation_data_signing_roots(d.data, dom.data, 0, n, out) : 0;
  if (rc != 0) return make_error(env, rc, 0);
  return enif_make_tuple2(env, atom_ok, bin);
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  atom_ok = enif_make_atom(env, "ok");
  atom_error = enif_make_atom(env, "error");
  atom_true = enif_make_atom(env, "true");
  atom_false = enif_make_atom(env, "false");
  const char* dev = getenv("MBLS_DEVICE");
  if (mbls_init(dev ? atoi(dev) : 0) != 0) return 1;
  /* MBLS_QUEUE=<max_sets>[,<max_wait_us>] starts the batching queue: verify and
   * (eth_)fast_aggregate_verify calls from concurrent dirty schedulers then share batches */
  const char* qs = getenv("MBLS_QUEUE");
  if (qs) {
    unsigned max_sets = 4096, wait_us = 500;
    sscanf(qs, "%u,%u", &max_sets, &wait_us);
    if (mbls_queue_start(max_sets, wait_us) != 0) return 1;
  }
  return 0;
}

static int upgrade(ErlNifEnv* env, void** priv, void** old_priv, ERL_NIF_TERM info) {
  (void)old_priv;
  return load(env, priv, info);
}

#define NIF_ENTRY(name, arity) {#name, arity, nif_##name, ERL_NIF_DIRTY_JOB_CPU_BOUND}

static ErlNifFunc nif_funcs[] = {
    NIF_ENTRY(sign, 2),
    NIF_ENTRY(aggregate, 1),
    NIF_ENTRY(aggregate_verify, 3),
    NIF_ENTRY(fast_aggregate_verify, 3),
    NIF_ENTRY(eth_fast_aggregate_verify, 3),
    NIF_ENTRY(eth_aggregate_pubkeys, 1),
    NIF_ENTRY(verify, 3),
    NIF_ENTRY(attestation_signing_roots, 2),
};

ERL_NIF_INIT(Elixir.Bls, nif_funcs, load, NULL, upgrade, NULL)
