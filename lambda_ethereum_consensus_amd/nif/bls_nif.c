/*
 * bls_nif.c — Erlang NIF `Elixir.Bls` backed by libmbls (include/mbls.h).
 *
 * Drop-in replacement for the reference's Rustler NIF native/bls_nif/src/lib.rs: the same
 * module and EXACTLY the same seven functions and arities (lib.rs:147-158), so the
 * reference's lib/bls.ex:1-62 loads it unchanged apart from the loader line (its
 * key_validate/1 stub stays unexported, as in the reference).  Term shapes:
 * {:ok, true|false|binary} / {:error, binary} (mbls_nif_common.h), except that a device or
 * internal failure raises {:bls_device_error, msg} instead of returning {:error, _} (a GPU
 * fault must not read as an invalid signature).  Modelled on the reference's own C NIF
 * native/libp2p_nif/libp2p.c (NIF table + ERL_NIF_INIT, :erlang.load_nif from
 * lib/libp2p/libp2p.ex:6-11).  Calls block on the GPU, so every entry is scheduled on a
 * dirty CPU scheduler (the reference runs them on a normal scheduler).
 *
 * The additive entries (validator table, index-addressed verification, signing roots) live
 * in the separate module `Elixir.Bls.Device` (bls_device_nif.c), so this table matches the
 * reference's one-to-one.
 *
 * Build (where Erlang headers exist):
 *   gcc -O2 -fPIC -shared -I$(ERLANG_INCLUDES) -I include -o priv/native/bls_nif.so \
 *       lambda_ethereum_consensus_amd/nif/bls_nif.c -L lambda_ethereum_consensus_amd/lib -lmbls
 */
#include <stdio.h>

#include "mbls_nif_common.h"

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

/* The engine must be usable when the module loads: a host without a GPU fails the load
 * (every Bls.* then raises :nif_not_loaded), there is no CPU fallback. */
static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  mbls_nif_atoms(env);
  if (mbls_nif_engine_start() != 0) return 1;
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

/* lib.rs:147-158, same order */
static ErlNifFunc nif_funcs[] = {
    NIF_ENTRY(sign, 2),
    NIF_ENTRY(aggregate, 1),
    NIF_ENTRY(aggregate_verify, 3),
    NIF_ENTRY(fast_aggregate_verify, 3),
    NIF_ENTRY(eth_fast_aggregate_verify, 3),
    NIF_ENTRY(eth_aggregate_pubkeys, 1),
    NIF_ENTRY(verify, 3),
};

ERL_NIF_INIT(Elixir.Bls, nif_funcs, load, NULL, upgrade, NULL)
