/*
 * bls_device_nif.c — Erlang NIF `Elixir.Bls.Device`: the engine's additive entries, kept out
 * of `Elixir.Bls` so that module's table stays the reference's (lib.rs:147-158).
 *
 *   pk_table_set(first, [pubkey48])                 -> {:ok, [:ok | {:error, msg}]}
 *       decode + KeyValidate the keys into validator rows first.., once;
 *       the per-key outcome is what Bls.* would report for that key
 *   pk_table_size()                                 -> non_neg_integer
 *   fast_aggregate_verify_indices([index], msg, sig)     -> {:ok, bool} | {:error, msg}
 *   eth_fast_aggregate_verify_indices([index], msg, sig) -> {:ok, bool} | {:error, msg}
 *       Bls.(eth_)fast_aggregate_verify over table rows: replaces the O(N*k) pubkey gather of
 *       predicates.ex:122-127 (feed it Accessors.get_committee_indices) and the per-call
 *       decompression of lib.rs:92-96; a row never set is {:error, "UnknownValidatorIndex"}
 *   eth_aggregate_pubkeys_indices([index])          -> {:ok, pubkey48} | {:error, msg}
 *       the sync-committee aggregate of accessors.ex:14-20 over table rows
 *   attestation_signing_roots(datas, domain)        -> {:ok, <<root::256, ...>>}
 *       compute_signing_root (misc.ex:243-260) of n concatenated 128-byte phase0
 *       AttestationData encodings under one 32-byte domain
 *   stats()                                         -> [{op, calls, sets, keys, errors, busy_us}]
 *       the engine's per-operation counters since load (mbls_stats_read), the measurements of
 *       the node's [:bls, :batch] telemetry events; a plain (non-dirty)
 *       NIF: it reads a few atomics
 *
 * The Elixir side is a new module with one stub per entry.  Errors map
 * as in bls_nif.c (device / internal failures raise).  Both NIFs link the same libmbls, so
 * they share one engine and one table.
 */
#include "mbls_nif_common.h"

static ERL_NIF_TERM nif_pk_table_set(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  unsigned first;
  mbls_bin* pks;
  size_t n;
  if (argc != 2 || !enif_get_uint(env, argv[0], &first) || !get_bin_list(env, argv[1], &pks, &n))
    return enif_make_badarg(env);
  uint8_t* packed = (uint8_t*)malloc(48 * (n ? n : 1));
  int32_t* st = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  ERL_NIF_TERM* terms = (ERL_NIF_TERM*)malloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
  int bad = !packed || !st || !terms;
  for (size_t i = 0; !bad && i < n; ++i) {
    if (pks[i].len != 48) bad = 1; /* table rows are 48-byte encodings */
    else memcpy(packed + 48 * i, pks[i].data, 48);
  }
  free(pks);
  if (bad) {
    free(packed);
    free(st);
    free(terms);
    return enif_make_badarg(env);
  }
  const int32_t rc = n ? mbls_pk_table_set(first, packed, (uint32_t)n, st) : 0;
  ERL_NIF_TERM out;
  if (rc != 0) {
    out = make_error(env, rc, 0);
  } else {
    for (size_t i = 0; i < n; ++i) terms[i] = st[i] == 0 ? atom_ok : make_error(env, st[i], 0);
    out = enif_make_tuple2(env, atom_ok, enif_make_list_from_array(env, terms, (unsigned)n));
  }
  free(packed);
  free(st);
  free(terms);
  return out;
}

static ERL_NIF_TERM nif_pk_table_size(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argv;
  if (argc != 0) return enif_make_badarg(env);
  return enif_make_uint(env, mbls_pk_table_size());
}

static ERL_NIF_TERM fav_indices(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[], int eth) {
  uint32_t* idx;
  size_t n;
  mbls_bin msg, sig;
  if (argc != 3 || !get_index_list(env, argv[0], &idx, &n)) return enif_make_badarg(env);
  if (!get_bin(env, argv[1], &msg) || !get_bin(env, argv[2], &sig)) {
    free(idx);
    return enif_make_badarg(env);
  }
  const uint32_t off[2] = {0, (uint32_t)n};
  int32_t res = 0;
  size_t got = 0;
  const int32_t rc = mbls_fast_aggregate_verify_indexed_batch(idx, off, &msg, &sig, 1, eth, &res, &got);
  free(idx);
  return bool_result(env, rc ? rc : res, got);
}
static ERL_NIF_TERM nif_fast_aggregate_verify_indices(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  return fav_indices(env, argc, argv, 0);
}
static ERL_NIF_TERM nif_eth_fast_aggregate_verify_indices(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  return fav_indices(env, argc, argv, MBLS_FAV_ETH);
}

static ERL_NIF_TERM nif_eth_aggregate_pubkeys_indices(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  uint32_t* idx;
  size_t n;
  if (argc != 1 || !get_index_list(env, argv[0], &idx, &n)) return enif_make_badarg(env);
  uint8_t out[48];
  const int32_t rc = mbls_eth_aggregate_pubkeys_indexed(idx, n, out);
  free(idx);
  return bytes_result(env, rc, 0, out, 48);
}

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
  mbls_nif_atoms(env);
  return mbls_nif_engine_start() == 0 ? 0 : 1;
}

static ERL_NIF_TERM nif_stats(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argv;
  if (argc != 0) return enif_make_badarg(env);
  mbls_op_stats st[MBLS_OP_COUNT];
  const int32_t n = mbls_stats_read(st, MBLS_OP_COUNT, 0);
  if (n < 0) return make_error(env, n, 0);
  ERL_NIF_TERM rows[MBLS_OP_COUNT];
  for (int32_t i = 0; i < n; ++i) {
    const ERL_NIF_TERM t[6] = {enif_make_atom(env, mbls_op_name(i)), enif_make_uint64(env, st[i].calls),
                               enif_make_uint64(env, st[i].sets),   enif_make_uint64(env, st[i].keys),
                               enif_make_uint64(env, st[i].errors), enif_make_uint64(env, st[i].ns / 1000)};
    rows[i] = enif_make_tuple_from_array(env, t, 6);
  }
  return enif_make_list_from_array(env, rows, (unsigned)n);
}

static int upgrade(ErlNifEnv* env, void** priv, void** old_priv, ERL_NIF_TERM info) {
  (void)old_priv;
  return load(env, priv, info);
}

#define NIF_ENTRY(name, arity) {#name, arity, nif_##name, ERL_NIF_DIRTY_JOB_CPU_BOUND}

static ErlNifFunc nif_funcs[] = {
    NIF_ENTRY(pk_table_set, 2),
    NIF_ENTRY(pk_table_size, 0),
    NIF_ENTRY(fast_aggregate_verify_indices, 3),
    NIF_ENTRY(eth_fast_aggregate_verify_indices, 3),
    NIF_ENTRY(eth_aggregate_pubkeys_indices, 1),
    NIF_ENTRY(attestation_signing_roots, 2),
    {"stats", 0, nif_stats, 0},
};

ERL_NIF_INIT(Elixir.Bls.Device, nif_funcs, load, NULL, upgrade, NULL)
