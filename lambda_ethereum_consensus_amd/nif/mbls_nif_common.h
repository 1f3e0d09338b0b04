/*
 * mbls_nif_common.h — term helpers shared by the two NIF modules over libmbls:
 * bls_nif.c (`Elixir.Bls`, the drop-in for native/bls_nif/src/lib.rs) and bls_device_nif.c
 * (`Elixir.Bls.Device`, the additive table / index / signing-root entries).
 *
 * Outcome mapping (lib.rs:7-12 Rustler `Result<T, String>` encoding):
 *   MBLS_TRUE / MBLS_FALSE        -> {:ok, true | false}
 *   MBLS_OK                       -> {:ok, binary}
 *   decode / argument errors      -> {:error, "<format!(\"{:?}\", err)>"}   (codes -1 .. -99)
 *   MBLS_ERR_DEVICE (-100),
 *   MBLS_ERR_ARGUMENT (-101) and
 *   MBLS_ERR_SCRATCH_PLAN (-102)  -> raised exception {:bls_device_error, "<msg>"}
 * The last row is deliberate: callers treat {:error, _} as "invalid signature"
 * (lib/bls.ex:56-60, predicates.ex:130-133, operations.ex:78-79), so a GPU fault must never
 * reject valid gossip or blocks; it raises in the calling process, as a panic inside the
 * reference's Rustler NIF does.
 */
#ifndef MBLS_NIF_COMMON_H_
#define MBLS_NIF_COMMON_H_

#include <erl_nif.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mbls.h"

static ERL_NIF_TERM atom_ok, atom_error, atom_true, atom_false, atom_device_error;

static inline void mbls_nif_atoms(ErlNifEnv* env) {
  atom_ok = enif_make_atom(env, "ok");
  atom_error = enif_make_atom(env, "error");
  atom_true = enif_make_atom(env, "true");
  atom_false = enif_make_atom(env, "false");
  atom_device_error = enif_make_atom(env, "bls_device_error");
}

static inline ERL_NIF_TERM make_msg(ErlNifEnv* env, int32_t code, size_t got) {
  char msg[192];
  size_t n = mbls_status_message(code, got, msg, sizeof msg);
  if (n >= sizeof msg) n = sizeof msg - 1;
  ERL_NIF_TERM bin;
  unsigned char* p = enif_make_new_binary(env, n, &bin);
  memcpy(p, msg, n);
  return bin;
}

static inline int is_internal(int32_t code) { return code <= MBLS_ERR_DEVICE; }

/* {:error, msg} for a reference-visible error; raise for a device / internal failure */
static inline ERL_NIF_TERM make_error(ErlNifEnv* env, int32_t code, size_t got) {
  if (is_internal(code))
    return enif_raise_exception(env, enif_make_tuple2(env, atom_device_error, make_msg(env, code, got)));
  return enif_make_tuple2(env, atom_error, make_msg(env, code, got));
}

static inline ERL_NIF_TERM bool_result(ErlNifEnv* env, int32_t code, size_t got) {
  if (code == MBLS_TRUE) return enif_make_tuple2(env, atom_ok, atom_true);
  if (code == MBLS_FALSE) return enif_make_tuple2(env, atom_ok, atom_false);
  return make_error(env, code, got);
}

static inline ERL_NIF_TERM bytes_result(ErlNifEnv* env, int32_t code, size_t got, const uint8_t* out, size_t len) {
  if (code != MBLS_OK) return make_error(env, code, got);
  ERL_NIF_TERM bin;
  unsigned char* p = enif_make_new_binary(env, len, &bin);
  memcpy(p, out, len);
  return enif_make_tuple2(env, atom_ok, bin);
}

static inline int get_bin(ErlNifEnv* env, ERL_NIF_TERM t, mbls_bin* b) {
  ErlNifBinary eb;
  if (!enif_inspect_binary(env, t, &eb)) return 0;
  b->data = eb.data;
  b->len = eb.size;
  return 1;
}

/* list of binaries -> malloc'd array (caller frees); 0 on badarg */
static inline int get_bin_list(ErlNifEnv* env, ERL_NIF_TERM list, mbls_bin** out, size_t* n) {
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

/* list of non-negative integers (validator indices) -> malloc'd uint32 array; 0 on badarg */
static inline int get_index_list(ErlNifEnv* env, ERL_NIF_TERM list, uint32_t** out, size_t* n) {
  unsigned len;
  if (!enif_get_list_length(env, list, &len)) return 0;
  uint32_t* a = (uint32_t*)malloc(sizeof(uint32_t) * (len ? len : 1));
  if (!a) return 0;
  ERL_NIF_TERM head, tail = list;
  for (unsigned i = 0; i < len; ++i) {
    unsigned v;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &v)) {
      free(a);
      return 0;
    }
    a[i] = v;
  }
  *out = a;
  *n = len;
  return 1;
}

/* Engine start shared by both modules' `load` (idempotent): MBLS_DEVICES="0,1,..." puts one
 * engine on each listed GPU (layer-1 batches are split over them), else MBLS_DEVICE=<n>
 * (default 0).  Returns 0 or a negative code. */
static inline int32_t mbls_nif_engine_start(void) {
  const char* list = getenv("MBLS_DEVICES");
  if (list && *list) {
    int32_t devs[64];
    uint32_t n = 0;
    const char* p = list;
    while (*p && n < 64) {
      char* end;
      long v = strtol(p, &end, 10);
      if (end == p) return MBLS_ERR_ARGUMENT;
      devs[n++] = (int32_t)v;
      p = (*end == ',') ? end + 1 : end;
    }
    return mbls_init_devices(devs, n);
  }
  const char* dev = getenv("MBLS_DEVICE");
  return mbls_init(dev ? atoi(dev) : 0);
}

#endif /* MBLS_NIF_COMMON_H_ */
