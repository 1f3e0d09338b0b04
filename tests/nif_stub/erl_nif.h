/* TEST-ONLY declarations of the erl_nif.h subset nif/bls_nif.c uses, so tests/test_abi.py can
 * type-check the shim with gcc -fsyntax-only (Erlang/OTP headers are not in this image).
 * Signatures follow the documented erl_nif C API; nothing here is linked or run. */
#ifndef MBLS_TEST_ERL_NIF_STUB_H
#define MBLS_TEST_ERL_NIF_STUB_H
#include <stddef.h>
typedef unsigned long ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct {
  size_t size;
  unsigned char* data;
  void* ref_bin;
  void* spare[2];
} ErlNifBinary;
typedef struct {
  const char* name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]);
  unsigned flags;
} ErlNifFunc;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM term, ERL_NIF_TERM* head, ERL_NIF_TERM* tail);
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* len);
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM bin_term, ErlNifBinary* bin);
ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env);
unsigned char* enif_make_new_binary(ErlNifEnv* env, size_t size, ERL_NIF_TERM* termp);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM e1, ERL_NIF_TERM e2);
#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                                       \
  const void* nif_init(void) {                                                                       \
    static const void* keep[] = {FUNCS, (const void*)LOAD, (const void*)UPGRADE};                    \
    return keep;                                                                                     \
  }
#endif
