/* TEST-ONLY stand-in for the erl_nif.h subset the NIF shims use (Erlang/OTP headers are not in
 * this image).  Signatures follow the documented erl_nif C API; fake_beam.c implements them
 * over a tiny term model so tests/test_nif.py can load a shim, read its function table and
 * call its entries on the CPU.  Nothing here ships. */
#ifndef MBLS_TEST_ERL_NIF_STUB_H
#define MBLS_TEST_ERL_NIF_STUB_H
#include <stddef.h>
#include <stdint.h>
typedef uintptr_t ERL_NIF_TERM;
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
/* the part of the real ErlNifEntry a test reads */
typedef struct {
  const char* name;
  int num_of_funcs;
  ErlNifFunc* funcs;
  int (*load)(ErlNifEnv*, void**, ERL_NIF_TERM);
  int (*upgrade)(ErlNifEnv*, void**, void**, ERL_NIF_TERM);
} ErlNifEntry;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM term, ERL_NIF_TERM* head, ERL_NIF_TERM* tail);
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* len);
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM bin_term, ErlNifBinary* bin);
int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* ip);
ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env);
ERL_NIF_TERM enif_raise_exception(ErlNifEnv* env, ERL_NIF_TERM reason);
unsigned char* enif_make_new_binary(ErlNifEnv* env, size_t size, ERL_NIF_TERM* termp);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM e1, ERL_NIF_TERM e2);
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned i);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, unsigned long i);
ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt);
#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                                      \
  const ErlNifEntry* nif_init(void) {                                                               \
    static ErlNifEntry entry = {#NAME, (int)(sizeof(FUNCS) / sizeof(FUNCS[0])), FUNCS, LOAD, UPGRADE}; \
    return &entry;                                                                                  \
  }
#endif
