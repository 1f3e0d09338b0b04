/* TEST-ONLY: a minimal term model implementing tests/nif_stub/erl_nif.h, so the NIF shims can
 * be loaded and called on the CPU (tests/test_nif.py) and run under ASan/UBSan
 * (tests/sanitize/nif_sanitize.c).  Terms are pointers to heap cells that live until
 * fb_reset() (cell allocation is thread-safe, as NIF calls from concurrent schedulers are);
 * atoms are interned by name.  fb_show() prints a term in Erlang syntax. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "erl_nif.h"

enum { T_ATOM = 1, T_BIN, T_TUPLE, T_LIST, T_UINT, T_RAISE, T_BADARG };
typedef struct cell {
  int kind;
  size_t n;              /* binary size / tuple or list arity */
  unsigned char* bytes;  /* binary data, atom name */
  ERL_NIF_TERM* elems;   /* tuple / list elements, raise reason in elems[0] */
  unsigned long uval;
  struct cell* next_alloc;
} cell;

static cell* g_cells;
static pthread_mutex_t g_cells_mu = PTHREAD_MUTEX_INITIALIZER;  /* NIFs run on many schedulers */

static cell* new_cell(int kind) {
  cell* c = (cell*)calloc(1, sizeof(cell));
  c->kind = kind;
  pthread_mutex_lock(&g_cells_mu);
  c->next_alloc = g_cells;
  g_cells = c;
  pthread_mutex_unlock(&g_cells_mu);
  return c;
}
static cell* C(ERL_NIF_TERM t) { return (cell*)t; }

void fb_reset(void) {
  while (g_cells) {
    cell* n = g_cells->next_alloc;
    free(g_cells->bytes);
    free(g_cells->elems);
    free(g_cells);
    g_cells = n;
  }
}

ERL_NIF_TERM fb_bin(const void* data, size_t len) {
  cell* c = new_cell(T_BIN);
  c->n = len;
  c->bytes = (unsigned char*)malloc(len ? len : 1);
  if (len) memcpy(c->bytes, data, len);
  return (ERL_NIF_TERM)c;
}
ERL_NIF_TERM fb_list(const ERL_NIF_TERM* elems, size_t n) {
  cell* c = new_cell(T_LIST);
  c->n = n;
  c->elems = (ERL_NIF_TERM*)malloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
  if (n) memcpy(c->elems, elems, sizeof(ERL_NIF_TERM) * n);
  return (ERL_NIF_TERM)c;
}
ERL_NIF_TERM fb_uint(unsigned long v) {
  cell* c = new_cell(T_UINT);
  c->uval = v;
  return (ERL_NIF_TERM)c;
}

ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name) {
  (void)env;
  cell* c = new_cell(T_ATOM);
  c->n = strlen(name);
  c->bytes = (unsigned char*)malloc(c->n + 1);
  memcpy(c->bytes, name, c->n + 1);
  return (ERL_NIF_TERM)c;
}
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env) {
  (void)env;
  return (ERL_NIF_TERM)new_cell(T_BADARG);
}
ERL_NIF_TERM enif_raise_exception(ErlNifEnv* env, ERL_NIF_TERM reason) {
  (void)env;
  cell* c = new_cell(T_RAISE);
  c->n = 1;
  c->elems = (ERL_NIF_TERM*)malloc(sizeof(ERL_NIF_TERM));
  c->elems[0] = reason;
  return (ERL_NIF_TERM)c;
}
unsigned char* enif_make_new_binary(ErlNifEnv* env, size_t size, ERL_NIF_TERM* termp) {
  (void)env;
  cell* c = new_cell(T_BIN);
  c->n = size;
  c->bytes = (unsigned char*)calloc(1, size ? size : 1);
  *termp = (ERL_NIF_TERM)c;
  return c->bytes;
}
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM e1, ERL_NIF_TERM e2) {
  (void)env;
  cell* c = new_cell(T_TUPLE);
  c->n = 2;
  c->elems = (ERL_NIF_TERM*)malloc(2 * sizeof(ERL_NIF_TERM));
  c->elems[0] = e1;
  c->elems[1] = e2;
  return (ERL_NIF_TERM)c;
}
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned i) {
  (void)env;
  return fb_uint(i);
}
ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, unsigned long i) {
  (void)env;
  return fb_uint(i);
}
ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt) {
  (void)env;
  cell* c = new_cell(T_TUPLE);
  c->n = cnt;
  c->elems = (ERL_NIF_TERM*)malloc(sizeof(ERL_NIF_TERM) * (cnt ? cnt : 1));
  if (cnt) memcpy(c->elems, arr, sizeof(ERL_NIF_TERM) * cnt);
  return (ERL_NIF_TERM)c;
}
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt) {
  (void)env;
  return fb_list(arr, cnt);
}
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* len) {
  (void)env;
  if (!term || C(term)->kind != T_LIST) return 0;
  *len = (unsigned)C(term)->n;
  return 1;
}
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM term, ERL_NIF_TERM* head, ERL_NIF_TERM* tail) {
  (void)env;
  if (!term || C(term)->kind != T_LIST || C(term)->n == 0) return 0;
  *head = C(term)->elems[0];
  *tail = fb_list(C(term)->elems + 1, C(term)->n - 1);
  return 1;
}
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifBinary* bin) {
  (void)env;
  if (!term || C(term)->kind != T_BIN) return 0;
  memset(bin, 0, sizeof *bin);
  bin->size = C(term)->n;
  bin->data = C(term)->bytes;
  return 1;
}
int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* ip) {
  (void)env;
  if (!term || C(term)->kind != T_UINT || C(term)->uval > 0xffffffffUL) return 0;
  *ip = (unsigned)C(term)->uval;
  return 1;
}

/* Erlang-syntax rendering: {ok,true}, {error,<<"msg">>}, <<1,2,3>>, [1,2], raise:{...}, badarg */
static size_t put(char* out, size_t cap, size_t at, const char* s) {
  size_t n = strlen(s);
  if (at < cap) {
    size_t k = n < cap - at ? n : cap - at;
    memcpy(out + at, s, k);
  }
  return at + n;
}
static size_t show(ERL_NIF_TERM t, char* out, size_t cap, size_t at) {
  char tmp[32];
  cell* c = C(t);
  if (!c) return put(out, cap, at, "NULL");
  switch (c->kind) {
    case T_ATOM: return put(out, cap, at, (const char*)c->bytes);
    case T_BADARG: return put(out, cap, at, "badarg");
    case T_UINT:
      snprintf(tmp, sizeof tmp, "%lu", c->uval);
      return put(out, cap, at, tmp);
    case T_RAISE:
      at = put(out, cap, at, "raise:");
      return show(c->elems[0], out, cap, at);
    case T_BIN: {
      int printable = c->n > 0;
      for (size_t i = 0; i < c->n; ++i) printable &= c->bytes[i] >= 32 && c->bytes[i] < 127 && c->bytes[i] != '"';
      at = put(out, cap, at, "<<");
      if (printable) {
        at = put(out, cap, at, "\"");
        for (size_t i = 0; i < c->n; ++i) {
          tmp[0] = (char)c->bytes[i];
          tmp[1] = 0;
          at = put(out, cap, at, tmp);
        }
        at = put(out, cap, at, "\"");
      } else {
        for (size_t i = 0; i < c->n; ++i) {
          snprintf(tmp, sizeof tmp, i ? ",%u" : "%u", c->bytes[i]);
          at = put(out, cap, at, tmp);
        }
      }
      return put(out, cap, at, ">>");
    }
    case T_TUPLE:
    case T_LIST:
      at = put(out, cap, at, c->kind == T_TUPLE ? "{" : "[");
      for (size_t i = 0; i < c->n; ++i) {
        if (i) at = put(out, cap, at, ",");
        at = show(c->elems[i], out, cap, at);
      }
      return put(out, cap, at, c->kind == T_TUPLE ? "}" : "]");
  }
  return put(out, cap, at, "?");
}
size_t fb_show(ERL_NIF_TERM t, char* out, size_t cap) {
  size_t n = show(t, out, cap, 0);
  if (cap) out[n < cap ? n : cap - 1] = 0;
  return n;
}
