"""TEST INFRASTRUCTURE: ctypes wrapper of the C restatement of the oracle (oracle/c,
libblsoracle.so) for the checks that are too large for the pure-Python oracle (the BASELINE
shapes: 512-key sets, 2,048-set epochs, 65,536-set gossip batches).  The C oracle is itself
checked against the Python oracle and the golden fixtures (tests/test_oracle_c.py); this
module is only ever the checker, never the thing measured.

Result codes follow include/mbls.h (1 true, 0 false, < 0 the error); `outcome()` turns them
into the ("ok", v) / ("error", msg) tuples of lambda_ethereum_consensus_amd.bls, with the
message strings of the reference NIF (`format!("{:?}", err)`)."""
from __future__ import annotations

import ctypes
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "c", "libblsoracle.so")

P, SZ, I32, U32, INT = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int

MESSAGES = {
    -1: "BlstError(BLST_BAD_ENCODING)",
    -2: "BlstError(BLST_POINT_NOT_ON_CURVE)",
    -3: "BlstError(BLST_POINT_NOT_IN_GROUP)",
    -4: "BlstError(BLST_PK_IS_INFINITY)",
    -5: "InvalidInfinityPublicKey",
    -9: "Empty public key vector",
}

_lib = None


def threads() -> int:
    """Host threads for the checker: the box's share for one GPU is 16 (gpurun), this
    container has 8."""
    return max(1, min(16, os.cpu_count() or 1))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(SO):
        subprocess.run(["make", "-C", os.path.dirname(SO)], check=True, timeout=300)
    L = ctypes.CDLL(SO)
    L.oracle_c_fav.argtypes = [P, P, SZ, ctypes.c_char_p, SZ, ctypes.c_char_p, SZ, INT]
    L.oracle_c_fav.restype = INT
    L.oracle_c_verify.argtypes = [ctypes.c_char_p, SZ, ctypes.c_char_p, SZ, ctypes.c_char_p, SZ]
    L.oracle_c_verify.restype = INT
    L.oracle_c_fav_batch.argtypes = [P, P, P, P, U32, INT, INT, P]
    L.oracle_c_verify_batch.argtypes = [P, P, P, U32, INT, P]
    L.oracle_c_av_batch.argtypes = [P, P, P, P, U32, INT, P]
    L.oracle_c_eth_aggregate_pubkeys.argtypes = [P, P, SZ, P]
    L.oracle_c_eth_aggregate_pubkeys.restype = INT
    L.oracle_c_aggregate_verify.argtypes = [P, P, SZ, P, P, SZ, ctypes.c_char_p, SZ]
    L.oracle_c_aggregate_verify.restype = INT
    L.oracle_c_table_build.argtypes = [P, U32, INT]
    L.oracle_c_table_build.restype = P
    L.oracle_c_table_free.argtypes = [P]
    L.oracle_c_fav_warm_batch.argtypes = [P, P, P, P, P, U32, INT, INT, P]
    _lib = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data


def _u8(b) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b)


# ------------------------------------------------------------------ packed batches -----
def fav_batch(pks48, key_off, msgs32, sigs96, eth=False, nthreads=None) -> np.ndarray:
    """(eth_)fast_aggregate_verify codes of packed sets (key_off[n+1])."""
    pk, m, s = _u8(pks48), _u8(msgs32), _u8(sigs96)
    off = np.ascontiguousarray(key_off, dtype=np.uint32)
    n = len(off) - 1
    out = np.zeros(n, dtype=np.int32)
    lib().oracle_c_fav_batch(_ptr(pk), _ptr(off), _ptr(m), _ptr(s), n, 1 if eth else 0, nthreads or threads(), _ptr(out))
    return out


def verify_batch(pks48, msgs32, sigs96, nthreads=None) -> np.ndarray:
    pk, m, s = _u8(pks48), _u8(msgs32), _u8(sigs96)
    n = len(s) // 96
    out = np.zeros(n, dtype=np.int32)
    lib().oracle_c_verify_batch(_ptr(pk), _ptr(m), _ptr(s), n, nthreads or threads(), _ptr(out))
    return out


def av_batch(pks48, msgs32, pair_off, sigs96, nthreads=None) -> np.ndarray:
    pk, m, s = _u8(pks48), _u8(msgs32), _u8(sigs96)
    off = np.ascontiguousarray(pair_off, dtype=np.uint32)
    n = len(off) - 1
    out = np.zeros(n, dtype=np.int32)
    lib().oracle_c_av_batch(_ptr(pk), _ptr(m), _ptr(off), _ptr(s), n, nthreads or threads(), _ptr(out))
    return out


# ------------------------------------------------------- lists of binaries (ragged) ----
def _arr(items):
    arr = (ctypes.c_char_p * max(len(items), 1))(*items)
    lens = (ctypes.c_size_t * max(len(items), 1))(*[len(k) for k in items])
    return ctypes.cast(arr, P), ctypes.cast(lens, P), arr, lens


def fav_code(pks, msg, sig, eth=False) -> int:
    a, l, _k1, _k2 = _arr(list(pks))
    return lib().oracle_c_fav(a, l, len(pks), msg, len(msg), sig, len(sig), 1 if eth else 0)


def fav_codes(sets, eth=False, nthreads=None):
    """codes of [(pks, msg, sig)], the sets spread over host threads (ctypes drops the GIL)"""
    with ThreadPoolExecutor(nthreads or threads()) as ex:
        return list(ex.map(lambda t: fav_code(t[0], t[1], t[2], eth), sets))


def av_code(pks, msgs, sig) -> int:
    a, l, _k1, _k2 = _arr(list(pks))
    b, lm, _k3, _k4 = _arr(list(msgs))
    return lib().oracle_c_aggregate_verify(a, l, len(pks), b, lm, len(msgs), sig, len(sig))


def eth_aggregate_pubkeys(pks):
    """("ok", 48 bytes) | ("error", msg) as Bls.eth_aggregate_pubkeys"""
    a, l, _k1, _k2 = _arr(list(pks))
    out = ctypes.create_string_buffer(48)
    rc = lib().oracle_c_eth_aggregate_pubkeys(a, l, len(pks), out)
    if rc == 2:
        return ("ok", out.raw)
    return ("error", message(rc, pks))


def message(code: int, pks=(), msgs=()):
    if code == -6:
        got = next(len(k) for k in pks if len(k) != 48)
        return f"InvalidByteLength {{ got: {got}, expected: 48 }}"
    if code == -7:
        got = next(len(m) for m in msgs if len(m) != 32)
        return f"InvalidMessageLength {{ got: {got}, expected: 32 }}"
    return MESSAGES[code]


def outcome(code: int, pks=(), msgs=()):
    if code in (0, 1):
        return ("ok", bool(code))
    return ("error", message(code, pks, msgs))


# ------------------------------------------------------------------- warm table -------
class Table:
    """Pre-decoded validator table (keys decompressed + KeyValidated once): the warm CPU path."""

    def __init__(self, pks48, nthreads=None):
        self.pk = _u8(pks48)
        self.n = len(self.pk) // 48
        self.h = lib().oracle_c_table_build(_ptr(self.pk), self.n, nthreads or threads())

    def fav_batch(self, idx, idx_off, msgs32, sigs96, eth=False, nthreads=None) -> np.ndarray:
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        off = np.ascontiguousarray(idx_off, dtype=np.uint32)
        m, s = _u8(msgs32), _u8(sigs96)
        n = len(off) - 1
        out = np.zeros(n, dtype=np.int32)
        lib().oracle_c_fav_warm_batch(self.h, _ptr(ix), _ptr(off), _ptr(m), _ptr(s), n, 1 if eth else 0,
                                      nthreads or threads(), _ptr(out))
        return out

    def __del__(self):
        try:
            lib().oracle_c_table_free(self.h)
        except Exception:
            pass
