"""Host-side mirror of the reference's Elixir `Bls` module (lib/bls.ex:1-62).

Same function names, argument meaning and outcomes: every call returns ``("ok", value)``
or ``("error", message)`` exactly where the reference NIF (native/bls_nif/src/lib.rs)
returns ``{:ok, value}`` / ``{:error, message}``; `valid` mirrors `Bls.valid?/3` and
`key_validate` keeps the reference's behaviour of not being exported by the NIF
(lib/bls.ex:47-49, lib.rs:147-158), i.e. it raises.

All arithmetic runs in libmbls.so's HIP kernels.  A device failure raises
`BlsDeviceError` (the reference would crash the calling process on a NIF panic); it is
never turned into `false`.

The `*_batch` functions are the batching-queue entry points: many
independent signature sets per device submission, results identical to the per-call API.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

from . import _lib

Result = Tuple[str, object]


class BlsDeviceError(RuntimeError):
    pass


class NifNotLoaded(RuntimeError):
    """`:erlang.nif_error(:nif_not_loaded)` — raised by `key_validate`, as in the reference."""


def _b(x) -> bytes:
    if isinstance(x, bytes):
        return x
    if isinstance(x, (bytearray, memoryview)):
        return bytes(x)
    raise TypeError("expected a binary (bytes), got %r" % type(x).__name__)  # badarg


def _bins(items: Sequence[bytes]):
    items = [_b(x) for x in items]
    arr = (_lib.mbls_bin * max(len(items), 1))()
    for i, x in enumerate(items):
        arr[i].data = ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p) if x else None
        arr[i].len = len(x)
    return arr, items  # keep `items` alive for the call


def _bin(x):
    x = _b(x)
    v = _lib.mbls_bin()
    v.data = ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p) if x else None
    v.len = len(x)
    return v, x


def _outcome(code: int, got: int, value=None) -> Result:
    if code == _lib.MBLS_ERR_DEVICE or code <= -100:
        raise BlsDeviceError(_lib.status_message(code, got))
    if code == _lib.MBLS_TRUE:
        return ("ok", True)
    if code == _lib.MBLS_FALSE:
        return ("ok", False)
    if code == _lib.MBLS_OK:
        return ("ok", value)
    return ("error", _lib.status_message(code, got))


# --------------------------------------------------------------------------- Bls.* ------

def sign(private_key: bytes, message: bytes) -> Result:
    """Bls.sign/2 (lib/bls.ex:7-10 -> lib.rs:14-29)."""
    lib = _lib.load()
    sk, _k = _bin(private_key)
    m, _m = _bin(message)
    out = ctypes.create_string_buffer(96)
    got = ctypes.c_size_t(0)
    rc = lib.mbls_bls_sign(sk, m, out, ctypes.byref(got))
    return _outcome(rc, got.value, out.raw)


def aggregate(signatures: Sequence[bytes]) -> Result:
    """Bls.aggregate/1 (lib/bls.ex:12-15 -> lib.rs:31-51)."""
    lib = _lib.load()
    arr, _keep = _bins(signatures)
    out = ctypes.create_string_buffer(96)
    got = ctypes.c_size_t(0)
    rc = lib.mbls_bls_aggregate(arr, len(signatures), out, ctypes.byref(got))
    return _outcome(rc, got.value, out.raw)


def verify(public_key: bytes, message: bytes, signature: bytes) -> Result:
    """Bls.verify/3 (lib/bls.ex:17-21 -> lib.rs:53-60)."""
    lib = _lib.load()
    pk, _a = _bin(public_key)
    m, _b2 = _bin(message)
    s, _c = _bin(signature)
    got = ctypes.c_size_t(0)
    return _outcome(lib.mbls_bls_verify(pk, m, s, ctypes.byref(got)), got.value)


def fast_aggregate_verify(public_keys: Sequence[bytes], message: bytes, signature: bytes) -> Result:
    """Bls.fast_aggregate_verify/3 (lib/bls.ex:23-27 -> lib.rs:84-100)."""
    lib = _lib.load()
    arr, _keep = _bins(public_keys)
    m, _m = _bin(message)
    s, _s = _bin(signature)
    got = ctypes.c_size_t(0)
    return _outcome(lib.mbls_bls_fast_aggregate_verify(arr, len(public_keys), m, s, ctypes.byref(got)), got.value)


def eth_fast_aggregate_verify(public_keys: Sequence[bytes], message: bytes, signature: bytes) -> Result:
    """Bls.eth_fast_aggregate_verify/3 (lib/bls.ex:29-33 -> lib.rs:102-119)."""
    lib = _lib.load()
    arr, _keep = _bins(public_keys)
    m, _m = _bin(message)
    s, _s = _bin(signature)
    got = ctypes.c_size_t(0)
    return _outcome(lib.mbls_bls_eth_fast_aggregate_verify(arr, len(public_keys), m, s, ctypes.byref(got)), got.value)


def aggregate_verify(public_keys: Sequence[bytes], messages: Sequence[bytes], signature: bytes) -> Result:
    """Bls.aggregate_verify/3 (lib/bls.ex:35-39 -> lib.rs:62-82)."""
    lib = _lib.load()
    pa, _kp = _bins(public_keys)
    ma, _km = _bins(messages)
    s, _s = _bin(signature)
    got = ctypes.c_size_t(0)
    rc = lib.mbls_bls_aggregate_verify(pa, len(public_keys), ma, len(messages), s, ctypes.byref(got))
    return _outcome(rc, got.value)


def eth_aggregate_pubkeys(public_keys: Sequence[bytes]) -> Result:
    """Bls.eth_aggregate_pubkeys/1 (lib/bls.ex:41-45 -> lib.rs:121-145)."""
    lib = _lib.load()
    arr, _keep = _bins(public_keys)
    out = ctypes.create_string_buffer(48)
    got = ctypes.c_size_t(0)
    rc = lib.mbls_bls_eth_aggregate_pubkeys(arr, len(public_keys), out, ctypes.byref(got))
    return _outcome(rc, got.value, out.raw)


def key_validate(public_key: bytes):
    """Bls.key_validate/1 is a stub the reference NIF never exports (lib/bls.ex:47-49)."""
    raise NifNotLoaded("nif_not_loaded")


def valid(public_key: bytes, message: bytes, signature: bytes) -> bool:
    """Bls.valid?/3 (lib/bls.ex:55-61): verify with errors mapped to false."""
    tag, v = verify(public_key, message, signature)
    return bool(v) if tag == "ok" else False


# --------------------------------------------------------------------------- batches ----

def _offsets(groups) -> "ctypes.Array":
    off = (ctypes.c_uint32 * (len(groups) + 1))()
    acc = 0
    for i, g in enumerate(groups):
        off[i] = acc
        acc += len(g)
    off[len(groups)] = acc
    return off


def _batch_results(codes, gots) -> List[Result]:
    return [_outcome(int(codes[i]), int(gots[i])) for i in range(len(codes))]


def verify_batch(sets: Sequence[Tuple[bytes, bytes, bytes]]) -> List[Result]:
    """Many `verify(pk, msg, sig)` calls in one device submission."""
    lib = _lib.load()
    n = len(sets)
    if n == 0:
        return []
    pa, _k1 = _bins([s[0] for s in sets])
    ma, _k2 = _bins([s[1] for s in sets])
    sa, _k3 = _bins([s[2] for s in sets])
    codes = (ctypes.c_int32 * n)()
    gots = (ctypes.c_size_t * n)()
    rc = lib.mbls_bls_verify_batch(pa, ma, sa, n, codes, gots)
    if rc:
        raise BlsDeviceError(_lib.status_message(rc))
    return _batch_results(codes, gots)


FAV_ETH, FAV_RLC = 1, 2  # include/mbls.h MBLS_FAV_*


def fast_aggregate_verify_batch(sets: Sequence[Tuple[Sequence[bytes], bytes, bytes]], eth: bool = False,
                                rlc: bool = False) -> List[Result]:
    """Many `(eth_)fast_aggregate_verify(pks, msg, sig)` calls in one device submission.
    rlc=True: opt-in random-linear-combination batch check; results equal
    the exact ones except with probability <= 2^-64 per batch."""
    lib = _lib.load()
    n = len(sets)
    if n == 0:
        return []
    groups = [list(s[0]) for s in sets]
    off = _offsets(groups)
    pa, _k1 = _bins([k for g in groups for k in g])
    ma, _k2 = _bins([s[1] for s in sets])
    sa, _k3 = _bins([s[2] for s in sets])
    codes = (ctypes.c_int32 * n)()
    gots = (ctypes.c_size_t * n)()
    flags = (FAV_ETH if eth else 0) | (FAV_RLC if rlc else 0)
    rc = lib.mbls_bls_fast_aggregate_verify_batch(pa, off, ma, sa, n, flags, codes, gots)
    if rc:
        raise BlsDeviceError(_lib.status_message(rc))
    return _batch_results(codes, gots)


def aggregate_verify_batch(sets: Sequence[Tuple[Sequence[bytes], Sequence[bytes], bytes]]) -> List[Result]:
    """Many `aggregate_verify(pks, msgs, sig)` calls in one device submission."""
    lib = _lib.load()
    n = len(sets)
    if n == 0:
        return []
    kg = [list(s[0]) for s in sets]
    mg = [list(s[1]) for s in sets]
    koff, moff = _offsets(kg), _offsets(mg)
    pa, _k1 = _bins([k for g in kg for k in g])
    ma, _k2 = _bins([m for g in mg for m in g])
    sa, _k3 = _bins([s[2] for s in sets])
    codes = (ctypes.c_int32 * n)()
    gots = (ctypes.c_size_t * n)()
    rc = lib.mbls_bls_aggregate_verify_batch(pa, koff, ma, moff, sa, n, codes, gots)
    if rc:
        raise BlsDeviceError(_lib.status_message(rc))
    return _batch_results(codes, gots)


# ------------------------------------------------------------ validator pubkey table ---

class PubkeyTable:
    """The engine's device-resident validator pubkey table (one per
    process, like the engine).  Rows are validator indices; `set` decodes and KeyValidates
    keys once, and `fast_aggregate_verify_batch` then verifies committees given as index
    lists with the outcomes the per-key-bytes API gives for the same keys, plus
    ``("error", "UnknownValidatorIndex")`` for a row that was never set."""

    def set(self, first: int, public_keys: Sequence[bytes]) -> List[int]:
        """Rows first.. <- public_keys (48-byte encodings); returns per-key codes (0 valid)."""
        lib = _lib.load()
        n = len(public_keys)
        if n == 0:
            return []
        for k in public_keys:
            if len(_b(k)) != 48:
                raise ValueError("table keys must be 48-byte encodings")
        buf = b"".join(public_keys)
        st = (ctypes.c_int32 * n)()
        rc = lib.mbls_pk_table_set(first, buf, n, st)
        if rc:
            raise BlsDeviceError(_lib.status_message(rc))
        return list(st)

    @property
    def size(self) -> int:
        return int(_lib.load().mbls_pk_table_size())

    def clear(self):
        rc = _lib.load().mbls_pk_table_clear()
        if rc:
            raise BlsDeviceError(_lib.status_message(rc))

    def eth_aggregate_pubkeys(self, indices: Sequence[int]) -> Result:
        """Bls.eth_aggregate_pubkeys over table rows (the sync committee as validator indices,
        accessors.ex:14-20); ("error", "UnknownValidatorIndex") for a row never set."""
        lib = _lib.load()
        n = len(indices)
        idx = (ctypes.c_uint32 * max(n, 1))(*indices)
        out = ctypes.create_string_buffer(48)
        rc = lib.mbls_eth_aggregate_pubkeys_indexed(idx, n, out)
        return _outcome(rc, 0, out.raw)

    def fast_aggregate_verify_batch(self, sets: Sequence[Tuple[Sequence[int], bytes, bytes]],
                                    eth: bool = False, rlc: bool = False) -> List[Result]:
        lib = _lib.load()
        n = len(sets)
        if n == 0:
            return []
        groups = [list(s[0]) for s in sets]
        off = _offsets(groups)
        flat = [i for g in groups for i in g]
        idx = (ctypes.c_uint32 * max(len(flat), 1))(*flat)
        ma, _k2 = _bins([s[1] for s in sets])
        sa, _k3 = _bins([s[2] for s in sets])
        codes = (ctypes.c_int32 * n)()
        gots = (ctypes.c_size_t * n)()
        flags = (FAV_ETH if eth else 0) | (FAV_RLC if rlc else 0)
        rc = lib.mbls_fast_aggregate_verify_indexed_batch(idx, off, ma, sa, n, flags, codes, gots)
        if rc:
            raise BlsDeviceError(_lib.status_message(rc))
        return _batch_results(codes, gots)


# ------------------------------------------------------------------- batching queue ----

class BatchingQueue:
    """The engine's coalescing queue as a context manager: while it runs,
    `verify` / `fast_aggregate_verify` / `eth_fast_aggregate_verify` below may be called from
    many threads at once (ctypes releases the GIL); concurrent calls share device batches and
    each returns what the per-call function returns."""

    def __init__(self, max_sets: int = 4096, max_wait_us: int = 500):
        self.max_sets, self.max_wait_us = max_sets, max_wait_us

    def __enter__(self):
        rc = _lib.load().mbls_queue_start(self.max_sets, self.max_wait_us)
        if rc:
            raise BlsDeviceError(_lib.status_message(rc))
        return self

    def __exit__(self, *exc):
        _lib.load().mbls_queue_stop()

    @staticmethod
    def stats():
        b, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _lib.load().mbls_queue_stats(ctypes.byref(b), ctypes.byref(n))
        return int(b.value), int(n.value)

    @staticmethod
    def verify(public_key: bytes, message: bytes, signature: bytes) -> Result:
        lib = _lib.load()
        pk, _a = _bin(public_key)
        m, _b2 = _bin(message)
        s, _c = _bin(signature)
        got = ctypes.c_size_t(0)
        return _outcome(lib.mbls_queue_verify(pk, m, s, ctypes.byref(got)), got.value)

    @staticmethod
    def fast_aggregate_verify(public_keys: Sequence[bytes], message: bytes, signature: bytes,
                              eth: bool = False) -> Result:
        lib = _lib.load()
        arr, _keep = _bins(public_keys)
        m, _m = _bin(message)
        s, _s = _bin(signature)
        got = ctypes.c_size_t(0)
        rc = lib.mbls_queue_fast_aggregate_verify(arr, len(public_keys), m, s, 1 if eth else 0, ctypes.byref(got))
        return _outcome(rc, got.value)

    @classmethod
    def eth_fast_aggregate_verify(cls, public_keys, message, signature) -> Result:
        return cls.fast_aggregate_verify(public_keys, message, signature, eth=True)
