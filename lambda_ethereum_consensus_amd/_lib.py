"""ctypes binding of libmbls.so (include/mbls.h).

The library is built in-tree (lambda_ethereum_consensus_amd/lib/libmbls.so) by
`__graft_entry__.build()` / `make -C lambda_ethereum_consensus_amd/csrc`.  Loading fails
loudly if it is missing: there is no CPU fallback for any `Bls` operation.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# MBLS_LIB_PATH: an alternative in-tree build of the same library (variant experiments)
LIB_PATH = os.environ.get("MBLS_LIB_PATH") or os.path.join(_HERE, "lib", "libmbls.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mbls.h")

MBLS_OK = 2
MBLS_TRUE = 1
MBLS_FALSE = 0
MBLS_ERR_DEVICE = -100
MBLS_ERR_SCRATCH_PLAN = -102


class mbls_bin(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class MblsLibraryMissing(RuntimeError):
    pass


_lib = None


def header_symbols():
    """Every function declared in include/mbls.h."""
    with open(HEADER_PATH) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mbls_[a-z0-9_]+)\s*\(", src)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MblsLibraryMissing(
            f"{LIB_PATH} not built; run `make -C lambda_ethereum_consensus_amd/csrc` (no CPU fallback exists)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    I32 = ctypes.c_int32
    U32 = ctypes.c_uint32
    SZ = ctypes.c_size_t
    PSZ = ctypes.POINTER(ctypes.c_size_t)
    B = mbls_bin
    PB = ctypes.POINTER(mbls_bin)
    sig = {
        "mbls_init": (I32, [I32]),
        "mbls_init_devices": (I32, [ctypes.POINTER(I32), U32]),
        "mbls_engine_count": (I32, []),
        "mbls_dev_select": (I32, [I32]),
        "mbls_plan_shards": (I32, [P, SZ, U32, P]),
        "mbls_dev_stream_wait_engine": (I32, [P]),
        "mbls_shutdown": (None, []),
        "mbls_status_message": (SZ, [I32, SZ, ctypes.c_char_p, SZ]),
        "mbls_version": (ctypes.c_char_p, []),
        "mbls_bls_sign": (I32, [B, B, P, PSZ]),
        "mbls_bls_aggregate": (I32, [PB, SZ, P, PSZ]),
        "mbls_bls_verify": (I32, [B, B, B, PSZ]),
        "mbls_bls_aggregate_verify": (I32, [PB, SZ, PB, SZ, B, PSZ]),
        "mbls_bls_fast_aggregate_verify": (I32, [PB, SZ, B, B, PSZ]),
        "mbls_bls_eth_fast_aggregate_verify": (I32, [PB, SZ, B, B, PSZ]),
        "mbls_bls_eth_aggregate_pubkeys": (I32, [PB, SZ, P, PSZ]),
        "mbls_bls_verify_batch": (I32, [PB, PB, PB, SZ, P, P]),
        "mbls_bls_fast_aggregate_verify_batch": (I32, [PB, P, PB, PB, SZ, I32, P, P]),
        "mbls_bls_aggregate_verify_batch": (I32, [PB, P, PB, P, PB, SZ, P, P]),
        "mbls_dev_fast_aggregate_verify": (I32, [P, P, U32, P, P, U32, I32, P, P]),
        "mbls_dev_verify": (I32, [P, P, P, U32, P, P]),
        "mbls_dev_aggregate_verify": (I32, [P, P, P, U32, P, U32, P, P]),
        "mbls_dev_aggregate_pubkeys": (I32, [P, P, U32, U32, P, P, P]),
        "mbls_dev_validate_pubkeys": (I32, [P, U32, P, P]),
        "mbls_dev_synchronize": (I32, [P]),
        "mbls_dev_sk_to_pk": (I32, [P, U32, P, P]),
        "mbls_dev_sign": (I32, [P, P, U32, P, P]),
        "mbls_dev_aggregate_signatures": (I32, [P, P, U32, U32, P, P, P]),
        "mbls_queue_start": (I32, [U32, U32]),
        "mbls_queue_stop": (I32, []),
        "mbls_queue_running": (I32, []),
        "mbls_queue_stats": (I32, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "mbls_queue_verify": (I32, [B, B, B, PSZ]),
        "mbls_queue_fast_aggregate_verify": (I32, [PB, SZ, B, B, I32, PSZ]),
        "mbls_pk_table_set": (I32, [U32, P, U32, P]),
        "mbls_dev_pk_table_set": (I32, [U32, P, U32, P, P]),
        "mbls_pk_table_size": (U32, []),
        "mbls_pk_table_clear": (I32, []),
        "mbls_fast_aggregate_verify_indexed_batch": (I32, [P, P, PB, PB, SZ, I32, P, P]),
        "mbls_dev_fast_aggregate_verify_indexed": (I32, [P, P, U32, P, P, U32, I32, P, P]),
        "mbls_dev_aggregate_pubkeys_indexed": (I32, [P, P, U32, U32, P, P, P]),
        "mbls_eth_aggregate_pubkeys_indexed": (I32, [P, SZ, P]),
        "mbls_comm_unique_id": (I32, [P]),
        "mbls_comm_init": (I32, [ctypes.c_char_p, I32, I32]),
        "mbls_comm_destroy": (I32, []),
        "mbls_dev_pk_table_set_sharded": (I32, [P, U32, P, P]),
        "mbls_dev_hash_tree_root_chunks": (I32, [P, U32, U32, P, P]),
        "mbls_dev_signing_roots": (I32, [P, P, U32, U32, P, P]),
        "mbls_dev_attestation_data_signing_roots": (I32, [P, P, U32, U32, P, P]),
        "mbls_hash_tree_root_chunks": (I32, [ctypes.c_char_p, U32, SZ, P]),
        "mbls_signing_roots": (I32, [ctypes.c_char_p, ctypes.c_char_p, U32, SZ, P]),
        "mbls_attestation_data_signing_roots": (I32, [ctypes.c_char_p, ctypes.c_char_p, U32, SZ, P]),
        "mbls_op_name": (ctypes.c_char_p, [I32]),
        "mbls_stats_read": (I32, [P, I32, I32]),
        "mbls_scratch_plan": (I32, [ctypes.c_uint64, ctypes.c_uint64, U32, U32, P, P, U32, P]),
        "mbls_scratch_kernel_gated": (I32, [I32]),
        "mbls_scratch_gate_stats": (I32, [P]),
        "mbls_scratch_info": (I32, [P]),
        "mbls_scratch_kernel": (ctypes.c_char_p, [I32]),
        "mbls_debug_fail_deferred": (I32, [I32, I32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class mbls_op_stats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("sets", ctypes.c_uint64), ("keys", ctypes.c_uint64),
                ("errors", ctypes.c_uint64), ("ns", ctypes.c_uint64)]


def stats(reset: bool = False) -> dict:
    """Per-operation batch counters (include/mbls.h mbls_stats_read; the measurements of the
    node's [:bls, :batch] telemetry events): {op: {calls, sets, keys, errors, ns}}.  No GPU needed."""
    lib = load()
    arr = (mbls_op_stats * 32)()
    n = lib.mbls_stats_read(ctypes.cast(arr, ctypes.c_void_p), 32, 1 if reset else 0)
    if n < 0:
        raise RuntimeError(status_message(n))
    return {lib.mbls_op_name(i).decode(): {f: int(getattr(arr[i], f)) for f, _ in mbls_op_stats._fields_}
            for i in range(n)}


def status_message(code: int, got: int = 0) -> str:
    lib = load()
    buf = ctypes.create_string_buffer(192)
    lib.mbls_status_message(code, got, buf, len(buf))
    return buf.value.decode()
