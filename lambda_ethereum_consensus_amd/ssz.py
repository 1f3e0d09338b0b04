"""Signing roots on the GPU: the step before the `Bls` path.

Mirrors the reference's `Misc.compute_signing_root/2`
(lib/lambda_ethereum_consensus/state_transition/misc.ex:243-260) and the `Ssz.hash_tree_root/1`
calls behind it (lib/ssz.ex:51-55) for the containers the verification path signs, batched:

* `compute_signing_roots(object_roots, domains)` - `compute_signing_root(<<_::256>> = root, domain)`
  (misc.ex:244-252): hash_tree_root(SigningData{object_root, domain}).
* `hash_tree_roots(objects)` - hash_tree_root of fixed-size containers given as their 32-byte
  field leaves (uint64 fields little-endian and zero padded, composite fields as their roots).
* `attestation_data_signing_roots(datas, domains)` - `compute_signing_root(data, domain)` for
  phase0 AttestationData SSZ encodings (128 bytes), the call at predicates.ex:118-121.

Every call is one device submission through libmbls (include/mbls.h); there is no host
hashing path.  A wrong-length input raises ValueError (the reference crashes on a bad pattern
match there: misc.ex:244).
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Union

from . import _lib
from .bls import BlsDeviceError

Bytes = Union[bytes, bytearray, memoryview]


def _pack(items: Sequence[Bytes], size: int, what: str) -> bytes:
    out = bytearray()
    for i, x in enumerate(items):
        x = bytes(x)
        if len(x) != size:
            raise ValueError(f"{what} {i}: expected {size} bytes, got {len(x)}")
        out += x
    return bytes(out)


def _domains(domains, n: int):
    """One domain for all (bytes) or one per object (sequence) -> (packed, stride)."""
    if isinstance(domains, (bytes, bytearray, memoryview)):
        return _pack([domains], 32, "domain"), 0
    if len(domains) != n:
        raise ValueError(f"expected {n} domains, got {len(domains)}")
    return _pack(domains, 32, "domain"), 32


def _split(out, n: int) -> List[bytes]:
    raw = bytes(out)
    return [raw[32 * i:32 * i + 32] for i in range(n)]


def compute_signing_roots(object_roots: Sequence[Bytes], domains) -> List[bytes]:
    n = len(object_roots)
    if n == 0:
        return []
    roots = _pack(object_roots, 32, "object_root")
    dom, stride = _domains(domains, n)
    out = ctypes.create_string_buffer(32 * n)
    rc = _lib.load().mbls_signing_roots(roots, dom, stride, n, ctypes.cast(out, ctypes.c_void_p))
    if rc:
        raise BlsDeviceError(_lib.status_message(rc))
    return _split(out, n)


def compute_signing_root(object_root: Bytes, domain: Bytes) -> bytes:
    return compute_signing_roots([object_root], domain)[0]


def hash_tree_roots(objects: Sequence[Sequence[Bytes]]) -> List[bytes]:
    """Roots of fixed-size containers of equal field count (1..16), fields as 32-byte leaves."""
    n = len(objects)
    if n == 0:
        return []
    leaves = len(objects[0])
    if not 1 <= leaves <= 16 or any(len(o) != leaves for o in objects):
        raise ValueError("every object needs the same number (1..16) of 32-byte leaves")
    chunks = _pack([leaf for o in objects for leaf in o], 32, "leaf")
    out = ctypes.create_string_buffer(32 * n)
    rc = _lib.load().mbls_hash_tree_root_chunks(chunks, leaves, n, ctypes.cast(out, ctypes.c_void_p))
    if rc:
        raise BlsDeviceError(_lib.status_message(rc))
    return _split(out, n)


def attestation_data_signing_roots(datas: Sequence[Bytes], domains) -> List[bytes]:
    n = len(datas)
    if n == 0:
        return []
    data = _pack(datas, 128, "AttestationData")
    dom, stride = _domains(domains, n)
    out = ctypes.create_string_buffer(32 * n)
    rc = _lib.load().mbls_attestation_data_signing_roots(data, dom, stride, n, ctypes.cast(out, ctypes.c_void_p))
    if rc:
        raise BlsDeviceError(_lib.status_message(rc))
    return _split(out, n)
