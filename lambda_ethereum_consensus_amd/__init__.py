"""lambda_ethereum_consensus_amd — MI355X-native BLS12-381 engine behind the `Bls` API.

Drop-in for the reference's `Bls` hot path (lib/bls.ex backed by native/bls_nif): the
arithmetic is hand-written HIP for gfx950 in `csrc/`, exposed through the C ABI of
`include/mbls.h` (libmbls.so).  `bls` mirrors the Elixir module for Python callers and
tests; `nif/bls_nif.c` is the Erlang NIF shim.
"""
from . import bls  # noqa: F401
from ._lib import LIB_PATH, load  # noqa: F401

__all__ = ["bls", "load", "LIB_PATH"]
