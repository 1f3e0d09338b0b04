"""CPU: the C-ABI library builds, loads, and exports every symbol include/mbls.h declares.
(No compute calls here — there is no GPU in this container.)"""
import ctypes
import os
import subprocess

import pytest

from lambda_ethereum_consensus_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "lambda_ethereum_consensus_amd", "csrc"), "-j3"],
                       check=True, timeout=1500)
    return ctypes.CDLL(_lib.LIB_PATH)


def test_header_declares_the_bls_surface():
    syms = _lib.header_symbols()
    for name in ("mbls_bls_sign", "mbls_bls_aggregate", "mbls_bls_verify", "mbls_bls_fast_aggregate_verify",
                 "mbls_bls_eth_fast_aggregate_verify", "mbls_bls_aggregate_verify", "mbls_bls_eth_aggregate_pubkeys",
                 "mbls_dev_fast_aggregate_verify"):
        assert name in syms


def test_library_exports_every_header_symbol(lib):
    missing = [s for s in _lib.header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_library_binding_and_messages(lib):
    l = _lib.load()
    assert b"gfx950" in l.mbls_version()
    assert _lib.status_message(-1) == "BlstError(BLST_BAD_ENCODING)"
    assert _lib.status_message(-6, 47) == "InvalidByteLength { got: 47, expected: 48 }"
    assert _lib.status_message(-9) == "Empty public key vector"


def test_code_objects_are_gfx950(lib):
    import re
    data = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", data))
    assert targets == {b"gfx950"}, targets


def test_nif_shim_type_checks():
    """nif/bls_nif.c (the drop-in `Elixir.Bls` NIF) and nif/bls_device_nif.c compile against include/mbls.h; Erlang
    headers are absent here, so a test-only declaration subset stands in (syntax/type check
    only, nothing is linked)."""
    import shutil
    import subprocess

    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for src in ("bls_nif.c", "bls_device_nif.c"):
        r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", "-std=gnu11",
                            "-I", os.path.join(root, "tests", "nif_stub"), "-I", os.path.join(root, "include"),
                            os.path.join(root, "lambda_ethereum_consensus_amd", "nif", src)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
