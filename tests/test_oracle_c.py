"""CPU: the C restatement of the oracle (oracle/c, the cpu_baseline "port") agrees with the
Python oracle on the golden fixtures and reproduces the RFC 9380 hash_to_G2 vector."""
import ctypes
import os
import subprocess

import pytest
import yaml

from tests import spec_runner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "c", "libblsoracle.so")


@pytest.fixture(scope="module")
def coracle():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle", "c")], check=True, timeout=300)
    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    SZ = ctypes.c_size_t
    lib.oracle_c_fav.argtypes = [P, P, SZ, ctypes.c_char_p, SZ, ctypes.c_char_p, SZ, ctypes.c_int]
    lib.oracle_c_fav.restype = ctypes.c_int
    lib.oracle_c_verify.argtypes = [ctypes.c_char_p, SZ, ctypes.c_char_p, SZ, ctypes.c_char_p, SZ]
    lib.oracle_c_verify.restype = ctypes.c_int
    lib.oracle_c_hash_to_g2.argtypes = [ctypes.c_char_p, ctypes.c_char_p, SZ, ctypes.c_char_p, SZ]
    return lib


def c_fav(lib, pks, msg, sig, eth):
    arr = (ctypes.c_char_p * max(len(pks), 1))(*pks)
    lens = (ctypes.c_size_t * max(len(pks), 1))(*[len(k) for k in pks])
    return lib.oracle_c_fav(ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p), len(pks),
                            msg, len(msg), sig, len(sig), 1 if eth else 0)


def expected_code(res):
    tag, v = res
    if tag == "ok":
        return 1 if v else 0
    return None  # some error


def test_rfc9380_hash_to_g2(coracle):
    kat = yaml.safe_load(open(os.path.join(ROOT, "tests", "golden", "kat.yaml")))
    for v in kat["hash_to_g2"]:
        out = ctypes.create_string_buffer(192)
        coracle.oracle_c_hash_to_g2(out, v["msg"].encode(), len(v["msg"]), v["dst"].encode(), len(v["dst"]))
        got = [out.raw[i:i + 48].hex() for i in range(0, 192, 48)]
        assert got == [v["x_c0"], v["x_c1"], v["y_c0"], v["y_c1"]]


def test_fixtures_verify_family(coracle):
    from oracle import bls12_381 as o

    n = 0
    for handler, case_dir in spec_runner.discover(os.path.join(ROOT, "tests", "golden", "bls")):
        if handler not in ("verify", "fast_aggregate_verify", "eth_fast_aggregate_verify"):
            continue
        inp, _ = spec_runner.load_case(case_dir)
        if handler == "verify":
            code = coracle.oracle_c_verify(inp["pubkey"], len(inp["pubkey"]), inp["message"], len(inp["message"]),
                                           inp["signature"], len(inp["signature"]))
            res = o.verify(inp["pubkey"], inp["message"], inp["signature"])
        else:
            eth = handler.startswith("eth")
            code = c_fav(coracle, inp["pubkeys"], inp["message"], inp["signature"], eth)
            fn = o.eth_fast_aggregate_verify if eth else o.fast_aggregate_verify
            res = fn(inp["pubkeys"], inp["message"], inp["signature"])
        exp = expected_code(res)
        if exp is None:
            assert code < 0, (case_dir, code, res)
        else:
            assert code == exp, (case_dir, code, res)
        n += 1
    assert n >= 40


def test_work_model_headline_unit_matches_oracle_count():
    """the roofline's per-key M-count (bench.py M_PER_KEY) lands within ±25% of the
    C restatement's own op count for decompress + G1 membership of a fixture key."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("work_model", os.path.join(ROOT, "tools", "work_model.py"))
    wm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(wm)
    m = wm.model()
    unit = m["units"]["public_key (decompress + G1 membership)"]
    assert 0.75 <= unit["bench_M"] / unit["oracle_M"] <= 1.25, unit
    assert m["mac_per_M"] == 300
