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


def test_c_oracle_aggregates_and_av_match_python_oracle():
    """The C entry points the BASELINE-shape GPU checks use (eth_aggregate_pubkeys,
    aggregate_verify, packed verify / AV batches, the pre-decoded warm table) agree with the
    Python oracle on small cases, including every error class."""
    import random

    import numpy as np

    from oracle import bls12_381 as o
    from tests import coracle

    rng = random.Random(99)
    sks = [rng.randrange(1, o.R) for _ in range(6)]
    pks = [o.sk_to_pk(s) for s in sks]
    bad = [b"\x80" + bytes(47), o.INFINITY_PUBKEY, pks[0][:47], (o.P | (1 << 383)).to_bytes(48, "big")]
    cases = [pks[:1], pks[:4], [pks[1], o.g1_compress(o.g1_neg(o.g1_uncompress(pks[1])))], [],
             [pks[0], bad[0], bad[1]], [pks[2], bad[2]], [bad[3]], [pks[3], pks[3]]]
    for ks in cases:
        assert coracle.eth_aggregate_pubkeys(ks) == o.eth_aggregate_pubkeys(ks), ks
    msgs = [bytes([i]) * 32 for i in range(6)]
    acc = None
    for s, m in zip(sks, msgs):
        acc = o.g2_add(acc, o.g2_uncompress(o.sign(s.to_bytes(32, "big"), m)[1]))
    sig = o.g2_compress(acc)
    av_cases = [(pks, msgs, sig), (pks, msgs[:5], sig), (pks, [msgs[1]] + msgs[1:], sig), ([], [], sig),
                (pks[:2], msgs[:2], o.INFINITY_SIGNATURE), (pks[:2], msgs[:2], bytes(96)),
                ([pks[0], bad[1]], msgs[:2], sig), (pks[:1], [bytes(31)], sig)]
    for ks, ms, sg in av_cases:
        assert coracle.outcome(coracle.av_code(ks, ms, sg), ks, ms) == o.aggregate_verify(ks, ms, sg)
    # packed batches: verify and AV (pairs = one key / message each)
    vs = [(pks[i], msgs[i], o.sign(sks[i].to_bytes(32, "big"), msgs[i])[1]) for i in range(4)]
    vs.append((pks[0], msgs[1], vs[0][2]))
    got = coracle.verify_batch(b"".join(v[0] for v in vs), b"".join(v[1] for v in vs), b"".join(v[2] for v in vs))
    assert got.tolist() == [1, 1, 1, 1, 0]
    off = np.array([0, 6, 8], dtype=np.uint32)
    sig2 = o.g2_compress(o.g2_add(o.g2_uncompress(vs[0][2]), o.g2_uncompress(vs[1][2])))
    got = coracle.av_batch(b"".join(pks) + pks[0] + pks[1], b"".join(msgs) + msgs[0] + msgs[1], off, sig + sig2)
    assert got.tolist() == [1, 1]
    # warm table == cold per-set outcome
    table = pks + [bad[0], bad[3]]
    t = coracle.Table(b"".join(table))
    sets = [([0, 1, 2], msgs[0]), ([3, 6], msgs[1]), ([], msgs[2]), ([7, 1], msgs[3]), ([5, 5], msgs[4])]
    sg = [o.sign((sum(sks[i] for i in ix if i < 6) % o.R or 1).to_bytes(32, "big"), m)[1] for ix, m in sets]
    idx = [i for ix, _ in sets for i in ix]
    ioff = np.cumsum([0] + [len(ix) for ix, _ in sets]).astype(np.uint32)
    for eth in (False, True):
        warm = t.fav_batch(idx, ioff, b"".join(m for _, m in sets), b"".join(sg), eth=eth).tolist()
        cold = [coracle.fav_code([table[i] for i in ix], m, s, eth) for (ix, m), s in zip(sets, sg)]
        assert warm == cold


def test_kat_sign_aggregate_vectors_verify_in_c(coracle):
    """The consensus-spec-tests sign / aggregate KATs (tests/golden/kat.yaml) verify true in the
    C restatement: every signature under its key, the 0xab.. aggregate under the three keys."""
    kat = yaml.safe_load(open(os.path.join(ROOT, "tests", "golden", "kat.yaml")))
    pk = {v["privkey"]: bytes.fromhex(v["pubkey"]) for v in kat["pubkeys"]}
    for v in kat["sign"]:
        m, s = bytes.fromhex(v["message"]), bytes.fromhex(v["signature"])
        assert coracle.oracle_c_verify(pk[v["privkey"]], 48, m, 32, s, 96) == 1
        assert coracle.oracle_c_verify(pk[v["privkey"]], 48, bytes(31) + b"\x01", 32, s, 96) == 0
    keys = [pk[v["privkey"]] for v in kat["sign"] if v["message"] == "ab" * 32]
    agg = bytes.fromhex(kat["aggregate"][0]["signature"])
    assert c_fav(coracle, keys, bytes.fromhex("ab" * 32), agg, False) == 1
    assert c_fav(coracle, keys[::-1][:2], bytes.fromhex("ab" * 32), agg, False) == 0


def test_device_algorithm_pairing_equals_the_restatement():
    """oracle/c's verify tails run the device's pairing algorithms (projective RCB steps, shared
    squarings, sparse lines, Granger-Scott squarings; r06, the CPU baseline's honest per-M cost):
    for 1, 2 and 4 pairs the reduced value of that Miller product equals the affine restatement's,
    coefficient by coefficient, and the cyclotomic / complex squarings equal general products."""
    import ctypes

    from tests import coracle

    L = coracle.lib()
    L.oracle_c_selftest_pairing.argtypes = [ctypes.c_uint32, ctypes.c_int]
    for seed in range(4):
        for n in (1, 2, 3, 4):
            assert L.oracle_c_selftest_pairing(seed, n) == 0, (seed, n)
