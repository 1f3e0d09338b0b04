"""GPU: the engine reproduces the published known-answer vectors the oracle is pinned to
(tests/golden/kat.yaml: consensus-spec-tests v1.3.0 general/phase0/bls sign / aggregate,
recalled and reproduced bit-exactly by the oracle) through the reference's own entry points:
Bls.sign (lib.rs:14-29), Bls.aggregate (lib.rs:31-51), Bls.verify (lib.rs:53-60) and
Bls.fast_aggregate_verify (lib.rs:84-100), plus the device Sign / SkToPk batch kernels."""
import os

import numpy as np
import pytest
import yaml

pytestmark = pytest.mark.gpu
KAT = yaml.safe_load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.yaml")))


def test_sign_kats_through_the_nif_entry():
    from lambda_ethereum_consensus_amd import bls

    for v in KAT["sign"]:
        got = bls.sign(bytes.fromhex(v["privkey"]), bytes.fromhex(v["message"]))
        assert got == ("ok", bytes.fromhex(v["signature"])), v["privkey"][:8]


def test_sign_and_pubkey_kats_through_the_device_batch():
    from lambda_ethereum_consensus_amd import device as D

    D.init(0)
    sks = b"".join(bytes.fromhex(v["privkey"]) for v in KAT["sign"])
    msgs = b"".join(bytes.fromhex(v["message"]) for v in KAT["sign"])
    n = len(KAT["sign"])
    d_sk, d_m, d_s = D.Buffer.from_host(sks), D.Buffer.from_host(msgs), D.Buffer(96 * n)
    D.sign(d_sk, d_m, d_s, n)
    assert d_s.to_numpy().reshape(n, 96).tobytes() == b"".join(bytes.fromhex(v["signature"]) for v in KAT["sign"])
    m = len(KAT["pubkeys"])
    d_sk2, d_pk = D.Buffer.from_host(b"".join(bytes.fromhex(v["privkey"]) for v in KAT["pubkeys"])), D.Buffer(48 * m)
    D.sk_to_pk(d_sk2, d_pk, m)
    assert d_pk.to_numpy().tobytes() == b"".join(bytes.fromhex(v["pubkey"]) for v in KAT["pubkeys"])


def test_aggregate_and_verify_kats():
    from lambda_ethereum_consensus_amd import bls

    for v in KAT["aggregate"]:
        assert bls.aggregate([bytes.fromhex(x) for x in v["signatures"]]) == ("ok", bytes.fromhex(v["signature"]))
    pk = {v["privkey"]: bytes.fromhex(v["pubkey"]) for v in KAT["pubkeys"]}
    sets = [(pk[v["privkey"]], bytes.fromhex(v["message"]), bytes.fromhex(v["signature"])) for v in KAT["sign"]]
    assert bls.verify_batch(sets) == [("ok", True)] * len(sets)
    assert bls.verify(sets[0][0], sets[1][1], sets[0][2]) == ("ok", sets[0][1] == sets[1][1])
    keys = [pk[v["privkey"]] for v in KAT["sign"] if v["message"] == "ab" * 32]
    agg = bytes.fromhex(KAT["aggregate"][0]["signature"])
    msg = bytes.fromhex("ab" * 32)
    assert bls.fast_aggregate_verify(keys, msg, agg) == ("ok", True)
    assert bls.eth_fast_aggregate_verify(keys, msg, agg) == ("ok", True)
    assert bls.fast_aggregate_verify(keys[:2], msg, agg) == ("ok", False)
    assert bls.fast_aggregate_verify(keys, bytes(32), agg) == ("ok", False)
    assert np.array_equal(np.frombuffer(bls.eth_aggregate_pubkeys(keys)[1], np.uint8),
                          np.frombuffer(bls.eth_aggregate_pubkeys(keys[::-1])[1], np.uint8))
