#!/usr/bin/env python3
"""Generate the BLS golden fixtures (consensus-spec-tests `data.yaml` schema) from the oracle.

Layout mirrors test/spec/vectors/tests/general/<fork>/bls/<handler>/small/<case>/data.yaml
(reference lib/spec/testcase.ex:39-49) so the same harness can later run the real
consensus-spec-tests v1.3.0 vectors dropped into tests/vectors/.  Outputs: `null` = the
call must return {:error, _} (runner semantics of lib/spec/runners/bls.ex:36-138).

Also writes tests/golden/kat.yaml: published known-answer vectors the oracle reproduces
(RFC 9380 expand_message_xmd / hash_to_curve J.10.1, consensus-spec-tests sign vectors).

Run:  python3 tests/golden/gen_fixtures.py   (deterministic; output committed)
"""
import os
import random
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as o  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "bls")
rng = random.Random(20250224)


def hx(b):
    return "0x" + bytes(b).hex()


def out_val(res):
    tag, v = res
    if tag == "error":
        return None
    if isinstance(v, bool):
        return v
    return hx(v)


def write(fork, handler, name, inp, output):
    d = os.path.join(OUT, fork, handler, name)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "data.yaml"), "w") as f:
        yaml.safe_dump({"input": inp, "output": output}, f, sort_keys=False)


# key material: the consensus-spec-tests generator's three private keys + random ones
SKS = [
    0x263DBD792F5B1BE47ED85F8938C0F29586AF0D3AC7B977F21C278FE1462040E3,
    0x47B8192D77BF871B62E87859D653922725724A5C031AFEABC60BCEF5FF665138,
    0x328388AFF0D4A5B7DC9205ABD374E7E98F3CD9F3418EDB4EAFDA5FB16473D216,
] + [rng.randrange(1, o.R) for _ in range(5)]
MSGS = [bytes(32), b"\x56" * 32, b"\xab" * 32] + [bytes(rng.randrange(256) for _ in range(32)) for _ in range(3)]
PKS = [o.sk_to_pk(sk) for sk in SKS]


def sig(sk, m):
    return o.sign(sk.to_bytes(32, "big"), m)[1]


def on_curve_not_in_g1():
    while True:
        x = rng.randrange(o.P)
        y = o.fp_sqrt(x ** 3 + 4)
        if y is not None and not o.g1_in_subgroup((x, y)):
            return o.g1_compress((x, y))


def on_curve_not_in_g2():
    while True:
        x = (rng.randrange(o.P), rng.randrange(o.P))
        y = o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2))
        if y is not None:
            return o.g2_compress((x, y))


def not_on_curve_g1():
    while True:
        x = rng.randrange(o.P)
        if o.fp_sqrt(x ** 3 + 4) is None:
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80
            return bytes(b)


def not_on_curve_g2():
    while True:
        x = (rng.randrange(o.P), rng.randrange(o.P))
        if o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2)) is None:
            b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
            b[0] |= 0x80
            return bytes(b)


def tamper(b, i=5):
    b = bytearray(b)
    b[i] ^= 0x01
    return bytes(b)


def neg_pk(pkb):
    p = o.g1_uncompress(pkb)
    return o.g1_compress(o.g1_neg(p))


def main():
    P_NOT_G1 = on_curve_not_in_g1()
    P_NOC = not_on_curve_g1()
    S_NOT_G2 = on_curve_not_in_g2()
    S_NOC = not_on_curve_g2()
    X_GE_P = bytes([0x9A]) + b"\xff" * 47  # flags + x >= p
    INF_PK, INF_SIG, NONE_SIG = o.INFINITY_PUBKEY, o.INFINITY_SIGNATURE, o.NONE_SIGNATURE

    # ---------------- sign
    for i, sk in enumerate(SKS[:3]):
        for j, m in enumerate(MSGS[:3]):
            write("phase0", "sign", f"sign_case_sk{i}_m{j}", {"privkey": hx(sk.to_bytes(32, "big")), "message": hx(m)},
                  out_val(o.sign(sk.to_bytes(32, "big"), m)))
    write("phase0", "sign", "sign_case_zero_privkey", {"privkey": hx(bytes(32)), "message": hx(MSGS[1])}, None)
    write("phase0", "sign", "sign_case_privkey_eq_r", {"privkey": hx(o.R.to_bytes(32, "big")), "message": hx(MSGS[1])}, None)

    # ---------------- verify
    cases = {
        "verify_valid_case": (PKS[0], MSGS[0], sig(SKS[0], MSGS[0])),
        "verify_valid_case_2": (PKS[1], MSGS[1], sig(SKS[1], MSGS[1])),
        "verify_wrong_message": (PKS[0], MSGS[1], sig(SKS[0], MSGS[0])),
        "verify_wrong_pubkey": (PKS[1], MSGS[0], sig(SKS[0], MSGS[0])),
        "verify_tampered_signature": (PKS[2], MSGS[2], tamper(sig(SKS[2], MSGS[2]), 50)),
        "verify_infinity_pubkey_and_infinity_signature": (INF_PK, MSGS[0], INF_SIG),
        "verify_infinity_signature": (PKS[0], MSGS[0], INF_SIG),
        "verify_none_signature": (PKS[0], MSGS[0], NONE_SIG),
        "verify_pubkey_not_in_g1": (P_NOT_G1, MSGS[0], sig(SKS[0], MSGS[0])),
        "verify_pubkey_not_on_curve": (P_NOC, MSGS[0], sig(SKS[0], MSGS[0])),
        "verify_pubkey_x_ge_p": (X_GE_P, MSGS[0], sig(SKS[0], MSGS[0])),
        "verify_signature_not_in_g2": (PKS[0], MSGS[0], S_NOT_G2),
        "verify_signature_not_on_curve": (PKS[0], MSGS[0], S_NOC),
        "verify_pubkey_wrong_length": (PKS[0][:47], MSGS[0], sig(SKS[0], MSGS[0])),
        "verify_signature_wrong_length": (PKS[0], MSGS[0], sig(SKS[0], MSGS[0])[:95]),
        "verify_message_wrong_length": (PKS[0], MSGS[0][:31], sig(SKS[0], MSGS[0])),
        "verify_sig_error_beats_pk_error": (PKS[0][:47], MSGS[0], S_NOC),
    }
    for name, (pk, m, s) in cases.items():
        write("phase0", "verify", name, {"pubkey": hx(pk), "message": hx(m), "signature": hx(s)},
              out_val(o.verify(pk, m, s)))

    # ---------------- aggregate
    s0, s1, s2 = sig(SKS[0], MSGS[0]), sig(SKS[1], MSGS[1]), sig(SKS[2], MSGS[2])
    agg_cases = {
        "aggregate_single_signature": [s0],
        "aggregate_three": [s0, s1, s2],
        "aggregate_with_none_signature": [s0, NONE_SIG, s1],
        "aggregate_infinity_signature": [INF_SIG],
        "aggregate_na_signatures": [],
        "aggregate_undecodable": [s0, S_NOC],
        "aggregate_not_in_g2_ok": [S_NOT_G2, s1],
        "aggregate_sum_to_infinity": [s0, o.g2_compress(o.g2_neg(o.g2_uncompress(s0)))],
        "aggregate_wrong_length": [s0, s1[:90]],
    }
    for name, sigs in agg_cases.items():
        write("phase0", "aggregate", name, [hx(s) for s in sigs], out_val(o.aggregate(sigs)))

    # ---------------- fast_aggregate_verify
    def fav_sig(idx, m):
        acc = sum(SKS[i] for i in idx) % o.R
        return o.sign(acc.to_bytes(32, "big"), m)[1]

    fav_cases = {
        "fast_aggregate_verify_valid_1": ([PKS[0]], MSGS[3], fav_sig([0], MSGS[3])),
        "fast_aggregate_verify_valid_3": (PKS[:3], MSGS[3], fav_sig([0, 1, 2], MSGS[3])),
        "fast_aggregate_verify_valid_8": (PKS[:8], MSGS[4], fav_sig(range(8), MSGS[4])),
        "fast_aggregate_verify_duplicate_keys": ([PKS[1], PKS[1], PKS[2]], MSGS[4], fav_sig([1, 1, 2], MSGS[4])),
        "fast_aggregate_verify_extra_pubkey": (PKS[:4], MSGS[3], fav_sig([0, 1, 2], MSGS[3])),
        "fast_aggregate_verify_wrong_message": (PKS[:3], MSGS[4], fav_sig([0, 1, 2], MSGS[3])),
        "fast_aggregate_verify_tampered_signature": (PKS[:3], MSGS[3], tamper(fav_sig([0, 1, 2], MSGS[3]), 40)),
        "fast_aggregate_verify_na_pubkeys_and_infinity_signature": ([], MSGS[0], INF_SIG),
        "fast_aggregate_verify_na_pubkeys_and_none_signature": ([], MSGS[0], NONE_SIG),
        "fast_aggregate_verify_infinity_pubkey": ([PKS[0], INF_PK], MSGS[3], fav_sig([0], MSGS[3])),
        "fast_aggregate_verify_keys_sum_to_infinity": ([PKS[0], neg_pk(PKS[0])], MSGS[3], INF_SIG),
        "fast_aggregate_verify_first_error_wins": ([PKS[0], P_NOC, P_NOT_G1], MSGS[3], fav_sig([0], MSGS[3])),
        "fast_aggregate_verify_first_error_wins_2": ([PKS[0], PKS[1][:10], P_NOC], MSGS[3], fav_sig([0], MSGS[3])),
        "fast_aggregate_verify_sig_not_in_g2": (PKS[:2], MSGS[3], S_NOT_G2),
        "fast_aggregate_verify_none_signature": (PKS[:2], MSGS[3], NONE_SIG),
    }
    for name, (pks, m, s) in fav_cases.items():
        inp = {"pubkeys": [hx(k) for k in pks], "message": hx(m), "signature": hx(s)}
        write("phase0", "fast_aggregate_verify", name, inp, out_val(o.fast_aggregate_verify(pks, m, s)))
        write("altair", "eth_fast_aggregate_verify", "eth_" + name, inp, out_val(o.eth_fast_aggregate_verify(pks, m, s)))

    # ---------------- aggregate_verify
    def av_sig(pairs):
        acc = None
        for i, m in pairs:
            acc = o.g2_add(acc, o.g2_uncompress(sig(SKS[i], m)))
        return o.g2_compress(acc)

    av_cases = {
        "aggregate_verify_valid": ([PKS[0], PKS[1], PKS[2]], MSGS[:3], av_sig([(0, MSGS[0]), (1, MSGS[1]), (2, MSGS[2])])),
        "aggregate_verify_valid_same_message": ([PKS[3], PKS[4]], [MSGS[5], MSGS[5]], av_sig([(3, MSGS[5]), (4, MSGS[5])])),
        "aggregate_verify_single": ([PKS[5]], [MSGS[4]], sig(SKS[5], MSGS[4])),
        "aggregate_verify_wrong_message": ([PKS[0], PKS[1]], [MSGS[0], MSGS[2]], av_sig([(0, MSGS[0]), (1, MSGS[1])])),
        "aggregate_verify_count_mismatch": ([PKS[0], PKS[1]], [MSGS[0]], av_sig([(0, MSGS[0]), (1, MSGS[1])])),
        "aggregate_verify_na_pubkeys_and_infinity_signature": ([], [], INF_SIG),
        "aggregate_verify_na_pubkeys_and_na_signature": ([], [], NONE_SIG),
        "aggregate_verify_infinity_pubkey": ([PKS[0], INF_PK], [MSGS[0], MSGS[1]], av_sig([(0, MSGS[0])])),
        "aggregate_verify_tampered_signature": ([PKS[0], PKS[1]], [MSGS[0], MSGS[1]], tamper(av_sig([(0, MSGS[0]), (1, MSGS[1])]), 70)),
        "aggregate_verify_message_wrong_length": ([PKS[0]], [MSGS[0][:20]], sig(SKS[0], MSGS[0])),
    }
    for name, (pks, ms, s) in av_cases.items():
        inp = {"pubkeys": [hx(k) for k in pks], "messages": [hx(m) for m in ms], "signature": hx(s)}
        write("phase0", "aggregate_verify", name, inp, out_val(o.aggregate_verify(pks, ms, s)))

    # ---------------- eth_aggregate_pubkeys
    eap_cases = {
        "eth_aggregate_pubkeys_valid_1": [PKS[0]],
        "eth_aggregate_pubkeys_valid_3": PKS[:3],
        "eth_aggregate_pubkeys_valid_8": PKS[:8],
        "eth_aggregate_pubkeys_empty_list": [],
        "eth_aggregate_pubkeys_infinity_pubkey": [PKS[0], INF_PK],
        "eth_aggregate_pubkeys_x40_pubkey": [PKS[0], bytes([0x40]) + bytes(47)],
        "eth_aggregate_pubkeys_not_in_g1": [PKS[0], P_NOT_G1],
        "eth_aggregate_pubkeys_sum_to_infinity": [PKS[1], neg_pk(PKS[1])],
        "eth_aggregate_pubkeys_duplicates": [PKS[2], PKS[2], PKS[2]],
    }
    for name, pks in eap_cases.items():
        write("altair", "eth_aggregate_pubkeys", name, [hx(k) for k in pks], out_val(o.eth_aggregate_pubkeys(pks)))

    # ---------------- published known-answer vectors
    kat = {
        "source": "RFC 9380 K.1 / J.10.1 and consensus-spec-tests v1.3.0 general/phase0/bls/sign (recalled, reproduced bit-exactly by the oracle)",
        "expand_message_xmd_sha256": [
            {"dst": "QUUX-V01-CS02-with-expander-SHA256-128", "msg": "", "len_in_bytes": 32,
             "uniform_bytes": "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"},
            {"dst": "QUUX-V01-CS02-with-expander-SHA256-128", "msg": "abc", "len_in_bytes": 32,
             "uniform_bytes": "d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615"},
        ],
        "hash_to_g2": [
            {"dst": "QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_", "msg": "",
             "x_c0": "0141ebfbdca40eb85b87142e130ab689c673cf60f1a3e98d69335266f30d9b8d4ac44c1038e9dcdd5393faf5c41fb78a",
             "x_c1": "05cb8437535e20ecffaef7752baddf98034139c38452458baeefab379ba13dff5bf5dd71b72418717047f5b0f37da03d",
             "y_c0": "0503921d7f6a12805e72940b963c0cf3471c7b2a524950ca195d11062ee75ec076daf2d4bc358c4b190c0c98064fdd92",
             "y_c1": "12424ac32561493f3fe3c260708a12b7c620e7be00099a974e259ddc7d1f6395c3c811cdd19f1e8dbf3e9ecfdcbab8d6"},
        ],
        "sign": [
            {"privkey": "263dbd792f5b1be47ed85f8938c0f29586af0d3ac7b977f21c278fe1462040e3", "message": "00" * 32,
             "signature": "b6ed936746e01f8ecf281f020953fbf1f01debd5657c4a383940b020b26507f6076334f91e2366c96e9ab279fb5158090352ea1c5b0c9274504f4f0e7053af24802e51e4568d164fe986834f41e55c8e850ce1f98458c0cfc9ab380b55285a55"},
        ],
        "pubkeys": [
            {"privkey": "263dbd792f5b1be47ed85f8938c0f29586af0d3ac7b977f21c278fe1462040e3",
             "pubkey": "a491d1b0ecd9bb917989f0e74f0dea0422eac4a873e5e2644f368dffb9a6e20fd6e10c1b77654d067c0618f6e5a7f79a"},
            {"privkey": "47b8192d77bf871b62e87859d653922725724a5c031afeabc60bcef5ff665138",
             "pubkey": "b301803f8b5ac4a1133581fc676dfedc60d891dd5fa99028805e5ea5b08d3491af75d0707adab3b70c6a6a580217bf81"},
            {"privkey": "328388aff0d4a5b7dc9205abd374e7e98f3cd9f3418edb4eafda5fb16473d216",
             "pubkey": "b53d21a4cfd562c469cc81514d4ce5a6b577d8403d32a394dc265dd190b47fa9f829fdd7963afdf972e5e77854051f6f"},
        ],
        "generators": {
            "g1": "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb",
            "g2": "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8",
        },
    }
    with open(os.path.join(ROOT, "tests", "golden", "kat.yaml"), "w") as f:
        yaml.safe_dump(kat, f, sort_keys=False)
    print("fixtures written under", OUT)


if __name__ == "__main__":
    main()
