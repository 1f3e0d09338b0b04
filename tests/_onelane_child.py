"""Child process of tests/test_gpu_parity.py (GPU): with MBLS_G2_CRITICAL_KEYS=0
(test_one_lane_cold_fav_path) every device-level fast_aggregate_verify takes the one-lane cold
verdict path (one-lane H(m), sig_miller, fav_verdict over projective key sums); without it
(test_lane_group_forms, MBLS_LG16 / MBLS_LG16_PREP forced) the small batches take the
lane-group latency path.  Compares ragged / invalid / eth-variant sets with the oracle.
Prints OK on success."""
import os
import random
import sys

import numpy as np

from oracle import bls12_381 as o


FORMS = ("fav_verdict_1l", "fav_verdict_lg8", "fav_verdict_lg16", "fav_verdict_lg6")
PATHS = ("path_prep_1l_table", "path_prep_lg", "path_prep_1l_cold", "path_miller_split", "path_miller_joint",
         "path_key_alt", "path_verify_key_alt", "path_lat_kstream2", "path_warm_fill", "path_warm_defer",
         "path_av_grouped", "path_av_onelane", "path_prep_split", "path_av_pipelined")


def check_forms(forms, paths, calls=2):
    """MBLS_EXPECT_FORM: the verdict form EVERY device call took (exactly `calls` verdict launches
    of that form, none of another); MBLS_EXPECT_PATHS "name=count,...": exact path counts of the
    same calls (a forced form must decide every call)."""
    want = os.environ.get("MBLS_EXPECT_FORM")
    if want and ":" in want:  # "form:count,...": a mix of forms, exact counts (a deferred table verdict)
        exp = {"fav_verdict_" + k: int(n) for k, n in (x.split(":") for x in want.split(","))}
        assert sum(exp.values()) == calls and all(forms[k] == n for k, n in exp.items()), (exp, forms)
        assert sum(forms.values()) == calls, forms
    elif want:
        assert forms["fav_verdict_" + want] == calls and sum(forms.values()) == calls, forms
    for item in filter(None, os.environ.get("MBLS_EXPECT_PATHS", "").split(",")):
        name, n = item.split("=")
        assert paths["path_" + name] == int(n), (name, paths)


def main():
    from lambda_ethereum_consensus_amd import bls
    from lambda_ethereum_consensus_amd import device as D

    rng = random.Random(23)
    sks = [rng.randrange(1, o.R) for _ in range(12)]
    pks = [o.sk_to_pk(s) for s in sks]
    sets = []
    for n in (1, 2, 3, 5, 8, 0, 7, 4):
        idx = [rng.randrange(len(sks)) for _ in range(n)]
        m = bytes(rng.randrange(256) for _ in range(32))
        s = o.sign((sum(sks[i] for i in idx) % o.R or 1).to_bytes(32, "big"), m)[1] if n else o.INFINITY_SIGNATURE
        sets.append(([pks[i] for i in idx], m, s))
    sets.append((sets[0][0], bytes(32), sets[0][2]))                       # wrong message
    sets.append((sets[1][0], sets[1][1], bytes(96)))                       # NONE signature
    sets.append((sets[2][0], sets[2][1], o.INFINITY_SIGNATURE))            # infinity signature
    p0 = o.g1_uncompress(pks[3])
    sets.append(([pks[3], o.g1_compress(o.g1_neg(p0))], sets[3][1], sets[3][2]))  # aggregate at infinity
    bad = bytearray(pks[4])
    bad[5] ^= 0x40
    sets.append(([pks[5], bytes(bad)], sets[4][1], sets[4][2]))           # undecodable / off-curve key
    n_sets = len(sets)
    keys = b"".join(k for s in sets for k in s[0])
    off = np.cumsum([0] + [len(s[0]) for s in sets]).astype(np.uint32)
    msgs = b"".join(s[1] for s in sets)
    sigs = b"".join(s[2] for s in sets)
    from tests import coracle

    D.prof_enable(True)
    forms = {k: 0 for k in FORMS}
    paths = {k: 0 for k in PATHS}
    for eth in (False, True):
        st = D.Buffer(4 * n_sets)
        bufs = [D.Buffer.from_host(x) for x in (keys, off, msgs, sigs)]
        D.synchronize()
        D.prof_reset()  # count exactly this device call's forms (not the uploads, not the host batch below)
        D.fast_aggregate_verify(*bufs, st, n_sets, eth=eth)
        D.synchronize()
        for k in FORMS:
            forms[k] += D.prof_read(k)[1]
        for k in PATHS:
            paths[k] += D.prof_read(k)[1]
        got = st.to_numpy(np.int32).tolist()
        fn = o.eth_fast_aggregate_verify if eth else o.fast_aggregate_verify
        exp = []
        for s in sets:
            tag, v = fn(*s)
            exp.append((1 if v else 0) if tag == "ok" else None)
        # exact codes (the error kind too) from the C restatement, itself checked against the
        # Python oracle above on every non-error outcome
        codes = coracle.fav_codes(sets, eth=eth)
        assert [c if e is None else e for c, e in zip(codes, exp)] == codes, (codes, exp)
        assert got == codes, (got, codes)
        # the same sets through the host batch API (lane-group latency path) agree
        assert [(("ok", bool(g)) if g >= 0 else None) for g in got] == \
            [(r if r[0] == "ok" else None) for r in bls.fast_aggregate_verify_batch(sets, eth=eth)]
        if not eth:
            cold_codes = codes
    D.prof_enable(False)
    check_forms(forms, paths)
    print("forms", forms, "paths", paths)
    # the same key lists as rows of the validator pubkey table (index-addressed, the table
    # gather's aggregation kernel): outcomes equal the cold path's (a row's status is its key's
    # decode result, ordered by list position like the cold keys)
    if keys:
        D.pk_table_set(0, D.Buffer.from_host(keys), len(keys) // 48)
        st = D.Buffer(4 * n_sets)
        D.fast_aggregate_verify_indexed(D.Buffer.from_host(np.arange(len(keys) // 48, dtype=np.uint32)),
                                        D.Buffer.from_host(off), D.Buffer.from_host(msgs), D.Buffer.from_host(sigs),
                                        st, n_sets)
        D.synchronize()
        assert st.to_numpy(np.int32).tolist() == cold_codes, (st.to_numpy(np.int32).tolist(), cold_codes)
    print("OK")


if __name__ == "__main__":
    sys.exit(main())
