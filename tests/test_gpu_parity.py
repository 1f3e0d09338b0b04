"""GPU parity vs the oracle on seeded random inputs: single calls, batches (including mixed
valid/invalid sets and ragged key counts) and the device-resident C-ABI entry points."""
import random

import pytest

from oracle import bls12_381 as o

pytestmark = pytest.mark.gpu
RNG = random.Random(7)


@pytest.fixture(scope="module")
def gbls():
    from lambda_ethereum_consensus_amd import bls

    return bls


def rand_msg():
    return bytes(RNG.randrange(256) for _ in range(32))


@pytest.fixture(scope="module")
def keys():
    sks = [RNG.randrange(1, o.R) for _ in range(24)]
    return sks, [o.sk_to_pk(s) for s in sks]


def sig_of(sk, m):
    return o.sign(sk.to_bytes(32, "big"), m)[1]


def test_sign_matches_oracle(gbls, keys):
    sks, _ = keys
    for sk in sks[:4]:
        m = rand_msg()
        assert gbls.sign(sk.to_bytes(32, "big"), m) == o.sign(sk.to_bytes(32, "big"), m)
    assert gbls.sign(bytes(31), bytes(32)) == o.sign(bytes(31), bytes(32))
    assert gbls.sign(o.R.to_bytes(32, "big"), bytes(32)) == ("error", "BlstError(BLST_BAD_ENCODING)")


def test_verify_batch_mixed(gbls, keys):
    sks, pks = keys
    sets = []
    for i in range(40):
        m = rand_msg()
        k = RNG.randrange(len(sks))
        s = sig_of(sks[k], m)
        kind = i % 5
        if kind == 1:
            m = rand_msg()  # wrong message
        elif kind == 2:
            s = bytearray(s)
            s[10] ^= 4
            s = bytes(s)
        elif kind == 3:
            k = (k + 1) % len(sks)  # wrong key
        sets.append((pks[k], m, s))
    got = gbls.verify_batch(sets)
    exp = [o.verify(*t) for t in sets]
    assert got == exp
    assert [gbls.verify(*t) for t in sets[:5]] == exp[:5]


def test_fast_aggregate_verify_batch_ragged(gbls, keys):
    sks, pks = keys
    sets = []
    for n in (1, 2, 3, 5, 8, 13, 24, 0, 7):
        idx = [RNG.randrange(len(sks)) for _ in range(n)]
        m = rand_msg()
        s = o.sign((sum(sks[i] for i in idx) % o.R or 1).to_bytes(32, "big"), m)[1] if n else o.INFINITY_SIGNATURE
        sets.append(([pks[i] for i in idx], m, s))
    # invalid variants: a bad key in the middle, opposite keys, not-in-group signature
    sets.append(([pks[0], pks[1][:40], pks[2]], rand_msg(), sets[0][2]))
    p0 = o.g1_uncompress(pks[3])
    sets.append(([pks[3], o.g1_compress(o.g1_neg(p0))], rand_msg(), o.INFINITY_SIGNATURE))
    for eth in (False, True):
        got = gbls.fast_aggregate_verify_batch(sets, eth=eth)
        fn = o.eth_fast_aggregate_verify if eth else o.fast_aggregate_verify
        assert got == [fn(*t) for t in sets]


def test_aggregate_verify_batch(gbls, keys):
    sks, pks = keys
    sets = []
    for n in (1, 2, 4, 16):
        idx = [RNG.randrange(len(sks)) for _ in range(n)]
        ms = [rand_msg() for _ in range(n)]
        acc = None
        for i, m in zip(idx, ms):
            acc = o.g2_add(acc, o.g2_uncompress(sig_of(sks[i], m)))
        sets.append(([pks[i] for i in idx], ms, o.g2_compress(acc)))
    sets.append((sets[1][0], sets[1][1][:1], sets[1][2]))  # count mismatch
    sets.append((sets[2][0], [sets[2][1][0], rand_msg()] + sets[2][1][2:], sets[2][2]))  # wrong message
    # odd pair counts (2-pair Miller lanes straddle set boundaries) and a bad key mid-set
    for n in (3, 5, 1):
        idx = [RNG.randrange(len(sks)) for _ in range(n)]
        ms = [rand_msg() for _ in range(n)]
        acc = None
        for i, m in zip(idx, ms):
            acc = o.g2_add(acc, o.g2_uncompress(sig_of(sks[i], m)))
        sets.append(([pks[i] for i in idx], ms, o.g2_compress(acc)))
    bad = bytearray(pks[5])
    bad[7] ^= 0x20
    sets.append(([pks[1], bytes(bad), pks[2]], [rand_msg() for _ in range(3)], sets[-1][2]))
    got = gbls.aggregate_verify_batch(sets)
    assert got == [o.aggregate_verify(*t) for t in sets]


def test_device_resident_aggregate_verify_pipelined(keys):
    """Back-to-back layer-2 aggregate_verify calls (r05: each takes its own stage of buffers and a
    triple of G2 streams, forking from the caller stream only for its inputs, so call i+1's keys
    and H(m) run beside call i's pairs and verdict): every call's statuses against the oracle,
    with the inputs of later calls different in size and content from earlier ones."""
    import numpy as np

    from lambda_ethereum_consensus_amd import device as D

    sks, pks = keys
    calls = []
    for c, per in enumerate((16, 3, 7, 16, 2)):
        key_bytes, offs, msgs, sigs, exp = b"", [0], b"", b"", []
        for s in range(5 + c):
            idx = [RNG.randrange(len(sks)) for _ in range(per)]
            ms = [rand_msg() for _ in range(per)]
            acc = None
            for i, m in zip(idx, ms):
                acc = o.g2_add(acc, o.g2_uncompress(sig_of(sks[i], m)))
            if (s + c) % 3 == 1:  # a wrong message in some sets
                ms[per // 2] = rand_msg()
            key_bytes += b"".join(pks[i] for i in idx)
            msgs += b"".join(ms)
            offs.append(offs[-1] + per)
            sigs += o.g2_compress(acc)
            exp.append(1 if (s + c) % 3 != 1 else 0)
        bufs = [D.Buffer.from_host(key_bytes), D.Buffer.from_host(msgs),
                D.Buffer.from_host(np.array(offs, dtype=np.uint32)), D.Buffer.from_host(sigs)]
        st = D.Buffer.from_host(np.full(len(exp), -77, dtype=np.int32).tobytes())
        D.aggregate_verify(bufs[0], bufs[1], bufs[2], bufs[3], st, len(exp))
        calls.append((bufs, st, exp))
    D.synchronize()
    for bufs, st, exp in calls:
        assert st.to_numpy(np.int32).tolist() == exp


def test_aggregates_match_oracle(gbls, keys):
    sks, pks = keys
    for n in (1, 3, 24):
        assert gbls.eth_aggregate_pubkeys(pks[:n]) == o.eth_aggregate_pubkeys(pks[:n])
    sigs = [sig_of(sks[i], rand_msg()) for i in range(6)]
    assert gbls.aggregate(sigs) == o.aggregate(sigs)
    assert gbls.aggregate([]) == ("error", "Empty signature vector")


def test_device_resident_fav(keys):
    import numpy as np

    from lambda_ethereum_consensus_amd import device as D

    sks, pks = keys
    n_sets, per = 6, 4
    key_bytes, offs, msgs, sigs, exp = b"", [0], b"", b"", []
    for s in range(n_sets):
        idx = [RNG.randrange(len(sks)) for _ in range(per)]
        m = rand_msg()
        sg = o.sign((sum(sks[i] for i in idx) % o.R).to_bytes(32, "big"), m)[1]
        if s == 2:
            m = rand_msg()
        key_bytes += b"".join(pks[i] for i in idx)
        offs.append(offs[-1] + per)
        msgs += m
        sigs += sg
        exp.append(1 if s != 2 else 0)
    st = D.Buffer(4 * n_sets)
    D.fast_aggregate_verify(D.Buffer.from_host(key_bytes), D.Buffer.from_host(np.array(offs, dtype=np.uint32)),
                            D.Buffer.from_host(msgs), D.Buffer.from_host(sigs), st, n_sets)
    D.synchronize()
    assert st.to_numpy(np.int32).tolist() == exp


def test_batch_telemetry_counts(gbls, keys):
    """mbls_stats_read ([:bls, :batch] telemetry): a host batch and a
    device-resident call count once each under their operation with the sets and keys they
    submitted; a nested single-set entry counts once; verdicts false are not errors."""
    import numpy as np

    from lambda_ethereum_consensus_amd import _lib
    from lambda_ethereum_consensus_amd import device as D

    sks, pks = keys
    m = rand_msg()
    sets = [([pks[0], pks[1], pks[2]], m, o.sign(((sks[0] + sks[1] + sks[2]) % o.R).to_bytes(32, "big"), m)[1]),
            ([pks[3]], rand_msg(), o.sign(sks[3].to_bytes(32, "big"), m)[1])]
    b0 = _lib.stats()
    assert gbls.fast_aggregate_verify_batch(sets) == [("ok", True), ("ok", False)]
    assert gbls.eth_fast_aggregate_verify(sets[0][0], sets[0][1], sets[0][2]) == ("ok", True)
    st = D.Buffer(8)
    D.fast_aggregate_verify(D.Buffer.from_host(b"".join(sets[0][0] + sets[1][0])),
                            D.Buffer.from_host(np.array([0, 3, 4], dtype=np.uint32)),
                            D.Buffer.from_host(sets[0][1] + sets[1][1]), D.Buffer.from_host(sets[0][2] + sets[1][2]),
                            st, 2)
    D.synchronize()
    b1 = _lib.stats()
    fav = {k: b1["fast_aggregate_verify"][k] - b0["fast_aggregate_verify"][k] for k in b1["verify"]}
    eth = {k: b1["eth_fast_aggregate_verify"][k] - b0["eth_fast_aggregate_verify"][k] for k in b1["verify"]}
    assert (fav["calls"], fav["sets"], fav["keys"], fav["errors"]) == (2, 4, 8, 0)
    assert (eth["calls"], eth["sets"], eth["keys"], eth["errors"]) == (1, 1, 3, 0)
    assert fav["ns"] > 0 and eth["ns"] > 0


def test_device_keygen_and_sign(keys):
    """SkToPk / Sign batch kernels vs the oracle (bench input generation relies on them)."""
    import numpy as np

    from lambda_ethereum_consensus_amd import device as D

    sks, pks = keys
    n = 8
    sk = b"".join(s.to_bytes(32, "big") for s in sks[:n])
    msgs = b"".join(rand_msg() for _ in range(n))
    d_sk = D.Buffer.from_host(sk)
    out_pk, out_sig = D.Buffer(48 * n), D.Buffer(96 * n)
    D.sk_to_pk(d_sk, out_pk, n)
    D.sign(d_sk, D.Buffer.from_host(msgs), out_sig, n)
    D.synchronize()
    got_pk = out_pk.to_numpy().tobytes()
    got_sig = out_sig.to_numpy().tobytes()
    for i in range(n):
        assert got_pk[48 * i:48 * i + 48] == pks[i]
        assert got_sig[96 * i:96 * i + 96] == sig_of(sks[i], msgs[32 * i:32 * i + 32])


def test_key_validation_torsion_points(gbls, keys):
    """Keys with small-order components (the incomplete-addition exceptional cases of the
    device membership ladder) and cofactor-cleared keys: same verdicts/errors as the oracle."""
    from tests.test_hostsim_arith import G1_COFACTOR, _random_e1_point

    rng = random.Random(78)
    n = G1_COFACTOR * o.R
    pts = []
    for div in (3, 11**2, 10177**2, 859267**2, 52437899**2, 3 * 11**2):
        for _ in range(8):
            t = o.g1_mul(_random_e1_point(rng), n // div)
            if t is not None:
                pts += [t, o.g1_add(o.g1_mul(o.G1_GEN, rng.randrange(1, o.R)), t)]
                break
    pts.append(o.g1_mul(_random_e1_point(rng), G1_COFACTOR))
    sks, pks = keys
    m = rand_msg()
    sig = sig_of(sks[0], m)
    sets = [([pks[0], o.g1_compress(pt)], m, sig) for pt in pts] + [([o.g1_compress(pt)], m, sig) for pt in pts]
    got = gbls.fast_aggregate_verify_batch(sets)
    exp = [o.fast_aggregate_verify(p, mm, s) for p, mm, s in sets]
    assert got == exp
    assert sum(1 for e in exp if e[0] == "error") >= 10


def test_device_validate_and_aggregate_pubkeys(keys):
    import numpy as np

    from lambda_ethereum_consensus_amd import device as D

    sks, pks = keys
    table = list(pks[:10]) + [o.INFINITY_PUBKEY, bytes(48)]
    st = D.Buffer(4 * len(table))
    D.validate_pubkeys(D.Buffer.from_host(b"".join(table)), st)
    D.synchronize()
    assert st.to_numpy(np.int32).tolist() == [0] * 10 + [-5, -1]
    offs = np.array([0, 3, 3, 10], dtype=np.uint32)
    out, st2 = D.Buffer(48 * 3), D.Buffer(4 * 3)
    D.aggregate_pubkeys(D.Buffer.from_host(b"".join(pks[:10])), D.Buffer.from_host(offs), out, st2, 3)
    D.synchronize()
    codes = st2.to_numpy(np.int32).tolist()
    ob = out.to_numpy().tobytes()
    assert codes == [2, -9, 2]
    assert ob[:48] == o.eth_aggregate_pubkeys(pks[:3])[1]
    assert ob[96:144] == o.eth_aggregate_pubkeys(pks[3:10])[1]


def test_pubkey_table_indexed_fav(gbls, keys):
    """Warm path: committees as table rows give the cold path's outcomes on
    the same key lists, including invalid rows, empty sets and rows never set."""
    sks, pks = keys
    bad = [bytes(48), o.INFINITY_PUBKEY, b"\x80" + bytes(47), b"\x9a" + bytes(47)]  # no flag / infinity / x=0 / x>=p?
    table = list(pks) + bad
    t = gbls.PubkeyTable()
    t.clear()
    codes = t.set(5, table)
    cold = [o.fast_aggregate_verify([k], bytes(32), bytes(96)) for k in table]
    assert [c == 0 for c in codes] == [c[0] == "ok" for c in cold]
    assert t.size == 5 + len(table)
    rows = {i: 5 + i for i in range(len(table))}
    sets, cold_sets = [], []
    for s in range(30):
        n = RNG.randrange(0, 6)
        members = [RNG.randrange(len(pks)) for _ in range(n)]
        m = rand_msg()
        sig = sig_of((sum(sks[i] for i in members) % o.R) or 1, m) if members else sig_of(1, m)
        kind = s % 6
        idx = [rows[i] for i in members]
        keyb = [table[i] for i in members]
        if kind == 1 and members:
            m = rand_msg()
        elif kind == 2:
            j = RNG.randrange(len(bad))
            idx.insert(RNG.randrange(len(idx) + 1), rows[len(pks) + j])
            keyb.insert(idx.index(rows[len(pks) + j]), table[len(pks) + j])
        elif kind == 3:
            sig = o.INFINITY_SIGNATURE if hasattr(o, "INFINITY_SIGNATURE") else sig
        sets.append((idx, m, sig))
        cold_sets.append((keyb, m, sig))
    for eth in (False, True):
        got = t.fast_aggregate_verify_batch(sets, eth=eth)
        exp = gbls.fast_aggregate_verify_batch(cold_sets, eth=eth)
        assert got == exp
    # rows never set (0..4) and past the table
    m = rand_msg()
    got = t.fast_aggregate_verify_batch([([rows[0], 2], m, sig_of(sks[0], m)), ([10**6], m, sig_of(1, m))])
    assert got == [("error", "UnknownValidatorIndex")] * 2
    t.clear()
    assert t.size == 0


def test_pubkey_table_aggregate_pubkeys(keys):
    import numpy as np

    from lambda_ethereum_consensus_amd import device as D

    sks, pks = keys
    D.init(0)
    d = D.Buffer.from_host(b"".join(pks))
    D.pk_table_set(0, d, len(pks))
    idx = np.array([3, 1, 4, 1, 5, 9, 2, 6], dtype=np.uint32)
    off = np.array([0, 3, 8], dtype=np.uint32)
    out, st = D.Buffer(96), D.Buffer(8)
    D.aggregate_pubkeys_indexed(D.Buffer.from_host(idx), D.Buffer.from_host(off), out, st, 2)
    D.synchronize()
    assert st.to_numpy(np.int32).tolist() == [2, 2]
    ob = out.to_numpy().tobytes()
    assert ob[:48] == o.eth_aggregate_pubkeys([pks[i] for i in idx[:3]])[1]
    assert ob[48:] == o.eth_aggregate_pubkeys([pks[i] for i in idx[3:]])[1]


def test_batching_queue_coalesces_concurrent_callers(gbls, keys):
    """concurrent single-set calls through the queue return the per-call
    outcomes and share device batches."""
    import threading

    sks, pks = keys
    calls = []
    for i in range(48):
        n = 1 + i % 4
        members = [(i * 7 + j) % len(pks) for j in range(n)]
        m = rand_msg()
        sig = sig_of(sum(sks[j] for j in members) % o.R, m)
        kind = i % 6
        ks = [pks[j] for j in members]
        if kind == 1:
            m = rand_msg()
        elif kind == 2:
            ks = ks + [bytes(47)]
        elif kind == 3:
            ks = []
        calls.append(("fav" if i % 2 else "eth", ks, m, sig))
    calls += [("verify", pks[i], bytes([i]) * 32, sig_of(sks[i], bytes([i]) * 32)) for i in range(8)]
    calls += [("verify", pks[0], bytes(32), b"\x00" * 95)]
    exp = []
    for kind, k, m, s in calls:
        if kind == "verify":
            exp.append(o.verify(k, m, s))
        elif kind == "eth":
            exp.append(o.eth_fast_aggregate_verify(k, m, s))
        else:
            exp.append(o.fast_aggregate_verify(k, m, s))
    got = [None] * len(calls)
    with gbls.BatchingQueue(max_sets=64, max_wait_us=20000) as Q:
        barrier = threading.Barrier(len(calls))

        def run(i):
            kind, k, m, s = calls[i]
            barrier.wait()
            if kind == "verify":
                got[i] = Q.verify(k, m, s)
            else:
                got[i] = Q.fast_aggregate_verify(k, m, s, eth=(kind == "eth"))

        th = [threading.Thread(target=run, args=(i,)) for i in range(len(calls))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        batches, sets = Q.stats()
    assert got == exp
    assert sets == len(calls)
    assert batches < len(calls) // 4  # coalesced


def _fav_sets(sks, pks, n, bad_every=0, rng=None):
    rng = rng or random.Random(5)
    sets = []
    for s in range(n):
        k = rng.randrange(1, 6)
        members = [rng.randrange(len(pks)) for _ in range(k)]
        m = bytes(rng.randrange(256) for _ in range(32))
        sig = sig_of(sum(sks[i] for i in members) % o.R or 1, m)
        if bad_every and s % bad_every == bad_every - 1:
            m = bytes(32) if m != bytes(32) else bytes([1]) * 32  # wrong message
        sets.append(([pks[i] for i in members], m, sig))
    return sets


def test_rlc_batch_check_matches_exact(gbls, keys):
    """SURVEY.md §8f-4 opt-in mode: a passing batch check gives every pairing-decided set
    true; a failing one falls back to the exact per-set path; both equal the exact verdicts."""
    sks, pks = keys
    valid = _fav_sets(sks, pks, 40)
    assert gbls.fast_aggregate_verify_batch(valid, rlc=True) == [("ok", True)] * 40
    mixed = _fav_sets(sks, pks, 40, bad_every=7) + [
        ([], bytes(32), o.INFINITY_SIGNATURE),            # eth: empty + infinity -> true
        ([pks[0]], bytes(32), o.INFINITY_SIGNATURE),      # pairing decides: false
        ([pks[1], pks[1][:40]], bytes(32), valid[0][2]),  # key length error
        ([pks[2]], bytes(32), bytes(96)),                 # NONE signature -> false
    ]
    for eth in (False, True):
        exact = gbls.fast_aggregate_verify_batch(mixed, eth=eth)
        assert gbls.fast_aggregate_verify_batch(mixed, eth=eth, rlc=True) == exact
        assert exact == [(o.eth_fast_aggregate_verify if eth else o.fast_aggregate_verify)(*s) for s in mixed]
    # single invalid set among many valid ones: the fallback must still find it
    one_bad = valid[:20] + [(valid[20][0], bytes([9]) * 32, valid[20][2])] + valid[21:]
    got = gbls.fast_aggregate_verify_batch(one_bad, rlc=True)
    assert got == [("ok", True)] * 20 + [("ok", False)] + [("ok", True)] * 19


def test_one_lane_cold_fav_path():
    """The cold-epoch verdict kernel (one lane per set over projective key sums with the
    precomputed signature-side Miller value, taken by large cold batches) on small
    invalid/edge cases, forced in a child process: MBLS_G2_CRITICAL_KEYS=0 sends the small
    batches down the cold path and MBLS_DEFER_VERDICT=0 launches their verdicts in the one-lane
    form at once (deferred, the synchronize would pick the lane-group form); the child asserts
    through the per-form launch counters that the one-lane kernel decided them."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MBLS_G2_CRITICAL_KEYS="0", MBLS_DEFER_VERDICT="0", MBLS_EXPECT_FORM="1l")
    r = subprocess.run([sys.executable, "-m", "tests._onelane_child"], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


@pytest.mark.parametrize("forms", [{"MBLS_LG16": "0", "MBLS_LG16_PREP": "0"}, {"MBLS_LG16": "1", "MBLS_LG16_PREP": "1"},
                                   {"MBLS_LG16": "1", "MBLS_LAT_SPLIT": "0"},
                                   {"MBLS_LG16": "0", "MBLS_LG16_PREP": "0", "MBLS_LG6_CHAIN": "1"},
                                   {"MBLS_LG16": "1", "MBLS_LG6_CHAIN": "1"},
                                   {"MBLS_LG16": "0", "MBLS_LG16_PREP": "0", "MBLS_LAT_SPLIT": "0", "MBLS_LG6": "0"},
                                   {"MBLS_LG16": "0", "MBLS_LG16_PREP": "0", "MBLS_LAT_SPLIT": "0"}],
                         ids=["8-lane", "16-lane", "16-lane-fused-prep", "8-lane-chain-6-lane", "6-lane-prep-16-lane",
                              "8-lane-verdict-padded", "8-lane-verdict-6-lane"])
def test_lane_group_forms(forms):
    """The latency path taken by small cold batches -- by default the split chain (signature
    chain on one stream; H(m) then the key-side Miller loop on another; a final product +
    final exponentiation kernel), with MBLS_LAT_SPLIT=0 the r02 fused prep + one verdict kernel --
    in the 8-lane and in the 16-lane group form (one Fp component per lane), each forced in a
    child process on the edge-case sets of tests/_onelane_child.py, vs the oracle; the child also
    compares the device path with the host batch API and checks the form counters.  The 8-lane
    verdict kernels run on 6-lane groups by default (mbls_k_lg6.hip, ten sets per wave), on
    padded 8-lane groups with MBLS_LG6=0; MBLS_LG6_CHAIN=1 moves the prep, key-side Miller loop
    and final kernel to 6-lane groups too (the 16-lane kernels then read the 6-lane prep's
    signature-side values, whose pad slots it writes as zero)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # the 8-lane form runs on 6-lane groups (its own counter, r05) in the fused verdict unless
    # MBLS_LG6=0, and in the split chain's final kernel only under MBLS_LG6_CHAIN=1
    six = forms.get("MBLS_LG6_CHAIN") == "1" or (forms.get("MBLS_LAT_SPLIT") == "0" and forms.get("MBLS_LG6") != "0")
    want = "lg16" if forms["MBLS_LG16"] == "1" else "lg6" if six else "lg8"
    env = dict(os.environ, **forms, MBLS_EXPECT_FORM=want)
    r = subprocess.run([sys.executable, "-m", "tests._onelane_child"], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


@pytest.mark.parametrize("lanes", ["8", "16", "32"])
def test_aggregate_lane_groups(lanes):
    """The per-set key sums with narrower lane groups (mbls_k_g1_aggregate / _idx: 64 / L sets per
    wave, the default only for batches of >= 2,048 sets) forced onto the edge-case sets of
    tests/_onelane_child.py -- ragged sets of 0..8 keys, an undecodable key, a sum at infinity --
    through the cold device path, the host batch API and the pubkey table, vs the oracle."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MBLS_AGG_LANES=lanes, MBLS_AGG_LANES_IDX=lanes)
    r = subprocess.run([sys.executable, "-m", "tests._onelane_child"], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


def test_multi_engine_split_and_pipelining():
    """Two engines in one process (mbls_init_devices with the box's one GPU listed twice):
    layer-1 batches split by key count over both, concurrent pipelined callers, the indexed
    batch over both engines' tables and the two-worker batching queue, all vs the C oracle
    (tests/_multi_engine_child.py, a fresh process)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", "-m", "tests._multi_engine_child"], cwd=root, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]


def test_caller_stream_join_then_copy():
    """verdicts written on the engine's G2 streams are visible to work the caller
    enqueues after mbls_dev_stream_wait_engine, and to mbls_dev_memcpy_d2h right away."""
    import numpy as np

    from lambda_ethereum_consensus_amd import device as D

    sks = [RNG.randrange(1, o.R) for _ in range(4)]
    pks = [o.sk_to_pk(s) for s in sks]
    n = 64
    msgs = [rand_msg() for _ in range(n)]
    sig = [sig_of(sum(sks) % o.R, m) for m in msgs]
    keyb = b"".join(pks) * n
    offs = np.arange(0, 4 * n + 1, 4, dtype=np.uint32)
    s = D.Stream()
    st = D.Buffer(4 * n)
    bad = bytearray(b"".join(msgs))
    bad[32 * 5] ^= 1
    D.fast_aggregate_verify(D.Buffer.from_host(keyb), D.Buffer.from_host(offs), D.Buffer.from_host(bytes(bad)),
                            D.Buffer.from_host(b"".join(sig)), st, n, stream=s)
    D.stream_wait_engine(s)
    got = st.to_numpy(np.int32).tolist()  # memcpy_d2h synchronises the engine first
    assert got == [1] * 5 + [0] + [1] * (n - 6)
