"""GPU helpers of tests/test_gpu_deferred.py (also run as a child process with
MBLS_DEFER_VERDICT=0): back-to-back cold configs[3] calls whose verdicts take the one-lane
deferred form, every call's status buffer compared with the C oracle.

The headline's steady state (bench.py) is a chain of 2,048 x 512-key cold
mbls_dev_fast_aggregate_verify calls with no synchronize between them: each call's verdict
kernel is launched by the NEXT call, in its one-lane form over projective key sums with the
precomputed signature-side Miller value (csrc/mbls_k_pair.hip mbls_k_fav_verdict with fsig,
engine flush_verdict(more=true)); only the last call's verdict, launched by the synchronize,
takes the lane-group form.  Reference semantics: native/bls_nif/src/lib.rs:84-119.
Prints OK on success when run as a module."""
from __future__ import annotations

import sys

import numpy as np

from tests import coracle

SENTINEL = -77


def _sentinel_status(D, n):
    st = D.Buffer(4 * n)
    fill = np.full(n, SENTINEL, dtype=np.int32)
    D._check(D._fns().mbls_dev_memcpy_h2d(st.ptr, fill.ctypes.data, fill.nbytes))
    return st


def epoch_inputs(D):
    from tests.test_gpu_baseline_shapes import build_epoch

    keys, off, msgs, sigs, expect = build_epoch(D)
    pk_b, s_b, m_b = keys.reshape(-1).tobytes(), sigs.reshape(-1).tobytes(), b"".join(msgs)
    base = {eth: coracle.fav_batch(pk_b, off, m_b, s_b, eth=eth) for eth in (False, True)}
    return pk_b, off, m_b, s_b, base


def oracle_for(pk_b, off, s_b, base, msgs_b, changed, eth):
    """Oracle codes of a batch that differs from the base epoch only in the messages of the
    `changed` sets: the base codes, with those sets re-verified by the oracle."""
    exp = base[eth].copy()
    if len(changed):
        ch = np.asarray(sorted(changed))
        pk = b"".join(pk_b[48 * int(off[p]):48 * int(off[p + 1])] for p in ch)
        cnt = np.array([int(off[p + 1] - off[p]) for p in ch], dtype=np.uint32)
        sub_off = np.zeros(len(ch) + 1, dtype=np.uint32)
        np.cumsum(cnt, out=sub_off[1:])
        m = b"".join(msgs_b[32 * p:32 * p + 32] for p in ch)
        s = b"".join(s_b[96 * p:96 * p + 96] for p in ch)
        exp[ch] = coracle.fav_batch(pk, sub_off, m, s, eth=eth)
    return exp


def variant_messages(m_b, n, call, count):
    """The epoch's messages with `count` call-specific sets given a wrong message."""
    rng = np.random.default_rng(1000 + call)
    pos = sorted(int(p) for p in rng.choice(n, size=count, replace=False))
    m = bytearray(m_b)
    for p in pos:
        m[32 * p + (call % 32)] ^= 0x5A
    return bytes(m), pos


def back_to_back(D, inputs, n_calls=4, defer=True):
    """n_calls cold epoch calls + one trailing call, no synchronize in between, each with its
    own status buffer (filled with a sentinel first) and its own wrong-message sets; call 2 is
    eth_fast_aggregate_verify.  Returns the per-kernel launch counts of the verdict forms."""
    pk_b, off, m_b, s_b, base = inputs
    n = len(off) - 1
    d_pk, d_off, d_s = D.Buffer.from_host(pk_b), D.Buffer.from_host(off), D.Buffer.from_host(s_b)
    calls = []
    for c in range(n_calls + 1):
        m, pos = variant_messages(m_b, n, c, 3 + 2 * c)
        calls.append((D.Buffer.from_host(m), m, pos, c == 2, _sentinel_status(D, n)))
    D.synchronize()
    D.prof_enable(True)
    D.prof_reset()
    for d_m, _m, _pos, eth, st in calls:
        D.fast_aggregate_verify(d_pk, d_off, d_m, d_s, st, n, eth=eth)
    D.synchronize()
    forms = {k: D.prof_read(k)[1] for k in ("fav_verdict", "fav_verdict_1l", "fav_verdict_lg8", "fav_verdict_lg16",
                                            "fav_verdict_lg6")}
    D.prof_enable(False)
    for c, (_d_m, m, pos, eth, st) in enumerate(calls):
        got = st.to_numpy(np.int32)
        exp = oracle_for(pk_b, off, s_b, base, m, pos, eth)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (c, [(int(i), int(got[i]), int(exp[i])) for i in bad[:10]])
        assert (exp[pos] != 1).all()  # every injected wrong message verdicts false (or a key error)
    # the one-lane form decided every call but the last (flushed by the synchronize)
    want_1l = n_calls + 1 if not defer else n_calls
    assert forms["fav_verdict"] == n_calls + 1, forms
    assert forms["fav_verdict_1l"] == want_1l, forms
    if defer:
        assert forms["fav_verdict_lg8"] + forms["fav_verdict_lg16"] + forms["fav_verdict_lg6"] == 1, forms
    for b in (d_pk, d_off, d_s):
        b.free()
    for d_m, *_rest in calls:
        d_m.free()
    return forms


def lifetime(D, inputs):
    """A deferred call whose caller overwrites key_off and frees its inputs right after the
    call returns (mbls_dev_memcpy_h2d / mbls_dev_free launch the verdict and drain first), and
    one whose verdict the next call launches in the one-lane form before the caller frees its
    key_off: both still match the oracle."""
    pk_b, off, m_b, s_b, base = inputs
    n = len(off) - 1
    d_pk, d_s = D.Buffer.from_host(pk_b), D.Buffer.from_host(s_b)
    garbage = np.random.default_rng(5).integers(0, 2 ** 32, size=n + 1, dtype=np.uint32)
    # (1) overwrite + free right after the call
    m1, pos1 = variant_messages(m_b, n, 11, 7)
    d_off1, d_m1, st1 = D.Buffer.from_host(off), D.Buffer.from_host(m1), _sentinel_status(D, n)
    D.fast_aggregate_verify(d_pk, d_off1, d_m1, d_s, st1, n)
    D._check(D._fns().mbls_dev_memcpy_h2d(d_off1.ptr, garbage.ctypes.data, garbage.nbytes))
    d_off1.free()
    d_m1.free()
    D.synchronize()
    got = st1.to_numpy(np.int32)
    exp = oracle_for(pk_b, off, s_b, base, m1, pos1, False)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    # (2) a second call launches the first one's verdict (one lane), then the first call's
    # key_off is overwritten and freed before anything synchronises
    m2, pos2 = variant_messages(m_b, n, 12, 9)
    d_off2, d_m2, st2 = D.Buffer.from_host(off), D.Buffer.from_host(m2), _sentinel_status(D, n)
    d_off3, st3 = D.Buffer.from_host(off), _sentinel_status(D, n)
    d_m3 = D.Buffer.from_host(m_b)
    D.prof_enable(True)
    D.prof_reset()
    D.fast_aggregate_verify(d_pk, d_off2, d_m2, d_s, st2, n)
    D.fast_aggregate_verify(d_pk, d_off3, d_m3, d_s, st3, n)
    D._check(D._fns().mbls_dev_memcpy_h2d(d_off2.ptr, garbage.ctypes.data, garbage.nbytes))
    d_off2.free()
    D.synchronize()
    one_lane = D.prof_read("fav_verdict_1l")[1]
    D.prof_enable(False)
    assert one_lane == 1, one_lane
    got2, got3 = st2.to_numpy(np.int32), st3.to_numpy(np.int32)
    exp2 = oracle_for(pk_b, off, s_b, base, m2, pos2, False)
    assert (got2 == exp2).all(), np.nonzero(got2 != exp2)[0][:10]
    assert (got3 == base[False]).all(), np.nonzero(got3 != base[False])[0][:10]


def main():
    from lambda_ethereum_consensus_amd import device as D

    import os

    D.init(0)
    inputs = epoch_inputs(D)
    forms = back_to_back(D, inputs, defer=os.environ.get("MBLS_DEFER_VERDICT", "1") != "0")
    print("forms", forms)
    print("OK")


if __name__ == "__main__":
    sys.exit(main())
