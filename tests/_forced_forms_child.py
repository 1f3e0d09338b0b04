"""Child process of tests/test_gpu_forced_forms.py (GPU): one scenario per run, chosen by
MBLS_SCENARIO, with the engine knobs of the parent's parametrisation in the environment.

* table_epoch -- tests/test_gpu_baseline_shapes.py::test_table_epoch_one_lane_prep (2,048-set
  table calls: the pipelined warm form) with the per-path counters on; MBLS_EXPECT_FORM /
  MBLS_EXPECT_PATHS pin the form EVERY call took (exact counts over its two calls).
* verify -- two Bls.verify device batches (invalid keys / signatures / messages mixed in) vs
  the C oracle, path counters pinned the same way.
* overwrite -- two engines (the box's GPU listed twice): a call enqueued on engine 0, then
  from the same thread after mbls_dev_select(1) its key buffer is overwritten through
  mbls_dev_memcpy_h2d (and, on a second call, through the stream-ordered
  mbls_dev_memcpy_h2d_async); the verdicts must be those of the ORIGINAL keys (the
  drain covers every engine, not the caller's).
Prints OK on success."""
import ctypes
import os
import random
import sys

import numpy as np

from tests import _onelane_child as oc
from tests import coracle


def read_paths(D):
    forms = {k: D.prof_read(k)[1] for k in oc.FORMS}
    paths = {k: D.prof_read(k)[1] for k in oc.PATHS}
    return forms, paths


def table_epoch(D):
    from tests import test_gpu_baseline_shapes as T

    D.prof_enable(True)
    D.prof_reset()
    T.test_table_epoch_one_lane_prep(D)
    forms, paths = read_paths(D)
    D.prof_enable(False)
    oc.check_forms(forms, paths, calls=2)
    print("forms", forms, "paths", paths)


def verify(D):
    from oracle import bls12_381 as o
    from tests import test_gpu_baseline_shapes as T

    rng = random.Random(41)
    n = 256
    _, pks = T.keygen(D, n, 41, b"forced-verify")
    import bench

    sk, s0 = bench.sks_for(n, 41, 0, b"forced-verify")
    msgs = [T.msg_of(i, b"forced-verify") for i in range(n)]
    sigs = T.sign_scalars(D, [s0 + i for i in range(n)], msgs)
    pks = pks.copy()
    pks[3] = np.frombuffer(T.not_in_g1(rng), np.uint8)
    pks[4] = np.frombuffer(o.INFINITY_PUBKEY, np.uint8)
    sigs[5] = np.zeros(96, np.uint8)
    sigs[6] = np.frombuffer(T.not_in_g2(rng), np.uint8)
    msgs[7] = T.msg_of(7, b"wrong")
    pk_b, m_b, s_b = pks.reshape(-1).tobytes(), b"".join(msgs), sigs.reshape(-1).tobytes()
    exp = coracle.verify_batch(pk_b, m_b, s_b)
    assert (exp == 1).sum() == n - 5, exp[:10]
    bufs = [D.Buffer.from_host(x) for x in (pk_b, m_b, s_b)]
    sts = [D.Buffer(4 * n) for _ in range(2)]
    D.prof_enable(True)
    D.prof_reset()
    for st in sts:
        D.verify(*bufs, st, n)
    D.synchronize()
    forms, paths = read_paths(D)
    D.prof_enable(False)
    for st in sts:
        assert st.to_numpy(np.int32).tolist() == exp.tolist()
    oc.check_forms(forms, paths, calls=2)
    print("forms", forms, "paths", paths)


def overwrite(D):
    from tests import test_gpu_baseline_shapes as T

    assert D.init_devices([0, 0]) == 2
    D.select(0)
    n_sets, kps = 96, 512
    s0, keys = T.keygen(D, n_sets * kps, 7, b"overwrite")
    off = np.arange(0, n_sets * kps + 1, kps, dtype=np.uint32)
    msgs = [T.msg_of(i, b"overwrite") for i in range(n_sets)]
    sigs = T.sign_scalars(D, [sum(s0 + j for j in range(s * kps, (s + 1) * kps)) % T.R for s in range(n_sets)], msgs)
    msgs[9] = T.msg_of(9, b"wrong")
    pk_b, m_b, s_b = keys.reshape(-1).tobytes(), b"".join(msgs), sigs.reshape(-1).tobytes()
    exp = coracle.fav_batch(pk_b, off, m_b, s_b).tolist()
    assert exp.count(1) == n_sets - 1 and exp[9] == 0
    junk = np.random.default_rng(5).integers(0, 256, size=len(pk_b), dtype=np.uint8)
    for mode in ("sync", "async"):
        D.select(0)
        d_pk, d_off, d_m, d_s = (D.Buffer.from_host(x) for x in (pk_b, off, m_b, s_b))
        st = D.Buffer(4 * (len(off) - 1))
        D.fast_aggregate_verify(d_pk, d_off, d_m, d_s, st, len(off) - 1)
        D.select(1)  # another engine of the process overwrites engine 0's input right away
        if mode == "sync":
            from lambda_ethereum_consensus_amd.device import _check, _fns

            _check(_fns().mbls_dev_memcpy_h2d(d_pk.ptr, junk.ctypes.data, junk.nbytes))
        else:
            keep = d_pk.write_async(junk)
        D.select(0)
        D.synchronize()
        D.select(1)
        D.synchronize()
        got = st.to_numpy(np.int32).tolist()
        assert got == exp, (mode, [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e][:8])
        assert d_pk.to_numpy().tobytes() == junk.tobytes()  # and the overwrite did land
        if mode == "async":
            del keep
    print("overwrite ok")


def table_overwrite(D):
    """The deferred G2 side of a pipelined table call (> 1,024 sets) reads the caller's
    signatures and messages when it launches: overwritten right away from another engine --
    synchronously and stream-ordered -- the verdicts must still be those of the original bytes."""
    from tests import test_gpu_baseline_shapes as T

    assert D.init_devices([0, 0]) == 2
    D.select(0)
    n_tab, n_sets, kps = 4096, 2048, 4
    s0, keys = T.keygen(D, n_tab, 11, b"tab-overwrite")
    D.pk_table_set(0, D.Buffer.from_host(keys.reshape(-1).tobytes()), n_tab)
    rng = np.random.default_rng(11)
    idx = rng.integers(0, n_tab, size=(n_sets, kps)).astype(np.uint32)
    ioff = np.arange(0, n_sets * kps + 1, kps, dtype=np.uint32)
    msgs = [T.msg_of(i, b"tab-overwrite") for i in range(n_sets)]
    sigs = T.sign_scalars(D, [int(sum(s0 + int(j) for j in row)) % T.R or 1 for row in idx], msgs)
    msgs[21] = T.msg_of(21, b"wrong")
    m_b, s_b = b"".join(msgs), sigs.reshape(-1).tobytes()
    exp = [1] * n_sets
    exp[21] = 0
    junk = np.random.default_rng(6).integers(0, 256, size=len(s_b), dtype=np.uint8)
    for mode in ("sync", "async"):
        D.select(0)
        d_idx, d_off, d_m, d_s = (D.Buffer.from_host(x) for x in (idx.reshape(-1), ioff, m_b, s_b))
        st = D.Buffer(4 * n_sets)
        D.prof_enable(True)
        D.prof_reset()
        D.fast_aggregate_verify_indexed(d_idx, d_off, d_m, d_s, st, n_sets)
        D.select(1)  # another engine overwrites the signatures the deferred prep has not read yet
        if mode == "sync":
            from lambda_ethereum_consensus_amd.device import _check, _fns

            _check(_fns().mbls_dev_memcpy_h2d(d_s.ptr, junk.ctypes.data, junk.nbytes))
        else:
            keep = d_s.write_async(junk)
        D.select(0)
        D.synchronize()
        deferred = D.prof_read("path_warm_defer")[1]
        D.prof_enable(False)
        D.select(1)
        D.synchronize()
        D.select(0)
        got = st.to_numpy(np.int32).tolist()
        assert deferred == 1, deferred  # the call did take the deferred path
        assert got == exp, (mode, [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e][:8])
        assert d_s.to_numpy().tobytes() == junk.tobytes()
        if mode == "async":
            del keep
    print("table overwrite ok")


def defer_error(D):
    """ADVICE r04 (medium / low): one engine's failed deferred launch stays that engine's -- the
    other engine's uploads, reads and frees succeed, the failing engine's synchronize reports it
    once -- and a status buffer written by engine 0's DEFERRED verdict reads back correctly from a
    thread that selected engine 1 (mbls_dev_memcpy_d2h drains every engine).  Run with
    MBLS_G2_CRITICAL_KEYS=0, so the small cold call takes the one-lane path whose verdict defers."""
    from lambda_ethereum_consensus_amd import _lib
    from lambda_ethereum_consensus_amd.device import _check, _fns
    from tests import test_gpu_baseline_shapes as T

    lib = _lib.load()
    assert D.init_devices([0, 0]) == 2
    D.select(0)
    buf = D.Buffer(64)
    data = np.arange(16, dtype=np.uint32)
    assert lib.mbls_debug_fail_deferred(1, -100) == 0
    _check(_fns().mbls_dev_memcpy_h2d(buf.ptr, data.ctypes.data, data.nbytes))  # engine 0: unaffected
    assert buf.to_numpy(np.uint32).tolist() == data.tolist()
    tmp = D.Buffer(64)
    tmp.free()
    D.select(1)
    assert _fns().mbls_dev_synchronize(None) == -100  # reported once, to its own engine
    assert _fns().mbls_dev_synchronize(None) == 0
    # a failed deferred launch of the CALLER's engine is recorded as MBLS_ERR_DEVICE,
    # the same code as a failed drain; the upload and the free must still take effect, and the
    # code is returned after them, once.
    D.select(0)
    data2 = np.arange(100, 116, dtype=np.uint32)
    assert lib.mbls_debug_fail_deferred(0, _lib.MBLS_ERR_DEVICE) == 0
    assert _fns().mbls_dev_memcpy_h2d(buf.ptr, data2.ctypes.data, data2.nbytes) == _lib.MBLS_ERR_DEVICE
    assert _fns().mbls_dev_synchronize(None) == 0  # consumed by the copy
    assert buf.to_numpy(np.uint32).tolist() == data2.tolist()  # ... which still took effect
    with open("/proc/self/maps") as f:  # the HIP runtime libmbls already mapped
        hip_path = next(ln.split()[-1] for ln in f if "libamdhip64.so" in ln)
    hip = ctypes.CDLL(hip_path)
    free_b, total_b = ctypes.c_size_t(), ctypes.c_size_t()
    big = D.Buffer(1 << 30)
    D.synchronize()
    assert hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)) == 0
    before = free_b.value
    assert lib.mbls_debug_fail_deferred(0, _lib.MBLS_ERR_DEVICE) == 0
    assert _fns().mbls_dev_free(big.ptr) == _lib.MBLS_ERR_DEVICE
    big.ptr = None
    assert hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)) == 0
    assert free_b.value >= before + (1 << 30) - (64 << 20), (before, free_b.value)  # freed
    assert _fns().mbls_dev_synchronize(None) == 0
    # a deferred verdict of engine 0 read back from engine 1's thread
    D.select(0)
    n_sets, kps = 64, 8
    s0, keys = T.keygen(D, n_sets * kps, 13, b"defer-err")
    off = np.arange(0, n_sets * kps + 1, kps, dtype=np.uint32)
    msgs = [T.msg_of(i, b"defer-err") for i in range(n_sets)]
    sigs = T.sign_scalars(D, [sum(s0 + j for j in range(s * kps, (s + 1) * kps)) % T.R for s in range(n_sets)], msgs)
    msgs[5] = T.msg_of(5, b"wrong")
    pk_b, m_b, s_b = keys.reshape(-1).tobytes(), b"".join(msgs), sigs.reshape(-1).tobytes()
    exp = coracle.fav_batch(pk_b, off, m_b, s_b).tolist()
    assert exp.count(1) == n_sets - 1
    d_pk, d_off, d_m, d_s = (D.Buffer.from_host(x) for x in (pk_b, off, m_b, s_b))
    st = D.Buffer(4 * n_sets)
    D.prof_enable(True)
    D.prof_reset()
    D.fast_aggregate_verify(d_pk, d_off, d_m, d_s, st, n_sets)
    D.select(1)
    got = st.to_numpy(np.int32).tolist()  # d2h from engine 1's thread: engine 0's verdict lands first
    D.select(0)
    D.synchronize()
    one_lane = D.prof_read("path_prep_1l_cold")[1]
    D.prof_enable(False)
    assert one_lane == 1, one_lane  # the call did take the deferred one-lane path
    assert got == exp, [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e][:8]
    print("defer error ok")


def av(D):
    """aggregate_verify through the device entry (dev_av) in the form the environment selects --
    one lane per pair couple (default) or grouped joint Miller loops (MBLS_AV_FORM=grouped) -- on sets
    whose pair counts cut groups of four every way (0, 1, 3, 4, 5, 7, 8, 16, 17 pairs), with an
    invalid key first / mid / last, NONE / infinity / not-in-G2 / undecodable signatures, a wrong
    message and a repeated message, every verdict vs the C oracle, the path counter pinned
    (MBLS_EXPECT_PATHS)."""
    from oracle import bls12_381 as o
    from tests import test_gpu_baseline_shapes as T

    rng = random.Random(43)
    sizes = [1, 3, 4, 5, 7, 8, 16, 17, 0, 2, 16, 16, 16, 16, 16, 1, 9]
    n_pairs = sum(sizes)
    s0, pks = T.keygen(D, n_pairs, 43, b"forced-av")
    msgs = [T.msg_of(i, b"forced-av") for i in range(n_pairs)]
    sig1 = T.sign_scalars(D, [s0 + i for i in range(n_pairs)], msgs)
    off = np.cumsum([0] + sizes).astype(np.uint32)
    n_sets = len(sizes)
    d_sig, ast = D.Buffer(96 * n_sets), D.Buffer(4 * n_sets)
    D.aggregate_signatures(D.Buffer.from_host(sig1.reshape(-1).tobytes()), D.Buffer.from_host(off), d_sig, ast, n_sets)
    D.synchronize()
    sigs = d_sig.to_numpy().reshape(n_sets, 96).copy()
    pks = pks.copy()
    pks[off[10]] = np.frombuffer(T.not_in_g1(rng), np.uint8)           # first key of set 10
    pks[off[11] + 8] = np.frombuffer(o.INFINITY_PUBKEY, np.uint8)      # mid
    pks[off[12] + 15] = np.frombuffer(T.x_ge_p(), np.uint8)            # last
    sigs[13] = np.zeros(96, np.uint8)                                  # NONE
    sigs[14] = np.frombuffer(T.not_in_g2(rng), np.uint8)
    sigs[15] = np.frombuffer(o.INFINITY_SIGNATURE, np.uint8)           # one pair, infinity signature
    sigs[8] = np.frombuffer(o.INFINITY_SIGNATURE, np.uint8)            # empty set
    sigs[9][0] &= 0x7F                                                 # undecodable
    msgs[off[6] + 7] = T.msg_of(1, b"other")                           # wrong message in a 16-pair set
    msgs[off[16] + 2] = msgs[off[16] + 1]                              # repeated message, wrong signature
    pk_b, m_b, s_b = pks.reshape(-1).tobytes(), b"".join(msgs), sigs.reshape(-1).tobytes()
    exp = coracle.av_batch(pk_b, m_b, off, s_b).tolist()
    assert exp[:6] == [1] * 6 and exp[7] == 1 and exp[8] == 0 and exp[6] == 0, exp
    st = D.Buffer(4 * n_sets)
    D.prof_enable(True)
    D.prof_reset()
    D.aggregate_verify(D.Buffer.from_host(pk_b), D.Buffer.from_host(m_b), D.Buffer.from_host(off),
                       D.Buffer.from_host(s_b), st, n_sets)
    D.synchronize()
    _forms, paths = read_paths(D)
    D.prof_enable(False)
    got = st.to_numpy(np.int32).tolist()
    assert got == exp, [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    oc.check_forms({}, paths, calls=1)
    print("av paths", paths)


def av_pipe(D):
    """Three back-to-back aggregate_verify device calls (the r05 cross-call pipeline: each on its
    own FAV stage and G2 stream triple), each with its own inputs, status buffer and injected
    failures, every verdict vs the C oracle; the use-once gate's counters (the calls' two-wave
    H(m) dispatches) are checked against the budget, and with MBLS_USE_ONCE_BUDGET set tight the
    gate must have made later H(m) dispatches wait for earlier ones -- with unchanged verdicts."""
    from oracle import bls12_381 as o
    from tests import test_gpu_baseline_shapes as T

    rng = random.Random(44)
    sizes = [1, 3, 4, 5, 7, 8, 16, 17, 0, 2, 16, 16, 9]
    n_pairs, n_sets = sum(sizes), len(sizes)
    s0, pks = T.keygen(D, n_pairs, 44, b"av-pipe")
    msgs = [T.msg_of(i, b"av-pipe") for i in range(n_pairs)]
    sig1 = T.sign_scalars(D, [s0 + i for i in range(n_pairs)], msgs)
    off = np.cumsum([0] + sizes).astype(np.uint32)
    d_sig, ast = D.Buffer(96 * n_sets), D.Buffer(4 * n_sets)
    D.aggregate_signatures(D.Buffer.from_host(sig1.reshape(-1).tobytes()), D.Buffer.from_host(off), d_sig, ast, n_sets)
    D.synchronize()
    base_sigs = d_sig.to_numpy().reshape(n_sets, 96).copy()
    calls = []
    for c in range(3):
        k, m, g = pks.copy(), list(msgs), base_sigs.copy()
        k[off[6 + c] + 2] = np.frombuffer(T.not_in_g1(rng), np.uint8)  # bad key, a different set per call
        m[off[10] + 3 + c] = T.msg_of(c, b"other")                      # wrong message
        g[(2 + c) % 6] = np.zeros(96, np.uint8)                         # NONE
        g[11 - c] = np.frombuffer(T.not_in_g2(rng), np.uint8)           # not in G2
        if c == 1:
            g[8] = np.frombuffer(o.INFINITY_SIGNATURE, np.uint8)        # empty set, infinity
        pk_b, m_b, s_b = k.reshape(-1).tobytes(), b"".join(m), g.reshape(-1).tobytes()
        exp = coracle.av_batch(pk_b, m_b, off, s_b).tolist()
        assert exp.count(1) <= n_sets - 4, (c, exp)
        calls.append(([D.Buffer.from_host(x) for x in (pk_b, m_b, off, s_b)], D.Buffer(4 * n_sets), exp))
    D.synchronize()
    before = D.scratch_gate_stats()
    D.prof_enable(True)
    D.prof_reset()
    for bufs, st, _ in calls:
        D.aggregate_verify(*bufs, st, n_sets)
    D.synchronize()
    _forms, paths = read_paths(D)
    D.prof_enable(False)
    after = D.scratch_gate_stats()
    for c, (_b, st, exp) in enumerate(calls):
        got = st.to_numpy(np.int32).tolist()
        assert got == exp, (c, [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e])
    oc.check_forms({}, paths, calls=3)
    plan = D.scratch_info()
    admitted = after["admitted"] - before["admitted"]
    waited = after["waited"] - before["waited"]
    assert admitted == 3, (before, after)  # one two-wave H(m) per call
    assert after["peak_live"] <= plan["use_once_budget"], (after, plan)
    min_waits = int(os.environ.get("MBLS_EXPECT_GATE_WAITS", "0"))
    assert waited >= min_waits, (waited, before, after)
    print("av pipe paths", paths, "gate", after, "waited", waited)


def main():
    from lambda_ethereum_consensus_amd import device as D

    sc = os.environ["MBLS_SCENARIO"]
    if sc not in ("overwrite", "table_overwrite", "defer_error"):
        D.init(0)
    {"table_epoch": table_epoch, "verify": verify, "overwrite": overwrite, "table_overwrite": table_overwrite,
     "defer_error": defer_error, "av": av, "av_pipe": av_pipe}[sc](D)
    print("OK")


if __name__ == "__main__":
    sys.exit(main())
