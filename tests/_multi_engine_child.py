"""Child process of test_gpu_parity.test_multi_engine_split_and_pipelining (a fresh process:
mbls_init_devices must come before any other engine call).

Two engines on the one GPU of the box (a repeated ordinal, include/mbls.h mbls_init_devices)
exercise the in-process split of layer-1 batches (contiguous key-balanced chunks, one host
thread per engine) and concurrent, pipelined layer-1 callers; every outcome is compared with
the C oracle (tests/coracle.py)."""
import os
import random
import sys
import threading

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MBLS_HW_QUEUES", "10")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from lambda_ethereum_consensus_amd import bls, device as D  # noqa: E402
from oracle import bls12_381 as o  # noqa: E402
from tests import coracle  # noqa: E402
from tests.test_gpu_baseline_shapes import keygen, msg_of, not_in_g1, sign_scalars  # noqa: E402


def main():
    assert D.init_devices([0, 0]) == 2
    assert D.init_devices([0, 0]) == 2  # idempotent for the same list
    rng = random.Random(8)
    kps, n_sets = 512, 192
    s0, pks = keygen(D, n_sets * kps, 8, b"multi")
    keys = [bytes(k) for k in pks]
    sets = []
    scal = []
    for s in range(n_sets):
        sets.append([keys[s * kps:(s + 1) * kps], msg_of(s, b"me"), None])
        scal.append(sum(s0 + s * kps + j for j in range(kps)) % o.R)
    sg = sign_scalars(D, scal, [x[1] for x in sets])
    for s in range(n_sets):
        sets[s][2] = bytes(sg[s])
    sets[10][0] = sets[10][0][:200] + [not_in_g1(rng)] + sets[10][0][201:]
    sets[150][1] = msg_of(1, b"wrong")
    sets[100][0] = sets[100][0][:70] + [sets[100][0][70][:47]] + sets[100][0][71:]
    sets = [tuple(x) for x in sets]
    exp = [coracle.outcome(c, s[0], [s[1]]) for c, s in zip(coracle.fav_codes(sets), sets)]
    # one call, split over the two engines (cost 192 x 528 > the split threshold)
    b = D.plan_shards([len(x[0]) for x in sets], 2)
    assert 0 < b[1] < n_sets
    assert bls.fast_aggregate_verify_batch(sets) == exp
    assert sum(1 for e in exp if e == ("ok", True)) == n_sets - 3
    # concurrent layer-1 callers (pipelined: the engine lock is released while they wait)
    out = [None] * 6
    chunks = [sets[i * 32:(i + 1) * 32] for i in range(6)]

    def run(i):
        out[i] = bls.fast_aggregate_verify_batch(chunks[i], eth=(i % 2 == 1))

    th = [threading.Thread(target=run, args=(i,)) for i in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i in range(6):
        want = [coracle.outcome(c, s[0], [s[1]]) for c, s in zip(coracle.fav_codes(chunks[i], eth=(i % 2 == 1)), chunks[i])]
        assert out[i] == want, i
    # Bls.verify batch split over the engines (one key per set)
    n_v = 4096
    vmsgs = [msg_of(i, b"v") for i in range(n_v)]
    vsig = sign_scalars(D, [s0 + i for i in range(n_v)], vmsgs)
    vsets = [(keys[i], vmsgs[i], bytes(vsig[i])) for i in range(n_v)]
    vsets[7] = (keys[7], vmsgs[8], vsets[7][2])
    got = bls.verify_batch(vsets)
    vexp = coracle.verify_batch(b"".join(x[0] for x in vsets), b"".join(x[1] for x in vsets),
                                b"".join(x[2] for x in vsets))
    assert got == [coracle.outcome(int(c)) for c in vexp]
    assert got.count(("ok", True)) == n_v - 1
    # validator table on both engines + an indexed batch split over them
    t = bls.PubkeyTable()
    t.clear()
    assert t.set(0, keys[:8192]) == [0] * 8192
    isets = []
    for s in range(96):
        idx = [rng.randrange(8192) for _ in range(kps)]
        m = msg_of(s, b"ix")
        isets.append((idx, m))
    isg = sign_scalars(D, [sum(s0 + i for i in x[0]) % o.R for x in isets], [x[1] for x in isets])
    isets = [(x[0], x[1], bytes(g)) for x, g in zip(isets, isg)]
    isets[3] = (isets[3][0][:90] + [9000] + isets[3][0][91:], isets[3][1], isets[3][2])
    got = t.fast_aggregate_verify_batch(isets)
    assert got[3] == ("error", "UnknownValidatorIndex")
    assert got[:3] + got[4:] == [("ok", True)] * 95
    # the batching queue's two workers over two engines
    with bls.BatchingQueue(max_sets=16, max_wait_us=2000) as Q:
        res = [None] * 40

        def q(i):
            res[i] = Q.fast_aggregate_verify(*sets[i])

        th = [threading.Thread(target=q, args=(i,)) for i in range(40)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    assert res == exp[:40]
    D.shutdown()
    print("OK")


if __name__ == "__main__":
    main()
