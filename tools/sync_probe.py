"""Host-side costs around one mainnet block on the GPU box: enqueue time of the two FAV calls,
the synchronize when the GPU is idle, and the block's device time (engine profiling events)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import bench  # noqa: E402
from lambda_ethereum_consensus_amd import device as D  # noqa: E402

D.init(0)
kps, n_att = 512, 128
d_pks, d_off, d_msgs, d_sigs, msgs, _ = bench.make_inputs(D, n_att + 1, kps, 7, 0)
pk_all, sig_all = d_pks.to_numpy(), d_sigs.to_numpy()
a = [D.Buffer.from_host(pk_all[:48 * kps * n_att]), D.Buffer.from_host(np.arange(0, kps * n_att + 1, kps, dtype=np.uint32)),
     D.Buffer.from_host(msgs[:32 * n_att]), D.Buffer.from_host(sig_all[:96 * n_att])]
b = [D.Buffer.from_host(pk_all[48 * kps * n_att:]), D.Buffer.from_host(np.array([0, kps], dtype=np.uint32)),
     D.Buffer.from_host(msgs[32 * n_att:]), D.Buffer.from_host(sig_all[96 * n_att:])]
st, st_s = D.Buffer(4 * n_att), D.Buffer(4)
for _ in range(3):
    D.fast_aggregate_verify(*a, st, n_att)
    D.fast_aggregate_verify(*b, st_s, 1, eth=True)
    D.synchronize()
t_enq, t_sync, t_idle, t_tot = [], [], [], []
for _ in range(20):
    t0 = time.perf_counter()
    D.fast_aggregate_verify(*a, st, n_att)
    D.fast_aggregate_verify(*b, st_s, 1, eth=True)
    t1 = time.perf_counter()
    D.synchronize()
    t2 = time.perf_counter()
    D.synchronize()
    t3 = time.perf_counter()
    t_enq.append(t1 - t0)
    t_tot.append(t2 - t0)
    t_idle.append(t3 - t2)
print({"enqueue_ms": round(1e3 * float(np.median(t_enq)), 3), "block_ms": round(1e3 * float(np.median(t_tot)), 3),
       "idle_sync_ms": round(1e3 * float(np.median(t_idle)), 3)})
