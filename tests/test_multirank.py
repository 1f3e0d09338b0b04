"""CPU: the N>1 bench path with world_size 2 over gloo (no GPU): per-rank inputs differ
(independent shards, no data-path collective) and the timed region is reduced with MAX."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import hashlib

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    elapsed, ok = bench.reduce_over_ranks(dist, 1.0 + rank, rank != 1 or True)
    # the per-rank key seed used by make_inputs: distinct per rank
    tag = (3).to_bytes(4, "big") + rank.to_bytes(4, "big")
    seed = hashlib.sha256(b"mbls-bench-sk" + tag).hexdigest()
    _, bad = bench.reduce_over_ranks(dist, 0.0, rank == 0)
    q.put((rank, elapsed, ok, bad, seed))
    dist.destroy_process_group()


def test_two_rank_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == [2.0, 2.0]  # max over ranks
    assert all(r[2] for r in res)
    assert [r[3] for r in res] == [False, False]  # one rank failing fails the job
    assert res[0][4] != res[1][4]  # independent per-rank shards


class _FakeComm:
    """Records the libmbls communicator calls bench.comm_setup makes (no GPU here)."""

    def __init__(self, rank):
        self.rank, self.calls = rank, []

    def comm_unique_id(self):
        assert self.rank == 0, "only rank 0 makes the RCCL id"
        return bytes(range(128))

    def comm_init(self, uid, rank, world):
        self.calls.append((uid, rank, world))


def _comm_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    fake = _FakeComm(rank)
    bench.comm_setup(fake, dist)
    q.put((rank, fake.calls))
    dist.destroy_process_group()


def test_sharded_table_comm_setup_two_ranks():
    """The sharded table build's RCCL id exchange: every rank joins with rank
    0's id, its own rank and the world size."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, [(bytes(range(128)), 0, 2)]), (1, [(bytes(range(128)), 1, 2)])]
