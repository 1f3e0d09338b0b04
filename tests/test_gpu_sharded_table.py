"""GPU: the RCCL sharded validator-table build -- rows validated per shard and
replicated by the all-gather equal a local build, and committees verified against the sharded
table equal the cold path.  The one-GPU box runs world = 1 (RCCL init + all-gather of one
shard); the world > 1 arithmetic runs on an 8-GPU node via the same child script."""
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_ranks(world):
    with tempfile.TemporaryDirectory() as tmp:
        idf = os.path.join(tmp, "id")
        procs = [subprocess.Popen([sys.executable, "-m", "tests._sharded_child", str(r), str(world), idf,
                                   os.path.join(tmp, f"out{r}")], cwd=ROOT, stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True) for r in range(world)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=180)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        return [p.returncode for p in procs], outs


def test_sharded_table_world1():
    rcs, outs = run_ranks(1)
    assert rcs == [0] and outs[0].strip().endswith("OK"), outs


def test_sharded_table_multi_gpu():
    """world = 2 with one rank per GPU (needs two devices: RCCL refuses two ranks on one GPU)."""
    from lambda_ethereum_consensus_amd import _lib

    if _lib.load().mbls_dev_device_count() < 2:
        pytest.skip("needs two GPUs")
    rcs, outs = run_ranks_on_devices(2)
    assert rcs == [0, 0] and all(o.strip().endswith("OK") for o in outs), outs


def run_ranks_on_devices(world):
    with tempfile.TemporaryDirectory() as tmp:
        idf = os.path.join(tmp, "id")
        procs = [subprocess.Popen([sys.executable, "-m", "tests._sharded_child", str(r), str(world), idf,
                                   os.path.join(tmp, f"out{r}")], cwd=ROOT, env=dict(os.environ, MBLS_TEST_DEVICE=str(r)),
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=180)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        return [p.returncode for p in procs], outs
