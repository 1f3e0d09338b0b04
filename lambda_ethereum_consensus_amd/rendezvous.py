"""Host-side rendezvous of the one-process-per-GPU deployment, standard library only.

SURVEY.md §8e: the ranks of a node exchange nothing on the data path; they need a barrier, the
max of a timed region, an AND of verdict checks, a gather of verdict chunks and -- for the
sharded validator-table build -- rank 0's 128-byte RCCL id.  bench.py used torch.distributed
(gloo) for that, but importing torch before libmbls loads maps PyTorch-ROCm's bundled
libamdhip64 / librccl (ROCm 7.0, same sonames as ROCm 7.2's), so libmbls then ran on a HIP
runtime and RCCL that no `-m gpu` test exercises.  This module replaces it
in the ranks' processes: a file-based group in a directory every rank of one launch agrees on
(torch.distributed.run keeps launching the ranks; it stays a separate process).

The group implements the subset of the torch.distributed API the bench uses -- get_rank,
get_world_size, barrier, all_gather_object, broadcast_object_list, destroy_process_group -- so
the callers read the same with either.  Objects travel as JSON (bytes as hex); one node only
(every rank sees the same file system).
"""
from __future__ import annotations

import json
import os
import time
import uuid

DEFAULT_TIMEOUT_S = 600.0


def _enc(o):
    if isinstance(o, (bytes, bytearray)):
        return {"__bytes__": bytes(o).hex()}
    if isinstance(o, (list, tuple)):
        return [_enc(x) for x in o]
    if isinstance(o, dict):
        return {str(k): _enc(v) for k, v in o.items()}
    if hasattr(o, "item") and not isinstance(o, (str, int, float, bool)):  # numpy scalars
        return o.item()
    return o


def _dec(o):
    if isinstance(o, dict):
        if set(o) == {"__bytes__"}:
            return bytes.fromhex(o["__bytes__"])
        return {k: _dec(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_dec(x) for x in o]
    return o


class FileGroup:
    """A group of `world` processes on one node meeting in directory `path`."""

    def __init__(self, rank: int, world: int, path: str, timeout_s: float = DEFAULT_TIMEOUT_S):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world, self.path, self.timeout_s = rank, world, path, timeout_s
        self._op = 0
        os.makedirs(path, exist_ok=True)
        self.gen = self._join()

    # -- generation: files a crashed earlier launch left in the same directory --
    # (MBLS_RDZV_DIR, a launch without torchrun, a reused pid) must never be read as this
    # launch's.  Rank 0 clears the directory and publishes a fresh nonce in `gen`; every other
    # rank joins with the nonce it reads there and a random token of its own (re-joining if `gen`
    # changes under it, i.e. it read a stale one first), rank 0 answers `ready.<nonce>` naming the
    # tokens it collected, a rank proceeds only on a ready marker that names ITS token, and every
    # op file carries the nonce.
    def _join(self) -> str:
        deadline = time.monotonic() + self.timeout_s
        if self.rank == 0:
            for f in os.listdir(self.path):
                try:
                    os.unlink(os.path.join(self.path, f))
                except OSError:
                    pass
            gen = f"{uuid.uuid4().hex}{os.getpid():x}"
            self._write("gen", gen)
            tokens = {}
            while len(tokens) < self.world - 1:
                for r in range(1, self.world):
                    if r not in tokens:
                        t = self._read(f"join.{r}.{gen}")
                        if t is not None:
                            tokens[r] = t
                if time.monotonic() > deadline:
                    raise TimeoutError(f"rendezvous: ranks did not join generation {gen} within {self.timeout_s} s")
                time.sleep(0.0005)
            self._write(f"ready.{gen}", {str(r): t for r, t in tokens.items()})
            return gen
        # a fresh token per process: a ready marker a crashed launch left can never name it
        token = uuid.uuid4().hex
        joined = None
        while True:
            gen = self._read("gen")
            if gen is not None and gen != joined:
                self._write(f"join.{self.rank}.{gen}", token)
                joined = gen
            if joined is not None:
                ready = self._read(f"ready.{joined}")
                if isinstance(ready, dict) and ready.get(str(self.rank)) == token:
                    return joined
            if time.monotonic() > deadline:
                raise TimeoutError(f"rendezvous: rank 0 did not publish a generation within {self.timeout_s} s")
            time.sleep(0.0005)

    def _read(self, name: str):
        try:
            with open(os.path.join(self.path, name)) as f:
                return _dec(json.load(f)["v"])
        except (OSError, ValueError, KeyError):
            return None

    # -- torch.distributed-compatible subset -------------------------------------------
    def get_rank(self) -> int:
        return self.rank

    def get_world_size(self) -> int:
        return self.world

    def barrier(self):
        self._exchange(None)

    def all_gather_object(self, out: list, obj):
        vals = self._exchange(obj)
        for i in range(self.world):
            out[i] = vals[i]

    def broadcast_object_list(self, objs: list, src: int = 0):
        vals = self._exchange(list(objs) if self.rank == src else None)
        objs[:] = vals[src]

    def destroy_process_group(self):
        """Leave the group; the last step removes the directory once every rank has left."""
        self._exchange(None)
        self._write(f"left.{self.gen}.{self.rank}", None)
        if self.rank == 0:
            deadline = time.monotonic() + self.timeout_s
            while not all(os.path.exists(os.path.join(self.path, f"left.{self.gen}.{r}")) for r in range(self.world)):
                if time.monotonic() > deadline:
                    return
                time.sleep(0.002)
            for f in os.listdir(self.path):
                try:
                    os.unlink(os.path.join(self.path, f))
                except OSError:
                    pass
            try:
                os.rmdir(self.path)
            except OSError:
                pass

    # -- helpers -------------------------------------------------------------------------
    def max_and_all(self, value: float, ok: bool):
        """(max of `value` over ranks, AND of `ok` over ranks)."""
        vals = self._exchange([float(value), bool(ok)])
        return max(v[0] for v in vals), all(v[1] for v in vals)

    def _write(self, name: str, obj):
        tmp = os.path.join(self.path, f".{name}.tmp")
        with open(tmp, "w") as f:
            json.dump({"v": _enc(obj)}, f)
        os.replace(tmp, os.path.join(self.path, name))  # atomic: a reader sees all or nothing

    def _exchange(self, obj):
        k = self._op
        self._op += 1
        self._write(f"{self.gen}.{k}.{self.rank}", obj)
        names = [os.path.join(self.path, f"{self.gen}.{k}.{r}") for r in range(self.world)]
        deadline = time.monotonic() + self.timeout_s
        vals = [None] * self.world
        have = [False] * self.world
        while not all(have):
            for r in range(self.world):
                if not have[r] and os.path.exists(names[r]):
                    with open(names[r]) as f:
                        vals[r] = _dec(json.load(f)["v"])
                    have[r] = True
            if all(have):
                break
            if time.monotonic() > deadline:
                missing = [r for r in range(self.world) if not have[r]]
                raise TimeoutError(f"rendezvous op {k}: ranks {missing} did not arrive within {self.timeout_s} s")
            time.sleep(0.0005)
        return vals


def rendezvous_dir(env=None) -> str:
    """The directory every rank of one torch.distributed.run launch derives alike: the launch's
    master address / port and run id, and the launching agent's pid (the ranks' common parent)."""
    env = os.environ if env is None else env
    base = env.get("MBLS_RDZV_DIR") or os.path.join(env.get("TMPDIR", "/tmp"), "mbls_rdzv")
    key = "_".join(str(x) for x in (env.get("MASTER_ADDR", "127.0.0.1"), env.get("MASTER_PORT", "0"),
                                    env.get("TORCHELASTIC_RUN_ID", "none"), os.getppid()))
    return os.path.join(base, key.replace("/", "_").replace(":", "_"))


def init_from_env(rank: int, world: int, env=None, timeout_s: float = DEFAULT_TIMEOUT_S) -> FileGroup:
    return FileGroup(rank, world, rendezvous_dir(env), timeout_s)


def runtime_libraries() -> dict:
    """Every HIP runtime, HSA runtime and RCCL this process has mapped (from /proc/self/maps;
    one path each when the process is sound): every bench line records them, so an N > 1 line
    and the `-m gpu` tests can be seen to run the same runtime."""
    want = {"libamdhip64": set(), "librccl": set(), "libhsa-runtime64": set()}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) < 6:
                    continue
                path = parts[-1]
                base = os.path.basename(path)
                for k in want:
                    if base.startswith(k + ".so"):
                        want[k].add(os.path.realpath(path))
    except OSError:
        pass
    return {k: sorted(v) for k, v in want.items()}
