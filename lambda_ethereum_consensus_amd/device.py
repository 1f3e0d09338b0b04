"""Device-resident batch calls (include/mbls.h layer 2) on HBM buffers owned by libmbls.

Device memory, streams and events come from libmbls.so's own HIP runtime
(`mbls_dev_malloc` & co.): PyTorch-ROCm bundles a different libamdhip64, and two HIP
runtimes cannot share a process, so torch is used only for `torch.distributed` (gloo) in
bench.py.  Used by bench.py (inputs already resident in HBM) and the GPU tests.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def _fns():
    lib = _lib.load()
    if not getattr(lib, "_dev_bound", False):
        P, I32, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t
        for name, res, args in (
            ("mbls_dev_device_count", I32, []),
            ("mbls_dev_malloc", P, [SZ]),
            ("mbls_dev_free", I32, [P]),
            ("mbls_dev_memcpy_h2d", I32, [P, P, SZ]),
            ("mbls_dev_memcpy_h2d_async", I32, [P, P, SZ, P]),
            ("mbls_dev_memcpy_d2h", I32, [P, P, SZ]),
            ("mbls_dev_stream_create", P, []),
            ("mbls_dev_stream_destroy", I32, [P]),
            ("mbls_dev_event_create", P, []),
            ("mbls_dev_event_destroy", I32, [P]),
            ("mbls_dev_event_record", I32, [P, P]),
            ("mbls_dev_event_elapsed_ms", ctypes.c_float, [P, P]),
            ("mbls_prof_enable", I32, [I32]),
            ("mbls_prof_reset", I32, []),
            ("mbls_prof_read", I32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]),
        ):
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        lib._dev_bound = True
    return lib


def _check(rc):
    if rc != 0:
        raise RuntimeError("libmbls device call failed: %s" % _lib.status_message(rc))


def init(device: int = 0):
    _check(_fns().mbls_init(device))


def init_devices(devices) -> int:
    """One engine per listed GPU ordinal in this process (include/mbls.h mbls_init_devices):
    layer-1 batches are then split by key count over all of them.  Returns the engine count."""
    devs = [int(d) for d in devices]
    arr = (ctypes.c_int32 * len(devs))(*devs)
    _check(_fns().mbls_init_devices(arr, len(devs)))
    return int(_fns().mbls_engine_count())


def engine_count() -> int:
    return int(_fns().mbls_engine_count())


def select(engine: int):
    """Layer-2 calls of this thread go to engine `engine` (its GPU owns the buffers)."""
    _check(_fns().mbls_dev_select(engine))


def plan_shards(key_counts, parts: int):
    """Contiguous, key-balanced chunks of sets (mbls_plan_shards): list of parts+1 bounds.
    key_counts None = one key per set of len n (pass n as an int)."""
    import numpy as np

    if isinstance(key_counts, int):
        n, off_ptr = key_counts, None
        off = None
    else:
        cnt = np.asarray(key_counts, dtype=np.uint32)
        n = len(cnt)
        off = np.zeros(n + 1, dtype=np.uint32)
        np.cumsum(cnt, out=off[1:])
        off_ptr = off.ctypes.data
    b = np.zeros(parts + 1, dtype=np.uint32)
    _check(_lib.load().mbls_plan_shards(off_ptr, n, parts, b.ctypes.data))
    return [int(x) for x in b]


class mbls_scratch_plan_t(ctypes.Structure):
    _fields_ = [("pool_bytes", ctypes.c_uint64), ("retain_default", ctypes.c_uint64),
                ("retain_bytes", ctypes.c_uint64), ("worst_retained", ctypes.c_uint64),
                ("worst_use_once", ctypes.c_uint64), ("queues", ctypes.c_uint32), ("max_frame", ctypes.c_uint32),
                ("max_retained_frame", ctypes.c_uint32), ("safe", ctypes.c_int32), ("applied", ctypes.c_int32),
                ("use_once_budget", ctypes.c_uint64)]


def _plan_dict(p):
    return {f: int(getattr(p, f)) for f, _ in mbls_scratch_plan_t._fields_}


def scratch_plan(pool_bytes: int, retain_default: int, queues: int, cus: int, frames, gated=None) -> dict:
    """The engine's scratch plan for given runtime limits and kernel frames (include/mbls.h
    mbls_scratch_plan; host-only, no GPU needed).  `gated`: one flag per frame, True where the
    engine's use-once gate admits the kernel (None: every frame gated)."""
    lib = _lib.load()
    fr = np.asarray(list(frames), dtype=np.uint32)
    g = None if gated is None else np.asarray([1 if x else 0 for x in gated], dtype=np.uint8)
    if g is not None and len(g) != len(fr):
        raise ValueError("gated needs one flag per frame")
    out = mbls_scratch_plan_t()
    _check(lib.mbls_scratch_plan(ctypes.c_uint64(pool_bytes), ctypes.c_uint64(retain_default), queues, cus,
                                 fr.ctypes.data if len(fr) else None,
                                 g.ctypes.data if g is not None and len(g) else None, len(fr), ctypes.byref(out)))
    return _plan_dict(out)


def scratch_info() -> dict:
    """The plan the calling thread's engine runs with (mbls_scratch_info)."""
    out = mbls_scratch_plan_t()
    _check(_lib.load().mbls_scratch_info(ctypes.byref(out)))
    return _plan_dict(out)


def scratch_kernels() -> list:
    """Kernels whose frames the engine prices (mbls_scratch_kernel)."""
    lib, out, i = _lib.load(), [], 0
    while True:
        n = lib.mbls_scratch_kernel(i)
        if not n:
            return out
        out.append(n.decode())
        i += 1


def scratch_gated_kernels() -> list:
    """Kernels whose every dispatch passes the engine's use-once gate (mbls_scratch_kernel_gated)."""
    lib = _lib.load()
    return [k for i, k in enumerate(scratch_kernels()) if lib.mbls_scratch_kernel_gated(i) == 1]


def scratch_gate_stats() -> dict:
    """The use-once gate of the calling thread's device (mbls_scratch_gate_stats)."""
    out = (ctypes.c_uint64 * 3)()
    _check(_lib.load().mbls_scratch_gate_stats(out))
    return {"admitted": int(out[0]), "waited": int(out[1]), "peak_live": int(out[2])}


def shutdown():
    _lib.load().mbls_shutdown()


def device_count() -> int:
    return int(_fns().mbls_dev_device_count())


class Buffer:
    """A device allocation with host<->device copies (bytes / numpy)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = _fns().mbls_dev_malloc(max(self.nbytes, 1))
        if not self.ptr:
            raise MemoryError("mbls_dev_malloc(%d) failed" % self.nbytes)

    @classmethod
    def from_host(cls, data) -> "Buffer":
        arr = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data)
        b = cls(arr.nbytes)
        if arr.nbytes:
            _check(_fns().mbls_dev_memcpy_h2d(b.ptr, arr.ctypes.data, arr.nbytes))
        return b

    def write_async(self, data, stream: "Stream" = None, offset: int = 0):
        """Stream-ordered overwrite (mbls_dev_memcpy_h2d_async): after every engine's work so far,
        no host drain.  Returns the host array, which must stay alive until `stream` completes."""
        arr = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data)
        if offset < 0 or offset + arr.nbytes > self.nbytes:
            raise ValueError("write past the buffer")
        if arr.nbytes:
            _check(_fns().mbls_dev_memcpy_h2d_async(self.ptr + offset, arr.ctypes.data, arr.nbytes, _h(stream)))
        return arr

    def to_numpy(self, dtype=np.uint8, count=None) -> np.ndarray:
        dt = np.dtype(dtype)
        n = self.nbytes // dt.itemsize if count is None else count
        out = np.empty(n, dtype=dt)
        if out.nbytes:
            _check(_fns().mbls_dev_memcpy_d2h(out.ctypes.data, self.ptr, out.nbytes))
        return out

    def free(self):
        if self.ptr:
            _fns().mbls_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self):
        self.handle = _fns().mbls_dev_stream_create()
        if not self.handle:
            raise RuntimeError("stream creation failed")

    def synchronize(self):
        _check(_fns().mbls_dev_synchronize(self.handle))


class Event:
    def __init__(self):
        self.handle = _fns().mbls_dev_event_create()

    def record(self, stream: "Stream" = None):
        _check(_fns().mbls_dev_event_record(self.handle, stream.handle if stream else None))

    def elapsed_ms(self, stop: "Event") -> float:
        return float(_fns().mbls_dev_event_elapsed_ms(self.handle, stop.handle))


def synchronize(stream: "Stream" = None):
    _check(_fns().mbls_dev_synchronize(stream.handle if stream else None))


def stream_wait_engine(stream: "Stream" = None):
    """Device-side join: `stream` waits for all work the engine has enqueued so far."""
    _check(_fns().mbls_dev_stream_wait_engine(stream.handle if stream else None))


def _h(stream):
    return stream.handle if stream is not None else None


FAV_ETH, FAV_RLC = 1, 2  # include/mbls.h MBLS_FAV_*


def _fav_flags(eth, rlc):
    return (FAV_ETH if eth else 0) | (FAV_RLC if rlc else 0)


def fast_aggregate_verify(pks48: Buffer, key_off: Buffer, msgs32: Buffer, sigs96: Buffer, status: Buffer,
                          n_sets: int, eth: bool = False, stream: Stream = None, rlc: bool = False):
    _check(_fns().mbls_dev_fast_aggregate_verify(pks48.ptr, key_off.ptr, pks48.nbytes // 48, msgs32.ptr, sigs96.ptr,
                                                 n_sets, _fav_flags(eth, rlc), status.ptr, _h(stream)))


def verify(pks48: Buffer, msgs32: Buffer, sigs96: Buffer, status: Buffer, n_sets: int, stream: Stream = None):
    _check(_fns().mbls_dev_verify(pks48.ptr, msgs32.ptr, sigs96.ptr, n_sets, status.ptr, _h(stream)))


def aggregate_verify(pks48: Buffer, msgs32: Buffer, key_off: Buffer, sigs96: Buffer, status: Buffer, n_sets: int,
                     stream: Stream = None):
    _check(_fns().mbls_dev_aggregate_verify(pks48.ptr, msgs32.ptr, key_off.ptr, pks48.nbytes // 48, sigs96.ptr, n_sets,
                                            status.ptr, _h(stream)))


def aggregate_pubkeys(pks48: Buffer, key_off: Buffer, out48: Buffer, status: Buffer, n_sets: int,
                      stream: Stream = None):
    _check(_fns().mbls_dev_aggregate_pubkeys(pks48.ptr, key_off.ptr, pks48.nbytes // 48, n_sets, out48.ptr, status.ptr,
                                             _h(stream)))


def aggregate_signatures(sigs96: Buffer, off: Buffer, out96: Buffer, status: Buffer, n_sets: int,
                         stream: Stream = None):
    _check(_fns().mbls_dev_aggregate_signatures(sigs96.ptr, off.ptr, sigs96.nbytes // 96, n_sets, out96.ptr,
                                                status.ptr, _h(stream)))


# multi-GPU validator-table build: RCCL communicator of the job
def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(_fns().mbls_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return buf.raw


def comm_init(unique_id: bytes, rank: int, world: int):
    if len(unique_id) != 128:
        raise ValueError("RCCL unique id is 128 bytes")
    _check(_fns().mbls_comm_init(unique_id, rank, world))


def comm_destroy():
    _check(_fns().mbls_comm_destroy())


def pk_table_set_sharded(pks48: Buffer, n: int, status: Buffer = None):
    """Every rank passes the same n keys; each validates 1/world of them, one RCCL all-gather
    replicates the rows (the local build when no communicator is set)."""
    _check(_fns().mbls_dev_pk_table_set_sharded(pks48.ptr, n, status.ptr if status else None, None))


# SSZ signing roots; domain_stride 0 = one shared domain, 32 = per object
def hash_tree_root_chunks(chunks32: Buffer, leaves: int, n: int, out32: Buffer, stream: Stream = None):
    _check(_fns().mbls_dev_hash_tree_root_chunks(chunks32.ptr, leaves, n, out32.ptr, _h(stream)))


def signing_roots(roots32: Buffer, domains32: Buffer, n: int, out32: Buffer, per_object_domain: bool = True,
                  stream: Stream = None):
    _check(_fns().mbls_dev_signing_roots(roots32.ptr, domains32.ptr, 32 if per_object_domain else 0, n, out32.ptr,
                                         _h(stream)))


def attestation_data_signing_roots(data128: Buffer, domains32: Buffer, n: int, out32: Buffer,
                                   per_object_domain: bool = True, stream: Stream = None):
    _check(_fns().mbls_dev_attestation_data_signing_roots(data128.ptr, domains32.ptr, 32 if per_object_domain else 0,
                                                          n, out32.ptr, _h(stream)))


def validate_pubkeys(pks48: Buffer, status: Buffer, stream: Stream = None):
    _check(_fns().mbls_dev_validate_pubkeys(pks48.ptr, pks48.nbytes // 48, status.ptr, _h(stream)))


def sk_to_pk(sk32: Buffer, out48: Buffer, n: int, stream: Stream = None):
    _check(_fns().mbls_dev_sk_to_pk(sk32.ptr, n, out48.ptr, _h(stream)))


def sign(sk32: Buffer, msgs32: Buffer, out96: Buffer, n: int, stream: Stream = None):
    _check(_fns().mbls_dev_sign(sk32.ptr, msgs32.ptr, n, out96.ptr, _h(stream)))


# ----- validator pubkey table ------------------------------------------
def pk_table_set(first: int, pks48: Buffer, n: int, status: Buffer = None):
    """Decode + KeyValidate n device-resident keys into table rows first..first+n-1 (sync)."""
    _check(_fns().mbls_dev_pk_table_set(first, pks48.ptr, n, status.ptr if status else None, None))


def fast_aggregate_verify_indexed(idx: Buffer, idx_off: Buffer, msgs32: Buffer, sigs96: Buffer, status: Buffer,
                                  n_sets: int, eth: bool = False, stream: Stream = None, rlc: bool = False):
    _check(_fns().mbls_dev_fast_aggregate_verify_indexed(idx.ptr, idx_off.ptr, idx.nbytes // 4, msgs32.ptr, sigs96.ptr,
                                                         n_sets, _fav_flags(eth, rlc), status.ptr, _h(stream)))


def aggregate_pubkeys_indexed(idx: Buffer, idx_off: Buffer, out48: Buffer, status: Buffer, n_sets: int,
                              stream: Stream = None):
    _check(_fns().mbls_dev_aggregate_pubkeys_indexed(idx.ptr, idx_off.ptr, idx.nbytes // 4, n_sets, out48.ptr,
                                                     status.ptr, _h(stream)))


# ----- per-kernel timing ------------------------------------------------------------------
def prof_enable(on: bool = True):
    _fns().mbls_prof_enable(1 if on else 0)


def prof_reset():
    _fns().mbls_prof_reset()


def prof_read(kernel: str):
    ms = ctypes.c_double(0)
    n = ctypes.c_uint64(0)
    _check(_fns().mbls_prof_read(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value
