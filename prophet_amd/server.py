"""Python mirror of the GPU-resident PS server (include/bpsr/server.h).

``PSServer`` keeps the request semantics of byteps/server/server.cc
(``BytePSHandler`` for pushes and pulls, engine lanes chosen like
``GetThreadID``) with an in-process transport: ``push(key, worker, data)`` /
``pull(key, out)`` take numpy arrays (host) or torch tensors (host or device).
Worker threads call them concurrently, as ps-lite's receive threads would.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .reducer import ReduceError, _check, load_library

FUSED, INCREMENTAL = 0, 1
HOST, DEVICE = 0, 1

SERVER_EXPORTS = (
    "byteps_server_config_from_env", "byteps_server_create", "byteps_server_create_sized",
    "byteps_server_destroy",
    "byteps_server_init_key", "byteps_server_push", "byteps_server_recv_slot",
    "byteps_server_push_ready", "byteps_server_pull", "byteps_server_pull_host_view",
    "byteps_server_pull_async", "byteps_server_push_async", "byteps_server_key_info",
    "byteps_server_debug_lane", "byteps_server_push_ready_many", "byteps_server_push_many",
    "byteps_server_pull_many", "byteps_server_pull_device_view", "byteps_server_stats",
    "byteps_server_pull_into_async",
    "byteps_server_key_hash", "byteps_server_group_config_from_env", "byteps_server_route",
    "byteps_server_group_create", "byteps_server_group_destroy", "byteps_server_group_route",
    "byteps_server_group_instance", "byteps_server_group_init_key", "byteps_server_group_push",
    "byteps_server_group_pull", "byteps_server_group_push_many", "byteps_server_group_pull_many",
    "byteps_server_order_after", "byteps_server_group_order_after",
    "byteps_server_group_pull_host_view",
)
SPLIT_HASH, SPLIT_RANGE = 0, 1
HASH_FNS = {"djb2": 0, "naive": 1, "sdbm": 2, "built_in": 3}
GROUP_MAX = 16

_vp, _sz, _int, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
# void cb(void* ctx, uint64_t key, const void* data, size_t len, int status)
PULL_CB = ctypes.CFUNCTYPE(None, _vp, _u64, _vp, _sz, _int)
# void cb(void* ctx, uint64_t key, int worker, int status)
PUSH_CB = ctypes.CFUNCTYPE(None, _vp, _u64, _int, _int)


class ServerConfig(ctypes.Structure):
    _fields_ = [("num_workers", _int), ("engine_lanes", _int), ("policy", _int),
                ("async_mode", _int), ("device", _int), ("enable_schedule", _int),
                ("engine_blocking", _int), ("release", _int)]


RELEASE_LAUNCH, RELEASE_DEVICE = 0, 1


class GroupConfig(ctypes.Structure):
    _fields_ = [("server", ServerConfig), ("num_servers", _int), ("devices", _int * 16),
                ("split", _int), ("hash_fn", _int), ("hash_coef", ctypes.c_uint32),
                ("split_min_bytes", _sz)]


def _lib():
    L = load_library()
    if not getattr(L, "_server_bound", False):
        P = ctypes.POINTER
        L.byteps_server_key_hash.argtypes = [_u64, _int, ctypes.c_uint32]
        L.byteps_server_key_hash.restype = _u64
        L.byteps_server_group_config_from_env.argtypes = [P(GroupConfig)]
        L.byteps_server_group_create.argtypes = [P(GroupConfig), P(_vp)]
        L.byteps_server_group_destroy.argtypes = [_vp]
        L.byteps_server_group_route.argtypes = [_vp, _u64, _sz, P(_int), P(_int), P(_sz), P(_sz),
                                                _int]
        L.byteps_server_route.argtypes = [P(GroupConfig), _u64, _sz, P(_int), P(_int), P(_sz),
                                          P(_sz), _int]
        L.byteps_server_group_instance.argtypes = [_vp, _int, P(_vp)]
        L.byteps_server_group_init_key.argtypes = [_vp, _u64, _sz, _int]
        L.byteps_server_group_push.argtypes = [_vp, _u64, _int, _vp, _sz, _int, _int]
        L.byteps_server_group_pull.argtypes = [_vp, _u64, _vp, _sz, _int]
        L.byteps_server_group_pull_host_view.argtypes = [_vp, _u64, ctypes.POINTER(_vp),
                                                         ctypes.POINTER(_sz)]
        L.byteps_server_group_push_many.argtypes = [_vp, P(_u64), P(_vp), P(_sz), _int, _int, _int,
                                                    _int]
        L.byteps_server_group_pull_many.argtypes = [_vp, P(_u64), P(_vp), P(_sz), _int, _int]
        L.byteps_server_order_after.argtypes = [_vp, P(_u64), _int, _vp]
        L.byteps_server_group_order_after.argtypes = [_vp, P(_u64), _int, _vp]
        L.byteps_server_config_from_env.argtypes = [ctypes.POINTER(ServerConfig)]
        L.byteps_server_create.argtypes = [ctypes.POINTER(ServerConfig), ctypes.POINTER(_vp)]
        L.byteps_server_destroy.argtypes = [_vp]
        L.byteps_server_init_key.argtypes = [_vp, _u64, _sz, _int]
        L.byteps_server_push.argtypes = [_vp, _u64, _int, _vp, _sz, _int, _int]
        L.byteps_server_recv_slot.argtypes = [_vp, _u64, _int, ctypes.POINTER(_vp)]
        L.byteps_server_push_ready.argtypes = [_vp, _u64, _int]
        L.byteps_server_pull.argtypes = [_vp, _u64, _vp, _sz, _int]
        L.byteps_server_pull_host_view.argtypes = [_vp, _u64, ctypes.POINTER(_vp),
                                                   ctypes.POINTER(_sz)]
        L.byteps_server_pull_device_view.argtypes = [_vp, _u64, ctypes.POINTER(_vp),
                                                     ctypes.POINTER(_sz)]
        L.byteps_server_pull_async.argtypes = [_vp, _u64, PULL_CB, _vp]
        L.byteps_server_pull_into_async.argtypes = [_vp, _u64, _vp, _sz, _int, PULL_CB, _vp]
        L.byteps_server_stats.argtypes = [_vp, ctypes.POINTER(_u64), _int]
        L.byteps_server_push_async.argtypes = [_vp, _u64, _int, _vp, _sz, _int, _int, PUSH_CB,
                                               _vp]
        L.byteps_server_key_info.argtypes = [_vp, _u64, ctypes.POINTER(_u64),
                                             ctypes.POINTER(_int), ctypes.POINTER(_int), _int]
        L.byteps_server_debug_lane.argtypes = [_vp, _int, _int, ctypes.POINTER(_u64), _int,
                                               ctypes.POINTER(_int)]
        L.byteps_server_push_ready_many.argtypes = [_vp, ctypes.POINTER(_u64), _int, _int]
        L.byteps_server_push_many.argtypes = [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_vp),
                                              ctypes.POINTER(_sz), _int, _int, _int, _int]
        L.byteps_server_pull_many.argtypes = [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_vp),
                                              ctypes.POINTER(_sz), _int, _int]
        L._server_bound = True
    return L


def _buf(x):
    """(pointer, nbytes, location) of a numpy array or torch tensor."""
    if isinstance(x, np.ndarray):
        assert x.flags["C_CONTIGUOUS"]
        return x.ctypes.data, x.nbytes, HOST
    if hasattr(x, "data_ptr"):
        loc = DEVICE if x.device.type == "cuda" else HOST
        return int(x.data_ptr()), x.numel() * x.element_size(), loc
    raise TypeError(f"unsupported buffer {type(x)!r}")


def _producer_events(xs) -> list:
    """The server copies and folds on streams of its own: whatever torch
    queued for these device tensors on the calling thread's current stream
    (the kernel that produced a push, a fill of a pull's destination) must run
    first.  Per device with work pending there, an event recorded on that
    stream, for byteps_server_order_after (the server's streams wait on the
    device, the host does not); a stream with nothing pending costs a query.
    Work on other torch streams is the caller's to order."""
    import torch
    seen, evs = set(), []
    for x in xs:
        if not hasattr(x, "data_ptr") or x.device.type != "cuda" or x.device in seen:
            continue
        seen.add(x.device)
        st = torch.cuda.current_stream(x.device)
        if not st.query():
            ev = torch.cuda.Event()
            ev.record(st)
            evs.append(ev)
    return evs


def _order_after(fn, handle, keys, xs) -> None:
    """byteps_server(_group)_order_after(keys, event) for the producer events
    of xs (nothing when no stream has work pending)."""
    evs = _producer_events(xs)
    if not evs:
        return
    n = len(keys)
    arr = (_u64 * max(1, n))(*keys)
    for ev in evs:
        _check(fn(handle, arr, n, ev.cuda_event))


def key_hash(key: int, fn: str = "djb2", coef: int = 1) -> int:
    """The reference's key hash (global.cc:491-523) through the C ABI."""
    return int(_lib().byteps_server_key_hash(key, HASH_FNS[fn], coef))


def make_group_config(num_workers: int, devices, engine_lanes: int = 4, policy: int = FUSED,
                      async_mode: bool = False, enable_schedule: bool = False,
                      engine_blocking: bool = False, split: str = "hash", hash_fn: str = "djb2",
                      hash_coef: int = 1, split_min_bytes: int = 0) -> GroupConfig:
    devices = list(devices)
    c = GroupConfig()
    c.server = ServerConfig(num_workers, engine_lanes, policy, int(async_mode), 0,
                            int(enable_schedule), int(engine_blocking))
    c.num_servers = len(devices)
    for i, d in enumerate(devices[:GROUP_MAX]):
        c.devices[i] = d
    c.split = {"hash": SPLIT_HASH, "range": SPLIT_RANGE}[split]
    c.hash_fn = HASH_FNS[hash_fn]
    c.hash_coef = hash_coef
    c.split_min_bytes = split_min_bytes
    return c


def _pieces(fn, *args) -> list[tuple[int, int, int]]:
    n = _int()
    cap = GROUP_MAX
    srv, off, ln = (_int * cap)(), (_sz * cap)(), (_sz * cap)()
    _check(fn(*args, ctypes.byref(n), srv, off, ln, cap))
    return [(srv[i], int(off[i]), int(ln[i])) for i in range(n.value)]


def route(cfg: GroupConfig, key: int, nbytes: int) -> list[tuple[int, int, int]]:
    """byteps_server_route: [(instance, offset, length)] of a key's pieces."""
    return _pieces(_lib().byteps_server_route, ctypes.byref(cfg), key, nbytes)


def group_config_from_env() -> GroupConfig:
    c = GroupConfig()
    _check(_lib().byteps_server_group_config_from_env(ctypes.byref(c)))
    return c


def config_from_env() -> ServerConfig:
    c = ServerConfig()
    _check(_lib().byteps_server_config_from_env(ctypes.byref(c)))
    return c


class PSServer:
    def __init__(self, num_workers: int, engine_lanes: int = 4, policy: int = FUSED,
                 async_mode: bool = False, device: int = 0, enable_schedule: bool = False,
                 engine_blocking: bool = False, release: int = RELEASE_LAUNCH):
        self.lib = _lib()
        self.cfg = ServerConfig(num_workers, engine_lanes, policy, int(async_mode), device,
                                int(enable_schedule), int(engine_blocking), int(release))
        self.handle = _vp()
        self._pending = {}
        _check(self.lib.byteps_server_create(ctypes.byref(self.cfg), ctypes.byref(self.handle)))

    @classmethod
    def from_env(cls) -> "PSServer":
        """The dedicated server process's server (byteps_server(),
        server.cc:339-400): byteps_server_config_from_env — device releases
        by default (each epoch's first release picks a consumer or lane
        launches, so copied and slot-written rounds mix freely, server.h);
        BPSR_SERVER_RELEASE=launch keeps one launch per round."""
        c = config_from_env()
        return cls(c.num_workers, c.engine_lanes, c.policy, bool(c.async_mode), c.device,
                   bool(c.enable_schedule), bool(c.engine_blocking), c.release)

    def init_key(self, key: int, nbytes: int, dtype: int) -> None:
        _check(self.lib.byteps_server_init_key(self.handle, key, nbytes, int(dtype)))

    def _order(self, keys, xs) -> None:
        _order_after(self.lib.byteps_server_order_after, self.handle, keys, xs)

    def order_after(self, event, keys=()) -> None:
        """byteps_server_order_after: the server's later device work on the
        lanes of ``keys`` (all lanes when empty) runs after ``event`` (a
        torch.cuda.Event or a raw hipEvent_t)."""
        n = len(keys)
        ev = getattr(event, "cuda_event", event)
        _check(self.lib.byteps_server_order_after(self.handle, (_u64 * max(1, n))(*keys), n, ev))

    def push(self, key: int, worker: int, data, dtype: int, nbytes: int | None = None) -> None:
        p, n, loc = _buf(data)
        self._order([key], [data])
        _check(self.lib.byteps_server_push(self.handle, key, worker, p,
                                           n if nbytes is None else nbytes, int(dtype), loc))

    def push_async(self, key: int, worker: int, data, dtype: int, callback=None,
                   nbytes: int | None = None) -> None:
        """Non-blocking push (byteps_server_push_async): returns once the copy is
        queued and the arrival recorded; ``callback(key, worker, status)`` runs on
        the responder thread when ``data`` may be reused.  ``data`` is kept
        alive until then."""
        p, n, loc = _buf(data)
        self._order([key], [data])

        def tramp(_ctx, k, w, status):
            try:
                if callback is not None:
                    callback(int(k), int(w), int(status))
            finally:
                self._pending.pop(token, None)
        cfn = PUSH_CB(tramp)
        token = id(cfn)
        self._pending[token] = (cfn, data)
        rc = self.lib.byteps_server_push_async(self.handle, key, worker, p,
                                               n if nbytes is None else nbytes, int(dtype),
                                               loc, cfn, None)
        if rc != 0:
            self._pending.pop(token, None)
        _check(rc)

    def recv_slot(self, key: int, worker: int) -> int:
        out = _vp()
        _check(self.lib.byteps_server_recv_slot(self.handle, key, worker, ctypes.byref(out)))
        return int(out.value)

    def push_ready(self, key: int, worker: int) -> None:
        _check(self.lib.byteps_server_push_ready(self.handle, key, worker))

    def pull(self, key: int, out, nbytes: int | None = None) -> None:
        p, n, loc = _buf(out)
        self._order([key], [out])
        _check(self.lib.byteps_server_pull(self.handle, key, p, n if nbytes is None else nbytes,
                                           loc))

    def pull_view(self, key: int) -> memoryview:
        """Zero-copy pull response (server.cc:42-70): a read-only memoryview of
        the pinned host mirror the server fills with one D2H per round.  Valid
        until this worker's next pull of the key returns (sync mode), or for the
        next num_workers pulls of the key (async mode)."""
        p, n = _vp(), _sz()
        _check(self.lib.byteps_server_pull_host_view(self.handle, key, ctypes.byref(p),
                                                     ctypes.byref(n)))
        buf = (ctypes.c_char * n.value).from_address(p.value)
        return memoryview(buf).cast("B").toreadonly()

    def pull_device_view(self, key: int) -> tuple[int, int]:
        """Zero-copy pull from HBM (byteps_server_pull_device_view): blocks until
        the round is finished and folded, counts the pull, and returns
        ``(device_pointer, nbytes)`` of the key's store — what a GPUDirect
        transport would send from.  Sync mode only; valid until this worker's
        next push of the key; read-only."""
        p, n = _vp(), _sz()
        _check(self.lib.byteps_server_pull_device_view(self.handle, key, ctypes.byref(p),
                                                       ctypes.byref(n)))
        return int(p.value), int(n.value)

    def pull_async(self, key: int, callback) -> None:
        """Non-blocking pull (byteps_server_pull_async; server.cc:286-305 queues
        it until the round finishes).  ``callback(key, view, status)`` runs on the
        server's responder thread with ``view`` a read-only memoryview of the
        round's host mirror (None unless status == 0); the pull is counted
        toward the key's re-arm just before the callback runs."""
        def tramp(_ctx, k, data, n, status):
            try:
                view = None
                if status == 0:
                    view = memoryview((ctypes.c_char * n).from_address(data)).cast("B") \
                        .toreadonly()
                callback(int(k), view, int(status))
            finally:
                self._pending.pop(token, None)
        cfn = PULL_CB(tramp)
        token = id(cfn)
        self._pending[token] = cfn          # keep the thunk alive until it ran
        rc = self.lib.byteps_server_pull_async(self.handle, key, cfn, None)
        if rc != 0:
            self._pending.pop(token, None)
        _check(rc)

    def pull_into_async(self, key: int, out, callback=None, nbytes: int | None = None) -> None:
        """Non-blocking pull into a device tensor (byteps_server_pull_into_async):
        the lane's issuer copies the finished round into ``out`` (batched with
        the other pulls that piled up); ``callback(key, status)`` runs on the
        responder thread once the bytes are there.  ``out`` is kept alive until
        then.  Work torch queued on ``out`` on the current stream (a fill, a
        kernel still reading it) is ordered before the copy."""
        p, n, loc = _buf(out)
        self._order([key], [out])

        def tramp(_ctx, k, _data, _n, status):
            try:
                if callback is not None:
                    callback(int(k), int(status))
            finally:
                self._pending.pop(token, None)
        cfn = PULL_CB(tramp)
        token = id(cfn)
        self._pending[token] = (cfn, out)
        rc = self.lib.byteps_server_pull_into_async(self.handle, key, p,
                                                    n if nbytes is None else nbytes, loc,
                                                    cfn, None)
        if rc != 0:
            self._pending.pop(token, None)
        _check(rc)

    def key_info(self, key: int):
        rounds, lane = _u64(), _int()
        order = (_int * self.cfg.num_workers)()
        _check(self.lib.byteps_server_key_info(self.handle, key, ctypes.byref(rounds),
                                               ctypes.byref(lane), order, self.cfg.num_workers))
        return int(rounds.value), int(lane.value), list(order)

    def stats(self) -> dict:
        """Launch telemetry since create (byteps_server_stats)."""
        out = (_u64 * 14)()
        _check(self.lib.byteps_server_stats(self.handle, out, 14))
        return {"fold_launches": out[0], "rounds_folded": out[1], "pull_launches": out[2],
                "pulls": out[3], "issuer_ns": out[4], "push_copy_launches": out[5],
                "consumer_launches": out[6], "key_releases": out[7],
                "service_pulls": out[8], "service_launches": out[9],
                "service_pushes": out[10], "consumers_retired": out[11],
                "epochs_closed": out[12], "lane_epochs": out[13]}

    # batched calls (server.h): one lane-wide launch for many keys
    def push_ready_many(self, keys, worker: int) -> None:
        arr = (_u64 * len(keys))(*keys)
        _check(self.lib.byteps_server_push_ready_many(self.handle, arr, len(keys), worker))

    def push_many(self, keys, worker: int, datas, dtype: int) -> None:
        bufs = [_buf(d) for d in datas]
        locs = {loc for _, _, loc in bufs}
        if len(locs) > 1:
            raise ValueError("push_many: all sources host, or all device")
        self._order(keys, datas)
        n = len(keys)
        _check(self.lib.byteps_server_push_many(
            self.handle, (_u64 * n)(*keys), (_vp * n)(*[p for p, _, _ in bufs]),
            (_sz * n)(*[b for _, b, _ in bufs]), n, worker, int(dtype), locs.pop() if n else 0))

    def pull_many(self, keys, outs) -> None:
        bufs = [_buf(o) for o in outs]
        locs = {loc for _, _, loc in bufs}
        if len(locs) > 1:
            raise ValueError("pull_many: all destinations host, or all device")
        self._order(keys, outs)
        n = len(keys)
        _check(self.lib.byteps_server_pull_many(
            self.handle, (_u64 * n)(*keys), (_vp * n)(*[p for p, _, _ in bufs]),
            (_sz * n)(*[b for _, b, _ in bufs]), n, locs.pop() if n else 0))

    def debug_lane(self, lane: int, pause: int = -1, max_log: int = 4096) -> list[int]:
        """Scheduling test hook (byteps_server_debug_lane): pause (1) / release
        (0) the lane's engine queue; returns the keys it issued so far, in order."""
        keys = (_u64 * max_log)()
        n = _int()
        _check(self.lib.byteps_server_debug_lane(self.handle, lane, pause, keys, max_log,
                                                 ctypes.byref(n)))
        return [int(keys[i]) for i in range(min(n.value, max_log))]

    def close(self) -> None:
        if self.handle and getattr(self, "_owned", True):
            self.lib.byteps_server_destroy(self.handle)
        self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class PSServerGroup:
    """The key space over several server instances (byteps_server_group_*,
    include/bpsr/server.h): whole keys by the reference's key hash
    (``split="hash"``), or large keys cut into per-instance owner ranges
    (``split="range"``).  Same push / pull / batched calls as PSServer."""

    def __init__(self, num_workers: int, devices, engine_lanes: int = 4, policy: int = FUSED,
                 async_mode: bool = False, enable_schedule: bool = False,
                 engine_blocking: bool = False, split: str = "hash", hash_fn: str = "djb2",
                 hash_coef: int = 1, split_min_bytes: int = 0):
        self.lib = _lib()
        c = make_group_config(num_workers, devices, engine_lanes, policy, async_mode,
                              enable_schedule, engine_blocking, split, hash_fn, hash_coef,
                              split_min_bytes)
        self.cfg = c
        self.handle = _vp()
        _check(self.lib.byteps_server_group_create(ctypes.byref(c), ctypes.byref(self.handle)))

    def route(self, key: int, nbytes: int) -> list[tuple[int, int, int]]:
        """[(instance, offset, length)] of the key's pieces."""
        return _pieces(self.lib.byteps_server_group_route, self.handle, key, nbytes)

    def instance(self, i: int) -> "PSServer":
        """Instance i as a non-owning PSServer (views, key_info of pieces)."""
        h = _vp()
        _check(self.lib.byteps_server_group_instance(self.handle, i, ctypes.byref(h)))
        srv = PSServer.__new__(PSServer)
        srv.lib, srv.cfg, srv.handle, srv._pending = self.lib, self.cfg.server, h, {}
        srv._owned = False
        return srv

    def init_key(self, key: int, nbytes: int, dtype: int) -> None:
        _check(self.lib.byteps_server_group_init_key(self.handle, key, nbytes, int(dtype)))

    def _order(self, keys, xs) -> None:
        _order_after(self.lib.byteps_server_group_order_after, self.handle, keys, xs)

    def push(self, key: int, worker: int, data, dtype: int, nbytes: int | None = None) -> None:
        p, n, loc = _buf(data)
        self._order([key], [data])
        _check(self.lib.byteps_server_group_push(self.handle, key, worker, p,
                                                 n if nbytes is None else nbytes, int(dtype), loc))

    def pull(self, key: int, out, nbytes: int | None = None) -> None:
        p, n, loc = _buf(out)
        self._order([key], [out])
        _check(self.lib.byteps_server_group_pull(self.handle, key, p,
                                                 n if nbytes is None else nbytes, loc))

    def pull_view(self, key: int) -> memoryview:
        """Zero-copy pull response of a whole (unsplit) key from the instance
        holding it (byteps_server_group_pull_host_view; PSServer.pull_view's
        validity rules)."""
        p, n = _vp(), _sz()
        _check(self.lib.byteps_server_group_pull_host_view(self.handle, key, ctypes.byref(p),
                                                           ctypes.byref(n)))
        buf = (ctypes.c_char * n.value).from_address(p.value)
        return memoryview(buf).cast("B").toreadonly()

    def push_many(self, keys, worker: int, datas, dtype: int) -> None:
        bufs = [_buf(d) for d in datas]
        locs = {loc for _, _, loc in bufs}
        if len(locs) > 1:
            raise ValueError("push_many: all sources host, or all device")
        self._order(keys, datas)
        n = len(keys)
        _check(self.lib.byteps_server_group_push_many(
            self.handle, (_u64 * n)(*keys), (_vp * n)(*[p for p, _, _ in bufs]),
            (_sz * n)(*[b for _, b, _ in bufs]), n, worker, int(dtype), locs.pop() if n else 0))

    def pull_many(self, keys, outs) -> None:
        bufs = [_buf(o) for o in outs]
        locs = {loc for _, _, loc in bufs}
        if len(locs) > 1:
            raise ValueError("pull_many: all destinations host, or all device")
        self._order(keys, outs)
        n = len(keys)
        _check(self.lib.byteps_server_group_pull_many(
            self.handle, (_u64 * n)(*keys), (_vp * n)(*[p for p, _, _ in bufs]),
            (_sz * n)(*[b for _, b, _ in bufs]), n, locs.pop() if n else 0))

    def close(self) -> None:
        if self.handle:
            self.lib.byteps_server_group_destroy(self.handle)
            self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


__all__ = ["PSServer", "PSServerGroup", "GroupConfig", "key_hash", "group_config_from_env",
           "make_group_config", "route", "ServerConfig", "config_from_env", "FUSED", "INCREMENTAL", "HOST",
           "DEVICE", "ReduceError", "SERVER_EXPORTS"]
