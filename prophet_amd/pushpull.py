"""End-to-end push_pull of whole gradient tensors over the GPU-resident PS server.

The worker side of byteps/common/operations.cc and the server side of
byteps/server/server.cc, with an in-process transport:

* ``declare`` — every worker registers its tensors in the same order; the
  position is the tensor's declared key (BytePSGlobal's declared-tensor list);
* ``init_tensor`` — ``InitTensor`` (operations.cc:219-316): the key list is
  ``(declared_key << 16) + i`` for the partitions of ``size`` bytes under the
  partition bound (global.cc:128-135, aligned down to 8 * local_size), and
  each partition is pushed once, blocking — the store's init round and the
  workers' global barrier (operations.cc:301-302);
* ``push_pull`` — ``EnqueueTensor`` (operations.cc:138-217) with
  ``PartitionTensor`` (:99-136): the tensor is cut into the same partitions,
  each one is pushed under its key and pulled back, and the aggregate lands at
  its offset of the output — optionally in the order the Prophet PUSH
  scheduler releases partitions (scheduled_queue.cc:217-296,
  ``prophet_amd.prophet.ProphetPushQueue``);
* ``push_pull(average=True)``, ``push_pull_async`` / ``poll`` /
  ``synchronize`` and ``broadcast`` (push_pull with zeros on the non-root
  ranks) — the byteps/torch API shapes (ops.py, __init__.py:244-272);
* the server front end decodes the request word like ``BytePSHandler``
  (``DepairDataHandleType``, server.h:77-88, of ``GetCommandType``'s Cantor
  pairing, common.cc:99-102) and hands the bytes to ``PSServer``.

Buffers may be host (numpy / CPU tensors) or device tensors; every byte of
arithmetic is the server's HIP fold.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field

from .buckets import (DEFAULT_PARTITION_BYTES, cantor_command, depair_command,
                      local_size_from_env, partition_bound, partition_bytes_from_env)
from .dtypes import DType, elem_size

K_DEFAULT_PUSH_PULL = 0     # RequestType::kDefaultPushPull (common.h:68-71)


class ServerFrontend:
    """The handler in front of the GPU-resident server: decodes the request
    word, checks one key per request (server.cc:150-171) and forwards."""

    def __init__(self, server, size: int | None = None):
        self.server = server
        cfg = getattr(server, "cfg", None)
        self.size = size if size is not None else (cfg.num_workers if cfg is not None else None)

    def push(self, cmd: int, key: int, worker: int, data, nbytes: int) -> None:
        req, dtype = depair_command(cmd)
        if req != K_DEFAULT_PUSH_PULL:       # server.cc:151 CHECK_EQ(type.requestType, ...)
            raise ValueError(f"request type {req} is not kDefaultPushPull")
        self.server.push(key, worker, data, dtype, nbytes=nbytes)

    def pull(self, key: int, out, nbytes: int) -> None:
        self.server.pull(key, out, nbytes=nbytes)


@dataclass
class Context:
    """BPSContext (common.h): one declared tensor's keys and partitions."""
    name: str
    declared_key: int
    size: int = 0
    dtype: int = 0
    key_list: list = field(default_factory=list)
    parts: list = field(default_factory=list)      # (key, offset, len) in bytes
    initialized: bool = False
    init_lock: threading.Lock = field(default_factory=threading.Lock)


class Worker:
    """One BytePS worker (its root device) talking to the server front end."""

    def __init__(self, rank: int, frontend: ServerFrontend,
                 partition_bytes: int | None = None, local_size: int | None = None):
        """``partition_bytes`` / ``local_size`` default to the reference's
        environment: BYTEPS_PARTITION_BYTES (global.cc:128-130, else 4,096,000)
        and BYTEPS_LOCAL_SIZE (communicator.cc:71-77, else 1); the bound is
        AlignTo(partition_bytes, 8 * local_size), rounded down (global.cc:135)."""
        self.rank = rank
        self.frontend = frontend
        if partition_bytes is None:
            partition_bytes = partition_bytes_from_env()
        if local_size is None:
            local_size = local_size_from_env()
        if local_size < 1:
            raise ValueError("local_size must be >= 1")
        self.bound = partition_bound(partition_bytes, local_size)
        if self.bound <= 0:
            raise ValueError(f"partition bound must be positive (BYTEPS_PARTITION_BYTES="
                             f"{partition_bytes}, local_size={local_size})")
        self.contexts: dict[str, Context] = {}
        self._declared: list[str] = []
        self._pool = None
        self._handles: dict[int, tuple] = {}
        self._next_handle = 0

    # ------------------------------------------------------------ declare/init
    def declare(self, name: str) -> int:
        """Register a tensor; its position is its declared key."""
        if name not in self.contexts:
            self.contexts[name] = Context(name, len(self._declared))
            self._declared.append(name)
        return self.contexts[name].declared_key

    def _partition(self, size: int):
        """PartitionTensor (operations.cc:99-136): [offset, len) under the bound."""
        out, acc = [], 0
        while acc < size:
            ln = min(self.bound, size - acc)
            out.append((acc, ln))
            acc += ln
        return out

    def init_tensor(self, name: str, data, dtype: int) -> Context:
        """InitTensor (operations.cc:219-316): keys, then one blocking init push
        per partition (every worker's init push of a key returns only once all
        of them arrived: the global barrier)."""
        self.declare(name)
        ctx = self.contexts[name]
        size = _nbytes(data)
        with ctx.init_lock:
            if ctx.initialized:
                return ctx
            if size <= 0:
                raise ValueError("init tensor size not larger than 0")      # operations.cc:229
            ctx.size, ctx.dtype = size, int(dtype)
            start = ctx.declared_key << 16
            ctx.parts = [(start + i, off, ln) for i, (off, ln) in enumerate(self._partition(size))]
            ctx.key_list = [k for k, _, _ in ctx.parts]
            assert len(ctx.key_list) == (size + self.bound - 1) // self.bound   # :257-259
            cmd = cantor_command(K_DEFAULT_PUSH_PULL, ctx.dtype)
            for key, off, ln in ctx.parts:
                self.frontend.push(cmd, key, self.rank, _slice(data, off, ln), ln)
            ctx.initialized = True
        return ctx

    # ---------------------------------------------------------------- push_pull
    def push_pull(self, name: str, tensor, output=None, order=None,
                  average: bool = False) -> None:
        """EnqueueTensor + the PUSH/PULL stages for one tensor: push every
        partition (in ``order`` — a list of partition indices — if given), then
        pull every partition into ``output`` (default: ``tensor`` itself, in
        place, as byteps_push_pull does).  ``average``: divide the sum by the
        number of workers afterwards, as byteps/torch's push_pull(average=True)
        does (floating dtypes only)."""
        ctx = self.contexts[name]
        if not ctx.initialized:
            raise RuntimeError(f"{name}: init_tensor first")
        if _nbytes(tensor) != ctx.size:
            raise ValueError(f"{name}: {_nbytes(tensor)} bytes, declared {ctx.size}")
        out = tensor if output is None else output
        if _nbytes(out) != ctx.size:
            raise ValueError(f"{name}: output tensor size does not match")   # operations.cc:151
        cmd = cantor_command(K_DEFAULT_PUSH_PULL, ctx.dtype)
        idx = range(len(ctx.parts)) if order is None else order
        for i in idx:
            key, off, ln = ctx.parts[i]
            self.frontend.push(cmd, key, self.rank, _slice(tensor, off, ln), ln)
        for key, off, ln in ctx.parts:
            self.frontend.pull(key, _slice(out, off, ln), ln)
        if average:
            size = getattr(self.frontend, "size", None)
            if not size:
                raise ValueError("average: the frontend does not know the worker count")
            _divide_(out, size)

    # byteps/torch/ops.py: push_pull_async -> handle, poll(handle),
    # synchronize(handle).  Calls run in call order on the worker's own
    # thread (BytePS's loops also take a worker's tensors one after another).
    def push_pull_async(self, name: str, tensor, output=None, average: bool = False) -> int:
        from concurrent.futures import ThreadPoolExecutor
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"bps{self.rank}")
        out = tensor if output is None else output
        fut = self._pool.submit(self.push_pull, name, tensor, out, None, average)
        self._next_handle += 1
        self._handles[self._next_handle] = (fut, out)
        return self._next_handle

    def poll(self, handle: int) -> bool:
        return self._handles[handle][0].done()

    def synchronize(self, handle: int):
        """Wait for the push_pull and return its output (errors re-raised)."""
        fut, out = self._handles.pop(handle)
        fut.result()
        return out

    def close(self) -> None:
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None

    def broadcast(self, name: str, tensor, root_rank: int, output=None):
        """Broadcast as BytePS does it (byteps/torch/__init__.py:264-272: "push +
        pull ... the non-root tensors all 0", no averaging): the root pushes its
        tensor, every other rank pushes zeros, everyone pulls the sum into
        ``output`` (a new buffer like ``tensor`` if not given; the source is
        left untouched, as test_mxnet.py:116-158 requires).  The tensor must
        have been through ``init_tensor``."""
        src = tensor if self.rank == root_rank else _zeros_like(tensor)
        out = _zeros_like(tensor) if output is None else output
        self.push_pull(name, src, output=out)
        return out

    def push_pull_iteration(self, tensors: dict, scheduler=None) -> list:
        """One training iteration: every declared tensor, gradients arriving in
        backward order (highest declared index first).  With a Prophet
        ``scheduler`` (``ProphetPushQueue``) the partitions are pushed in the
        groups it releases; then every partition is pulled back in place.
        Returns the release groups as lists of (declared key, partition)."""
        from .prophet import PushTask, release_groups
        ctxs = [self.contexts[n] for n in self._declared if n in tensors]
        arrivals = []
        for c in sorted(ctxs, key=lambda c: -c.declared_key):
            for i, (key, off, ln) in enumerate(c.parts):
                arrivals.append(PushTask(c.declared_key, i, ln, len(c.parts), key))
        if scheduler is None:
            groups = [arrivals]
        else:
            scheduler.reset()
            groups = release_groups(scheduler, arrivals)
        by_key = {c.declared_key: c for c in ctxs}
        for g in groups:
            for t in g:
                c = by_key[t.grad]
                key, off, ln = c.parts[t.part]
                self.frontend.push(cantor_command(K_DEFAULT_PUSH_PULL, c.dtype), key, self.rank,
                                   _slice(tensors[c.name], off, ln), ln)
        for c in ctxs:
            for key, off, ln in c.parts:
                self.frontend.pull(key, _slice(tensors[c.name], off, ln), ln)
        return [[(t.grad, t.part) for t in g] for g in groups]


def _nbytes(x) -> int:
    if hasattr(x, "nbytes") and not hasattr(x, "data_ptr"):
        return int(x.nbytes)                               # numpy
    return int(x.numel() * x.element_size())               # torch


def _divide_(x, size: int) -> None:
    """In-place x /= size for a floating tensor or array."""
    if hasattr(x, "data_ptr"):                             # torch
        if not x.is_floating_point():
            raise ValueError("average needs a floating dtype")
        x.div_(size)
        return
    import numpy as np
    if not np.issubdtype(x.dtype, np.floating):
        raise ValueError("average needs a floating dtype")
    x /= size


def _zeros_like(x):
    if hasattr(x, "data_ptr"):                             # torch
        import torch
        return torch.zeros_like(x)
    import numpy as np
    return np.zeros_like(x)


def _slice(x, off: int, ln: int):
    """Byte range [off, off+ln) of a contiguous buffer, as a view of the same
    kind (pulls write through it, so a copy would lose the result)."""
    if hasattr(x, "data_ptr"):                             # torch
        import torch
        if not x.is_contiguous():
            raise ValueError("push_pull needs contiguous tensors")
        return x.reshape(-1).view(torch.uint8)[off:off + ln]
    import numpy as np
    if not x.flags["C_CONTIGUOUS"]:
        raise ValueError("push_pull needs contiguous arrays")
    return x.reshape(-1).view(np.uint8)[off:off + ln]


__all__ = ["ServerFrontend", "Worker", "Context", "K_DEFAULT_PUSH_PULL", "DType", "elem_size"]
