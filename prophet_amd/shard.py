"""Key-space sharding of the aggregated parameter vector across the GPUs of a node.

Ownership follows the reference's intra-node reduce-scatter split
(byteps/common/core_loops.cc:208-211, 233-247): with ``E`` elements and ``G``
GPUs, ``per = E // G``; GPU ``g`` owns ``[g*per, (g+1)*per)`` and the last GPU
(the reference's NCCL root, nccl_manager.cc:62-64) also owns the
``E - per*G`` tail elements.  A bucket whose byte range crosses an ownership
boundary is split; every piece is reduced by its owner with the same left fold,
so the sharded result is bit-identical to the unsharded one.

Data path (one process per GPU, torch.distributed over RCCL/xGMI):
  * device-resident pushes already on their owner: local fold only, no
    collective (``ShardedReducer.reduce_owned``);
  * pushes that landed on one GPU: grouped point-to-point send/recv moves each
    owner its slice of every worker's bucket (RCCL has no scatter primitive:
    ``dist.batch_isend_irecv``), then the owner folds
    (``ShardedReducer.scatter_reduce``);
  * optional return leg: all-gather of the owned results
    (``ShardedReducer.allgather``, mirrors core_loops.cc:249-254);
  * worker local reduce: every GPU holds a full gradient; each owner receives
    its slice from every GPU and folds them in rank order
    (``ShardedReducer.reduce_scatter`` / ``allreduce``): a deterministic,
    bit-reproducible replacement for ncclReduceScatter + ncclAllGather.

Two transports.  With a :class:`ShardComm` (the C ABI of include/bpsr/shard.h:
RCCL grouped send/recv, or an in-process group of GPUs) every call is ONE
native call — transfers and the HIP fold inside libbpsr.so, the same entry
points a ``core_loops.cc``-shaped C++ caller binds.  Without one, the
transfers are ``torch.distributed`` point-to-point ops (any backend — the CPU
tests run them over gloo with an injected checker fold) and the fold is the
HIP fold through the reduce C ABI.  Both give the same bits: the rank-order
left fold of the same slices.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Callable, Sequence


def owner_ranges(n_elems: int, world: int) -> list[tuple[int, int]]:
    """[start, end) element range owned by each GPU (core_loops.cc:210-211)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    per = n_elems // world
    out = [(g * per, (g + 1) * per) for g in range(world)]
    out[-1] = (out[-1][0], n_elems)   # tail to the last GPU (the NCCL root)
    return out


def owner_of(elem: int, n_elems: int, world: int) -> int:
    per = n_elems // world
    if per == 0:
        return world - 1
    return min(elem // per, world - 1)


@dataclass(frozen=True)
class Piece:
    """Part of a bucket owned by one GPU, in elements."""
    owner: int
    bucket: int
    start: int        # global element index
    length: int       # elements
    bucket_offset: int  # element offset inside the bucket


def split_buckets(bucket_elems: Sequence[int], world: int) -> list[Piece]:
    """Cut consecutive buckets of a flattened vector at ownership boundaries."""
    total = sum(bucket_elems)
    ranges = owner_ranges(total, world)
    pieces, pos = [], 0
    for b, n in enumerate(bucket_elems):
        s, e = pos, pos + n
        for g, (os_, oe) in enumerate(ranges):
            lo, hi = max(s, os_), min(e, oe)
            if lo < hi:
                pieces.append(Piece(g, b, lo, hi - lo, lo - s))
        pos = e
    return pieces


# --------------------------------------------------------------------------
# C ABI (include/bpsr/shard.h)

SHARD_EXPORTS = (
    "byteps_shard_owner_range", "byteps_shard_reduce_root_of", "byteps_shard_get_unique_id",
    "byteps_shard_comm_init", "byteps_shard_comm_wrap", "byteps_shard_comm_init_local",
    "byteps_shard_comm_destroy", "byteps_shard_comm_info", "byteps_shard_reduce_scatter",
    "byteps_shard_allgather", "byteps_shard_scatter_reduce", "byteps_shard_reduce_root",
    "byteps_shard_broadcast", "byteps_shard_rccl_version",
)
UNIQUE_ID_BYTES = 128

_vp, _sz, _int, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64


def _lib():
    from .reducer import load_library
    L = load_library()
    if not getattr(L, "_shard_bound", False):
        P = ctypes.POINTER
        L.byteps_shard_owner_range.argtypes = [_sz, _int, _int, P(_sz), P(_sz)]
        L.byteps_shard_reduce_root_of.argtypes = [_u64, P(_int), _int]
        L.byteps_shard_get_unique_id.argtypes = [_vp]
        L.byteps_shard_comm_init.argtypes = [_vp, _int, _int, _int, P(_vp)]
        L.byteps_shard_comm_wrap.argtypes = [_vp, P(_vp)]
        L.byteps_shard_comm_init_local.argtypes = [_int, P(_int), P(_vp)]
        L.byteps_shard_comm_destroy.argtypes = [_vp]
        L.byteps_shard_comm_info.argtypes = [_vp, P(_int), P(_int), P(_int)]
        L.byteps_shard_reduce_scatter.argtypes = [_vp, _vp, P(_vp), _vp, _sz, _int, _int, _vp]
        L.byteps_shard_allgather.argtypes = [_vp, _vp, _vp, _sz, _int, _vp]
        L.byteps_shard_scatter_reduce.argtypes = [_vp, _int, P(_vp), _int, P(_vp), _vp, _sz,
                                                  _int, _int, _vp]
        L.byteps_shard_reduce_root.argtypes = [_vp, _int, _vp, P(_vp), _vp, _sz, _int, _int, _vp]
        L.byteps_shard_broadcast.argtypes = [_vp, _int, _vp, _sz, _int, _vp]
        L.byteps_shard_rccl_version.argtypes = [P(_int)]
        L._shard_bound = True
    return L


def _check(rc):
    from .reducer import _check as chk
    chk(rc)


def owner_range_native(n_elems: int, world: int, rank: int) -> tuple[int, int]:
    """byteps_shard_owner_range (must equal :func:`owner_ranges`)."""
    lo, hi = _sz(), _sz()
    _check(_lib().byteps_shard_owner_range(n_elems, world, rank, ctypes.byref(lo),
                                           ctypes.byref(hi)))
    return int(lo.value), int(hi.value)


def rccl_version() -> int:
    """byteps_shard_rccl_version: ncclGetVersion of the RCCL the library bound."""
    v = _int()
    _check(_lib().byteps_shard_rccl_version(ctypes.byref(v)))
    return int(v.value)


def reduce_roots_from_env(env=None) -> list[int]:
    """BYTEPS_REDUCE_ROOTS exactly as global.cc:217-229 reads it: ``roots_ss >>
    i`` (skips leading whitespace, optional sign, digits) repeated, ignoring
    one ',' after each number; stops at the first token that is not a number.
    Empty when unset (reduce-scatter mode, IsUsingReduce() false)."""
    v = (os.environ if env is None else env).get("BYTEPS_REDUCE_ROOTS")
    out: list[int] = []
    if not v:
        return out
    i, n = 0, len(v)
    while True:
        while i < n and v[i].isspace():
            i += 1
        j = i
        if j < n and v[j] in "+-":
            j += 1
        k = j
        while k < n and v[k].isdigit():
            k += 1
        if k == j:
            return out
        out.append(int(v[i:k]))
        i = k
        if i < n and v[i] == ",":
            i += 1


def reduce_root_of(key: int, roots: Sequence[int]) -> int:
    """GetReduceRootByKey (global.h:107-108) through the C ABI."""
    arr = (_int * len(roots))(*roots)
    rc = _lib().byteps_shard_reduce_root_of(key, arr, len(roots))
    if rc < 0:
        _check(rc)
    return int(rc)


def _ptr(x) -> int:
    if x is None:
        return 0
    return x if isinstance(x, int) else int(x.data_ptr())


def _ptrs(xs) -> ctypes.Array:
    xs = list(xs)
    return (_vp * max(1, len(xs)))(*[_ptr(x) for x in xs])


def _stream(x, stream):
    from .reducer import _stream_of
    return _stream_of(x, stream)


def _dtype(x, dtype):
    if dtype is not None:
        return int(dtype)
    from .dtypes import from_torch
    return int(from_torch(x.dtype))


class ShardComm:
    """``byteps_shard_comm``: an RCCL communicator (created here, or wrapped)
    or one rank of an in-process group of GPUs.  Methods take torch device
    tensors (or raw device pointers with explicit ``elems``/``dtype``) and run
    on the tensors' current stream unless ``stream`` is given."""

    def __init__(self, handle: int):
        self.lib = _lib()
        self.handle = _vp(handle)
        w, r, d = _int(), _int(), _int()
        _check(self.lib.byteps_shard_comm_info(self.handle, ctypes.byref(w), ctypes.byref(r),
                                               ctypes.byref(d)))
        self.world, self.rank, self.device = w.value, r.value, d.value

    # ------------------------------------------------------------ creation
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        _check(_lib().byteps_shard_get_unique_id(buf))
        return buf.raw

    @classmethod
    def init(cls, uid: bytes, world: int, rank: int, device: int) -> "ShardComm":
        h = _vp()
        _check(_lib().byteps_shard_comm_init(ctypes.create_string_buffer(uid, UNIQUE_ID_BYTES),
                                             world, rank, device, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def from_group(cls, group=None, device: int | None = None) -> "ShardComm":
        """NcclManager::ConstructRings (nccl_manager.cc:74-127): rank 0 makes
        the unique id, the torch.distributed group (any backend) carries it
        to every rank, every rank initialises its RCCL communicator."""
        import torch
        import torch.distributed as dist
        rank = dist.get_rank(group)
        world = dist.get_world_size(group)
        if device is None:
            device = torch.cuda.current_device()
        obj = [cls.unique_id() if rank == 0 else None]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(obj, src=src, group=group)
        return cls.init(obj[0], world, rank, device)

    @classmethod
    def wrap(cls, nccl_comm: int) -> "ShardComm":
        """A caller-owned ncclComm_t (e.g. torch's ``ProcessGroupNCCL._comm_ptr()``)."""
        h = _vp()
        _check(_lib().byteps_shard_comm_wrap(nccl_comm, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def local_group(cls, devices: Sequence[int]) -> list["ShardComm"]:
        """In-process group: one communicator per rank (rank r on devices[r]),
        each to be driven by its own thread."""
        n = len(devices)
        hs = (_vp * n)()
        _check(_lib().byteps_shard_comm_init_local(n, (_int * n)(*devices), hs))
        return [cls(hs[i]) for i in range(n)]

    def close(self) -> None:
        if self.handle:
            h, self.handle = self.handle, _vp()
            _check(self.lib.byteps_shard_comm_destroy(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------- calls
    def owner_range(self, n_elems: int) -> tuple[int, int]:
        return owner_range_native(n_elems, self.world, self.rank)

    def reduce_scatter(self, local, recv_slots, dst, elems: int | None = None, dtype=None,
                       mode: int = 0, stream=None) -> None:
        """byteps_shard_reduce_scatter: ``dst`` = rank-order fold of this
        rank's slice of every rank's ``local``."""
        e = local.numel() if elems is None else elems
        _check(self.lib.byteps_shard_reduce_scatter(
            self.handle, _ptr(local), _ptrs(recv_slots if recv_slots is not None else []),
            _ptr(dst), e, _dtype(local, dtype), mode, _stream(local, stream)))

    def allgather(self, owned, full, elems: int | None = None, dtype=None, stream=None) -> None:
        e = full.numel() if elems is None else elems
        _check(self.lib.byteps_shard_allgather(self.handle, _ptr(owned), _ptr(full), e,
                                               _dtype(full, dtype), _stream(full, stream)))

    def scatter_reduce(self, root: int, pushes, recv_slots, dst, elems: int, dtype,
                       mode: int = 0, stream=None, n: int | None = None) -> None:
        n = len(pushes) if pushes is not None else (n if n is not None else len(recv_slots))
        _check(self.lib.byteps_shard_scatter_reduce(
            self.handle, root, _ptrs(pushes or []), n,
            _ptrs(recv_slots if recv_slots is not None else []), _ptr(dst), elems, int(dtype),
            mode, _stream(dst, stream)))

    def reduce_root(self, root: int, local, recv_slots, dst, elems: int | None = None,
                    dtype=None, mode: int = 0, stream=None) -> None:
        e = local.numel() if elems is None else elems
        _check(self.lib.byteps_shard_reduce_root(
            self.handle, root, _ptr(local), _ptrs(recv_slots if recv_slots is not None else []),
            _ptr(dst), e, _dtype(local, dtype), mode, _stream(local, stream)))

    def broadcast(self, root: int, buf, elems: int | None = None, dtype=None,
                  stream=None) -> None:
        e = buf.numel() if elems is None else elems
        _check(self.lib.byteps_shard_broadcast(self.handle, root, _ptr(buf), e,
                                               _dtype(buf, dtype), _stream(buf, stream)))


FoldFn = Callable[[object, list], None]   # fold(dst_tensor, [src_tensors])


def _gpu_fold():
    from .dtypes import from_torch
    from .reducer import GpuReducer
    red = GpuReducer()

    def fold(dst, srcs):
        red.sum_n(dst, srcs, dst.numel() * dst.element_size(), from_torch(dst.dtype))
    return fold


class ShardedReducer:
    """One instance per rank.  With ``comm`` (a :class:`ShardComm`) every
    operation is one call into the shard C ABI.  Otherwise transfers are
    torch.distributed P2P ops and ``fold`` defaults to the HIP fold through the
    reduce C ABI (there is no CPU fallback in the product path; CPU tests
    inject their own checker fold to exercise the plumbing over gloo)."""

    def __init__(self, n_elems: int, group=None, fold: FoldFn | None = None,
                 comm: "ShardComm | None" = None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.comm = comm
        if comm is not None:
            self.world, self.rank = comm.world, comm.rank
        else:
            self.world = dist.get_world_size(group) if dist.is_initialized() else 1
            self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_elems = n_elems
        self.ranges = owner_ranges(n_elems, self.world)
        self.lo, self.hi = self.ranges[self.rank]
        self.fold = fold if (fold is not None or comm is not None) else _gpu_fold()

    @property
    def owned(self) -> int:
        return self.hi - self.lo

    def reduce_owned(self, dst, srcs) -> None:
        """Fold this rank's owned slice: ``dst``/``srcs`` hold only the slice."""
        self.fold(dst, list(srcs))

    def scatter_reduce(self, root: int, pushes, recv_slots, dst) -> None:
        """``root`` holds the full flattened pushes of N workers (list of 1-D
        tensors of n_elems); every rank receives its slice of each push into
        ``recv_slots[k]`` (its own arena) with grouped P2P, then folds into
        ``dst`` (owned slice).  The root copies its own slice locally (native:
        folds it straight from ``pushes``)."""
        if self.comm is not None:
            dt = pushes[0] if pushes else recv_slots[0]
            self.comm.scatter_reduce(root, pushes, recv_slots, dst, self.n_elems,
                                     _dtype(dt, None), n=len(recv_slots))
            return
        dist = self.dist
        ops = []
        if self.rank == root:
            for g, (lo, hi) in enumerate(self.ranges):
                if g == root or hi == lo:
                    continue
                for k, p in enumerate(pushes):
                    ops.append(dist.P2POp(dist.isend, p[lo:hi], g, self.group))
            for k, p in enumerate(pushes):
                recv_slots[k].copy_(p[self.lo:self.hi])
        elif self.owned:
            for k in range(len(recv_slots)):
                ops.append(dist.P2POp(dist.irecv, recv_slots[k], root, self.group))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        if self.owned:
            self.fold(dst, list(recv_slots))

    def reduce_from_host(self, host_pushes, recv_slots, dst) -> None:
        """Pushes that start in host memory (ps-lite receive buffers / BytePS
        shm, server.cc:174, shared_memory.cc:28-49) land straight on their
        owner: each rank copies only ITS slice of every worker's push host ->
        its own HBM (``recv_slots[k]``, non-blocking from pinned memory) and
        folds it — no collective, and the node's PCIe links work in parallel,
        one per GPU (the scatter over xGMI is the fallback for
        pushes that already sit on one GPU)."""
        if not self.owned:
            return
        for k, h in enumerate(host_pushes):
            recv_slots[k].copy_(h[self.lo:self.hi], non_blocking=True)
        self.fold(dst, list(recv_slots))

    def reduce_scatter(self, local_full, recv_slots, dst) -> None:
        """Worker local reduce (REDUCE stage, core_loops.cc:184-247): every rank
        holds its own full gradient vector ``local_full`` (n_elems); rank g
        receives slice g of every rank's vector into ``recv_slots[r]`` (grouped
        point-to-point over RCCL/xGMI) and folds them in RANK order into ``dst``.
        Unlike ncclReduceScatter, whose summation order follows the ring, the
        result is a fixed left fold: bit-reproducible and equal to the oracle."""
        if self.comm is not None:
            self.comm.reduce_scatter(local_full, recv_slots, dst)
            return
        dist = self.dist
        ops = []
        for g, (lo, hi) in enumerate(self.ranges):
            if g != self.rank and hi > lo:
                ops.append(dist.P2POp(dist.isend, local_full[lo:hi], g, self.group))
        if self.owned:
            for r in range(self.world):
                if r != self.rank:
                    ops.append(dist.P2POp(dist.irecv, recv_slots[r], r, self.group))
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        if self.owned:
            recv_slots[self.rank].copy_(local_full[self.lo:self.hi])
            self.fold(dst, list(recv_slots))

    def allreduce(self, local_full, out_full, recv_slots=None, owned=None) -> None:
        """Deterministic all-reduce = reduce_scatter (P2P + HIP fold in rank
        order) + allgather (core_loops.cc:248-261 return leg)."""
        import torch
        if recv_slots is None:
            recv_slots = [torch.empty(self.owned, dtype=local_full.dtype, device=local_full.device)
                          for _ in range(self.world)]
        if owned is None:
            owned = torch.empty(self.owned, dtype=local_full.dtype, device=local_full.device)
        self.reduce_scatter(local_full, recv_slots, owned)
        self.allgather(owned, out_full)

    def allgather(self, owned_result, full_out) -> None:
        """Return leg: every rank gets the whole reduced vector (core_loops.cc:249-254).
        Uses all_gather on equal-size chunks plus a broadcast of the tail."""
        if self.comm is not None:
            self.comm.allgather(owned_result, full_out)
            return
        dist = self.dist
        per = self.n_elems // self.world
        if per:
            chunks = list(full_out[: per * self.world].split(per))
            dist.all_gather(chunks, owned_result[:per].contiguous(), group=self.group)
        tail = self.n_elems - per * self.world
        if tail:
            last = self.world - 1
            t = full_out[per * self.world:]
            if self.rank == last:
                t.copy_(owned_result[per:])
            dist.broadcast(t, src=last, group=self.group)
