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
"""
from __future__ import annotations

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


FoldFn = Callable[[object, list], None]   # fold(dst_tensor, [src_tensors])


def _gpu_fold():
    from .dtypes import from_torch
    from .reducer import GpuReducer
    red = GpuReducer()

    def fold(dst, srcs):
        red.sum_n(dst, srcs, dst.numel() * dst.element_size(), from_torch(dst.dtype))
    return fold


class ShardedReducer:
    """One instance per rank.  ``fold`` defaults to the HIP fold through the C
    ABI (there is no CPU fallback in the product path; CPU tests inject their
    own checker fold to exercise the distributed plumbing over gloo)."""

    def __init__(self, n_elems: int, group=None, fold: FoldFn | None = None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_elems = n_elems
        self.ranges = owner_ranges(n_elems, self.world)
        self.lo, self.hi = self.ranges[self.rank]
        self.fold = fold or _gpu_fold()

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
        ``dst`` (owned slice).  The root copies its own slice locally."""
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
