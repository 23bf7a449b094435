"""Host-to-host streaming reduction: pinned host pushes -> HBM -> fold -> host.

The reference path starts and ends in host memory (pushes arrive through
ps-lite into host buffers, byteps/server/server.cc:174; the worker stages
through pinned shm, shared_memory.cc:28-49, with D2H/H2D copy loops,
core_loops.cc:372-437 and 566-610).  ``StreamingReducer`` runs that path on
one GPU with three HIP streams and a ring of device chunk slots:

    h2d stream:      chunk c of every worker's bucket -> slot c % depth
    compute stream:  fold(slot) -> out slot           (byteps_reduce_sum_n)
    d2h stream:      out slot -> host result chunk

so PCIe transfers in both directions overlap the fold.  ``zero_copy=True``
instead runs ONE fold whose loads and stores go straight to the pinned host
pages over PCIe (device addresses from ``hipHostGetDevicePointer``): no device
staging and no copy engines, the same PCIe ceiling (config 2's workload: 51.8
vs 51.0 GiB/s), but the kernel holds the CUs for the whole
transfer, so it suits a GPU with nothing else to run.  Chunks are multiples
of 16 bytes and of 8 elements, so the fp16 F16C body/tail split
(cpu_reducer.cc:103,118) falls exactly where an unchunked call would put it,
and the result is bit-identical to one ``sum_n`` over the whole bucket.
"""
from __future__ import annotations

from .dtypes import elem_size
from .reducer import GpuReducer, MODE_REFERENCE


class StreamingReducer:
    def __init__(self, n_workers: int, chunk_bytes: int = 32 << 20, depth: int = 3,
                 device=None, reducer: GpuReducer | None = None, zero_copy: bool = False):
        import torch
        self.torch = torch
        self.zero_copy = zero_copy
        self.dev = torch.device(device if device is not None else "cuda")
        self.n_workers = n_workers
        self.chunk = max(128, (int(chunk_bytes) // 128) * 128)
        self.depth = depth
        self.red = reducer or GpuReducer()
        self.slots = [[torch.empty(self.chunk, dtype=torch.uint8, device=self.dev)
                       for _ in range(n_workers)] for _ in range(depth)]
        self.outs = [torch.empty(self.chunk, dtype=torch.uint8, device=self.dev)
                     for _ in range(depth)]
        self.s_h2d = torch.cuda.Stream(self.dev)
        self.s_cmp = torch.cuda.Stream(self.dev)
        self.s_d2h = torch.cuda.Stream(self.dev)
        E = torch.cuda.Event
        self.ev_h2d = [E() for _ in range(depth)]
        self.ev_cmp = [E() for _ in range(depth)]
        self.ev_d2h = [E() for _ in range(depth)]
        self._used = [False] * depth

    def reduce(self, host_srcs, host_dst, length: int, dtype: int,
               mode: int = MODE_REFERENCE) -> None:
        """``host_dst[:length] = fold(host_srcs[k][:length])``; host tensors
        should be pinned (uint8 views).  Blocks until the result is in host_dst."""
        torch = self.torch
        if len(host_srcs) != self.n_workers:
            raise ValueError("expected one host buffer per worker")
        if self.zero_copy:
            srcs = [_Dev(_host_device_ptr(h)) for h in host_srcs]
            with torch.cuda.stream(self.s_cmp):
                self.red.sum_n(_Dev(_host_device_ptr(host_dst)), srcs, length, dtype, mode,
                               stream=self.s_cmp)
            self.s_cmp.synchronize()
            return
        es = elem_size(dtype)
        step = self.chunk // (8 * es) * (8 * es)      # whole 8-element groups
        if step == 0:
            raise ValueError("chunk too small")
        off, c = 0, 0
        while off < length:
            ln = min(step, length - off)
            i = c % self.depth
            slot, out = self.slots[i], self.outs[i]
            with torch.cuda.stream(self.s_h2d):
                if self._used[i]:
                    self.s_h2d.wait_event(self.ev_cmp[i])   # slot inputs consumed
                for k in range(self.n_workers):
                    slot[k][:ln].copy_(host_srcs[k][off: off + ln], non_blocking=True)
                self.ev_h2d[i].record(self.s_h2d)
            with torch.cuda.stream(self.s_cmp):
                self.s_cmp.wait_event(self.ev_h2d[i])
                if self._used[i]:
                    self.s_cmp.wait_event(self.ev_d2h[i])   # out slot drained
                self.red.sum_n(out, [s[:ln] for s in slot], ln, dtype, mode, stream=self.s_cmp)
                self.ev_cmp[i].record(self.s_cmp)
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(self.ev_cmp[i])
                host_dst[off: off + ln].copy_(out[:ln], non_blocking=True)
                self.ev_d2h[i].record(self.s_d2h)
            self._used[i] = True
            off += ln
            c += 1
        self.s_d2h.synchronize()


class _Dev:
    """A device address in the shape the reducer takes (``data_ptr()``)."""
    def __init__(self, p: int):
        self.p = p

    def data_ptr(self) -> int:
        return self.p


_hip = None


def _host_device_ptr(t) -> int:
    """Device address of a pinned host tensor (hipHostGetDevicePointer); raises
    for memory the device cannot address (pageable host memory)."""
    import ctypes
    from .reducer import EARGS, ReduceError
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.c_void_p, ctypes.c_uint]
    p = ctypes.c_void_p()
    rc = _hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(int(t.data_ptr())), 0)
    if rc != 0 or not p.value:
        _hip.hipGetLastError()     # do not leave the error for torch's next check
        raise ReduceError(EARGS, f"zero_copy needs pinned host buffers (hipHostGetDevicePointer "
                                 f"returned {rc})")
    return int(p.value)
