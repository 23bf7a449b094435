"""Prophet's PUSH-stage scheduler — the native one in libbpsr.so
(include/bpsr/prophet.h, prophet_amd/csrc/bpsr_prophet.cpp), behind the
interface of BytePSScheduledQueue's PUSH queue
(byteps/common/scheduled_queue.cc:94-108 addTask, :217-296 getTask,
:362-371 reportFinish).

It decides which partitions reach the server together: the release groups a
batched fold launch (``byteps_reduce_plan``) or a block-queue release
(``byteps_reduce_blockq_release_range``) receives.  The algorithm, its
deviations from the reference and its thread-safety are documented in the
header; ``oracle/prophet_oracle.py`` restates it in Python and the tests
compare the two task for task.  There is no Python fallback: a missing
``libbpsr.so`` raises.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass

from .buckets import DEFAULT_PARTITION_BYTES, PROPHET_CHECKPOINTS, partition_all
from .reducer import _check, load_library

# scheduled_queue.h:84-85
BACKWARD_EXEC = (16, 15, 9, 10, 12, 18, 15, 21, 30, 25, 20, 5, 0)

PHASE_CREDIT = -1      # BYTEPS_PROPHET_CREDIT
PHASE_FIFO = -2        # BYTEPS_PROPHET_FIFO
_PHASE_NAMES = {PHASE_CREDIT: "credit", PHASE_FIFO: "fifo"}


@dataclass(frozen=True, order=True)
class PushTask:
    grad: int          # gradient index; the reference's priority is -grad
    part: int          # partition index inside the gradient
    len: int           # bytes
    total_partnum: int = 1
    key: int = 0
    scheduled: bool = True   # the tensor name matches Z_keyword (else: FIFO)


class _Config(ctypes.Structure):
    _fields_ = [("batch_size", ctypes.c_int64), ("net_b", ctypes.c_int64),
                ("credit", ctypes.c_int64), ("checkpoints", ctypes.POINTER(ctypes.c_int32)),
                ("ncheckpoints", ctypes.c_int32), ("backward_exec", ctypes.POINTER(ctypes.c_double))]


class _Task(ctypes.Structure):
    _fields_ = [("grad", ctypes.c_int32), ("part", ctypes.c_int32), ("len", ctypes.c_int64),
                ("total_partnum", ctypes.c_int32), ("scheduled", ctypes.c_int32),
                ("key", ctypes.c_uint64), ("handle", ctypes.c_uint64)]


class _State(ctypes.Structure):
    _fields_ = [("pointer", ctypes.c_int32), ("expected", ctypes.c_int32),
                ("sizepointer", ctypes.c_int32), ("dequeue", ctypes.c_int32),
                ("meetzero", ctypes.c_int32), ("stack_depth", ctypes.c_int32),
                ("credit", ctypes.c_int64), ("budget_left", ctypes.c_double)]


PROPHET_EXPORTS = (
    "byteps_prophet_create", "byteps_prophet_destroy", "byteps_prophet_add_task",
    "byteps_prophet_get_task", "byteps_prophet_report_finish", "byteps_prophet_pending",
    "byteps_prophet_get_state", "byteps_prophet_reset", "byteps_prophet_release_groups",
    "byteps_prophet_profile", "byteps_prophet_estimate_net_b",
    "byteps_prophet_loop_create", "byteps_prophet_loop_begin", "byteps_prophet_loop_push",
    "byteps_prophet_loop_push_many", "byteps_prophet_loop_release_calls",
    "byteps_prophet_loop_end", "byteps_prophet_loop_destroy",
)

_BOUND = None


def _ck(rc: int) -> None:
    if rc < 0:
        _check(rc)


def _lib():
    global _BOUND
    if _BOUND is None:
        L = load_library()
        vp, P = ctypes.c_void_p, ctypes.POINTER
        L.byteps_prophet_create.argtypes = [P(_Config), P(vp)]
        L.byteps_prophet_destroy.argtypes = [vp]
        L.byteps_prophet_add_task.argtypes = [vp, P(_Task)]
        L.byteps_prophet_get_task.argtypes = [vp, P(_Task), P(ctypes.c_int32)]
        L.byteps_prophet_report_finish.argtypes = [vp, ctypes.c_int64]
        L.byteps_prophet_pending.argtypes = [vp, P(ctypes.c_uint64)]
        L.byteps_prophet_get_state.argtypes = [vp, P(_State)]
        L.byteps_prophet_reset.argtypes = [vp]
        L.byteps_prophet_loop_create.argtypes = [vp, vp, P(ctypes.c_int32), ctypes.c_int32,
                                                 ctypes.c_int32, vp, ctypes.c_int, P(vp)]
        L.byteps_prophet_loop_begin.argtypes = [vp, vp]
        L.byteps_prophet_loop_push.argtypes = [vp, P(_Task)]
        L.byteps_prophet_loop_push_many.argtypes = [vp, P(_Task), ctypes.c_int32]
        L.byteps_prophet_loop_release_calls.argtypes = [vp, P(ctypes.c_uint64)]
        L.byteps_prophet_loop_end.argtypes = [vp, ctypes.c_double]
        L.byteps_prophet_loop_destroy.argtypes = [vp]
        L.byteps_prophet_estimate_net_b.argtypes = [P(ctypes.c_int64)] * 3 + [
            ctypes.c_int32, P(ctypes.c_double)]
        L.byteps_prophet_profile.argtypes = [P(ctypes.c_int64), ctypes.c_int32,
                                             P(ctypes.c_int32), P(ctypes.c_double), ctypes.c_int32]
        L.byteps_prophet_release_groups.argtypes = [
            vp, P(_Task), ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
            P(_Task), P(ctypes.c_int32), P(ctypes.c_int32)]
        for name in PROPHET_EXPORTS:
            getattr(L, name).restype = ctypes.c_int
        _BOUND = L
    return _BOUND


class ProphetPushQueue:
    """One PUSH queue (the root device's, scheduled_queue.cc:69-72), native.

    ``batch_size`` = Z_BATCH_SIZE, ``net_b`` = Z_NET_B (the constructor
    multiplies it by 125), ``credit`` = Z_CREDIT bytes.  ``phase`` is the phase
    of the last released task: its budget block index, "credit" or "fifo"."""

    def __init__(self, batch_size: int, net_b: int, credit: int,
                 checkpoints=PROPHET_CHECKPOINTS, backward_exec=BACKWARD_EXEC):
        if len(backward_exec) != len(checkpoints):
            raise ValueError("backward_exec needs one entry per checkpoint")
        self._L = _lib()
        cps = (ctypes.c_int32 * len(checkpoints))(*checkpoints)
        ex = (ctypes.c_double * len(backward_exec))(*backward_exec)
        cfg = _Config(int(batch_size), int(net_b), int(credit), cps, len(checkpoints), ex)
        h = ctypes.c_void_p()
        _ck(self._L.byteps_prophet_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.checkpoints = tuple(checkpoints)
        self.phase = None
        self._lock = threading.Lock()          # guards the handle -> task map
        self._live: dict[int, PushTask] = {}
        self._next = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._L.byteps_prophet_destroy(h)
            self._h = None

    def _to_c(self, t: PushTask) -> _Task:
        with self._lock:
            hid = self._next
            self._next += 1
            self._live[hid] = t
        return _Task(t.grad, t.part, t.len, t.total_partnum, int(t.scheduled), t.key, hid)

    def add_task(self, t: PushTask) -> None:
        c = self._to_c(t)
        rc = self._L.byteps_prophet_add_task(self._h, ctypes.byref(c))
        if rc:
            with self._lock:
                del self._live[c.handle]
            _ck(rc)

    def get_task(self) -> PushTask | None:
        """One getTask() poll: the released task, or None."""
        out, ph = _Task(), ctypes.c_int32()
        rc = self._L.byteps_prophet_get_task(self._h, ctypes.byref(out), ctypes.byref(ph))
        _ck(rc if rc < 0 else 0)
        if rc == 0:
            return None
        self.phase = _PHASE_NAMES.get(ph.value, ph.value)
        with self._lock:
            return self._live.pop(out.handle)

    def report_finish(self, size: int) -> None:
        _ck(self._L.byteps_prophet_report_finish(self._h, int(size)))

    def pending(self) -> int:
        n = ctypes.c_uint64()
        _ck(self._L.byteps_prophet_pending(self._h, ctypes.byref(n)))
        return n.value

    def reset(self) -> None:
        _ck(self._L.byteps_prophet_reset(self._h))

    def state(self) -> dict:
        s = _State()
        _ck(self._L.byteps_prophet_get_state(self._h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in _State._fields_}


def _stream_ptr(stream) -> int:
    if stream is None:
        return 0
    return int(getattr(stream, "cuda_stream", stream))


class PushLoop:
    """The PUSH loop as a native thread (byteps_prophet_loop_*; core_loops.cc
    RunPushLoopOnce -> reportFinish): ``queue`` (a ProphetPushQueue) releases
    partitions, the loop releases the blocks of ``blockq``
    (``GpuReducer.make_blockq``) that they complete, one release_range per run
    of consecutive blocks on ``release_stream``.  ``block_of[i]`` is the block
    of table partition i; push each partition with its table index.
    Per iteration: ``begin(consumer_stream)``, ``push(task, index)`` per
    partition as its bytes land, ``end()``.  By default a library thread
    drains the scheduler and issues the releases (the reference's shape; at
    config 3 as fast as a hand-written loop).
    ``inline=True``: each push does it in the caller's thread — fewer host
    cycles and no thread hand-off, but then that thread must not block
    on the device (``torch.cuda.synchronize``, a ``hipFree`` — which Python's
    garbage collector can trigger at any allocation) between ``begin`` and its
    last push: the consumer would wait for releases the blocked thread cannot
    issue, until its timeout."""

    def __init__(self, queue: ProphetPushQueue, blockq, block_of, release_stream=None,
                 inline: bool = False, host_release: bool = False):
        """``host_release=True``: complete blocks are released from the host
        (``BlockQueue.release_host``, no stream work) — for pushes whose bytes
        are already visible to the device when ``push`` is called.  Otherwise
        the loop thread (``inline=False``) needs ``release_stream``: the stream
        the pushes' copies are queued on (None is refused — the library would
        read it as the loop thread's own per-thread stream)."""
        if release_stream is None and not inline and not host_release:
            raise ValueError("PushLoop: release_stream is required with the loop thread and "
                             "stream releases (the stream the pushes' copies are queued on)")
        self._L = _lib()
        self.queue, self.blockq = queue, blockq
        bo = (ctypes.c_int32 * max(len(block_of), 1))(*block_of)
        h = ctypes.c_void_p()
        flags = (1 if inline else 0) | (2 if host_release else 0)
        _ck(self._L.byteps_prophet_loop_create(queue._h, blockq.handle, bo, len(block_of),
                                               blockq.nblocks, _stream_ptr(release_stream),
                                               flags, ctypes.byref(h)))
        self._h = h

    def begin(self, consumer_stream=None) -> None:
        """Reset the scheduler and launch the iteration's consumer on
        ``consumer_stream`` (None: the library's consumer stream — then
        ``end`` orders the current torch stream after the consumer)."""
        self._on_library_stream = consumer_stream is None
        _ck(self._L.byteps_prophet_loop_begin(self._h, _stream_ptr(consumer_stream)))

    def push(self, task: PushTask, index: int) -> None:
        c = _Task(task.grad, task.part, task.len, task.total_partnum, int(task.scheduled),
                  task.key, int(index))
        _ck(self._L.byteps_prophet_loop_push(self._h, ctypes.byref(c)))

    def make_batch(self, tasks, indices):
        """A reusable native array of (task, table index) pairs for
        ``push_many`` (build it once per arrival set, push it every iteration)."""
        arr = (_Task * max(len(tasks), 1))()
        for i, (t, ix) in enumerate(zip(tasks, indices)):
            arr[i] = _Task(t.grad, t.part, t.len, t.total_partnum, int(t.scheduled), t.key,
                           int(ix))
        return arr, len(tasks)

    def push_many(self, batch) -> None:
        """Push partitions that landed together (``make_batch``'s result, or a
        list of (task, index) pairs): one scheduler drain, their release groups
        released together."""
        if not isinstance(batch, tuple):
            pairs = list(batch)
            batch = self.make_batch([t for t, _ in pairs], [i for _, i in pairs])
        arr, n = batch
        _ck(self._L.byteps_prophet_loop_push_many(self._h, arr, int(n)))

    def release_calls(self) -> int:
        """Release kernels (or host releases) issued since the loop was made."""
        n = ctypes.c_uint64()
        _ck(self._L.byteps_prophet_loop_release_calls(self._h, ctypes.byref(n)))
        return n.value

    def end(self, timeout_s: float = 10.0) -> None:
        """Wait until every block has been released; with the consumer on the
        library's stream, the current torch stream then waits for it (on the
        device, ``BlockQueue.join`` — also with overlapping launches), so
        later torch work sees the folded outputs."""
        _ck(self._L.byteps_prophet_loop_end(self._h, float(timeout_s)))
        if getattr(self, "_on_library_stream", False):
            self.blockq.join()      # torch's current stream, after the consumer

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._L.byteps_prophet_loop_destroy(h)
            self._h = None

    def __del__(self):
        self.close()


def profile_checkpoints(tic_us) -> tuple[tuple, tuple]:
    """Prophet's pre-run profile (scheduled_queue.cc:110-167), native
    (``byteps_prophet_profile``): the first time each gradient i reached the
    PUSH queue in one profiled iteration (``tic_us[i]``, microseconds) ->
    ``(checkpoints, backward_exec)`` for ``ProphetPushQueue``: a block boundary
    wherever the gap before a gradient exceeds twice the mean gap, each block's
    budget the compute gap that follows it (ms; the constructor scales it by
    batch/64 and Z_NET_B * 125)."""
    L = _lib()
    n = len(tic_us)
    tics = (ctypes.c_int64 * max(n, 1))(*[int(t) for t in tic_us])
    cap = n + 2
    cps = (ctypes.c_int32 * cap)()
    ex = (ctypes.c_double * cap)()
    k = L.byteps_prophet_profile(tics, n, cps, ex, cap)
    _ck(k)
    return tuple(cps[:k]), tuple(ex[:k])


def estimate_net_b(sizes, start_us, finish_us) -> float:
    """Prophet's bandwidth monitor (reportFinish(size, priority),
    scheduled_queue.cc:373-398), native: the fastest profiled push as Z_NET_B
    (Mb/s) = max of size * 8 / (finish - start) over the pushes."""
    L = _lib()
    n = len(sizes)
    arr = lambda xs: (ctypes.c_int64 * max(n, 1))(*[int(x) for x in xs])  # noqa: E731
    out = ctypes.c_double()
    _ck(L.byteps_prophet_estimate_net_b(arr(sizes), arr(start_us), arr(finish_us), n,
                                        ctypes.byref(out)))
    return out.value


def queue_from_profile(tic_us, batch_size: int, credit: int, net_b: float | None = None,
                       push_sizes=None, push_start_us=None, push_finish_us=None):
    """A PUSH queue configured the way Prophet's pre-run pass configures it:
    checkpoints and block budgets from the gradients' first-arrival times
    (``profile_checkpoints``) and Z_NET_B from the profiled pushes
    (``estimate_net_b``) unless given."""
    cps, ex = profile_checkpoints(tic_us)
    if net_b is None:
        net_b = estimate_net_b(push_sizes, push_start_us, push_finish_us)
    return ProphetPushQueue(batch_size=batch_size, net_b=int(net_b), credit=credit,
                            checkpoints=cps, backward_exec=ex)


def model_checkpoints(n_tensors: int, checkpoints=PROPHET_CHECKPOINTS) -> tuple:
    """The reference hard-codes a 157-gradient model; a model with more
    gradients gets its last checkpoint extended to ``n_tensors - 1`` (same rule
    as buckets.prophet_blocks) so every gradient is collected."""
    cps = list(checkpoints)
    if cps[-1] < n_tensors - 1:
        cps[-1] = n_tensors - 1
    return tuple(cps)


def backward_arrivals(sizes_bytes, bound: int = DEFAULT_PARTITION_BYTES) -> list[PushTask]:
    """PUSH tasks of one iteration in the order the backward pass enqueues
    them: highest gradient index first, partitions in order
    (operations.cc:99-136 partitioning, priority = -declared index)."""
    parts = partition_all(list(sizes_bytes), bound=bound)
    nparts = {}
    for p in parts:
        nparts[p.tensor] = nparts.get(p.tensor, 0) + 1
    parts.sort(key=lambda p: (-p.tensor, p.part))
    return [PushTask(p.tensor, p.part, p.len, nparts[p.tensor], p.key) for p in parts]


def release_groups(queue: ProphetPushQueue, arrivals, finish_immediately: bool = True,
                   max_idle: int = 1_000_000, with_phase: bool = False):
    """Drive ``queue`` through one iteration in native code
    (``byteps_prophet_release_groups``): one arrival per scheduler poll, in
    the given (backward) order; a release group is a run of consecutive
    successful polls — what one batched reduce launch receives.  ``with_phase``
    returns ``(phase, group)`` pairs (groups also split at phase changes),
    phase being the budget block index, "credit" or "fifo".  The queue must be
    empty; it is not reset first."""
    arrivals = list(arrivals)
    n = len(arrivals)
    arr = (_Task * max(n, 1))(*[queue._to_c(t) for t in arrivals])
    rel = (_Task * max(n, 1))()
    starts = (ctypes.c_int32 * (n + 1))()
    phases = (ctypes.c_int32 * max(n, 1))()
    unset = (1 << 64) - 1
    for i in range(n):
        rel[i].handle = unset
    ng = queue._L.byteps_prophet_release_groups(
        queue._h, arr, n, int(finish_immediately), int(with_phase), int(max_idle),
        rel, starts, phases)
    if ng < 0:
        # The native queue keeps what it accepted and did not release (e.g.
        # "no progress"): those handles stay live for later get_task() polls.
        # Released ones (written to rel) and — when the queue holds nothing,
        # as after a refused arrival — every handle of this call are dropped.
        held = queue.pending() > 0
        with queue._lock:
            released = {rel[i].handle for i in range(n) if rel[i].handle != unset}
            for c in arr[:n]:
                if c.handle in released or not held:
                    queue._live.pop(c.handle, None)
        _ck(ng)
    groups = []
    with queue._lock:
        for g in range(ng):
            tasks = [queue._live.pop(rel[i].handle) for i in range(starts[g], starts[g + 1])]
            ph = _PHASE_NAMES.get(phases[g], phases[g])
            groups.append((ph, tasks) if with_phase else tasks)
        if ng:
            queue.phase = _PHASE_NAMES.get(phases[ng - 1], phases[ng - 1])
    return groups


__all__ = ["PushTask", "ProphetPushQueue", "BACKWARD_EXEC", "PHASE_CREDIT", "PHASE_FIFO",
           "model_checkpoints", "backward_arrivals", "release_groups", "profile_checkpoints",
           "estimate_net_b", "queue_from_profile", "PushLoop", "PROPHET_EXPORTS"]
