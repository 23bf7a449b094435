"""End-to-end push_pull (prophet_amd/pushpull.py) on the CPU with a recording
stand-in for the server: keys (operations.cc:237-247), partitions
(operations.cc:99-136), the request word (common.cc:99-102 / server.h:77-88),
reassembly at the right offsets, and the Prophet release order.  The GPU test
(tests/test_pushpull_gpu.py) runs the same path against the real server."""
import threading

import numpy as np
import pytest

from prophet_amd.buckets import cantor_command, resnet50_param_sizes
from prophet_amd.dtypes import DType
from prophet_amd.prophet import ProphetPushQueue, model_checkpoints
from prophet_amd.pushpull import ServerFrontend, Worker


class FakeServer:
    """Sums int32 pushes per key once every worker pushed (the init round
    stores the last push); a pull returns the current store."""

    def __init__(self, n_workers):
        self.n = n_workers
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self.store, self.pending, self.inited, self.log = {}, {}, set(), []

    def push(self, key, worker, data, dtype, nbytes=None):
        assert dtype == DType.INT32 and nbytes == data.nbytes
        with self.cv:
            self.log.append((key, worker, nbytes))
            self.pending.setdefault(key, {})[worker] = data.view(np.int32).copy()
            if len(self.pending[key]) == self.n:
                vals = list(self.pending.pop(key).values())
                self.store[key] = vals[-1] if key not in self.inited else sum(vals)
                self.inited.add(key)
                self.cv.notify_all()
            elif key not in self.inited:
                self.cv.wait_for(lambda: key in self.inited)     # init barrier

    def pull(self, key, out, nbytes=None):
        with self.cv:
            self.cv.wait_for(lambda: key not in self.pending)
            out.view(np.int32)[:] = self.store[key]


def test_keys_partitions_and_reassembly():
    srv = FakeServer(2)
    fe = ServerFrontend(srv)
    ws = [Worker(r, fe, partition_bytes=1000) for r in range(2)]
    sizes = {"a": 10, "b": 777, "c": 250}               # int32 elements
    data = {w.rank: {k: np.arange(n, dtype=np.int32) * (w.rank + 1) for k, n in sizes.items()}
            for w in ws}

    def run(w):
        for k in sizes:
            w.declare(k)
        for k in sizes:
            w.init_tensor(k, data[w.rank][k], DType.INT32)
        for k in sizes:
            w.push_pull(k, data[w.rank][k])
    ts = [threading.Thread(target=run, args=(w,)) for w in ws]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    c = ws[0].contexts["b"]
    assert c.declared_key == 1
    # bound 1000 aligned down to 8: 1000; 3108 bytes -> 4 partitions, keys (1<<16)+i
    assert c.key_list == [(1 << 16) + i for i in range(4)]
    assert [ln for _, _, ln in c.parts] == [1000, 1000, 1000, 108]
    for w in ws:
        for k, n in sizes.items():
            assert (data[w.rank][k] == np.arange(n) * 3).all(), (w.rank, k)


def test_request_word_is_decoded():
    seen = []

    class S:
        def push(self, key, worker, data, dtype, nbytes=None):
            seen.append(dtype)
    fe = ServerFrontend(S())
    fe.push(cantor_command(0, int(DType.FLOAT16)), 5, 0, np.zeros(4, np.uint8), 4)
    assert seen == [DType.FLOAT16]
    with pytest.raises(ValueError):
        fe.push(cantor_command(1, 0), 5, 0, np.zeros(4, np.uint8), 4)


def test_prophet_iteration_order():
    """Gradients arrive in backward order; with the Prophet PUSH queue the
    partitions go out in its release groups (scheduled_queue.cc:217-296):
    every partition exactly once, the result still the full sum."""
    sizes = [max(1, n // 256) for n in resnet50_param_sizes()]     # 161 tensors, small
    srv = FakeServer(1)
    w = Worker(0, ServerFrontend(srv), partition_bytes=2048)
    tensors = {f"g{i}": np.full(n, i, np.int32) for i, n in enumerate(sizes)}
    for name in tensors:
        w.declare(name)
    for name, t in tensors.items():
        w.init_tensor(name, t, DType.INT32)
    srv.log.clear()
    q = ProphetPushQueue(batch_size=64, net_b=100, credit=1 << 14,
                         checkpoints=model_checkpoints(len(sizes)))
    groups = w.push_pull_iteration(tensors, scheduler=q)
    flat = [x for g in groups for x in g]
    nparts = sum(len(w.contexts[n].parts) for n in tensors)
    assert len(flat) == len(set(flat)) == nparts
    assert len(groups) > 1
    cps = model_checkpoints(len(sizes))
    assert all(g >= cps[-2] + 1 for g, _ in groups[0])   # the last block goes first
    pushed = [k for k, _, _ in srv.log]
    want = [w.contexts[f"g{g}"].parts[p][0] for g, p in flat]
    assert pushed == want
    for i, n in enumerate(sizes):
        assert (tensors[f"g{i}"] == i).all()          # one worker: the sum is itself


def test_broadcast_is_push_pull_with_zeros():
    """byteps/torch/__init__.py:264-272: non-root ranks push zeros, everyone
    pulls the root's tensor; sources untouched."""
    N, root = 3, 1
    srv = FakeServer(N)
    fe = ServerFrontend(srv)
    workers = [Worker(r, fe, partition_bytes=64) for r in range(N)]
    src = {r: np.full(50, 10 * r + 1, np.int32) for r in range(N)}
    out = {}

    def run(w):
        w.init_tensor("p", src[w.rank], DType.INT32)
        out[w.rank] = w.broadcast("p", src[w.rank], root)

    ts = [threading.Thread(target=run, args=(w,)) for w in workers]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    for r in range(N):
        assert np.array_equal(out[r], src[root])
        assert np.array_equal(src[r], np.full(50, 10 * r + 1, np.int32))


def test_average_divides_by_worker_count():
    """push_pull(average=True) as byteps/torch's: the sum / size; integer
    tensors refuse (no true division in place)."""
    class FloatFake(FakeServer):
        def push(self, key, worker, data, dtype, nbytes=None):
            with self.cv:
                self.pending.setdefault(key, {})[worker] = data.view(np.float32).copy()
                if len(self.pending[key]) == self.n:
                    vals = list(self.pending.pop(key).values())
                    self.store[key] = vals[-1] if key not in self.inited else sum(vals)
                    self.inited.add(key)
                    self.cv.notify_all()
                elif key not in self.inited:
                    self.cv.wait_for(lambda: key in self.inited)

        def pull(self, key, out, nbytes=None):
            with self.cv:
                self.cv.wait_for(lambda: key not in self.pending)
                out.view(np.float32)[:] = self.store[key]

    N = 4
    srv = FloatFake(N)
    fe = ServerFrontend(srv, size=N)
    workers = [Worker(r, fe, partition_bytes=64) for r in range(N)]
    vals = {r: np.full(40, float(r + 1), np.float32) for r in range(N)}

    def run(w):
        w.init_tensor("g", vals[w.rank], DType.FLOAT32)
        w.push_pull("g", vals[w.rank], average=True)

    ts = [threading.Thread(target=run, args=(w,)) for w in workers]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    for r in range(N):
        assert np.array_equal(vals[r], np.full(40, 2.5, np.float32))
    from prophet_amd.pushpull import _divide_
    with pytest.raises(ValueError):
        _divide_(np.zeros(3, np.int32), 2)


def test_push_pull_async_handles():
    """push_pull_async / poll / synchronize (byteps/torch/ops.py): several
    tensors in flight per worker, results as the synchronous call's."""
    N = 3
    srv = FakeServer(N)
    fe = ServerFrontend(srv, size=N)
    workers = [Worker(r, fe, partition_bytes=64) for r in range(N)]
    names = [f"t{i}" for i in range(4)]
    vals = {(r, n): np.arange(30, dtype=np.int32) * (r + 1) + i
            for r in range(N) for i, n in enumerate(names)}

    def run(w):
        for n in names:
            w.init_tensor(n, vals[(w.rank, n)], DType.INT32)
        hs = [w.push_pull_async(n, vals[(w.rank, n)]) for n in names]
        assert all(isinstance(w.poll(h), bool) for h in hs)
        for h in hs:
            w.synchronize(h)
        w.close()

    ts = [threading.Thread(target=run, args=(w,)) for w in workers]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    for i, n in enumerate(names):
        want = sum(np.arange(30, dtype=np.int32) * (r + 1) + i for r in range(N))
        for r in range(N):
            assert np.array_equal(vals[(r, n)], want)


def test_partition_bytes_and_local_size_from_env(monkeypatch):
    """BYTEPS_PARTITION_BYTES / BYTEPS_LOCAL_SIZE change the key lists exactly
    as the reference's bound does: AlignTo(atoi(bytes), 8 * local_size)
    rounded down (global.cc:128-135, communicator.cc:71-77)."""
    monkeypatch.setenv("BYTEPS_PARTITION_BYTES", "1000063")
    monkeypatch.setenv("BYTEPS_LOCAL_SIZE", "8")
    srv = FakeServer(1)
    w = Worker(0, ServerFrontend(srv))
    assert w.bound == 1_000_063 // 64 * 64 == 1_000_000
    x = np.arange(750_001, dtype=np.int32)               # 3,000,004 B
    ctx = w.init_tensor("g", x, DType.INT32)
    assert ctx.key_list == [0, 1, 2, 3]
    assert [ln for _, _, ln in ctx.parts] == [1_000_000] * 3 + [4]
    w.declare("h")
    ctx2 = w.init_tensor("h", np.zeros(10, np.int32), DType.INT32)
    assert ctx2.key_list == [1 << 16]
    # the ResNet-50 fp16 set under this bound: partitions per tensor
    from prophet_amd.buckets import partition_all
    parts = partition_all([n * 2 for n in resnet50_param_sizes()], bound=w.bound)
    want = sum(-(-n * 2 // 1_000_000) for n in resnet50_param_sizes())
    assert len(parts) == want and want > 165           # more keys than the default's 165


@pytest.mark.parametrize("env,bound", [
    ({}, 4_096_000),                                          # defaults
    ({"BYTEPS_LOCAL_SIZE": "8"}, 4_096_000),                  # 4096000 % 64 == 0
    ({"BYTEPS_PARTITION_BYTES": "4096001", "BYTEPS_LOCAL_SIZE": "3"}, 4_095_984),
    ({"BYTEPS_PARTITION_BYTES": " 2048000xyz"}, 2_048_000),   # atoi
    ({"BYTEPS_PARTITION_BYTES": "100", "BYTEPS_LOCAL_SIZE": "8"}, 64),
])
def test_partition_bound_env_cases(monkeypatch, env, bound):
    for k in ("BYTEPS_PARTITION_BYTES", "BYTEPS_LOCAL_SIZE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert Worker(0, ServerFrontend(FakeServer(1))).bound == bound


def test_partition_bound_env_zero_is_refused(monkeypatch):
    monkeypatch.setenv("BYTEPS_PARTITION_BYTES", "63")
    monkeypatch.setenv("BYTEPS_LOCAL_SIZE", "8")      # AlignTo(63, 64) == 0
    with pytest.raises(ValueError, match="positive"):
        Worker(0, ServerFrontend(FakeServer(1)))
    # explicit arguments still override the environment
    assert Worker(0, ServerFrontend(FakeServer(1)), partition_bytes=1000, local_size=1).bound == 1000
