"""GPU-resident PS server (include/bpsr/server.h) against the reference's
server semantics (byteps/server/server.cc:147-308): concurrent worker threads,
random arrival order, several rounds, both policies; results bit-exact with the
oracle's left fold in the recorded arrival order."""
import random
import threading
import time

import numpy as np
import pytest

from golden_util import assert_bytes_match
from oracle.oracle import PortReducer
from prophet_amd import synth
from prophet_amd.dtypes import DType, elem_size

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(180)]


@pytest.fixture(scope="module")
def port():
    assert torch.cuda.is_available()
    return PortReducer(nthreads=4)


def data(dt, n, worker, rnd, key):
    return np.ascontiguousarray(synth.bucket(dt, n, worker, "normal", 1000 * rnd + 37 * key)) \
        .view(np.uint8)


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16], ids=lambda d: DType(d).name)
def test_sync_rounds_concurrent_workers(port, policy, dt):
    from prophet_amd.server import PSServer
    N, R = 8, 3
    sizes = [1, 7, 1000, 65_536 + 3, 1_000_003]    # elements per key
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=4, policy=policy)
    bar = threading.Barrier(N + 1)
    errors = []
    results = {}

    def worker(w):
        try:
            rng = random.Random(w)
            for rnd in range(R + 1):               # round 0 = init pushes
                keys = list(range(len(sizes)))
                if rnd > 0:
                    # init pushes block until every worker's arrived, so they go
                    # in declaration order like BytePS's InitTensor (operations.cc:219)
                    rng.shuffle(keys)
                for j in keys:
                    time.sleep(rng.random() * 0.002)
                    srv.push(j, w, data(dt, sizes[j], w, rnd, j), dt)
                bar.wait()                          # main thread reads arrival orders
                bar.wait()
                if rnd == 0:
                    continue
                for j in keys:
                    out = np.zeros(sizes[j] * es, np.uint8)
                    srv.pull(j, out)
                    results[(w, rnd, j)] = out
        except Exception as e:  # surfaced below
            errors.append(e)
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    orders = {}
    for rnd in range(R + 1):
        bar.wait()
        for j in range(len(sizes)):
            rounds, lane, order = srv.key_info(j)
            assert rounds == rnd
            orders[(rnd, j)] = order
        bar.wait()
    for t in ts:
        t.join()
    assert not errors, errors
    for rnd in range(1, R + 1):
        for j, n in enumerate(sizes):
            order = orders[(rnd, j)]
            assert sorted(order) == list(range(N))
            ins = [data(dt, n, w, rnd, j) for w in order]
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, ins, n * es, dt)
            for w in range(N):
                assert_bytes_match(dt, results[(w, rnd, j)], want, nan_class_f32_f64=False,
                                   what=f"round {rnd} key {j} worker {w}")
    srv.close()


def test_fused_equals_incremental_in_same_order(port):
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT16, 5, 300_001
    outs = []
    for policy in (0, 1):
        srv = PSServer(N, policy=policy)
        init = [threading.Thread(target=srv.push, args=(0, w, data(dt, n, w, 0, 0), dt))
                for w in range(N)]    # init round: each push blocks until all arrived
        for t in init:
            t.start()
        for t in init:
            t.join()
        for w in (3, 0, 4, 1, 2):
            srv.push(0, w, data(dt, n, w, 1, 0), dt)
        out = np.zeros(n * 2, np.uint8)
        srv.pull(0, out)
        assert srv.key_info(0)[2] == [3, 0, 4, 1, 2]
        outs.append(out)
        srv.close()
    assert np.array_equal(outs[0], outs[1])
    want = np.zeros(n * 2, np.uint8)
    port.sum_n(want, [data(dt, n, w, 1, 0) for w in (3, 0, 4, 1, 2)], n * 2, dt)
    assert np.array_equal(outs[0], want)


def test_pull_blocks_until_round_complete():
    from prophet_amd.server import PSServer
    N, n, dt = 3, 4096, DType.INT32
    srv = PSServer(N)
    init = [threading.Thread(target=srv.push, args=(7, w, np.zeros(n, np.int32), dt))
            for w in range(N)]
    for t in init:
        t.start()
    for t in init:
        t.join()
    got = {}

    def puller():
        out = np.zeros(n, np.int32)
        srv.pull(7, out)
        got["v"] = out

    srv.push(7, 0, np.full(n, 1, np.int32), dt)
    srv.push(7, 1, np.full(n, 2, np.int32), dt)
    t = threading.Thread(target=puller)
    t.start()
    time.sleep(0.3)
    assert "v" not in got                     # round not finished: pull queued
    srv.push(7, 2, np.full(n, 4, np.int32), dt)
    t.join(timeout=10)
    assert (got["v"] == 7).all()
    srv.close()


def test_async_mode_sums_into_store():
    from prophet_amd.server import PSServer
    N, n, dt = 4, 10_001, DType.INT64
    srv = PSServer(N, async_mode=True)
    init = np.arange(n, dtype=np.int64)
    ts = [threading.Thread(target=srv.push, args=(1, w, init, dt)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for w in range(N):
        srv.push(1, w, np.full(n, w + 1, np.int64), dt)
    out = np.zeros(n, np.int64)
    srv.pull(1, out)                      # async: answered immediately
    assert np.array_equal(out, init + 10)
    srv.close()


def test_zero_copy_slot_path(port):
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 4, 77_777
    red = GpuReducer()
    srv = PSServer(N)
    srv.init_key(5, n * 4, dt)
    for rnd in range(2):
        ins = [data(dt, n, w, rnd, 5) for w in range(N)]
        dev = [torch.from_numpy(x).cuda() for x in ins]
        ths = []
        for w in range(N):
            slot = srv.recv_slot(5, w)
            red.copy(slot, dev[w], n * 4)
            red.sync()
            ths.append(threading.Thread(target=srv.push_ready, args=(5, w)))
            ths[-1].start()
        for t in ths:
            t.join()
        if rnd == 0:
            continue
        out = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
        srv.pull(5, out)
        order = srv.key_info(5)[2]
        want = np.zeros(n * 4, np.uint8)
        port.sum_n(want, [ins[w] for w in order], n * 4, dt)
        assert np.array_equal(out.cpu().numpy(), want)
    srv.close()


def test_engine_lanes_least_loaded_sticky():
    """server.h:138-162 GetThreadID: least accumulated bytes, sticky per key."""
    from prophet_amd.server import PSServer
    srv = PSServer(2, engine_lanes=3)
    sizes = [4000, 1000, 1000, 500, 3000, 100]
    load = [0, 0, 0]
    for k, s in enumerate(sizes):
        srv.init_key(k, s, DType.UINT8)
        want = min(range(3), key=lambda i: (load[i], i))
        load[want] += s
        assert srv.key_info(k)[1] == want
    srv.close()


def _init_round(srv, dt, N, sizes):
    for j, n in enumerate(sizes):
        ts = [threading.Thread(target=srv.push, args=(j, w, data(dt, n, w, 0, j), dt))
              for w in range(N)]       # init pushes block until all arrived
        for t in ts:
            t.start()
        for t in ts:
            t.join()


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
def test_pull_host_view_rounds(port, policy):
    """Zero-copy pull responses (byteps_server_pull_host_view, server.cc:42-70):
    one D2H per round into a pinned mirror; every worker's view is bit-exact
    with the oracle's fold in arrival order; a round-r view still holds round r
    after round r+1 finished (two mirrors by round parity); views and copying
    pulls count toward the same re-arm (server.cc:105-113)."""
    from prophet_amd.server import PSServer
    dt, N = DType.FLOAT32, 4
    sizes = [5, 1_000_003, 4_096_000 // 4]
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2, policy=policy)
    _init_round(srv, dt, N, sizes)
    held = {}
    for rnd in range(1, 5):
        for j, n in enumerate(sizes):
            order = random.Random(rnd * 10 + j).sample(range(N), N)
            for w in order:
                srv.push(j, w, data(dt, n, w, rnd, j), dt)
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, rnd, j) for w in order], n * es, dt)
            assert srv.key_info(j)[2] == order
            for w in range(N):
                if w == N - 1 and rnd % 2:          # a copying pull counts too
                    out = np.zeros(n * es, np.uint8)
                    srv.pull(j, out)
                    got = out
                else:
                    v = srv.pull_view(j)
                    assert v.readonly and v.nbytes == n * es
                    got = np.frombuffer(v, np.uint8)
                assert np.array_equal(got, want), f"round {rnd} key {j} worker {w}"
            if (rnd - 1, j) in held:   # previous round's view: other mirror, intact
                v0, w0 = held.pop((rnd - 1, j))
                assert np.array_equal(np.frombuffer(v0, np.uint8), w0)
            held[(rnd, j)] = (v, want.copy())
    srv.close()


def test_pull_host_view_async_and_errors(port):
    from prophet_amd.server import PSServer
    from prophet_amd.reducer import ReduceError
    dt, N, n = DType.FLOAT32, 2, 70_001
    with pytest.raises(ReduceError):
        with PSServer(N) as srv:
            srv.pull_view(99)                         # key not inited (server.cc:282)
    srv = PSServer(N, async_mode=True)
    init = data(dt, n, 0, 0, 0)          # same init data from both: store = it
    ts = [threading.Thread(target=srv.push, args=(0, w, init, dt)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    acc = init.view(np.float32).copy()
    for w in (1, 0, 1):
        srv.push(0, w, data(dt, n, w, 7, 0), dt)
        acc += data(dt, n, w, 7, 0).view(np.float32)
        v = srv.pull_view(0)                           # async: answered at once
        assert np.array_equal(np.frombuffer(v, np.uint8), acc.view(np.uint8))
    srv.close()


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
def test_pull_async_queued_until_round_finishes(port, policy):
    """byteps_server_pull_async: pulls issued before the round's pushes are
    queued (q_pull_reqmeta_, server.cc:303-304) and answered by the responder
    once the round finishes (server.cc:100-114) — never earlier; views are
    bit-exact with the oracle fold in arrival order; callbacks count toward the
    re-arm together with blocking pulls, so the next round proceeds."""
    from prophet_amd.server import PSServer
    dt, N = DType.FLOAT16, 4
    sizes = [3, 262_147]
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2, policy=policy)
    _init_round(srv, dt, N, sizes)
    for rnd in range(1, 4):
        got, fired = {}, threading.Semaphore(0)

        def cb(key, view, status, w=None):
            got[(w, key)] = (status, None if view is None else bytes(view))
            fired.release()
        nasync = 0
        for j in range(len(sizes)):
            for w in range(N):
                if rnd == 2 and w == 0:
                    continue                       # this one pulls blocking, below
                srv.pull_async(j, lambda k, v, st, w=w: cb(k, v, st, w))
                nasync += 1
        wants = {}
        for j, n in enumerate(sizes):
            order = random.Random(rnd * 7 + j).sample(range(N), N)
            for i, w in enumerate(order):
                if i == N - 1:
                    time.sleep(0.05)
                    assert not any(k[1] == j for k in got), "answered before the round finished"
                srv.push(j, w, data(dt, n, w, rnd, j), dt)
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, rnd, j) for w in order], n * es, dt)
            wants[j] = want
            if rnd == 2:
                out = np.zeros(n * es, np.uint8)
                srv.pull(j, out)
                got[(0, j)] = (0, out.tobytes())
        for _ in range(nasync):
            assert fired.acquire(timeout=30)
        for j in range(len(sizes)):
            for w in range(N):
                st, b = got[(w, j)]
                assert st == 0
                assert np.array_equal(np.frombuffer(b, np.uint8), wants[j]), (rnd, j, w)
        for j in range(len(sizes)):
            assert srv.key_info(j)[0] == rnd
    srv.close()


def test_pull_async_cancelled_at_shutdown_and_async_mode(port):
    from prophet_amd.reducer import ECANCELED
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 1000
    srv = PSServer(N)
    _init_round(srv, dt, N, [n])
    seen = []
    done = threading.Event()
    srv.pull_async(0, lambda k, v, st: (seen.append((k, v, st)), done.set()))
    srv.push(0, 1, data(dt, n, 1, 1, 0), dt)       # round 1 never completes
    srv.close()
    assert done.wait(10) and seen == [(0, None, ECANCELED)]

    srv = PSServer(N, async_mode=True)
    init = data(dt, n, 0, 0, 0)
    ts = [threading.Thread(target=srv.push, args=(0, w, init, dt)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    srv.push(0, 0, data(dt, n, 0, 5, 0), dt)
    box = []
    ev = threading.Event()
    srv.pull_async(0, lambda k, v, st: (box.append((st, bytes(v))), ev.set()))
    assert ev.wait(10)
    want = (init.view(np.float32) + data(dt, n, 0, 5, 0).view(np.float32)).view(np.uint8)
    assert box[0][0] == 0 and np.array_equal(np.frombuffer(box[0][1], np.uint8), want)
    srv.close()


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
def test_push_async_rounds(port, policy):
    """byteps_server_push_async: arrival order = call order (init: the store is
    the LAST call's data, server.cc:175-199), the fold runs behind the H2D copies
    on the device, the acknowledgement (server.cc:255) comes once the bytes are
    in HBM — the test then scribbles over the sender's buffer, and the round's
    result must not change; blocking pulls, views and async pulls all agree."""
    from prophet_amd.server import PSServer
    dt, N = DType.FLOAT32, 4
    sizes = [9, 500_003]
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2, policy=policy)
    acks = threading.Semaphore(0)
    status = []

    def ack(key, w, st, buf=None):
        status.append(st)
        if buf is not None:
            buf[:] = 0xEE                       # the sender reuses its buffer
        acks.release()
    for j, n in enumerate(sizes):                # init round, non-blocking
        for w in range(N):
            b = data(dt, n, w, 0, j).copy()
            srv.push_async(j, w, b, dt, lambda k, ww, st, b=b: ack(k, ww, st, b))
    for _ in range(N * len(sizes)):
        assert acks.acquire(timeout=30)
    for rnd in range(1, 4):
        for j, n in enumerate(sizes):
            order = random.Random(100 * rnd + j).sample(range(N), N)
            for w in order:
                b = data(dt, n, w, rnd, j).copy()
                srv.push_async(j, w, b, dt, lambda k, ww, st, b=b: ack(k, ww, st, b))
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, rnd, j) for w in order], n * es, dt)
            for w in range(N):
                if w == 0:
                    out = np.zeros(n * es, np.uint8)
                    srv.pull(j, out)
                else:
                    out = np.frombuffer(srv.pull_view(j), np.uint8)
                assert np.array_equal(out, want), (rnd, j, w)
            assert srv.key_info(j)[2] == order
        for _ in range(N * len(sizes)):
            assert acks.acquire(timeout=30)
    assert status and all(st == 0 for st in status)
    # round 1's expected values were built from the init stores: init = last call
    srv.close()


def test_push_async_init_store_is_last_call(port):
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT16, 3, 4099
    srv = PSServer(N)
    done = threading.Semaphore(0)
    for w in (2, 0, 1):                          # worker 1's init push arrives last
        srv.push_async(0, w, data(dt, n, w, 0, 0), dt, lambda k, ww, st: done.release())
    for _ in range(N):
        assert done.acquire(timeout=30)
    for w in range(N):
        srv.push_async(0, w, np.zeros(n * 2, np.uint8), dt)
    out = np.zeros(n * 2, np.uint8)
    srv.pull(0, out)                             # 0 + 0 + 0 in fp16: +0 bits
    assert not out.any()
    assert srv.key_info(0)[0] == 1
    srv.close()


def test_push_async_error_returns_buffer(port):
    """A state-machine error (a second init push from one worker) is reported
    by push_async itself, after its queued copy has finished."""
    from prophet_amd.reducer import ReduceError
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 1000
    srv = PSServer(N)
    srv.push_async(0, 0, data(dt, n, 0, 0, 0), dt)
    with pytest.raises(ReduceError):
        srv.push_async(0, 0, data(dt, n, 0, 0, 0), dt)
    srv.close()
