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


@pytest.mark.parametrize("schedule", [False, True], ids=["fifo", "schedule"])
@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16], ids=lambda d: DType(d).name)
def test_sync_rounds_concurrent_workers(port, policy, dt, schedule):
    """... also with BYTEPS_SERVER_ENABLE_SCHEDULE (engine threads issuing
    queued folds by priority, queue.h:68-97): same bits."""
    from prophet_amd.server import PSServer
    N, R = 8, 3
    sizes = [1, 7, 1000, 65_536 + 3, 1_000_003]    # elements per key
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=4, policy=policy, enable_schedule=schedule)
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


def test_pull_into_async_rules_and_cancel(port):
    """byteps_server_pull_into_async: refused for pageable host memory, in async mode,
    with scheduling or engine blocking, and for more bytes than the key; a
    pull parked for a round that never finishes is answered ECANCELED at
    shutdown; one queued after the round finished is copied and answered."""
    from prophet_amd.reducer import ECANCELED, ReduceError
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 5003
    dev = torch.device("cuda:0")
    for kw in ({"async_mode": True}, {"enable_schedule": True}, {"engine_blocking": True}):
        srv = PSServer(N, **kw)
        srv.init_key(1, n * 4, dt)
        with pytest.raises(ReduceError):
            srv.pull_into_async(1, torch.empty(n * 4, dtype=torch.uint8, device=dev))
        srv.close()
    srv = PSServer(N)
    srv.push_async(1, 0, data(dt, n, 0, 0, 1), dt)         # init: worker 1 arrives last
    srv.push(1, 1, data(dt, n, 1, 0, 1), dt)
    with pytest.raises(ReduceError):                       # host memory
        srv.pull_into_async(1, np.zeros(n * 4, np.uint8))
    with pytest.raises(ReduceError):                       # more than the key
        srv.pull_into_async(1, torch.empty(n * 4 + 4, dtype=torch.uint8, device=dev))
    got, done = [], threading.Semaphore(0)

    def cb(k, st):
        got.append((k, st))
        done.release()
    out = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    srv.pull_into_async(1, out, cb)                        # parked until round 1 finishes
    time.sleep(0.2)
    assert got == []
    for w in (1, 0):                                       # round 1, worker 1 first
        srv.push(1, w, data(dt, n, w, 1, 1), dt)
    assert done.acquire(timeout=30)
    assert got == [(1, 0)]
    torch.cuda.synchronize()
    want = np.zeros(n * 4, np.uint8)
    port.sum_n(want, [data(dt, n, w, 1, 1) for w in (1, 0)], n * 4, dt)
    assert np.array_equal(out.cpu().numpy(), want)
    pinned = torch.zeros(n * 4, dtype=torch.uint8, pin_memory=True)
    srv.pull_into_async(1, pinned, cb)      # the round is finished: at once, into pinned host
    assert done.acquire(timeout=30)         # memory through its device view
    assert np.array_equal(pinned.numpy(), want)
    srv.push(1, 0, data(dt, n, 0, 2, 1), dt)               # round 2: one push of two
    srv.pull_into_async(1, out, cb)                        # parked: never finishes
    time.sleep(0.2)
    assert len(got) == 2
    srv.close()
    assert done.acquire(timeout=30)
    assert got[2] == (1, ECANCELED)


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


def test_push_async_init_acks_wait_for_all_init_pushes(port):
    """server.cc:184-198: init pushes are answered only once all NumWorkers
    init pushes are in (a barrier for the workers, operations.cc:301-302).
    A worker that pushes its round-1 push before the other init pushes
    arrived waits inside the call (its slot still holds the init push), and
    the round is then folded normally."""
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 100_003
    srv = PSServer(N)
    acks = []
    got = threading.Semaphore(0)

    def ack(k, w, st, tag):
        acks.append((tag, w, st))
        got.release()
    srv.push_async(0, 0, data(dt, n, 0, 0, 0), dt, lambda k, w, st: ack(k, w, st, "init"))
    time.sleep(0.3)
    assert acks == []                      # worker 1's init push is missing
    early = threading.Thread(target=srv.push_async,
                             args=(0, 0, data(dt, n, 0, 1, 0), dt,
                                   lambda k, w, st: ack(k, w, st, "r1")))
    early.start()
    time.sleep(0.3)
    assert early.is_alive() and acks == []   # held: its slot still holds the init push
    srv.push_async(0, 1, data(dt, n, 1, 0, 0), dt, lambda k, w, st: ack(k, w, st, "init"))
    early.join(timeout=30)
    assert not early.is_alive()
    for _ in range(3):
        assert got.acquire(timeout=30)
    assert sorted(acks[:2]) == [("init", 0, 0), ("init", 1, 0)]
    assert acks[2] == ("r1", 0, 0)
    srv.push(0, 1, data(dt, n, 1, 1, 0), dt)
    out = np.zeros(n * 4, np.uint8)
    srv.pull(0, out)
    assert srv.key_info(0)[2] == [0, 1]
    want = np.zeros(n * 4, np.uint8)
    port.sum_n(want, [data(dt, n, w, 1, 0) for w in (0, 1)], n * 4, dt)
    assert np.array_equal(out, want)
    srv.close()


def test_pull_answer_then_immediate_next_round_push():
    """The responder counts a pull BEFORE calling back (server.cc:100-113
    counts under the lock that sends the answer).  Each worker pushes the next
    round the moment its answers arrive, so a round can complete right after
    the last answer; a count made after the callback would then land on the
    new round, re-arm the key one pull early and leave a worker's pull
    unanswered.  Pulls of a round are issued once every worker has pushed it
    (after that barrier every earlier answer, hence every earlier count, is
    done)."""
    from prophet_amd.server import PSServer
    N, n, R, keys = 3, 4099, 40, 2
    dt = DType.INT32
    srv = PSServer(N, engine_lanes=2)
    for j in range(keys):
        ts = [threading.Thread(target=srv.push, args=(j, w, np.zeros(n, np.int32), dt))
              for w in range(N)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    errors, results = [], {}
    bar = threading.Barrier(N)

    def worker(w):
        try:
            for r in range(1, R + 1):
                for j in range(keys):
                    srv.push_async(j, w, np.full(n, 100 * r + w, np.int32), dt)
                bar.wait(timeout=60)
                evs = []
                for j in range(keys):
                    ev = threading.Event()
                    box = {}

                    def cb(k, view, st, box=box, ev=ev):
                        box["v"] = None if view is None else np.frombuffer(view, np.int32).copy()
                        box["st"] = st
                        ev.set()
                    srv.pull_async(j, cb)
                    evs.append((j, ev, box))
                for j, ev, box in evs:
                    assert ev.wait(30), f"worker {w} round {r} key {j}: no answer"
                    assert box["st"] == 0
                    results[(w, r, j)] = box["v"]
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=150)
    assert not any(t.is_alive() for t in ts), "deadlock"
    assert not errors, errors[:3]
    assert len(results) == N * R * keys
    for (w, r, j), v in results.items():
        assert (v == sum(100 * r + k for k in range(N))).all(), (w, r, j)
    srv.close()


def test_schedule_issue_order():
    """BYTEPS_SERVER_ENABLE_SCHEDULE (queue.h:68-97): with the lane held, queued
    SUM_RECV / COPY_MERGED jobs leave by (fewest counted pushes on the key,
    oldest) — a key whose round is complete (ClearCounter, server.cc:269-271)
    first — and the results stay the arrival-order folds."""
    from prophet_amd.server import PSServer
    dt, N, n = DType.INT32, 3, 10_000
    srv = PSServer(N, engine_lanes=1, policy=1, enable_schedule=True)
    for j in range(3):
        ts = [threading.Thread(target=srv.push, args=(j, w, np.zeros(n, np.int32), dt))
              for w in range(N)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert srv.debug_lane(0) == []                  # the init round is not queued
    srv.debug_lane(0, pause=1)
    val = lambda j, w: np.full(n, 1 + 10 * j + 100 * w, np.int32)   # noqa: E731
    srv.push(0, 0, val(0, 0), dt)                   # first arrival: accumulator, no job
    srv.push(0, 1, val(0, 1), dt)                   # job a: SUM_RECV key 0 (count 1)
    srv.push(1, 0, val(1, 0), dt)
    srv.push(1, 1, val(1, 1), dt)                   # job b: key 1
    srv.push(1, 2, val(1, 2), dt)                   # jobs c, d: SUM_RECV + COPY_MERGED, cleared
    srv.push(2, 0, val(2, 0), dt)
    srv.push(2, 1, val(2, 1), dt)                   # job e: key 2 (count 1)
    assert srv.debug_lane(0) == []                  # held: nothing issued yet
    srv.debug_lane(0, pause=0)
    out = np.zeros(n, np.int32)
    srv.pull(1, out)                                # key 1's round finished
    assert (out == sum(1 + 10 + 100 * w for w in range(N))).all()
    for j in (0, 2):
        srv.push(j, 2, val(j, 2), dt)
    for j in (0, 2):
        srv.pull(j, out)
        assert (out == sum(1 + 10 * j + 100 * w for w in range(N))).all()
    log = srv.debug_lane(0)
    assert log[:5] == [1, 1, 1, 0, 2], log
    srv.close()


def test_async_mode_pulls_never_torn(port):
    """Async mode: a blocking pull's copy is ordered before the lane's later
    folds (no fold lands mid-copy), and views come from a ring of
    num_workers + 1 mirrors, so the last num_workers views stay intact."""
    from prophet_amd.server import PSServer
    dt, N, n = DType.INT32, 3, 8 << 20
    srv = PSServer(N, async_mode=True, engine_lanes=1)
    ts = [threading.Thread(target=srv.push, args=(0, w, np.zeros(n, np.int32), dt))
          for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ones = np.ones(n, np.int32)
    stop = threading.Event()
    pushes = []

    def pusher():
        while not stop.is_set():
            srv.push(0, len(pushes) % N, ones, dt)
            pushes.append(1)
    t = threading.Thread(target=pusher)
    t.start()
    try:
        out = np.zeros(n, np.int32)
        seen = []
        for _ in range(12):
            srv.pull(0, out)
            assert (out == out[0]).all(), "torn pull"
            seen.append(int(out[0]))
        assert seen == sorted(seen)
        views = []
        for _ in range(N):
            v = np.frombuffer(srv.pull_view(0), np.int32)
            assert (v == v[0]).all(), "torn view"
            views.append((v, int(v[0])))
        for v, first in views:                 # the ring kept every one of them
            assert (v == first).all()
    finally:
        stop.set()
        t.join()
    srv.close()


def _fast_bucket(n, seed):
    return np.random.default_rng(seed).standard_normal(n, dtype=np.float32).view(np.uint8)


@pytest.mark.parametrize("transport", ["host", "device_zero_copy"])
@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
@pytest.mark.parametrize("layout", ["1key", "17keys"])
def test_cfg1_two_workers_64mib(port, policy, layout, transport):
    """BASELINE config 1 at its own workload: 2 workers push fp32 64 MiB each,
    as ONE key, or split into BytePS's 4,096,000-B partitions (17 keys,
    global.cc:128-135) on 4 engine lanes; each worker pushes then pulls every
    key from its own thread; 2 rounds after init.  ``host``: pushes from host
    buffers, copying pulls.  ``device_zero_copy``: each round's bytes written
    straight into the receive slots (recv_slot, as an RDMA transport would),
    announced with push_ready, pulled as device views of the store.  Every
    pulled byte equals the oracle's left fold in the recorded arrival order
    (server.cc:147-308)."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    red = GpuReducer(device=0)
    zc = transport == "device_zero_copy"
    dt, N, B, R = DType.FLOAT32, 2, 64 << 20, 2
    parts = [(0, B)] if layout == "1key" else \
        [(o, min(4_096_000, B - o)) for o in range(0, B, 4_096_000)]
    assert len(parts) == (1 if layout == "1key" else 17)
    srv = PSServer(N, engine_lanes=4, policy=policy)
    ins = {(w, r): _fast_bucket(B // 4, 1000 + 10 * r + w) for w in range(N) for r in range(R + 1)}
    outs = {(w, r): np.zeros(B, np.uint8) for w in range(N) for r in range(1, R + 1)}
    orders = {}
    errors = []
    bar = threading.Barrier(N + 1)

    def worker(w):
        try:
            for r in range(R + 1):
                if zc and r > 0:
                    src = torch.from_numpy(ins[(w, r)]).cuda()
                    torch.cuda.synchronize()
                    for j, (o, ln) in enumerate(parts):   # the transport's write
                        red.copy(srv.recv_slot(j, w), src[o:o + ln], ln)
                    torch.cuda.synchronize()
                    for j in range(len(parts)):
                        srv.push_ready(j, w)
                    del src
                else:
                    for j, (o, ln) in enumerate(parts):
                        srv.push(j, w, ins[(w, r)][o:o + ln], dt)
                bar.wait()
                bar.wait()
                if r == 0:
                    continue
                for j, (o, ln) in enumerate(parts):
                    if zc:
                        ptr, nb = srv.pull_device_view(j)
                        assert nb == ln
                        outs[(w, r)][o:o + ln] = _read_device(red, ptr, nb)
                    else:
                        srv.pull(j, outs[(w, r)][o:o + ln])
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    for r in range(R + 1):
        bar.wait()
        for j in range(len(parts)):
            rounds, _, order = srv.key_info(j)
            assert rounds == r
            orders[(r, j)] = order
        bar.wait()
    for t in ts:
        t.join()
    assert not errors, errors
    for r in range(1, R + 1):
        want = np.zeros(B, np.uint8)
        for j, (o, ln) in enumerate(parts):
            order = orders[(r, j)]
            assert sorted(order) == [0, 1]
            port.sum_n(want[o:o + ln], [ins[(w, r)][o:o + ln] for w in order], ln, dt)
        for w in range(N):
            assert np.array_equal(outs[(w, r)], want), (r, w)
    srv.close()


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
@pytest.mark.parametrize("dt", [DType.FLOAT16, DType.FLOAT32], ids=lambda d: DType(d).name)
def test_batched_calls_many_keys(port, policy, dt):
    """push_many / push_ready_many / pull_many (server.h batched calls): 6
    worker threads x 40 keys of mixed sizes on 3 lanes, device-resident, three
    rounds (the first from host buffers through push_many's per-key path);
    every pulled byte equals the oracle's fold in the recorded arrival order,
    and the rounds complete in any interleaving of the workers' batches."""
    from prophet_amd.server import PSServer
    N, R = 6, 3
    sizes = [1 + (j * 7919) % 70_000 for j in range(40)]
    es = elem_size(dt)
    keys = list(range(100, 100 + len(sizes)))
    srv = PSServer(N, engine_lanes=3, policy=policy)
    dev = torch.device("cuda:0")
    host = {(w, r, j): data(dt, n, w, r, j) for w in range(N) for r in range(R + 1)
            for j, n in enumerate(sizes)}
    outs = {(w, r): [torch.empty(n * es, dtype=torch.uint8, device=dev) for n in sizes]
            for w in range(N) for r in range(1, R + 1)}
    bar = threading.Barrier(N + 1)
    errors, orders = [], {}

    def worker(w):
        try:
            srv.push_many(keys, w, [host[(w, 0, j)] for j in range(len(sizes))], dt)   # init
            for r in range(1, R + 1):
                if r == 1:      # host sources, per-key copies
                    srv.push_many(keys, w, [host[(w, r, j)] for j in range(len(sizes))], dt)
                else:           # device slots written directly, then one ready call
                    for j, k in enumerate(keys):
                        slot = srv.recv_slot(k, w)
                        _copy_to_ptr(slot, torch.from_numpy(host[(w, r, j)]).to(dev))
                    srv.push_ready_many(keys, w)
                srv.pull_many(keys, outs[(w, r)])
                bar.wait(timeout=120)
                bar.wait(timeout=120)
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    for r in range(1, R + 1):
        bar.wait(timeout=240)
        for j, k in enumerate(keys):
            rounds, _, order = srv.key_info(k)
            assert rounds == r
            orders[(r, j)] = order
        bar.wait(timeout=120)
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    for r in range(1, R + 1):
        for j, n in enumerate(sizes):
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [host[(w, r, j)] for w in orders[(r, j)]], n * es, dt)
            for w in range(N):
                assert_bytes_match(dt, outs[(w, r)][j].cpu().numpy(), want,
                                   nan_class_f32_f64=False, what=f"r{r} key {j} w{w}")
    srv.close()


@pytest.mark.parametrize("combine", ["1", "0"], ids=["issuer", "per_call"])
@pytest.mark.parametrize("dt", [DType.FLOAT16, DType.FLOAT32], ids=lambda d: DType(d).name)
def test_single_key_calls_issuer_batches(port, dt, combine, monkeypatch):
    """Single-key calls from 8 worker threads — push_ready into written slots
    and copying pulls into device memory, 60 keys on 4 lanes, three rounds —
    through the lanes' issuer threads (rounds and pulls that pile up go out as
    one batched launch each) and with BPSR_SERVER_COMBINE=0 (every call issues
    its own): every pulled byte equals the oracle's fold in the recorded
    arrival order.  With the issuer, every round is folded once and every pull
    answered once (telemetry), in no more launches than rounds."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_COMBINE", combine)
    N, R = 8, 3
    sizes = [1 + (j * 7919) % 50_000 for j in range(60)]
    es = elem_size(dt)
    keys = list(range(7, 7 + len(sizes)))
    srv = PSServer(N, engine_lanes=4)
    dev = torch.device("cuda:0")
    host = {(w, r, j): data(dt, n, w, r, j) for w in range(N) for r in range(R + 1)
            for j, n in enumerate(sizes)}
    outs = {(w, r): [torch.empty(n * es, dtype=torch.uint8, device=dev) for n in sizes]
            for w in range(N) for r in range(1, R + 1)}
    bar = threading.Barrier(N + 1)
    errors, orders = [], {}

    def worker(w):
        try:
            for j, k in enumerate(keys):    # init pushes, device sources
                srv.push(k, w, torch.from_numpy(host[(w, 0, j)]).to(dev), dt)
            for r in range(1, R + 1):
                for j, k in enumerate(keys):
                    _copy_to_ptr(srv.recv_slot(k, w), torch.from_numpy(host[(w, r, j)]).to(dev))
                bar.wait(timeout=120)       # every slot written: the round's pushes
                for k in keys:
                    srv.push_ready(k, w)
                for j, k in enumerate(keys):
                    srv.pull(k, outs[(w, r)][j])
                bar.wait(timeout=120)
                bar.wait(timeout=120)
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    st0 = srv.stats()     # init rounds count no fold (their store is a copy)
    for r in range(1, R + 1):
        bar.wait(timeout=240)
        bar.wait(timeout=240)
        for j, k in enumerate(keys):
            rounds, _, order = srv.key_info(k)
            assert rounds == r
            orders[(r, j)] = order
        bar.wait(timeout=120)
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    st = srv.stats()
    srv.close()
    for r in range(1, R + 1):
        for j, n in enumerate(sizes):
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [host[(w, r, j)] for w in orders[(r, j)]], n * es, dt)
            for w in range(N):
                assert_bytes_match(dt, outs[(w, r)][j].cpu().numpy(), want,
                                   nan_class_f32_f64=False, what=f"r{r} key {j} w{w}")
    folded = st["rounds_folded"] - st0["rounds_folded"]
    pulls = st["pulls"] - st0["pulls"]
    assert folded == R * len(keys) and pulls == R * len(keys) * N
    assert st["fold_launches"] - st0["fold_launches"] <= folded
    assert st["pull_launches"] - st0["pull_launches"] <= pulls


@pytest.mark.parametrize("combine,pull_mode", [("1", "blocking"), ("0", "blocking"),
                                               ("1", "into_async")],
                         ids=["issuer", "per_call", "issuer_pull_into_async"])
def test_push_async_device_copies_batched(port, combine, pull_mode, monkeypatch):
    """Non-blocking pushes of device data (server.h: after the init round the
    copies are the lane issuer's, batched): 6 worker threads x 50 keys x 3
    rounds, fp16, every push acknowledged once, then device pulls — blocking,
    or all queued with pull_into_async (parked until the round finishes,
    copied by the issuer) — every pulled byte equals the oracle's fold in
    arrival order; with the issuer the copies went out in fewer launches than
    pushes."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_COMBINE", combine)
    dt, N, R = DType.FLOAT16, 6, 3
    sizes = [1 + (j * 6007) % 40_000 for j in range(50)]
    keys = list(range(300, 300 + len(sizes)))
    srv = PSServer(N, engine_lanes=3)
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    outs = {(w, r): [torch.empty(n * 2, dtype=torch.uint8, device=dev) for n in sizes]
            for w in range(N) for r in range(1, R + 1)}
    torch.cuda.synchronize()
    acks = threading.Semaphore(0)
    bad = []

    def ack(k, w, st):
        if st:
            bad.append((k, w, st))
        acks.release()
    bar = threading.Barrier(N + 1)
    errors, orders = [], {}

    def worker(w):
        try:
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, 0, j)], dt)          # init round: blocking
            for r in range(1, R + 1):
                for j, k in enumerate(keys):
                    srv.push_async(k, w, src[(w, r, j)], dt, ack)
                if pull_mode == "into_async":   # every pull queued, answered later
                    got = threading.Semaphore(0)
                    for j, k in enumerate(keys):
                        srv.pull_into_async(k, outs[(w, r)][j],
                                            lambda kk, st: (bad.append((kk, st)) if st else None,
                                                            got.release()))
                    for _ in keys:
                        assert got.acquire(timeout=60)
                else:
                    for j, k in enumerate(keys):
                        srv.pull(k, outs[(w, r)][j])
                bar.wait(timeout=120)
                bar.wait(timeout=120)
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    st0 = srv.stats()
    for r in range(1, R + 1):
        bar.wait(timeout=240)
        for j, k in enumerate(keys):
            rounds, _, order = srv.key_info(k)
            assert rounds == r
            orders[(r, j)] = order
        bar.wait(timeout=120)
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    for _ in range(N * R * len(keys)):
        assert acks.acquire(timeout=30)
    assert not bad, bad[:5]
    st = srv.stats()
    srv.close()
    for r in range(1, R + 1):
        for j, n in enumerate(sizes):
            want = np.zeros(n * 2, np.uint8)
            port.sum_n(want, [data(dt, n, w, r, j) for w in orders[(r, j)]], n * 2, dt)
            for w in range(N):
                assert_bytes_match(dt, outs[(w, r)][j].cpu().numpy(), want,
                                   nan_class_f32_f64=False, what=f"r{r} key {j} w{w}")
    if combine == "1":
        launches = st.get("push_copy_launches", 0) - st0.get("push_copy_launches", 0)
        assert 1 <= launches <= N * R * len(keys)


@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16], ids=lambda d: DType(d).name)
def test_mixed_push_async_and_push_many_same_keys(port, dt):
    """Combining mode, the advisor's round-3 race: half the workers push device
    data with push_async (their copies into the slots queue on the lane
    issuer), the other half with push_many on the SAME keys.  A push_many that
    completes a round must not issue its fold ahead of a copy still queued on
    the issuer: every pulled byte equals the oracle's fold in the recorded
    arrival order, over several rounds of large keys (slow copies)."""
    from prophet_amd.server import PSServer
    N, R = 6, 4
    sizes = [(256 << 10) + 17 * j for j in range(24)]   # elements per key
    keys = list(range(900, 900 + len(sizes)))
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2)
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    outs = {(w, r): [torch.empty(n * es, dtype=torch.uint8, device=dev) for n in sizes]
            for w in range(N) for r in range(1, R + 1)}
    torch.cuda.synchronize()
    acks = threading.Semaphore(0)
    bad = []

    def ack(k, w, st):
        if st:
            bad.append((k, w, st))
        acks.release()
    bar = threading.Barrier(N + 1)
    errors, orders = [], {}

    def worker(w):
        try:
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, 0, j)], dt)          # init round: blocking
            for r in range(1, R + 1):
                if w % 2 == 0:
                    for j, k in enumerate(keys):
                        srv.push_async(k, w, src[(w, r, j)], dt, ack)
                    got = threading.Semaphore(0)
                    for j, k in enumerate(keys):
                        srv.pull_into_async(k, outs[(w, r)][j],
                                            lambda kk, st: (bad.append((kk, st)) if st else None,
                                                            got.release()))
                    for _ in keys:
                        assert got.acquire(timeout=60)
                else:
                    srv.push_many(keys, w, [src[(w, r, j)] for j in range(len(keys))], dt)
                    srv.pull_many(keys, outs[(w, r)])
                bar.wait(timeout=120)
                bar.wait(timeout=120)
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    for r in range(1, R + 1):
        bar.wait(timeout=240)
        for j, k in enumerate(keys):
            rounds, _, order = srv.key_info(k)
            assert rounds == r
            orders[(r, j)] = order
        bar.wait(timeout=120)
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    for _ in range((N // 2) * R * len(keys)):
        assert acks.acquire(timeout=30)
    assert not bad, bad[:5]
    srv.close()
    for r in range(1, R + 1):
        for j, n in enumerate(sizes):
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, r, j) for w in orders[(r, j)]], n * es, dt)
            for w in range(N):
                assert_bytes_match(dt, outs[(w, r)][j].cpu().numpy(), want,
                                   nan_class_f32_f64=False, what=f"r{r} key {j} w{w}")


def _copy_to_ptr(ptr, src):
    """Device copy of tensor `src` to raw device pointer `ptr` (the transport
    writing into a receive slot)."""
    from prophet_amd.reducer import GpuReducer
    GpuReducer().copy(ptr, src, src.numel() * src.element_size())
    torch.cuda.synchronize()


def test_batched_calls_async_mode(port):
    """Async mode through the batched calls: every push_many sums into the
    store; pull_many answers at once with the store as it stands."""
    from prophet_amd.server import PSServer
    dt, N = DType.INT32, 3
    sizes = [5, 40_000, 1_000_003]
    keys = [7, 8, 9]
    srv = PSServer(N, async_mode=True, engine_lanes=2)
    dev = torch.device("cuda:0")
    init = [torch.zeros(n, dtype=torch.int32, device=dev) for n in sizes]
    ts = [threading.Thread(target=srv.push_many, args=(keys, w, init, dt)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    for w in range(N):
        srv.push_many(keys, w, [torch.full((n,), w + 1, dtype=torch.int32, device=dev)
                                for n in sizes], dt)
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for n in sizes]
    srv.pull_many(keys, outs)
    for o in outs:
        assert (o == 6).all()
    srv.close()


def _read_device(red, ptr, nbytes):
    out = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    red.copy(out, ptr, nbytes)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("batched", [False, True], ids=["single", "push_many"])
@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
def test_pull_device_view_rounds(port, policy, batched):
    """byteps_server_pull_device_view: the store's own HBM, no copy (what a
    GPUDirect transport sends from).  Every round's view is bit-exact with the
    oracle's fold in arrival order — pushes one by one or through push_many
    (one batched fold per lane, the round published behind the lane's mark);
    views and copying pulls count toward the same re-arm (server.cc:105-113)."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    red = GpuReducer(device=0)
    dt, N = DType.FLOAT32, 3
    sizes = [3, 1_000_003, 4_096_000 // 4]
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2, policy=policy)
    _init_round(srv, dt, N, sizes)
    for rnd in range(1, 5):
        order = random.Random(rnd).sample(range(N), N)
        for w in order:
            if batched:
                srcs = [torch.from_numpy(data(dt, n, w, rnd, j)).cuda()
                        for j, n in enumerate(sizes)]
                torch.cuda.synchronize()               # the server's copies use its own streams
                srv.push_many(list(range(len(sizes))), w, srcs, dt)
                torch.cuda.synchronize()
                del srcs
            else:
                for j, n in enumerate(sizes):
                    srv.push(j, w, data(dt, n, w, rnd, j), dt)
        for j, n in enumerate(sizes):
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, rnd, j) for w in order], n * es, dt)
            for w in range(N):
                if w == 0 and rnd % 2:                 # a copying pull counts too
                    out = np.zeros(n * es, np.uint8)
                    srv.pull(j, out)
                    got = out
                else:
                    ptr, nb = srv.pull_device_view(j)
                    assert nb == n * es and ptr
                    got = _read_device(red, ptr, nb)
                assert np.array_equal(got, want), f"round {rnd} key {j} worker {w}"
    srv.close()


def test_pull_device_view_held_until_own_push(port):
    """A worker's device view still holds round r while the other workers push
    round r + 1 — the store is rewritten only by the fold its own push
    completes — and async mode refuses device views."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    red = GpuReducer(device=0)
    dt, N, n = DType.FLOAT32, 3, 500_001
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=1)
    _init_round(srv, dt, N, [n])
    for w in range(N):
        srv.push(0, w, data(dt, n, w, 1, 0), dt)
    want1 = np.zeros(n * es, np.uint8)
    port.sum_n(want1, [data(dt, n, w, 1, 0) for w in range(N)], n * es, dt)
    views = [srv.pull_device_view(0) for _ in range(N)]      # every worker pulls round 1
    assert len({p for p, _ in views}) == 1
    ptr, nb = views[-1]
    for w in range(N - 1):                                    # round 2 without worker N-1
        srv.push(0, w, data(dt, n, w, 2, 0), dt)
    torch.cuda.synchronize()
    assert np.array_equal(_read_device(red, ptr, nb), want1)   # still round 1
    srv.push(0, N - 1, data(dt, n, N - 1, 2, 0), dt)            # completes round 2
    want2 = np.zeros(n * es, np.uint8)
    port.sum_n(want2, [data(dt, n, w, 2, 0) for w in range(N)], n * es, dt)
    p2, _ = srv.pull_device_view(0)
    assert np.array_equal(_read_device(red, p2, nb), want2)
    srv.close()
    from prophet_amd.reducer import ReduceError
    with PSServer(2, async_mode=True) as a:
        _init_round(a, dt, 2, [16])
        with pytest.raises(ReduceError, match="sync mode"):
            a.pull_device_view(0)


@pytest.mark.parametrize("fail_after", [0, 1], ids=["init_copy", "round_fold"])
def test_fold_failure_fails_waiters_instead_of_hanging(monkeypatch, fail_after):
    """with scheduling off a fold that cannot be issued must fail
    the key (fail_key), else the other workers wait forever.  Fault injection
    (BPSR_SERVER_FAIL_AFTER=n: the (n+1)-th fold issue fails): 0 = the init
    copy fails while worker 0's init push waits for the barrier; 1 = round 1's
    fused fold fails while worker 0 waits in a pull.  Every waiter returns the
    error; later calls on the key return it too."""
    from prophet_amd.reducer import EHIP, ReduceError
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_FAIL_AFTER", str(fail_after))
    dt, n = DType.FLOAT32, 4096
    srv = PSServer(2, engine_lanes=1)
    out = {}

    def waiter():
        try:
            if fail_after == 0:
                srv.push(5, 0, data(dt, n, 0, 0, 5), dt)          # blocks: init barrier
            else:
                srv.pull(5, np.zeros(n * 4, np.uint8))           # blocks: round 1
            out["w"] = 0
        except ReduceError as e:
            out["w"] = e.code
    if fail_after == 1:
        t0 = threading.Thread(target=srv.push, args=(5, 0, data(dt, n, 0, 0, 5), dt))
        t0.start()
        srv.push(5, 1, data(dt, n, 1, 0, 5), dt)                 # init round completes
        t0.join(timeout=60)
        srv.push(5, 0, data(dt, n, 0, 1, 5), dt)                 # round 1, first arrival
    t = threading.Thread(target=waiter)
    t.start()
    time.sleep(0.2)                                              # the waiter is blocked
    if fail_after == 0:
        with pytest.raises(ReduceError) as ei:
            srv.push(5, 1, data(dt, n, 1, 1, 5), dt)             # completes -> copy fails
        assert ei.value.code == EHIP and "injected" in str(ei.value)
    else:
        # the round's fold is the lane issuer's (server.h): the completing push
        # may return before the fold is issued; the failure then reaches the
        # waiting pull and every later call on the key
        try:
            srv.push(5, 1, data(dt, n, 1, 1, 5), dt)             # completes -> fold fails
        except ReduceError as e:
            assert e.code == EHIP and "injected" in str(e)
    t.join(timeout=30)
    assert not t.is_alive(), "waiter hung after the failed fold"
    assert out["w"] == EHIP
    with pytest.raises(ReduceError) as ei:
        srv.pull(5, np.zeros(n * 4, np.uint8))
    assert ei.value.code == EHIP
    srv.close()


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
def test_engine_blocking_mode(port, policy):
    """BYTEPS_SERVER_ENGINE_BLOCKING (server.cc:205-262, 284-285): a push
    returns once its copy / sum / fold has completed, and a pull is answered
    at once from the store as it stands — a pull before the round's last push
    sees the previous round (the reference's ungated SendPullResponse), one
    after it sees the new left fold; pulls are not counted, so any number of
    them never blocks the next round."""
    from prophet_amd.server import PSServer, config_from_env
    dt, n, N = DType.FLOAT32, 70_001, 3
    srv = PSServer(N, engine_lanes=2, policy=policy, engine_blocking=True)
    init = [data(dt, n, w, 0, 9) for w in range(N)]
    ts = [threading.Thread(target=srv.push, args=(9, w, init[w], dt)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    out = np.zeros(n * 4, np.uint8)
    srv.pull(9, out)
    assert any(np.array_equal(out, x) for x in init)    # init store = last init arrival
    prev = out.copy()
    for rnd in (1, 2, 3):
        ins = [data(dt, n, w, rnd, 9) for w in range(N)]
        order = [(rnd + k) % N for k in range(N)]
        for i, w in enumerate(order):
            srv.push(9, w, ins[w], dt)
            if i < N - 1:
                for _ in range(2):                       # ungated, uncounted pulls
                    srv.pull(9, out)
                    assert np.array_equal(out, prev), (rnd, i)
        want = np.zeros(n * 4, np.uint8)
        port.sum_n(want, [ins[w] for w in order], want.nbytes, dt)
        srv.pull(9, out)
        assert np.array_equal(out, want), rnd
        view = np.frombuffer(srv.pull_view(9), np.uint8)
        assert np.array_equal(view, want), rnd
        prev = want
    srv.close()
    import os
    os.environ["BYTEPS_SERVER_ENGINE_BLOCKING"] = "1"
    try:
        assert config_from_env().engine_blocking == 1
    finally:
        del os.environ["BYTEPS_SERVER_ENGINE_BLOCKING"]


def test_blocking_device_calls_from_a_callback(port):
    """Blocking device pushes and pulls are served by the lane issuer and the
    responder (the caller waits without a HIP call).  One made from inside a
    callback — on the responder thread itself — takes the direct path instead
    of waiting on itself: a pull_async callback that makes the other worker's
    blocking device pull completes, and both answers are the oracle's fold."""
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 100_003
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=1)
    _init_round(srv, dt, N, [n])
    dev = torch.device("cuda", 0)
    for rnd in range(1, 3):
        out = torch.zeros(n * es, dtype=torch.uint8, device=dev)
        res, fired = {}, threading.Semaphore(0)

        def cb(key, view, status):
            res["async"] = (status, None if view is None else bytes(view))
            srv.pull(key, out)                      # blocking, on the responder thread
            torch.cuda.synchronize()
            res["blocking"] = out.cpu().numpy().tobytes()
            fired.release()
        srv.pull_async(0, cb)
        ins = [data(dt, n, w, rnd, 0) for w in range(N)]
        for w in range(N):                          # blocking device pushes
            srv.push(0, w, torch.from_numpy(ins[w].copy()).to(dev), dt)
        assert fired.acquire(timeout=60)
        want = np.zeros(n * es, np.uint8)
        port.sum_n(want, ins, n * es, dt)
        assert res["async"][0] == 0
        assert np.array_equal(np.frombuffer(res["async"][1], np.uint8), want)
        assert np.array_equal(np.frombuffer(res["blocking"], np.uint8), want)
        assert srv.key_info(0)[0] == rnd
    srv.close()


def test_order_after_orders_running_producer_without_host_wait():
    """The Python entry orders the caller's producers with an event the
    server's streams wait on (byteps_server_order_after), not a host stall: a
    producer still running on the caller's stream (a long spin, then the
    fill) is ordered before the pushes, which return while it still runs, and
    the round folds the filled values."""
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 1 << 20
    srv = PSServer(N)
    dev = torch.device("cuda:0")
    xs = [torch.zeros(n, device=dev) for _ in range(N)]
    torch.cuda.synchronize()
    srv.push_async(5, 0, xs[0], dt)                     # init round (answered when all are in)
    srv.push(5, 1, xs[1], dt)
    torch.cuda.synchronize()
    torch.cuda._sleep(400_000_000)                      # ~0.2 s on the current stream
    xs[0].fill_(1.5)
    xs[1].fill_(2.25)
    acks = threading.Semaphore(0)
    for w in range(N):
        srv.push_async(5, w, xs[w], dt, lambda k, ww, st: acks.release())
    still_running = not torch.cuda.current_stream(dev).query()
    out = torch.empty(n, device=dev)
    srv.pull(5, out)
    for _ in range(N):
        assert acks.acquire(timeout=30)
    assert still_running, "the pushes waited for the producer on the host"
    assert torch.all(out == 3.75)
    srv.close()


@pytest.mark.parametrize("service", ["1", "0"], ids=["copy_service", "lane_copies"])
def test_blocking_device_pulls_through_copy_service(port, service, monkeypatch):
    """Blocking pulls into this device's memory (combining mode) are served by
    the pull copy service (a persistent kernel fed through a pinned job ring):
    bit-exact at every size, from one element to a key of many 256 KiB jobs,
    into destinations at byte offsets 0..2 (vector, word and byte copies);
    across the service's idle exit and relaunch (a pause between rounds); and
    behind order_after — the destination's previous writer (a long spin, then
    a fill on the caller's stream) lands before the copy.  PyTorch's default
    stream does not wait for a running service.  BPSR_SERVER_PULL_SERVICE=0
    serves the same pulls with lane copies."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_PULL_SERVICE", service)
    dt, N, R = DType.FLOAT16, 3, 3
    sizes = [1, 8, 1001, 131_072 + 5, 1_500_007]                # elements per key
    keys = list(range(70, 70 + len(sizes)))
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2)
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    bufs = {(w, j): torch.zeros(n * es + 8, dtype=torch.uint8, device=dev)
            for w in range(N) for j, n in enumerate(sizes)}
    torch.cuda.synchronize()
    bar = threading.Barrier(N + 1)
    errors, pulled, stream_s = [], {}, []

    def worker(w):
        try:
            rng = random.Random(900 + w)
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, 0, j)], dt)              # init round
            for r in range(1, R + 1):
                order = list(range(len(keys)))
                rng.shuffle(order)
                for j in order:
                    srv.push(keys[j], w, src[(w, r, j)], dt)
                bar.wait(timeout=120)                           # main reads the orders
                for j in order:
                    off = (w + j + r) % 3
                    n = sizes[j] * es
                    dst = bufs[(w, j)][off:off + n]
                    if j == len(sizes) - 1 and w == 0:
                        torch.cuda._sleep(50_000_000)           # the previous writer, still running
                    dst.fill_(0xAB)
                    srv.pull(keys[j], dst)
                    if r == R and w == 0:   # right after a pull: the service is running
                        t0 = time.perf_counter()
                        x = torch.ones(1024, device=dev)
                        x.add_(1)
                        torch.cuda.current_stream(dev).synchronize()
                        stream_s.append(time.perf_counter() - t0)
                    pulled[(w, r, j)] = dst.cpu().numpy().copy()
                bar.wait(timeout=120)
                if r == 1:
                    time.sleep(0.05)                            # the service exits idle
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    orders = {}
    try:
        for r in range(1, R + 1):
            bar.wait(timeout=120)
            for j, k in enumerate(keys):
                rounds, _, order = srv.key_info(k)
                assert rounds == r and sorted(order) == list(range(N))
                orders[(r, j)] = order
            bar.wait(timeout=120)
    except threading.BrokenBarrierError:
        raise AssertionError(f"worker failed: {errors}")
    finally:
        for t in ts:
            t.join(timeout=60)
    assert not errors, errors
    st = srv.stats()
    srv.close()
    for r in range(1, R + 1):
        for j, n in enumerate(sizes):
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, r, j) for w in orders[(r, j)]], n * es, dt)
            for w in range(N):
                assert_bytes_match(dt, pulled[(w, r, j)], want, nan_class_f32_f64=False,
                                   what=f"r{r} key {j} w{w}")
    total = N * R * len(keys)
    if service == "1":
        assert st["service_pulls"] == total
        assert st["service_launches"] >= 2                      # the idle exit, then a relaunch
    else:
        assert st["service_pulls"] == 0 and st["service_launches"] == 0
    # the default stream's work did not wait for the running service
    assert len(stream_s) == len(keys) and sorted(stream_s)[len(keys) // 2] < 0.05, stream_s


def test_copy_service_give_up_falls_back_to_lane_copies(port, monkeypatch):
    """The copy service's give-up path: with BPSR_COPYSVC_TEST_STALL_MS the
    service's copiers hold every job 3 x that many ms and a job is given up
    after that many ms.  The pull that met the stalled service still
    completes, through the key's lane stream, and every later pull goes to
    lane copies directly; every pulled byte equals the oracle's left fold; the
    held job is never copied once the pull has returned."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_PULL_SERVICE", "1")
    monkeypatch.setenv("BPSR_COPYSVC_TEST_STALL_MS", "100")
    dt, N, R = DType.FLOAT32, 2, 3
    sizes = [1, 1001, 300_007]
    keys = list(range(140, 140 + len(sizes)))
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=2)
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    torch.cuda.synchronize()
    acks = threading.Semaphore(0)

    def push_all(r, j, k):       # a blocking push may wait for the other workers'
        for w in range(N):
            srv.push_async(k, w, src[(w, r, j)], dt, lambda kk, ww, st: acks.release())
        for _ in range(N):
            assert acks.acquire(timeout=30)

    for j, k in enumerate(keys):
        push_all(0, j, k)                                       # init round
    first_s = None
    for r in range(1, R + 1):
        for j, k in enumerate(keys):
            push_all(r, j, k)
            _, _, order = srv.key_info(k)
            want = np.zeros(sizes[j] * es, np.uint8)
            port.sum_n(want, [data(dt, sizes[j], w, r, j) for w in order], sizes[j] * es, dt)
            for w in range(N):
                out = torch.full((sizes[j],), -1.0, device=dev)
                t0 = time.perf_counter()
                srv.pull(k, out)
                if first_s is None:
                    first_s = time.perf_counter() - t0
                    first_out = out                             # the held job's destination
                assert_bytes_match(dt, out.cpu().numpy().view(np.uint8), want,
                                   nan_class_f32_f64=False, what=f"r{r} key {j} w{w}")
            if r == 1 and j == 0:
                # The copiers hold every job 3 x 100 ms and would then copy it.
                # The give-up waited for the service launch to end (the stop
                # dropped the held job), so the buffer the fallback filled is
                # the caller's again: a late service copy would overwrite the
                # marker written here.
                first_out.fill_(-7.0)
                torch.cuda.synchronize()
                time.sleep(0.45)
                assert torch.all(first_out == -7.0), "the copy service wrote after its give-up"
    st = srv.stats()
    srv.close()
    assert first_s >= 0.09, first_s                            # the first pull met the stall
    assert st["service_pulls"] == 0 and st["service_launches"] >= 1
    assert st["pulls"] == N * R * len(keys)


def test_device_sync_bounded_while_threads_pull_through_service(port):
    """include/bpsr/server.h: a device-wide synchronisation elsewhere in the
    process (torch.cuda.synchronize = hipDeviceSynchronize) waits for a
    running copy service at most its remaining age plus one relaunch's (the
    service's age limit is 1 ms).  8 worker threads push and pull 4 device
    keys through the service continuously while the main thread times 150
    device synchronisations; every pulled byte of the last round equals the
    oracle's fold in the recorded arrival order."""
    import sys
    from prophet_amd.server import PSServer
    dt, N = DType.FLOAT32, 8
    sizes = [16, 1000, 65_536, 300_007]
    keys = list(range(200, 200 + len(sizes)))
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=4)
    dev = torch.device("cuda:0")
    src = {(w, j): torch.from_numpy(data(dt, n, w, 5, j)).to(dev)
           for w in range(N) for j, n in enumerate(sizes)}
    outs = {(w, j): torch.empty(n, dtype=torch.float32, device=dev)
            for w in range(N) for j, n in enumerate(sizes)}
    torch.cuda.synchronize()
    stop = threading.Event()
    flag = [False]
    bar = threading.Barrier(N, action=lambda: flag.__setitem__(0, stop.is_set()))
    errors, rounds = [], [0] * N

    def worker(w):
        try:
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, j)], dt)                 # init round
            while True:
                bar.wait(timeout=60)
                if flag[0]:
                    return
                for j, k in enumerate(keys):
                    srv.push(k, w, src[(w, j)], dt)
                for j, k in enumerate(keys):
                    srv.pull(k, outs[(w, j)])
                rounds[w] += 1
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    old_switch = sys.getswitchinterval()
    sys.setswitchinterval(1e-4)          # the timing thread gets the GIL back promptly
    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    sync_s = []
    try:
        for t in ts:
            t.start()
        t_end = time.perf_counter() + 30
        while srv.stats()["service_pulls"] < 200 and time.perf_counter() < t_end and not errors:
            time.sleep(0.001)
        for _ in range(150):
            if errors:
                break
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            sync_s.append(time.perf_counter() - t0)
            time.sleep(0.002)
    finally:
        stop.set()
        for t in ts:
            t.join(timeout=60)
        sys.setswitchinterval(old_switch)
    assert not errors, errors
    st = srv.stats()
    orders = {j: srv.key_info(k)[2] for j, k in enumerate(keys)}
    srv.close()
    assert st["service_pulls"] >= 1000, st
    sync_s.sort()
    # before the age limit (2 s) a synchronisation under continuous pulls
    # waited for the whole launch
    assert sync_s[len(sync_s) // 2] < 0.004 and sync_s[-1] < 0.010, sync_s[-10:]
    for j, n in enumerate(sizes):
        want = np.zeros(n * es, np.uint8)
        port.sum_n(want, [data(dt, n, w, 5, j) for w in orders[j]], n * es, dt)
        for w in range(N):
            assert_bytes_match(dt, outs[(w, j)].cpu().numpy().view(np.uint8), want,
                               nan_class_f32_f64=False, what=f"key {j} w{w}")


def test_copy_service_many_rounds_racing_pullers(port):
    """The pull copy service under load: 4 worker threads, 24 keys of random
    sizes (1 element … 700 K fp32, so jobs of 1 … 11 chunks), 12 rounds; each
    worker pushes every key, then pulls every key into its own device buffer
    in its own random order, sometimes pausing past the service's idle exit —
    thousands of jobs from racing posters, relaunches included.  Every pulled
    byte equals the oracle's left fold in the recorded arrival order."""
    from prophet_amd.server import PSServer
    dt, N, R = DType.FLOAT32, 4, 12
    rng0 = random.Random(77)
    sizes = [rng0.choice([1, 3, 1000, 16_384, 70_001, 300_000, 700_000]) for _ in range(24)]
    keys = list(range(200, 200 + len(sizes)))
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=4)
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    outs = {(w, j): torch.empty(n * es, dtype=torch.uint8, device=dev)
            for w in range(N) for j, n in enumerate(sizes)}
    torch.cuda.synchronize()
    bar = threading.Barrier(N + 1)
    errors, pulled = [], {}

    def worker(w):
        try:
            rng = random.Random(300 + w)
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, 0, j)], dt)
            for r in range(1, R + 1):
                order = list(range(len(keys)))
                rng.shuffle(order)
                for j in order:
                    srv.push(keys[j], w, src[(w, r, j)], dt)
                bar.wait(timeout=120)
                rng.shuffle(order)
                for j in order:
                    if rng.random() < 0.02:
                        time.sleep(0.002)                # past the idle exit
                    srv.pull(keys[j], outs[(w, j)])
                    pulled[(w, r, j)] = outs[(w, j)].cpu().numpy().copy()
                bar.wait(timeout=120)
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    orders = {}
    try:
        for r in range(1, R + 1):
            bar.wait(timeout=120)
            for j, k in enumerate(keys):
                orders[(r, j)] = srv.key_info(k)[2]
            bar.wait(timeout=120)
    except threading.BrokenBarrierError:
        raise AssertionError(f"worker failed: {errors}")
    finally:
        for t in ts:
            t.join(timeout=60)
    assert not errors, errors
    st = srv.stats()
    srv.close()
    for r in range(1, R + 1):
        for j, n in enumerate(sizes):
            want = np.zeros(n * es, np.uint8)
            port.sum_n(want, [data(dt, n, w, r, j) for w in orders[(r, j)]], n * es, dt)
            for w in range(N):
                assert_bytes_match(dt, pulled[(w, r, j)], want, nan_class_f32_f64=False,
                                   what=f"r{r} key {j} w{w}")
    assert st["service_pulls"] == N * R * len(keys)
    assert st["service_pushes"] == N * (R + 1) * len(keys)     # device pushes too
    assert st["service_launches"] >= 2


def test_service_push_waits_for_running_producer():
    """A blocking device push served by the copy service (no stream of the
    server's is involved) still honours the order_after event PSServer hands
    over: the producer still running on the caller's stream (a long spin, then
    the fill) lands before the service copies the data, and the round folds
    the filled values."""
    from prophet_amd.server import PSServer
    dt, N, n = DType.FLOAT32, 2, 1 << 20
    srv = PSServer(N)
    dev = torch.device("cuda:0")
    xs = [torch.zeros(n, device=dev) for _ in range(N)]
    torch.cuda.synchronize()
    ts = [threading.Thread(target=srv.push, args=(9, w, xs[w], dt)) for w in range(N)]
    for t in ts:                                         # init round
        t.start()
    for t in ts:
        t.join(timeout=60)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)                      # ~0.1 s on the current stream
    xs[0].fill_(1.5)
    xs[1].fill_(2.25)
    srv.push(9, 0, xs[0], dt)                            # blocking: through the service
    srv.push(9, 1, xs[1], dt)
    out = torch.empty(n, device=dev)
    srv.pull(9, out)
    st = srv.stats()
    srv.close()
    assert st["service_pushes"] >= 2
    assert torch.all(out == 3.75)


def _ptr_copy(ptr, src):
    from prophet_amd.reducer import GpuReducer
    GpuReducer().copy(ptr, src, src.numel() * src.element_size())


@pytest.mark.parametrize("N,dt", [(8, DType.FLOAT32), (8, DType.FLOAT16), (16, DType.FLOAT32),
                                  (16, DType.BFLOAT16)],
                         ids=["8-FLOAT32", "8-FLOAT16", "16-FLOAT32", "16-BFLOAT16"])
def test_device_release_rounds_bit_exact(port, N, dt, monkeypatch):
    """BPSR_SERVER_RELEASE=device: after the init round one keyed block queue
    folds every key, a round's last push_ready stores the release word (no
    launch); blocking device pushes land through the copy service and are
    released the same way; non-blocking device pushes (lane copies) pass the
    consumer with a skip word and fold with a lane launch behind their copies.
    8 worker threads, keys arriving in a different random order per worker and
    round (never block order), 3 rounds from the slots (push_ready), 1 of
    blocking device pushes and 1 of non-blocking ones; pulls as device views,
    blocking device copies and host copies.  Every pull equals the oracle's
    left fold in the recorded arrival order; one consumer launch per round;
    lane folds only in the non-blocking round.  16 workers: the wide keyed
    queue (the order's positions 8..15 in each block's second release word)
    keeps device releases — the same counts, bit-exact (bf16 included)."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "device")
    R = 5
    sizes = [1, 7, 1000, 4096 + 5, 65_536 + 3, 300_001]        # elements per key
    keys = list(range(40, 40 + len(sizes)))
    es = elem_size(dt)
    srv = PSServer(N, engine_lanes=3)
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    torch.cuda.synchronize()
    # the workers' device work goes on non-blocking streams: the legacy NULL
    # stream would wait for the epoch's consumer, which waits for the workers
    streams = [torch.cuda.Stream(device=dev) for _ in range(N)]
    bar = threading.Barrier(N + 1)
    errors, pulled = [], {}

    def worker(w):
        torch.cuda.set_stream(streams[w])
        try:
            rng = random.Random(500 + w)
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, 0, j)], dt)             # init round
            for r in range(1, R + 1):
                order = list(range(len(keys)))
                rng.shuffle(order)
                for j in order:
                    time.sleep(rng.random() * 0.0005)
                    if r == 3:                                 # blocking device pushes
                        srv.push(keys[j], w, src[(w, r, j)], dt)
                    elif r == 4:                               # non-blocking: lane copies
                        srv.push_async(keys[j], w, src[(w, r, j)], dt)
                    else:                                      # the transport wrote the slot
                        # (a stream sync, never a device-wide one: the epoch's
                        # consumer is running and waits for this thread's releases)
                        ptr = srv.recv_slot(keys[j], w)
                        st = torch.cuda.current_stream(dev)
                        x = src[(w, r, j)]
                        GpuReducer().copy(ptr, x, x.numel() * x.element_size(), stream=st)
                        st.synchronize()
                        srv.push_ready(keys[j], w)
                outs = []
                for j, k in enumerate(keys):
                    n = sizes[j] * es
                    if w % 3 == 0:                             # zero-copy view of the store
                        p, ln = srv.pull_device_view(k)
                        assert ln == n
                        o = torch.empty(n, dtype=torch.uint8, device=dev)
                        GpuReducer().copy(o, p, n)
                        torch.cuda.current_stream(dev).synchronize()
                        outs.append(o.cpu().numpy())
                    elif w % 3 == 1:
                        o = torch.empty(n, dtype=torch.uint8, device=dev)
                        srv.pull(k, o)
                        outs.append(o.cpu().numpy())
                    else:
                        o = np.zeros(n, np.uint8)
                        srv.pull(k, o)
                        outs.append(o)
                pulled[(w, r)] = outs
                bar.wait(timeout=120)
                bar.wait(timeout=120)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    st0 = None
    try:
        for r in range(1, R + 1):
            try:
                bar.wait(timeout=240)
            except threading.BrokenBarrierError:
                raise AssertionError(f"a worker failed: {errors}")
            assert not errors, errors
            for j, k in enumerate(keys):
                rounds, _, order = srv.key_info(k)
                assert rounds == r and sorted(order) == list(range(N))
                n = sizes[j] * es
                want = np.zeros(n, np.uint8)
                port.sum_n(want, [data(dt, sizes[j], w, r, j) for w in order], n, dt)
                for w in range(N):
                    assert_bytes_match(dt, pulled[(w, r)][j], want, nan_class_f32_f64=False,
                                       what=f"r{r} key {k} w{w}")
            if r == 1:
                st0 = srv.stats()
            bar.wait(timeout=120)
    finally:
        for t in ts:
            t.join(timeout=60)
    assert not errors, errors
    st = srv.stats()
    srv.close()
    # lane-copied rounds fold with launches (the non-blocking round; also the
    # blocking-push round when BPSR_SERVER_PULL_SERVICE=0 takes the service away)
    import os
    copied = 1 if os.environ.get("BPSR_SERVER_PULL_SERVICE", "1") != "0" else 2
    assert st["key_releases"] == (R - copied) * len(keys)
    # one epoch per round: a consumer epoch, or — the copied round, when the
    # consumer launched ahead for it retired idle first — a lane epoch
    assert st["consumer_launches"] + st["lane_epochs"] == R, st
    assert 1 <= st["fold_launches"] - st0["fold_launches"] <= copied * len(keys)


def test_device_release_epoch_launched_ahead_and_retired(port, monkeypatch):
    """Device releases launch each epoch's consumer once the previous epoch
    has begun (kq_launch_ahead), behind it on the keyed queue, so it is
    resident before the next round's first push; an epoch launched ahead that
    no round begins within 1 ms is retired (skip words: its tiles pass,
    nothing is stored) and the next round launches its own.  Rounds back to
    back and after idle gaps, 4 workers, fp16: every pull equals the oracle's
    left fold in the recorded order; consumer_launches counts the begun
    epochs only (one per round), the idle gaps show as retirements; a
    device-wide sync and destroy with an idle consumer launched ahead return
    at once instead of waiting for the release timeout."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "device")
    monkeypatch.setenv("BPSR_SERVER_RELEASE_TIMEOUT_S", "3")
    dt, N, R = DType.FLOAT16, 4, 6
    sizes = [5, 4096 + 1, 100_003]
    keys = [70, 71, 72]
    es = elem_size(dt)
    dev = torch.device("cuda:0")
    src = {(w, r, j): torch.from_numpy(data(dt, n, w, r, j)).to(dev)
           for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    torch.cuda.synchronize()
    srv = PSServer(N, engine_lanes=2)
    st = torch.cuda.Stream(device=dev)      # never the legacy NULL stream (server.h)
    closed = False
    try:
        with torch.cuda.stream(st):
            for j, k in enumerate(keys):                 # init round: blocking pushes
                ts = [threading.Thread(target=srv.push, args=(k, w, src[(w, 0, j)], dt))
                      for w in range(N)]
                for t in ts:
                    t.start()
                for t in ts:
                    t.join(timeout=60)
            for r in range(1, R + 1):
                for j, k in enumerate(keys):             # the transport writes the slots
                    for w in range(N):
                        x = src[(w, r, j)]                   # the key's bytes (uint8)
                        GpuReducer().copy(srv.recv_slot(k, w), x, x.numel(), stream=st)
                st.synchronize()
                if r in (4, 5):
                    time.sleep(0.01)                     # idle: the epoch launched ahead retires
                for j, k in enumerate(keys):
                    for w in range(N):
                        srv.push_ready(k, w)
                for j, k in enumerate(keys):
                    _, _, order = srv.key_info(k)
                    n = sizes[j] * es
                    want = np.zeros(n, np.uint8)
                    port.sum_n(want, [data(dt, sizes[j], w, r, j) for w in order], n, dt)
                    for w in range(N):
                        o = torch.empty(n, dtype=torch.uint8, device=dev)
                        srv.pull(k, o)
                        assert np.array_equal(o.cpu().numpy(), want), (r, k, w)
                if r == 1:
                    st0 = srv.stats()
        stats = srv.stats()
        t0 = time.time()
        torch.cuda.synchronize()          # the epoch launched ahead is idle: it retires
        sync_s = time.time() - t0
        t0 = time.time()
        srv.close()
        closed = True
        close_s = time.time() - t0
    finally:
        if not closed:
            srv.close()
    assert stats["key_releases"] == R * len(keys), stats
    assert stats["consumer_launches"] == R, stats            # begun epochs only
    assert stats["consumers_retired"] >= 2, stats             # the two idle gaps at least
    assert stats["fold_launches"] == st0["fold_launches"], stats  # no lane folds
    assert sync_s < 1.0 and close_s < 1.0, (sync_s, close_s)


@pytest.mark.parametrize("release", [None, "launch"], ids=["env-default", "launch"])
def test_server_from_env_folds_by_device_releases(port, release, monkeypatch):
    """The dedicated server process (server.cc:339-400) builds its server from
    the environment (byteps_server_config_from_env): device releases by
    default (round 6: a server whose pushes are copied runs no consumer, and
    no key has to come every epoch, server.h) — one consumer launch per
    round, no fold launches — and BPSR_SERVER_RELEASE=launch keeps launches.
    4 workers, push_ready rounds from the slots, pulls into device memory:
    bit-exact with the oracle's left fold in the recorded order either way."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import RELEASE_DEVICE, PSServer
    monkeypatch.delenv("BPSR_SERVER_RELEASE", raising=False)
    if release:
        monkeypatch.setenv("BPSR_SERVER_RELEASE", release)
    monkeypatch.setenv("DMLC_NUM_WORKER", "4")
    dt, N, R = DType.FLOAT32, 4, 3
    sizes = [3, 4096 + 1, 200_003]
    keys = [11, 12, 13]
    es = elem_size(dt)
    srv = PSServer.from_env()
    assert srv.cfg.release == RELEASE_DEVICE and srv.cfg.num_workers == N
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)      # never the legacy NULL stream (server.h)
    with torch.cuda.stream(st):
        for j, k in enumerate(keys):                     # init round: blocking pushes
            ts = [threading.Thread(target=srv.push, args=(k, w, data(dt, sizes[j], w, 0, j), dt))
                  for w in range(N)]
            for t in ts:
                t.start()
            for t in ts:
                t.join(timeout=60)
        st0 = None
        for r in range(1, R + 1):
            for j, k in enumerate(keys):
                for w in range(N):
                    x = torch.from_numpy(data(dt, sizes[j], w, r, j)).to(dev)
                    GpuReducer().copy(srv.recv_slot(k, w), x, x.numel(), stream=st)  # bytes (uint8)
                    st.synchronize()
                    srv.push_ready(k, w)
            for j, k in enumerate(keys):
                _, _, order = srv.key_info(k)
                want = np.zeros(sizes[j] * es, np.uint8)
                port.sum_n(want, [data(dt, sizes[j], w, r, j) for w in order], sizes[j] * es, dt)
                for w in range(N):
                    o = torch.empty(sizes[j] * es, dtype=torch.uint8, device=dev)
                    srv.pull(k, o)
                    st.synchronize()
                    assert np.array_equal(o.cpu().numpy(), want), (r, k, w)
            if r == 1:
                st0 = srv.stats()
    s1 = srv.stats()
    srv.close()
    if release is None:
        assert s1["consumer_launches"] == R and s1["key_releases"] == R * len(keys)
        assert s1["fold_launches"] == st0["fold_launches"]
    else:
        assert s1["consumer_launches"] == 0 and s1["key_releases"] == 0


def test_order_after_orders_device_released_push_ready(port, monkeypatch):
    """with device releases a push_ready round is released by a
    host store, which no lane stream orders.  The transport writes the slots
    on its own stream behind a long spin, hands the event to order_after and
    signals the arrivals at once (no host wait): the release waits for the
    event first, so the consumer folds the written bytes — the oracle's sum —
    not the slots' previous contents."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "device")
    dt, N, n = DType.FLOAT32, 2, 1 << 20
    key = 91
    srv = PSServer(N)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    zeros = [torch.zeros(n, device=dev) for _ in range(N)]
    ts = [threading.Thread(target=srv.push, args=(key, w, zeros[w], dt)) for w in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    ins = [data(dt, n, w, 1, key) for w in range(N)]
    src = [torch.from_numpy(x).to(dev) for x in ins]
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        torch.cuda._sleep(300_000_000)                  # the producer, still running
        for w in range(N):
            GpuReducer().copy(srv.recv_slot(key, w), src[w], n * 4, stream=st)
        ev = torch.cuda.Event()
        ev.record(st)
    srv.order_after(ev, [key])
    still_running = not st.query()
    for w in range(N):
        srv.push_ready(key, w)
    out = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    srv.pull(key, out)
    got = out.cpu().numpy()
    want = np.zeros(n * 4, np.uint8)
    port.sum_n(want, ins, n * 4, dt)      # two fp32 operands: either order, one sum
    stt = srv.stats()
    srv.pull(key, out)                    # the round's other pull (it re-arms after N)
    srv.close()
    assert still_running, "the producer finished before the releases: nothing was ordered"
    assert stt["key_releases"] == 1 and stt["consumer_launches"] == 1, stt
    assert np.array_equal(got, want)


def test_device_release_server_mixed_copied_and_slot_written_rounds(port, monkeypatch):
    """Device releases on, the per-epoch release choice (server.h): copied
    rounds (pushes from host memory, the ps-lite shape) before any round comes
    through the slots fold with launches and build no keyed queue — no
    consumer waits beside the lanes (config 1 took 4x longer with one, r05s55);
    the first push_ready round builds it; from then on an epoch opened by a
    copied round is a lane epoch (no consumer) and one opened by a
    slot-written round a consumer epoch.  Rounds: init (copied), copied,
    push_ready, push_ready, copied, copied, push_ready: every pull exact
    against the oracle's fold in the recorded order; the slot-written rounds
    are device-released, the copied ones fold with launches, and the copied
    run after the queue exists has at least one lane epoch."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "device")
    dt, N, n = DType.FLOAT32, 2, 70_001
    srv = PSServer(N)
    dev = torch.device("cuda:0")
    out = np.zeros(n * 4, np.uint8)
    kinds = ["copied", "copied", "slot", "slot", "copied", "copied", "slot"]
    stats = []
    for r, kind in enumerate(kinds):
        if kind == "copied":                             # host data: copied by the lanes
            for k in (1, 2):
                ts = [threading.Thread(target=srv.push, args=(k, w, data(dt, n, w, r, k), dt))
                      for w in range(N)]
                for t in ts:
                    t.start()
                for t in ts:
                    t.join(timeout=60)
        else:                                            # the transport wrote the slots, all
            for k in (1, 2):                             # before the first release (a NULL-
                for w in range(N):                       # stream copy waits for a running
                    x = torch.from_numpy(data(dt, n, w, r, k)).to(dev)   # consumer; one
                    _ptr_copy(srv.recv_slot(k, w), x)    # launched ahead and idle retires
            torch.cuda.current_stream(dev).synchronize()  # within 1 ms)
            for k in (1, 2):
                for w in range(N):
                    srv.push_ready(k, w)
        if r > 0:                                        # the init round has no pulls
            for k in (1, 2):
                want = np.zeros(n * 4, np.uint8)
                port.sum_n(want, [data(dt, n, w, r, k) for w in srv.key_info(k)[2]], n * 4, dt)
                for w in range(N):
                    srv.pull(k, out)
                    assert np.array_equal(out, want), (r, kind, k, w)
        stats.append(srv.stats())
    srv.close()
    # copied rounds before the first slot-written one: launches, no queue
    assert stats[1]["key_releases"] == 0 and stats[1]["consumer_launches"] == 0, stats[1]
    slots = sum(1 for k in kinds if k == "slot")
    assert stats[-1]["key_releases"] == 2 * slots, stats[-1]
    for r in (4, 5):                                     # copied rounds: lane folds
        assert stats[r]["fold_launches"] > stats[r - 1]["fold_launches"], (r, stats)
        assert stats[r]["key_releases"] == stats[r - 1]["key_releases"], (r, stats)
    assert stats[-1]["lane_epochs"] >= 1, stats[-1]


@pytest.mark.parametrize("pulls", ["device", "mixed", "mixed8"])
def test_device_release_mixed_kinds_and_late_keys_stress(port, monkeypatch, pulls):
    """The per-epoch release choice under concurrency (server.h): 4 worker
    threads, 5 keys, 8 rounds; every (round, key, worker) push is, at random,
    written into the slot by the "transport" (push_ready), a non-blocking
    device push (lane copy) or a blocking host push (copied), keys arrive in
    a different random order per worker and round, and in two rounds one key
    comes 150 ms late (its epoch closes without it).  Rounds with any copied
    push fold with lane launches, the others on the device; epochs open as
    consumer or lane epochs as their first release decides.  Every pull of
    every round equals the oracle's left fold in the recorded arrival order.
    pulls="mixed": each pull is, at random, a copy into a device tensor, a
    copy into host memory or a host view of the store's mirror (the mirror's
    D2H waits for a device-released round's epoch on the lane's d2h stream),
    with other kind and late-key draws.  pulls="mixed8": the same with 8
    workers (the release word's widest single-word order)."""
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "device")
    dt, N, R = DType.FLOAT32, 4, 8
    sizes = [3, 1000, 4096 + 1, 65_536, 200_003]
    keys = list(range(300, 300 + len(sizes)))
    es = elem_size(dt)
    rng0 = random.Random({"device": 4242, "mixed": 77}.get(pulls, 5))
    if pulls == "mixed8":
        N = 8
    kind = {(r, j, w): rng0.choice(("slot", "slot", "async", "host"))
            for r in range(1, R + 1) for j in range(len(keys)) for w in range(N)}
    pkind = {(r, j, w): "device" if pulls == "device" else rng0.choice(("device", "host", "view"))
             for r in range(1, R + 1) for j in range(len(keys)) for w in range(N)}
    late = {(3, 1), (6, 4)} if pulls == "device" else {(2, 0), (5, 2), (7, 3)}
    srv = PSServer(N, engine_lanes=2)
    dev = torch.device("cuda:0")
    host = {(w, r, j): data(dt, n, w, r, j)
            for w in range(N) for r in range(R + 1) for j, n in enumerate(sizes)}
    src = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(N)]
    bar = threading.Barrier(N + 1)
    errors, pulled = [], {}

    def worker(w):
        torch.cuda.set_stream(streams[w])
        try:
            rng = random.Random(900 + w)
            for j, k in enumerate(keys):
                srv.push(k, w, src[(w, 0, j)], dt)       # init round
            for r in range(1, R + 1):
                order = list(range(len(keys)))
                rng.shuffle(order)
                for j in order:
                    if (r, j) in late and w == 0:
                        time.sleep(0.15)
                    kd = kind[(r, j, w)]
                    if kd == "slot":
                        st = torch.cuda.current_stream(dev)
                        x = src[(w, r, j)]
                        GpuReducer().copy(srv.recv_slot(keys[j], w), x, x.numel(), stream=st)
                        st.synchronize()
                        srv.push_ready(keys[j], w)
                    elif kd == "async":
                        srv.push_async(keys[j], w, src[(w, r, j)], dt)
                    else:
                        srv.push(keys[j], w, host[(w, r, j)], dt)
                outs = []
                for j, k in enumerate(keys):
                    pk = pkind[(r, j, w)]
                    if pk == "view":
                        outs.append(np.frombuffer(srv.pull_view(k), np.uint8).copy())
                    elif pk == "host":
                        o = np.empty(sizes[j] * es, np.uint8)
                        srv.pull(k, o)
                        outs.append(o)
                    else:
                        o = torch.empty(sizes[j] * es, dtype=torch.uint8, device=dev)
                        srv.pull(k, o)
                        outs.append(o.cpu().numpy())
                pulled[(w, r)] = outs
                bar.wait(timeout=120)
                bar.wait(timeout=120)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    try:
        for r in range(1, R + 1):
            try:
                bar.wait(timeout=240)
            except threading.BrokenBarrierError:
                raise AssertionError(f"a worker failed: {errors}")
            assert not errors, errors
            for j, k in enumerate(keys):
                rounds, _, order = srv.key_info(k)
                assert rounds == r and sorted(order) == list(range(N)), (r, k, order)
                n = sizes[j] * es
                want = np.zeros(n, np.uint8)
                port.sum_n(want, [host[(w, r, j)] for w in order], n, dt)
                for w in range(N):
                    assert_bytes_match(dt, pulled[(w, r)][j], want, nan_class_f32_f64=False,
                                       what=f"r{r} key {k} w{w}")
            bar.wait(timeout=120)
    finally:
        for t in ts:
            t.join(timeout=60)
    st = srv.stats()
    srv.close()
    assert not errors, errors
    assert st["key_releases"] > 0 and st["fold_launches"] > 0, st


def test_device_release_epoch_closes_for_a_missing_key(port, monkeypatch):
    """No key has to be pushed in every epoch (server.h): a round in which
    key 2 is not pushed in time leaves its epoch open only until the host
    closes it, 100 ms after its first release — key 2 gets a skip word, key
    1's round is folded and pulled exactly, nothing fails (the reference folds
    every key on its own) and device releases stay on.  Key 2's late round
    (copied pushes) then folds exactly in a later epoch; every later round is
    exact, and the keys' rounds are device-released in one epoch again by
    round 4.  Round 0 (init) is copied pushes,
    round 1 push_ready (the first slot-written round builds the keyed queue).
    The device timeout is set low (0.5 s) to show the host close comes first."""
    from prophet_amd.server import PSServer
    monkeypatch.setenv("BPSR_SERVER_RELEASE", "device")
    monkeypatch.setenv("BPSR_SERVER_RELEASE_TIMEOUT_S", "0.5")
    dt, N, n = DType.FLOAT32, 2, 50_003
    srv = PSServer(N)
    for k in (1, 2):                                     # init round, both keys
        ts = [threading.Thread(target=srv.push, args=(k, w, data(dt, n, w, 0, k), dt))
              for w in range(N)]                         # (an init push waits for the others)
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
    dev = torch.device("cuda:0")
    out = np.zeros(n * 4, np.uint8)

    def slot_round(r, keys):
        for k in keys:                                   # every slot written before the
            for w in range(N):                           # first release (the epoch's consumer
                x = torch.from_numpy(data(dt, n, w, r, k)).to(dev)   # then waits; NULL-stream
                _ptr_copy(srv.recv_slot(k, w), x)                   # work would wait for it)
        torch.cuda.current_stream(dev).synchronize()
        for k in keys:
            for w in range(N):
                srv.push_ready(k, w)

    def check(r, k):
        want = np.zeros(n * 4, np.uint8)
        port.sum_n(want, [data(dt, n, w, r, k) for w in srv.key_info(k)[2]], n * 4, dt)
        for w in range(N):
            srv.pull(k, out)
            assert np.array_equal(out, want), (r, k, w)

    slot_round(1, (1, 2))
    for k in (1, 2):
        check(1, k)
    # round 2: key 1 only; key 2 does not come before the epoch closes
    t0 = time.time()
    slot_round(2, (1,))
    check(2, 1)                                          # answered once the epoch is closed
    waited = time.time() - t0
    for w in range(N):                                   # key 2's round 2, late, copied
        srv.push(2, w, data(dt, n, w, 2, 2), dt)
    check(2, 2)
    st2 = srv.stats()
    # Epochs are not rounds: key 2's late round went to the epoch after the
    # closed one, where key 1's round 3 lands too, so round 3 of the two keys
    # sits in neighbouring epochs (key 1's may be a lane epoch, opened by key
    # 2's copied round) until a close skips key 1 once more; round 4 is in step.
    slot_round(3, (1, 2))
    for k in (1, 2):
        check(3, k)
    st3 = srv.stats()
    slot_round(4, (1, 2))
    for k in (1, 2):
        check(4, k)
    st4 = srv.stats()
    srv.close()
    assert st2["epochs_closed"] >= 1, st2
    assert waited < 0.45, waited                         # the host close, not the device timeout
    assert st4["key_releases"] - st3["key_releases"] == 2, (st3, st4)   # in step again
