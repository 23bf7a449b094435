"""GPU parity of the persistent block consumer (byteps_reduce_blockq_*).

One launch per iteration folds every block of the table, starting each block
once it (and every block before it) is released.  Bar: bit-exact with the CPU
oracle for every block, in every iteration, whichever way the blocks are
released (all up front, one by one from another stream after their pushes
land by DMA, from a captured hipGraph), and a launch whose releases never come
stops by itself and reports BYTEPS_REDUCE_ETIMEOUT.
"""
import json

import numpy as np
import pytest

from oracle.oracle import PortReducer
from prophet_amd import synth
from prophet_amd.dtypes import DType, elem_size

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def red(dev):
    from prophet_amd.reducer import GpuReducer
    return GpuReducer(device=0)


@pytest.fixture(scope="module")
def port():
    return PortReducer(nthreads=8)


class Table:
    """Receive slots + outputs for a list of blocks of (n_elems, n_sources, class)."""

    def __init__(self, dev, dt, blocks, offsets=False):
        self.dt, self.es = dt, elem_size(dt)
        self.blocks = []     # per block: list of (dst, [srcs], len)
        self.views = []      # flat: (dst tensor, [src tensors], len, n_elems, N, class)
        for bi, blk in enumerate(blocks):
            out = []
            for ne, N, cls in blk:
                L = ne * self.es
                o = (self.es * (len(self.views) % 3)) if offsets else 0
                srcs = [torch.empty(L + 16, dtype=torch.uint8, device=dev)[o:o + L]
                        for _ in range(N)]
                dst = torch.full((L + 16,), 0x5A, dtype=torch.uint8, device=dev)[o:o + L]
                out.append((dst, srcs, L))
                self.views.append((dst, srcs, L, ne, N, cls))
            self.blocks.append(out)

    def host_inputs(self, seed):
        """Pinned host pushes and the oracle's fold of every bucket."""
        pushes, wants = [], []
        for i, (dst, srcs, L, ne, N, cls) in enumerate(self.views):
            ins = [np.ascontiguousarray(synth.bucket(self.dt, ne, k, cls, seed + i)).view(np.uint8)
                   for k in range(N)]
            pushes.append([torch.from_numpy(x).pin_memory() for x in ins])
            w = np.full(L, 0x5A, np.uint8)
            if L:
                PortReducer(nthreads=8).sum_n(w, ins, L, self.dt)
            wants.append(w)
        return pushes, wants

    def upload(self, pushes, stream=None):
        for (dst, srcs, L, *_), ps in zip(self.views, pushes):
            for s, p in zip(srcs, ps):
                if L:
                    s.copy_(p, non_blocking=True)

    def check(self, wants):
        for i, ((dst, _, L, *_), w) in enumerate(zip(self.views, wants)):
            got = dst.cpu().numpy()
            if not np.array_equal(got, w):
                bad = np.flatnonzero(got != w)
                raise AssertionError(f"bucket {i}: {len(bad)} bytes differ, first at {bad[0]}")


# ragged buckets, an empty block, element-only buckets, > 8 sources
MIXED = [
    [(100_000, 8, "special"), (4099, 9, "normal"), (1, 1, "normal")],
    [],
    [(70_001, 32, "bits"), (0, 8, "normal"), (257, 12, "special")],
    [(300_000, 5, "normal")],
    [(9, 8, "bits"), (3 * 1024 + 5, 2, "normal"), (1 << 20, 8, "normal")],
]


# consumer shapes: 0 = dispatch-ordered (one workgroup per tile, gated on the
# released mark), 1 = persistent (one workgroup per CU sweeping the table)
SHAPES = pytest.mark.parametrize("shape", [0, 1], ids=["dispatch", "persistent"])


@SHAPES
@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16, DType.BFLOAT16, DType.INT32,
                                DType.FLOAT64, DType.UINT8], ids=lambda d: DType(d).name)
def test_release_all_three_iterations(red, dev, dt, shape):
    """Release every block up front; the queue re-arms itself between launches."""
    tab = Table(dev, dt, MIXED, offsets=True)
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=shape)
    for it in range(3):
        pushes, wants = tab.host_inputs(100 * it + 7)
        tab.upload(pushes)
        torch.cuda.synchronize()
        q.release(-1)
        q.launch()
        q.status()
        torch.cuda.synchronize()
        tab.check(wants)
    q.close()


@pytest.mark.parametrize("occ", [0, 1, 2, 4])
def test_live_release_after_dma(red, dev, occ):
    """The consumer is launched first (occ 0: dispatch-ordered, else
    persistent workgroups per CU); a copy stream then pushes each block's
    data by H2D DMA and releases the block behind it.  Every block must see
    its own freshly landed bytes (acquire after the release), over iterations
    whose data differ."""
    from prophet_amd.buckets import resnet50_param_sizes, prophet_blocks
    dt = DType.FLOAT16
    sizes = resnet50_param_sizes()
    groups = prophet_blocks(len(sizes))
    # every ResNet-50 gradient of every block, at a quarter of its size (test time)
    blocks = [[(max(1, sizes[i] // 4), 8, "normal") for i in g] for g in groups]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=occ, timeout_s=5.0)
    # launched on a caller's stream: the library forks the consumer onto its
    # own consumer stream (a hardware queue of its own, include/bpsr/reduce.h),
    # so the copy stream's DMA and releases never queue behind it
    comp, copy = torch.cuda.Stream(priority=-100), torch.cuda.Stream()
    for it in range(2):
        pushes, wants = tab.host_inputs(1000 * it + 3)
        torch.cuda.synchronize()
        q.launch(comp)
        k = 0
        with torch.cuda.stream(copy):
            for b, blk in enumerate(tab.blocks):
                for dst, srcs, L in blk:
                    for s, p in zip(srcs, pushes[k]):
                        s.copy_(p, non_blocking=True)
                    k += 1
                q.release(b, copy)
        comp.synchronize()
        copy.synchronize()
        q.status(comp)
        tab.check(wants)
    q.close()


@SHAPES
def test_out_of_order_release_waits_for_prefix(red, dev, shape):
    """Blocks released last-to-first from a side stream: nothing past an
    unreleased block is started, and the result is still exact."""
    dt = DType.FLOAT32
    blocks = [[(200_000 + 17 * b, 8, "normal")] for b in range(6)]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=shape)
    pushes, wants = tab.host_inputs(55)
    tab.upload(pushes)
    torch.cuda.synchronize()
    comp, side = torch.cuda.Stream(priority=-100), torch.cuda.Stream()
    q.launch(comp)
    for b in reversed(range(len(blocks))):
        q.release(b, side)
    comp.synchronize()
    q.status(comp)
    tab.check(wants)
    q.close()


@SHAPES
def test_missing_release_times_out_and_recovers(red, dev, shape):
    """Blocks 0-1 released, block 2 never: the launch gives up after its
    timeout, reports ETIMEOUT once, has folded the released blocks, and the
    queue works normally afterwards."""
    from prophet_amd.reducer import ETIMEOUT, ReduceError
    dt = DType.FLOAT32
    blocks = [[(500_000, 8, "normal")], [(123_457, 8, "normal")], [(400_000, 8, "normal")],
              [(1000, 8, "normal")]]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=shape, timeout_s=0.2)
    pushes, wants = tab.host_inputs(77)
    tab.upload(pushes)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    q.release(0, s)
    q.release(1, s)
    q.launch(s)
    with pytest.raises(ReduceError) as ei:
        q.status(s)
    assert ei.value.code == ETIMEOUT
    for i in (0, 1):
        assert np.array_equal(tab.views[i][0].cpu().numpy(), wants[i])
    q.status(s)  # cleared
    q.release(-1, s)
    q.launch(s)
    q.status(s)
    tab.check(wants)
    q.close()


@SHAPES
def test_graph_replay_matches_plans(red, dev, port, shape):
    """Release + launch captured into a hipGraph and replayed on new data:
    bit-identical with one plan per block (ResNet-50 fp16 Prophet blocks)."""
    from prophet_amd.buckets import resnet50_param_sizes, prophet_blocks
    dt = DType.FLOAT16
    sizes = resnet50_param_sizes()
    groups = prophet_blocks(len(sizes))
    blocks = [[(sizes[i], 8, "normal") for i in g] for g in groups]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=shape)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        q.release(-1, side)
        q.launch(side)
    gen = torch.Generator(device=dev)
    for it in range(2):
        gen.manual_seed(it)
        for dst, srcs, L, *_ in tab.views:
            for s in srcs:
                s.view(torch.float16).copy_(torch.randn(L // 2, generator=gen, device=dev))
        g.replay()
        torch.cuda.synchronize()
        q.status()
        got = [v[0].clone() for v in tab.views]
        plans = [red.make_plan(blk, dt) for blk in tab.blocks]
        for p in plans:
            p.launch()
        torch.cuda.synchronize()
        for a, v in zip(got, tab.views):
            assert torch.equal(a, v[0])
        for p in plans:
            p.close()
        if it == 1:     # and the oracle, on every bucket of the replayed iteration
            for i, (a, (dst, srcs, L, *_)) in enumerate(zip(got, tab.views)):
                want = np.zeros(L, np.uint8)
                port.sum_n(want, [s.cpu().numpy() for s in srcs], L, dt)
                assert np.array_equal(a.cpu().numpy(), want), f"bucket {i}"
    q.close()


def test_bad_tables_rejected(red, dev):
    from prophet_amd.reducer import EARGS, ReduceError
    import ctypes
    from prophet_amd.reducer import BucketDesc, _vp, _int
    h = _vp()
    descs = (BucketDesc * 1)()
    for ends in ([2], [0, 2], []):
        arr = (_int * max(1, len(ends)))(*ends)
        rc = red.lib.byteps_reduce_blockq_create(descs, 1, arr, len(ends), 0, 0, ctypes.byref(h))
        assert rc == EARGS
    assert red.lib.byteps_reduce_blockq_release(None, 0, None) == EARGS


@SHAPES
def test_epochs_back_to_back_iterations(red, dev, shape):
    """Epoch-numbered releases: three iterations enqueued without a host
    sync — consumer k launched from a caller's stream, its releases on a side stream,
    the next iteration's launch queued right behind — every launch folds its
    own iteration's data (each iteration rewrites the inputs by a device copy
    ordered after the previous launch and before its releases)."""
    dt = DType.FLOAT32
    blocks = [[(150_000 + 31 * b, 8, "normal"), (4099, 8, "normal")] for b in range(5)]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=shape, timeout_s=5.0)
    comp, side = torch.cuda.Stream(priority=-100), torch.cuda.Stream()
    staged, wants, outs = [], [], []
    for it in range(3):
        pushes, w = tab.host_inputs(300 + it)
        staged.append([[p.to(dev) for p in ps] for ps in pushes])
        wants.append(w)
    torch.cuda.synchronize()
    for it in range(3):
        q.launch(comp)
        done = torch.cuda.Event()
        k = 0
        with torch.cuda.stream(side):
            for b, blk in enumerate(tab.blocks):
                for dst, srcs, L in blk:
                    for s, p in zip(srcs, staged[it][k]):
                        s.copy_(p, non_blocking=True)
                    k += 1
                q.release(b, side)
        done.record(comp)
        side.wait_event(done)            # next iteration's data after this consumer
        with torch.cuda.stream(comp):
            outs.append([v[0].clone() for v in tab.views])
    torch.cuda.synchronize()
    q.status(comp)
    for it in range(3):
        for i, (o, w) in enumerate(zip(outs[it], wants[it])):
            assert np.array_equal(o.cpu().numpy(), w), (it, i)
    q.close()


def test_release_range_and_capture_rule(red, dev):
    """release_range releases several blocks with one kernel; a captured launch
    must have every block released before it (its epoch is fixed at capture)."""
    from prophet_amd.reducer import EARGS, ReduceError
    dt = DType.FLOAT16
    blocks = [[(70_000 + b, 8, "normal")] for b in range(7)]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    pushes, wants = tab.host_inputs(9)
    tab.upload(pushes)
    torch.cuda.synchronize()
    comp, side = torch.cuda.Stream(priority=-100), torch.cuda.Stream()
    q.launch(comp)
    q.release_range(4, 3, side)          # out of order, in ranges
    q.release_range(0, 4, side)
    comp.synchronize()
    q.status(comp)
    tab.check(wants)
    with pytest.raises(ReduceError):
        q.release_range(5, 3, side)      # past the last block
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with pytest.raises(ReduceError) as ei:
        with torch.cuda.graph(g, stream=s):
            q.launch(s)                  # nothing released for this epoch
    assert ei.value.code == EARGS
    torch.cuda.synchronize()
    q.close()


def test_live_release_never_behind_consumer_any_stream_pair():
    """Regression: stream priority does not separate hardware queues — with
    torch's pooled streams the 5th and 9th (high, normal) pairs of a process
    shared one, and a live release queued behind the spinning consumer timed
    out (tools/pushloop_diag.py).  The consumer now always runs on the
    library's consumer stream (its own hardware queue), forked from the
    caller's stream: for 12 successive pool pairs, launch on the high-priority
    stream, release on the normal one after the consumer started — every
    iteration completes, bit-exact."""
    import time as _time
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    red = GpuReducer(device=0)
    dev = torch.device("cuda:0")
    n, N = 1 << 16, 4
    ins = [[torch.randn(n, device=dev) for _ in range(N)] for _ in range(2)]
    outs = [torch.zeros(n, device=dev) for _ in range(2)]
    bq = red.make_blockq([[(outs[b], ins[b], n * 4)] for b in range(2)], DType.FLOAT32)
    bq.config(wg_per_cu=0, timeout_s=1.0)
    refs = []
    for b in range(2):
        r = ins[b][0].clone()
        for x in ins[b][1:]:
            r.add_(x)
        refs.append(r)
    for i in range(12):
        cons = torch.cuda.Stream(priority=-100)
        rel = torch.cuda.Stream()
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        bq.launch(cons)
        _time.sleep(0.002)
        bq.release(0, rel)
        bq.release(1, rel)
        torch.cuda.synchronize()
        bq.status(cons)                               # raises on a timeout
        assert all(torch.equal(o, r) for o, r in zip(outs, refs)), i
    bq.close()


# ------------------------------------------------- host releases (no stream) --


@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16, DType.INT32],
                         ids=lambda d: DType(d).name)
def test_host_releases_live_three_iterations(red, dev, dt):
    """Data resident, consumer launched first, then every block released from
    the HOST in a shuffled order (byteps_reduce_blockq_release_host, forwarded
    by the launch's helper workgroup): bit-exact with the oracle, 3 epochs."""
    tab = Table(dev, dt, MIXED, offsets=True)
    q = red.make_blockq(tab.blocks, dt)
    q.host_releases(True)
    rng = np.random.default_rng(5)
    for it in range(3):
        pushes, wants = tab.host_inputs(300 * it + 11)
        tab.upload(pushes)
        torch.cuda.synchronize()          # data complete and visible: host releases allowed
        q.launch()
        for b in rng.permutation(len(MIXED)):
            q.release_host(int(b))
        q.status()
        torch.cuda.synchronize()
        tab.check(wants)
    q.close()


def test_host_releases_after_device_copies_and_mixed_with_stream_releases(red, dev):
    """Blocks 0-1 land by device copies on a side stream and are released from
    the host once an event says they landed; blocks 2-4 are released on the
    stream as before.  Both kinds in one launch, exact; then a pre-released
    iteration (releases before the launch) through the host path."""
    dt = DType.FLOAT32
    tab = Table(dev, dt, MIXED)
    q = red.make_blockq(tab.blocks, dt)
    q.host_releases(True)
    pushes, wants = tab.host_inputs(901)
    staged = [[p.to(dev) for p in ps] for ps in pushes]
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    q.launch()
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        for (dst, srcs, L, *_), st in zip(tab.views, staged):
            for s_, x in zip(srcs, st):
                if L:
                    s_.copy_(x)
        ev.record(side)
    q.release_range(2, 3, side)            # stream-ordered, behind the copies
    ev.synchronize()                       # host knows blocks 0-1 landed
    q.release_host(0, 2)
    q.status()
    torch.cuda.synchronize()
    tab.check(wants)
    pushes, wants = tab.host_inputs(902)
    tab.upload(pushes)
    torch.cuda.synchronize()
    q.release_host(0, len(MIXED))         # before the launch
    q.launch()
    q.status()
    torch.cuda.synchronize()
    tab.check(wants)
    q.close()


def test_host_release_missing_times_out_and_recovers(red, dev):
    from prophet_amd.reducer import ETIMEOUT, ReduceError
    dt = DType.FLOAT32
    blocks = [[(500_000, 8, "normal")], [(123_457, 8, "normal")], [(400_000, 8, "normal")]]
    tab = Table(dev, dt, blocks)
    q = red.make_blockq(tab.blocks, dt)
    q.config(timeout_s=0.2)
    q.host_releases(True)
    pushes, wants = tab.host_inputs(78)
    tab.upload(pushes)
    torch.cuda.synchronize()
    q.launch()
    q.release_host(0, 2)                  # block 2 never
    with pytest.raises(ReduceError) as ei:
        q.status()
    assert ei.value.code == ETIMEOUT
    for i in (0, 1):
        assert np.array_equal(tab.views[i][0].cpu().numpy(), wants[i])
    q.status()                            # cleared
    q.launch()
    q.release_host(0, 3)
    q.status()
    tab.check(wants)
    q.close()


def test_host_releases_rules(red, dev):
    """Persistent consumers refuse host releases (and vice versa); releasing
    from the host before enabling it, or outside the table, is EARGS."""
    from prophet_amd.reducer import EARGS, ReduceError
    dt = DType.FLOAT32
    tab = Table(dev, dt, [[(4096, 2, "normal")], [(4096, 2, "normal")]])
    q = red.make_blockq(tab.blocks, dt)
    with pytest.raises(ReduceError) as ei:
        q.release_host(0)
    assert ei.value.code == EARGS
    q.config(wg_per_cu=1)
    with pytest.raises(ReduceError):
        q.host_releases(True)
    q.config(wg_per_cu=0)
    q.host_releases(True)
    with pytest.raises(ReduceError):
        q.config(wg_per_cu=2)
    with pytest.raises(ReduceError):
        q.release_host(1, 2)
    # a captured launch cannot carry the host-release helper: refused, even
    # with every block pre-released from the host
    q.release_host(0, 2)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with pytest.raises(ReduceError) as ei:
        with torch.cuda.graph(g, stream=s):
            q.launch(s)
    assert ei.value.code == EARGS and "host releases" in str(ei.value)
    torch.cuda.synchronize()
    q.host_releases(False)
    q.config(wg_per_cu=1)
    q.close()


# ------------------------------------- overlapping launches (round 5) --
# byteps_reduce_blockq_overlap: consecutive launches alternate between the
# device's two consumer queues, each dispatched only once every workgroup of
# the previous launch has started.  The tables below have
# more tiles than the consumer's resident slots (2 per CU), so a launch is
# enqueued while its predecessor still has workgroups to dispatch.


def _quarter_resnet(dev, dt=DType.FLOAT16):
    from prophet_amd.buckets import prophet_blocks, resnet50_param_sizes
    sizes = resnet50_param_sizes()
    return Table(dev, dt, [[(max(1, sizes[i] // 4), 8, "normal") for i in g]
                           for g in prophet_blocks(len(sizes))])


def test_overlap_releases_after_previous_iteration_no_deadlock(red, dev):
    """The pattern that deadlocks two freely overlapping launches: iteration
    k's inputs are rewritten, and its blocks released, on a side stream that
    first waits for every earlier launch (join) — so k's releases need k - 1
    to finish.  Launch k is enqueued before them, while k - 1 may still have
    workgroups to dispatch.  Four iterations of one queue with data changing
    every iteration, each output copied out after a join (and the next
    iteration's releases after that copy): bit-exact, no timeout (1 s)."""
    tab = _quarter_resnet(dev)
    q = red.make_blockq(tab.blocks, DType.FLOAT16)
    q.config(wg_per_cu=0, timeout_s=1.0)
    q.overlap(True)
    cons, side, out_s = q.stream(), torch.cuda.Stream(), torch.cuda.Stream()
    staged, wants, outs = [], [], []
    for it in range(4):
        pushes, w = tab.host_inputs(700 + it)
        staged.append([[p.to(dev) for p in ps] for ps in pushes])
        wants.append(w)
    torch.cuda.synchronize()
    for it in range(4):
        q.join(side)                     # side: after every launch so far (k - 1)
        q.launch(cons)                   # k: enqueued before its releases
        k = 0
        with torch.cuda.stream(side):
            for b, blk in enumerate(tab.blocks):
                for dst, srcs, L in blk:
                    for s, p in zip(srcs, staged[it][k]):
                        s.copy_(p, non_blocking=True)
                    k += 1
                q.release(b, side)
        q.join(out_s)
        with torch.cuda.stream(out_s):
            outs.append([v[0].clone() for v in tab.views])
        # the caller's side of the contract: the next iteration's releases
        # (which let its tiles rewrite the outputs) only after this read
        side.wait_stream(out_s)
    torch.cuda.synchronize()
    q.status(cons)
    for it in range(4):
        for i, (o, w) in enumerate(zip(outs[it], wants[it])):
            assert np.array_equal(o.cpu().numpy(), w), (it, i)
    q.close()


def test_overlap_two_queues_live_and_classic_interleaved(red, dev):
    """Two tables: A overlaps, B does not (its launches stay stream-ordered on
    consumer queue 0 and wait for A's dispatch when A went to queue 1).  Six
    rounds of A, B launched back to back with live releases from another
    stream after each launch, then host releases on A: every output exact."""
    dt = DType.FLOAT32
    ta = Table(dev, dt, MIXED, offsets=True)
    tb = _quarter_resnet(dev)
    qa = red.make_blockq(ta.blocks, dt)
    qb = red.make_blockq(tb.blocks, DType.FLOAT16)
    for q in (qa, qb):
        q.config(wg_per_cu=0, timeout_s=2.0)
    qa.overlap(True)
    pa, wa = ta.host_inputs(41)
    pb, wb = tb.host_inputs(42)
    ta.upload(pa)
    tb.upload(pb)
    torch.cuda.synchronize()
    cons, rel = qa.stream(), torch.cuda.Stream()
    for _ in range(6):
        for t in (ta, tb):
            for dst, *_ in t.views:
                dst.fill_(0x5A)
        torch.cuda.synchronize()
        qa.launch(cons)
        qb.launch(cons)
        qa.release(-1, rel)
        qb.release(-1, rel)
        qa.join()
        torch.cuda.synchronize()
        qa.status(cons)
        qb.status(cons)
        ta.check(wa)
        tb.check(wb)
    qa.host_releases(True)
    for _ in range(3):
        qa.launch(cons)
        qa.release_host(0, len(MIXED))
    qa.status(cons)
    torch.cuda.synchronize()
    ta.check(wa)
    qa.close()
    qb.close()


def test_overlap_rules(red, dev):
    """Overlap needs the dispatch-ordered consumer (EARGS for a persistent
    one, and a persistent config is refused while overlap is on); off again
    restores stream-ordered launches: the launch stream then sees the
    output without a join."""
    from prophet_amd.reducer import EARGS, ReduceError
    dt = DType.FLOAT32
    tab = Table(dev, dt, [[(65_536, 4, "normal")], [(4096, 2, "normal")]])
    q = red.make_blockq(tab.blocks, dt)
    q.config(wg_per_cu=1)
    with pytest.raises(ReduceError) as ei:
        q.overlap(True)
    assert ei.value.code == EARGS
    q.config(wg_per_cu=0)
    q.overlap(True)
    with pytest.raises(ReduceError) as ei:
        q.config(wg_per_cu=2)
    assert ei.value.code == EARGS
    q.overlap(False)
    pushes, wants = tab.host_inputs(5)
    tab.upload(pushes)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    q.release(-1, s)
    q.launch(s)                          # classic: forks and joins back into s
    with torch.cuda.stream(s):
        got = [v[0].clone() for v in tab.views]
    s.synchronize()
    q.status(s)
    for g, w in zip(got, wants):
        assert np.array_equal(g.cpu().numpy(), w)
    q.close()


def test_releases_on_streams_sharing_the_launch_streams_hardware_queue():
    """Round 6 (false dependencies): with GPU_MAX_HW_QUEUES=1
    every normal-priority stream — the NULL stream included — shares ONE
    in-order hardware queue, so a wait for the consumer queued on the launch
    stream at launch time would sit ahead of every release (and of the copies
    before it) on any other stream: the r05s76 stall, made deterministic.  A
    launch now joins back only once its epoch is fully released: each case
    (a caller-stream launch with copies and a release on another stream, the
    r05s76 NULL-stream test with mixed stream and host releases, the PUSH loop
    on caller streams) completes exactly, well inside the 2-s consumer timeout.
    Runs in a subprocess: the queue count is read when HIP starts."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "blockq_shared_hwq_case.py")],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert [x["case"] for x in lines] == ["caller_stream", "null_mixed", "push_loop"], r.stdout
    for x in lines:
        assert x["ok"], x
        assert x["s"] < 1.5, x          # no consumer timeout on the way
    assert r.stdout.strip().endswith("ok"), r.stdout + r.stderr
