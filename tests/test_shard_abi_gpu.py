"""The shard C ABI (include/bpsr/shard.h) on the GPU, against the oracle.

* In-process groups (``byteps_shard_comm_init_local``): W ranks on cuda:0,
  one host thread each, the same C++ code path a multi-GPU server process
  runs — rank-order reduce-scatter + all-gather, in place and out of place,
  the landed-bucket scatter, reduce-to-root (BYTEPS_REDUCE_ROOTS) and
  broadcast, ragged and tiny sizes, and a rank that sends the wrong size.
* RCCL: a world-1 communicator made through the ABI (unique id + init), one
  wrapped from torch's ProcessGroupNCCL, and (>= 2 GPUs) one rank per GPU.

Every result is compared bit for bit with the oracle's left fold
(oracle/bpsr_oracle.c via oracle.oracle.PortReducer) of each owner's slice in
rank (or worker) order."""
import os
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dt():
    from prophet_amd.dtypes import DType
    return DType


def _vec(dt, E, who, cls, seed):
    from prophet_amd import synth
    return np.ascontiguousarray(synth.bucket(dt, E, who, cls, seed)).view(np.uint8).copy()


def _fold(dt, arrays):
    """Oracle left fold of byte arrays, in list order."""
    from oracle.oracle import PortReducer
    want = np.zeros(arrays[0].nbytes, np.uint8)
    if want.nbytes:
        PortReducer(nthreads=4).sum_n(want, list(arrays), want.nbytes, dt)
    return want


def _sliced_fold(dt, vecs, E, world):
    """Each owner's slice folded on its own, in rank order, put together."""
    from prophet_amd.dtypes import elem_size
    from prophet_amd.shard import owner_ranges
    es = elem_size(dt)
    out = np.zeros(E * es, np.uint8)
    for lo, hi in owner_ranges(E, world):
        if hi > lo:
            out[lo * es:hi * es] = _fold(dt, [v[lo * es:hi * es] for v in vecs])
    return out


def _dev(a):
    return torch.from_numpy(a).to("cuda:0")


def _threads(world, fn):
    """Run fn(rank) on `world` threads; re-raise the first failure."""
    errs, out = [None] * world, [None] * world

    def body(r):
        try:
            s = torch.cuda.Stream(device=0)
            with torch.cuda.stream(s):
                out[r] = fn(r, s)
            s.synchronize()
        except BaseException as e:   # noqa: BLE001 - reported below
            errs[r] = e
    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
        assert not t.is_alive(), "shard group thread hung"
    for e in errs:
        if e is not None:
            raise e
    return out


CASES = [("FLOAT32", "normal"), ("FLOAT16", "special"), ("BFLOAT16", "bits"),
         ("INT32", "bits"), ("FLOAT64", "uniform100")]


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("dtname,cls", CASES)
def test_local_group_allreduce_rank_order(world, dtname, cls):
    """reduce_scatter + allgather (PostNcclCalls REDUCE then BROADCAST)."""
    from prophet_amd.dtypes import elem_size
    from prophet_amd.shard import ShardComm, owner_ranges
    dt = getattr(_dt(), dtname)
    es = elem_size(dt)
    E = 100_003
    vecs = [_vec(dt, E, r, cls, 700 + world) for r in range(world)]
    want = _sliced_fold(dt, vecs, E, world)
    comms = ShardComm.local_group([0] * world)
    ranges = owner_ranges(E, world)

    def rank(r, s):
        lo, hi = ranges[r]
        local = _dev(vecs[r])
        recv = [torch.empty((hi - lo) * es, dtype=torch.uint8, device="cuda:0")
                for _ in range(world)]
        recv[r] = None
        owned = torch.empty((hi - lo) * es, dtype=torch.uint8, device="cuda:0")
        full = torch.empty(E * es, dtype=torch.uint8, device="cuda:0")
        comms[r].reduce_scatter(local, recv, owned, elems=E, dtype=dt, stream=s)
        comms[r].allgather(owned, full, elems=E, dtype=dt, stream=s)
        s.synchronize()
        return owned.cpu().numpy(), full.cpu().numpy()
    res = _threads(world, rank)
    for r, (owned, full) in enumerate(res):
        lo, hi = ranges[r]
        assert np.array_equal(owned, want[lo * es:hi * es]), f"rank {r} owned slice"
        assert np.array_equal(full, want), f"rank {r} gathered vector"
    for c in comms:
        c.close()


def test_local_group_in_place_like_reference():
    """PostNcclCalls with task->tensor == task->output: each owner folds into
    its slice of its own vector (dst = p + lo; ranks > 0 alias a later
    source), then the all-gather runs in place (owned = full + lo)."""
    from prophet_amd.shard import ShardComm, ShardedReducer, owner_ranges
    DType = _dt()
    world, E = 3, 65_537
    vecs = [_vec(DType.FLOAT32, E, r, "normal", 91) for r in range(world)]
    want = _sliced_fold(DType.FLOAT32, vecs, E, world)
    comms = ShardComm.local_group([0] * world)
    ranges = owner_ranges(E, world)

    def rank(r, s):
        lo, hi = ranges[r]
        p = _dev(vecs[r]).view(torch.float32)
        recv = [torch.empty(hi - lo, device="cuda:0") for _ in range(world)]
        comms[r].reduce_scatter(p, recv, p[lo:hi], stream=s)
        comms[r].allgather(p[lo:hi], p, stream=s)
        s.synchronize()
        a = p.cpu().numpy().view(np.uint8).copy()
        # ShardedReducer over the same communicator: the same bits again
        q = _dev(vecs[r]).view(torch.float32)
        out = torch.empty(E, device="cuda:0")
        ShardedReducer(E, comm=comms[r]).allreduce(q, out)
        s.synchronize()
        return a, out.cpu().numpy().view(np.uint8).copy()
    for r, (a, b) in enumerate(_threads(world, rank)):
        assert np.array_equal(a, want), f"rank {r} in place"
        assert np.array_equal(b, want), f"rank {r} ShardedReducer(comm)"
    for c in comms:
        c.close()


@pytest.mark.parametrize("dtname,cls", [("FLOAT32", "normal"), ("FLOAT16", "special")])
def test_local_group_scatter_reduce(dtname, cls):
    """Config 4's exchange: 5 workers' vectors landed on rank 1, each owner
    receives its slice of every push and folds them in worker order."""
    from prophet_amd.dtypes import elem_size
    from prophet_amd.shard import ShardComm, owner_ranges
    dt = getattr(_dt(), dtname)
    es = elem_size(dt)
    world, E, NW, root = 3, 50_001, 5, 1
    pushes = [_vec(dt, E, k, cls, 333) for k in range(NW)]
    want = np.zeros(E * es, np.uint8)
    ranges = owner_ranges(E, world)
    for lo, hi in ranges:
        want[lo * es:hi * es] = _fold(dt, [p[lo * es:hi * es] for p in pushes])
    comms = ShardComm.local_group([0] * world)

    def rank(r, s):
        lo, hi = ranges[r]
        ps = [_dev(p) for p in pushes] if r == root else None
        recv = [torch.empty((hi - lo) * es, dtype=torch.uint8, device="cuda:0")
                for _ in range(NW)]
        dst = torch.empty((hi - lo) * es, dtype=torch.uint8, device="cuda:0")
        comms[r].scatter_reduce(root, ps, recv, dst, E, dt, stream=s, n=NW)
        s.synchronize()
        return dst.cpu().numpy()
    for r, got in enumerate(_threads(world, rank)):
        lo, hi = ranges[r]
        assert np.array_equal(got, want[lo * es:hi * es]), f"owner {r}"
    for c in comms:
        c.close()


def test_local_group_reduce_root_and_broadcast():
    """BYTEPS_REDUCE_ROOTS mode (core_loops.cc:212-218): every key's whole
    partition is folded on GetReduceRootByKey(key), then broadcast back; the
    root folds in place into its own vector (dst = local)."""
    from prophet_amd.shard import ShardComm, reduce_root_of
    DType = _dt()
    world, E = 4, 40_000
    roots = [1, 3]
    comms = ShardComm.local_group([0] * world)
    for key in ((7 << 16) + 0, (7 << 16) + 1, (12 << 16) + 3):
        root = reduce_root_of(key, roots)
        vecs = [_vec(DType.FLOAT16, E, r, "bits", key & 0xFFFF) for r in range(world)]
        want = _fold(DType.FLOAT16, vecs)

        def rank(r, s):
            p = _dev(vecs[r]).view(torch.float16)
            recv = [torch.empty(E, dtype=torch.float16, device="cuda:0") for _ in range(world)]
            comms[r].reduce_root(root, p, recv if r == root else None, p, stream=s)
            comms[r].broadcast(root, p, stream=s)
            s.synchronize()
            return p.cpu().numpy().view(np.uint8).copy()
        for r, got in enumerate(_threads(world, rank)):
            assert np.array_equal(got, want), f"key {key} rank {r} (root {root})"
    for c in comms:
        c.close()


@pytest.mark.parametrize("E", [0, 1, 2, 5])
def test_local_group_tiny_sizes(E):
    """Fewer elements than ranks: per = 0, the last rank owns everything."""
    from prophet_amd.shard import ShardComm
    DType = _dt()
    world = 3
    vecs = [_vec(DType.INT32, max(E, 1), r, "bits", 5)[:E * 4] for r in range(world)]
    want = _sliced_fold(DType.INT32, vecs, E, world) if E else np.zeros(0, np.uint8)
    comms = ShardComm.local_group([0] * world)

    def rank(r, s):
        local = torch.from_numpy(vecs[r].copy()).to("cuda:0")
        own = E if r == world - 1 else 0
        recv = [torch.empty(max(own, 1) * 4, dtype=torch.uint8, device="cuda:0")
                for _ in range(world)]
        dst = torch.empty(max(own, 1) * 4, dtype=torch.uint8, device="cuda:0")
        full = torch.zeros(max(E, 1) * 4, dtype=torch.uint8, device="cuda:0")
        comms[r].reduce_scatter(local, recv, dst, elems=E, dtype=DType.INT32, stream=s)
        comms[r].allgather(dst, full, elems=E, dtype=DType.INT32, stream=s)
        s.synchronize()
        return full.cpu().numpy()[:E * 4]
    for r, got in enumerate(_threads(world, rank)):
        assert np.array_equal(got, want), r
    for c in comms:
        c.close()


def test_local_group_size_mismatch_fails_without_hanging():
    """A rank that sends a different size than its peer expects: both calls
    return (EARGS on the receiver) instead of hanging."""
    from prophet_amd.reducer import ReduceError
    from prophet_amd.shard import ShardComm
    DType = _dt()
    comms = ShardComm.local_group([0, 0])
    errs = [None, None]

    def rank(r, s):
        E = 1000 if r == 0 else 1200
        local = torch.zeros(E, device="cuda:0")
        recv = [torch.empty(E, device="cuda:0") for _ in range(2)]
        try:
            comms[r].reduce_scatter(local, recv, torch.empty(E, device="cuda:0"),
                                    dtype=DType.FLOAT32, stream=s)
        except ReduceError as e:
            errs[r] = e.code
    _threads(2, rank)
    assert any(e == -2 for e in errs), errs


def test_local_group_timeout_breaks_group():
    """Only one rank of two makes the call: it returns ETIMEOUT after
    BPSR_SHARD_TIMEOUT_S instead of hanging, and the group refuses later
    calls (own process: the timeout is read once)."""
    code = r"""
import torch, sys
sys.path.insert(0, %r)
from prophet_amd.shard import ShardComm
from prophet_amd.reducer import ReduceError
c = ShardComm.local_group([0, 0])
x = torch.zeros(1000, device="cuda:0")
codes = []
for _ in range(2):
    try:
        c[0].reduce_scatter(x, [None, torch.empty(500, device="cuda:0")], torch.empty(500, device="cuda:0"))
        codes.append(0)
    except ReduceError as e:
        codes.append(e.code)
print(codes)
""" % ROOT
    env = dict(os.environ, BPSR_SHARD_TIMEOUT_S="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "[-5, -5]"


def _rccl_world1_checks(comm):
    """One rank: reduce_scatter is a copy, scatter_reduce folds 8 landed
    pushes (the config-2 round on a comm), reduce_root folds 1, broadcast and
    allgather are copies; everything through RCCL's group calls."""
    from prophet_amd.shard import ShardedReducer
    DType = _dt()
    E = 1_000_003
    for dt, cls in ((DType.FLOAT32, "normal"), (DType.FLOAT16, "special")):
        pushes = [_vec(dt, E, k, cls, 808) for k in range(8)]
        es = pushes[0].nbytes // E
        want = _fold(dt, pushes)
        ps = [_dev(p) for p in pushes]
        dst = torch.empty(E * es, dtype=torch.uint8, device="cuda:0")
        comm.scatter_reduce(0, ps, [None] * 8, dst, E, dt)
        full = torch.empty_like(dst)
        comm.allgather(dst, full, elems=E, dtype=dt)
        rs = torch.empty_like(dst)
        comm.reduce_scatter(ps[3], [None], rs, elems=E, dtype=dt)
        comm.broadcast(0, rs, elems=E, dtype=dt)
        torch.cuda.synchronize()
        assert np.array_equal(dst.cpu().numpy(), want)
        assert np.array_equal(full.cpu().numpy(), want)
        assert np.array_equal(rs.cpu().numpy(), pushes[3])
    out = torch.empty(E, device="cuda:0")
    x = torch.randn(E, device="cuda:0")
    ShardedReducer(E, comm=comm).allreduce(x, out)
    torch.cuda.synchronize()
    assert torch.equal(out, x)


def test_rccl_world1_through_abi():
    from prophet_amd.shard import ShardComm
    uid = ShardComm.unique_id()
    assert len(uid) == 128
    comm = ShardComm.init(uid, 1, 0, 0)
    assert (comm.world, comm.rank, comm.device) == (1, 0, 0)
    _rccl_world1_checks(comm)
    comm.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_wrap_torch_process_group_comm():
    """A caller-owned RCCL communicator (torch's ProcessGroupNCCL, as
    core_loops.cc would pass NcclManager::GetComm) wrapped, not owned."""
    import torch.distributed as dist
    from prophet_amd.shard import ShardComm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda", 0)
    if dist.is_initialized():       # a group another test left behind
        dist.destroy_process_group()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        t = torch.ones(4, device=dev)
        dist.all_reduce(t)          # the communicator exists after the first collective
        torch.cuda.synchronize()
        be = dist.group.WORLD._get_backend(dev)
        ptr = be._comm_ptr()
        assert ptr, "ProcessGroupNCCL has no communicator"
        comm = ShardComm.wrap(ptr)
        assert (comm.world, comm.rank, comm.device) == (1, 0, 0)
        _rccl_world1_checks(comm)
        comm.close()                # frees the wrapper only; torch's comm lives on
        dist.all_reduce(t)
        torch.cuda.synchronize()
        assert t[0].item() == 1.0
    finally:
        dist.destroy_process_group()


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        torch.cuda.set_device(rank)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from prophet_amd.dtypes import DType
        from prophet_amd.shard import ShardComm, ShardedReducer
        comm = ShardComm.from_group(device=rank)
        E = 1_000_003
        x = torch.from_numpy(_vec(DType.FLOAT32, E, rank, "normal", 55)).to(rank) \
            .view(torch.float32)
        out = torch.empty(E, device=f"cuda:{rank}")
        ShardedReducer(E, comm=comm).allreduce(x, out)
        torch.cuda.synchronize()
        q.put((rank, out.cpu().numpy().view(np.uint8).tobytes()))
        comm.close()
    except Exception as e:  # fail fast instead of a queue timeout
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rccl_multi_gpu_one_rank_per_gpu():
    """RCCL grouped send/recv between processes, one per GPU (the unique id
    carried over a gloo group, as NcclManager carries it over its socket)."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs (RCCL refuses two ranks on one GPU)")
    import torch.multiprocessing as mp
    world = min(n, 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    DType = _dt()
    want = _sliced_fold(DType.FLOAT32, [_vec(DType.FLOAT32, 1_000_003, r, "normal", 55)
                                        for r in range(world)], 1_000_003, world)
    for r in range(world):
        assert isinstance(res[r], bytes), res[r]
        assert res[r] == want.tobytes(), r
