"""Key-space sharding: ownership math (core_loops.cc:208-247) and the
multi-process data path over gloo (world_size 2, 3 and 8 — the driver's node size — on CPU).

The local fold in these CPU tests is the oracle (test infrastructure), injected
into ShardedReducer; the product default is the HIP fold (tests/test_parity_gpu.py
covers it on the GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from prophet_amd.buckets import partition_all, vgg16_param_sizes
from prophet_amd.shard import owner_of, owner_ranges, split_buckets


def test_owner_ranges_match_reference_split():
    # core_loops.cc:210-211: per = len/nccl_size/unit; tail to the root (last)
    assert owner_ranges(10, 4) == [(0, 2), (2, 4), (4, 6), (6, 10)]
    assert owner_ranges(8, 8) == [(i, i + 1) for i in range(8)]
    assert owner_ranges(3, 4) == [(0, 0), (0, 0), (0, 0), (0, 3)]
    vgg = sum(vgg16_param_sizes())
    r = owner_ranges(vgg, 8)
    assert all(hi - lo == 17_294_693 for lo, hi in r)
    for e in (0, 1, 17_294_692, 17_294_693, vgg - 1):
        g = owner_of(e, vgg, 8)
        assert r[g][0] <= e < r[g][1]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_split_buckets_covers_exactly(world):
    sizes = [p.len // 4 for p in partition_all([n * 4 for n in vgg16_param_sizes()])]
    pieces = split_buckets(sizes, world)
    total = sum(sizes)
    cover = np.zeros(total, dtype=np.int8)
    ranges = owner_ranges(total, world)
    starts = np.cumsum([0] + sizes)
    for p in pieces:
        assert ranges[p.owner][0] <= p.start and p.start + p.length <= ranges[p.owner][1]
        assert starts[p.bucket] + p.bucket_offset == p.start
        cover[p.start: p.start + p.length] += 1
    assert (cover == 1).all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fold():
    from oracle.oracle import PortReducer
    from prophet_amd.dtypes import from_torch
    port = PortReducer(nthreads=1)

    def fold(dst, srcs):
        a = dst.numpy().view(np.uint8)
        ins = [s.contiguous().numpy().view(np.uint8) for s in srcs]
        assert port.sum_n(a, ins, a.nbytes, from_torch(dst.dtype)) == 0
    return fold


def _worker(rank, world, port, n_elems, n_workers, q, mode="scatter"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from prophet_amd import synth
        from prophet_amd.dtypes import DType
        from prophet_amd.shard import ShardedReducer
        sr = ShardedReducer(n_elems, fold=_oracle_fold())
        root = 0
        pushes = None
        if rank == root or mode == "host":   # "host": every rank sees the shm pushes
            pushes = [torch.from_numpy(synth.bucket(DType.FLOAT32, n_elems, k, "normal", 77))
                      for k in range(n_workers)]
        slots = [torch.empty(sr.owned, dtype=torch.float32) for _ in range(n_workers)]
        owned = torch.empty(sr.owned, dtype=torch.float32)
        if mode == "host":
            sr.reduce_from_host(pushes, slots, owned)
        else:
            sr.scatter_reduce(root, pushes, slots, owned)
        full = torch.empty(n_elems, dtype=torch.float32)
        sr.allgather(owned, full)
        q.put((rank, full.numpy().tobytes()))
    except Exception as e:      # fail fast instead of a queue timeout
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("mode", ["scatter", "host"])
def test_scatter_reduce_allgather_gloo(world, mode):
    """Pushes on rank 0 scattered to owners (scatter_reduce), or read from host
    memory by every owner directly (reduce_from_host): the gathered result is
    the unsharded left fold, bit for bit."""
    n_elems, n_workers = 10_007, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_elems, n_workers, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # unsharded left fold by the oracle
    from oracle.oracle import PortReducer
    from prophet_amd import synth
    from prophet_amd.dtypes import DType
    ins = [np.ascontiguousarray(synth.bucket(DType.FLOAT32, n_elems, k, "normal", 77)).view(np.uint8)
           for k in range(n_workers)]
    want = np.zeros(n_elems * 4, np.uint8)
    PortReducer().sum_n(want, ins, want.nbytes, DType.FLOAT32)
    for r in range(world):
        assert results[r] == want.tobytes(), f"rank {r}"


def _worker_allreduce(rank, world, port, n_elems, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from prophet_amd import synth
        from prophet_amd.dtypes import DType
        from prophet_amd.shard import ShardedReducer
        sr = ShardedReducer(n_elems, fold=_oracle_fold())
        mine = torch.from_numpy(synth.bucket(DType.FLOAT16, n_elems, rank, "bits", 91)).view(torch.float16)
        out = torch.empty(n_elems, dtype=torch.float16)
        sr.allreduce(mine, out)
        q.put((rank, out.numpy().tobytes()))
    except Exception as e:      # fail fast instead of a queue timeout
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_local_reduce_allreduce_rank_order_gloo(world):
    """Worker local reduce (core_loops.cc:184-261) as P2P + fold + all-gather:
    every rank ends with the oracle's left fold in rank order (fp16 per-step RNE)."""
    n_elems = 9_999
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_allreduce, args=(r, world, port, n_elems, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.oracle import PortReducer
    from prophet_amd import synth
    from prophet_amd.dtypes import DType
    ins = [np.ascontiguousarray(synth.bucket(DType.FLOAT16, n_elems, r, "bits", 91)).view(np.uint8)
           for r in range(world)]
    want = np.zeros(n_elems * 2, np.uint8)
    PortReducer().sum_n(want, ins, want.nbytes, DType.FLOAT16)
    for r in range(world):
        assert results[r] == want.tobytes(), f"rank {r}"


def _worker_bench_leg(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        res = bench.scatter_leg(torch.device("cpu"), world, rank, 4, reps=2, n_elems=20_011,
                                fold=_oracle_fold())
        q.put((rank, res))
    except Exception as e:      # fail fast instead of a queue timeout
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_scatter_leg_gloo(world):
    """bench.py's config-4 leg (reported beside `value` at N > 1 GPUs): scatter
    from GPU 0, owner fold, all-gather; the root's check against torch's left
    fold passes and every rank reports the same max-over-ranks times."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_bench_leg, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert isinstance(results[r], dict), results[r]
    assert results[0]["exact_vs_torch_fold"] is True
    assert len({results[r]["scatter_fold_ms"] for r in range(world)}) == 1
