"""Key-space sharding across processes with the HIP fold (row a11/f2/e).

* ``nccl`` (RCCL over xGMI), one rank per GPU: ``scatter_reduce`` +
  ``allgather`` (config 4's exchange, core_loops.cc:234-254) and the worker
  local reduce ``allreduce`` (core_loops.cc:184-261), bit-exact with the
  oracle.  Needs >= 2 GPUs; skipped on a 1-GPU box.
* ``gloo`` ranks sharing the one GPU: the same collectives move CPU tensors
  and every rank folds its owned slice ON THE GPU through the C ABI — the
  multi-rank HIP fold on any box.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_want(dt, n_elems, n_workers, cls, seed):
    from oracle.oracle import PortReducer
    from prophet_amd import synth
    from prophet_amd.dtypes import elem_size
    es = elem_size(dt)
    ins = [np.ascontiguousarray(synth.bucket(dt, n_elems, k, cls, seed)).view(np.uint8)
           for k in range(n_workers)]
    want = np.zeros(n_elems * es, np.uint8)
    PortReducer(nthreads=4).sum_n(want, ins, want.nbytes, dt)
    return want.tobytes()


def _rank_main(rank, world, port, backend, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        if backend == "nccl":
            torch.cuda.set_device(rank)
            dev = torch.device("cuda", rank)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
            comm_dev = dev
        else:
            dev = torch.device("cuda", 0)
            dist.init_process_group("gloo", rank=rank, world_size=world)
            comm_dev = torch.device("cpu")
        from prophet_amd import synth
        from prophet_amd.dtypes import DType, from_torch
        from prophet_amd.reducer import GpuReducer
        from prophet_amd.shard import ShardedReducer
        red = GpuReducer(device=dev.index)

        def hip_fold(dst, srcs):
            """Owner fold on the GPU through the C ABI (CPU tensors staged in)."""
            if dst.device.type == "cuda":
                red.sum_n(dst, srcs, dst.numel() * dst.element_size(), from_torch(dst.dtype))
                return
            d = torch.empty(dst.shape, dtype=dst.dtype, device=dev)
            ss = [s.to(dev) for s in srcs]
            red.sum_n(d, ss, d.numel() * d.element_size(), from_torch(dst.dtype))
            dst.copy_(d.cpu())

        res = {}
        # config 4's exchange: N pushes land on rank 0, scatter to owners, fold, gather
        E, NW = 1_000_003, 5
        sr = ShardedReducer(E, fold=hip_fold)
        pushes = None
        if rank == 0:
            pushes = [torch.from_numpy(synth.bucket(DType.FLOAT32, E, k, "normal", 61))
                      .to(comm_dev) for k in range(NW)]
        slots = [torch.empty(sr.owned, device=comm_dev) for _ in range(NW)]
        owned = torch.empty(sr.owned, device=comm_dev)
        sr.scatter_reduce(0, pushes, slots, owned)
        full = torch.empty(E, device=comm_dev)
        sr.allgather(owned, full)
        res["scatter"] = full.cpu().numpy().tobytes()
        # worker local reduce: every rank's own fp16 gradient, rank-order fold
        E2 = 777_777
        sr2 = ShardedReducer(E2, fold=hip_fold)
        mine = torch.from_numpy(synth.bucket(DType.FLOAT16, E2, rank, "bits", 62)) \
            .view(torch.float16).to(comm_dev)
        out = torch.empty(E2, dtype=torch.float16, device=comm_dev)
        sr2.allreduce(mine, out)
        res["allreduce"] = out.cpu().numpy().tobytes()
        if comm_dev.type == "cuda":
            torch.cuda.synchronize()
        q.put((rank, res))
    except Exception as e:  # fail fast instead of a queue timeout
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(world, backend):
    import torch.multiprocessing as mp
    from prophet_amd.dtypes import DType
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, backend, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_s = _oracle_want(DType.FLOAT32, 1_000_003, 5, "normal", 61)
    want_a = _oracle_want(DType.FLOAT16, 777_777, world, "bits", 62)
    for r in range(world):
        assert isinstance(results[r], dict), results[r]
        assert results[r]["scatter"] == want_s, f"rank {r} scatter"
        assert results[r]["allreduce"] == want_a, f"rank {r} allreduce"


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_hip_fold_gloo_ranks_one_gpu(world):
    _run(world, "gloo")


def test_sharded_nccl_multi_gpu():
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs (RCCL ranks one per GPU)")
    _run(min(n, 4), "nccl")


def test_cfg4_vgg16_full_size_owner_slices_one_gpu():
    """BASELINE config 4 at its own size on one GPU: the 8-way fp32 VGG-16 set
    (138,357,544 elements per worker) cut by the reference's reduce-scatter
    ownership for G = 8 (core_loops.cc:208-211), each owner's slice folded by
    the HIP fold as its GPU would; the slices put together equal torch's left
    fold of the whole set bit for bit, and sampled windows equal the oracle."""
    from oracle.oracle import PortReducer
    from prophet_amd.buckets import vgg16_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.reducer import GpuReducer
    from prophet_amd.shard import owner_ranges
    dev = torch.device("cuda:0")
    E, N, G = sum(vgg16_param_sizes()), 8, 8
    assert E == 138_357_544
    gen = torch.Generator(device=dev)
    gen.manual_seed(44)
    pushes = [torch.randn(E, device=dev, generator=gen) for _ in range(N)]
    out = torch.empty(E, device=dev)
    red = GpuReducer(device=0)
    ranges = owner_ranges(E, G)
    assert all(hi - lo == 17_294_693 for lo, hi in ranges)
    for lo, hi in ranges:
        red.sum_n(out[lo:hi], [p[lo:hi] for p in pushes], (hi - lo) * 4, DType.FLOAT32)
    ref = pushes[0].clone()
    for p in pushes[1:]:
        ref.add_(p)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    port = PortReducer(nthreads=4)
    W = 50_000
    for lo, hi in ranges:                 # each shard's first and last window
        for a in (lo, hi - W):
            ins = [p[a:a + W].cpu().numpy().view(np.uint8) for p in pushes]
            want = np.zeros(W * 4, np.uint8)
            port.sum_n(want, ins, W * 4, DType.FLOAT32)
            assert np.array_equal(out[a:a + W].cpu().numpy().view(np.uint8), want), a
