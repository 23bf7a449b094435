"""GPU tests of the paths around the kernel: host-streamed reduction (cfg5
shape, small), the sharded reducer on one rank, the HBM slot arena."""
import numpy as np
import pytest

from golden_util import assert_bytes_match
from oracle.oracle import PortReducer
from prophet_amd import synth
from prophet_amd.dtypes import DType, elem_size

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def red():
    assert torch.cuda.is_available()
    from prophet_amd.reducer import GpuReducer
    return GpuReducer(device=0)


@pytest.mark.parametrize("dt", [DType.BFLOAT16, DType.FLOAT16, DType.FLOAT32, DType.INT8],
                         ids=lambda d: DType(d).name)
@pytest.mark.parametrize("extra", [0, 1, 7])
@pytest.mark.parametrize("zero_copy", [False, True], ids=["sdma", "zerocopy"])
def test_streaming_reducer_bit_exact(red, dt, extra, zero_copy):
    from prophet_amd.stream import StreamingReducer
    es = elem_size(dt)
    n = 300_007
    L = n * es + (extra % es if es > 1 else 0)
    N = 5
    ins = [np.ascontiguousarray(synth.bucket(dt, n + 1, k, "special" if dt in (DType.FLOAT16, DType.BFLOAT16, DType.FLOAT32) else "normal", 31))
           .view(np.uint8)[:L].copy() for k in range(N)]
    host = [torch.from_numpy(x).pin_memory() for x in ins]
    out = torch.zeros(L, dtype=torch.uint8).pin_memory()
    sr = StreamingReducer(N, chunk_bytes=64 * 1024 + 48, depth=3, reducer=red,
                          zero_copy=zero_copy)
    sr.reduce(host, out, L, dt)
    want = np.zeros(L, np.uint8)
    PortReducer(nthreads=4).sum_n(want, ins, L, dt)
    assert_bytes_match(dt, out.numpy(), want, nan_class_f32_f64=False)


def test_streaming_zero_copy_rejects_pageable(red):
    from prophet_amd.reducer import ReduceError
    from prophet_amd.stream import StreamingReducer
    sr = StreamingReducer(2, reducer=red, zero_copy=True)
    host = [torch.zeros(64, dtype=torch.uint8) for _ in range(2)]     # not pinned
    with pytest.raises(ReduceError):
        sr.reduce(host, torch.zeros(64, dtype=torch.uint8).pin_memory(), 64, DType.UINT8)


@pytest.fixture
def gloo_world1():
    """A world-1 gloo default group for the test, destroyed after it (a group
    left behind would make a later init_process_group fail)."""
    import os
    import socket
    import torch.distributed as dist
    made = False
    if not dist.is_initialized():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=0, world_size=1)
        made = True
    yield
    if made and dist.is_initialized():
        dist.destroy_process_group()


def test_sharded_reduce_from_host_single_rank(red, gloo_world1):
    """reduce_from_host: the owner's slice of pinned host pushes straight to its
    HBM slots, HIP fold; equal to torch's left fold."""
    import torch.distributed as dist
    from prophet_amd.shard import ShardedReducer
    n = 200_003
    sr = ShardedReducer(n)
    dev = torch.device("cuda:0")
    host = [torch.randn(n).pin_memory() for _ in range(6)]
    slots = [torch.empty(sr.owned, device=dev) for _ in range(6)]
    owned = torch.empty(sr.owned, device=dev)
    sr.reduce_from_host(host, slots, owned)
    torch.cuda.synchronize()
    ref = host[0].clone()
    for h in host[1:]:
        ref.add_(h)
    assert torch.equal(owned.cpu(), ref)


def test_sharded_reducer_single_rank(red, gloo_world1):
    import torch.distributed as dist
    from prophet_amd.shard import ShardedReducer
    n = 100_003
    sr = ShardedReducer(n)            # default fold = HIP via the C ABI
    dev = torch.device("cuda:0")
    pushes = [torch.randn(n, device=dev) for _ in range(4)]
    slots = [torch.empty(n, device=dev) for _ in range(4)]
    owned = torch.empty(n, device=dev)
    sr.scatter_reduce(0, pushes, slots, owned)
    ref = pushes[0].clone()
    for p in pushes[1:]:
        ref.add_(p)
    torch.cuda.synchronize()
    assert torch.equal(owned, ref)
    full = torch.empty(n, device=dev)
    sr.allgather(owned, full)
    assert torch.equal(full, ref)


def test_arena_slots_are_skewed_and_disjoint():
    from prophet_amd.arena import BucketArena
    a = BucketArena(9, 1 << 20, torch.device("cuda:0"))
    ptrs = [s.data_ptr() for s in a.slots()]
    assert all(b - a_ == a.stride for a_, b in zip(ptrs, ptrs[1:]))
    assert a.stride % (1 << 20) != 0
    assert all(s.numel() == 1 << 20 for s in a.slots())


@pytest.mark.timeout(600)
def test_cfg5_full_size_streamed_bf16(red):
    """BASELINE config 5 at its own size: 16 workers x 256 MiB bf16 (4 GiB of
    pinned host pushes) streamed H2D -> fold -> D2H by StreamingReducer.  The
    whole 256 MiB result equals torch's own bf16 left fold (per-step RNE, the
    build's bf16 rule), and a strided set of windows equals the CPU
    restatement (parity for bf16 is pinned by the restatement only: the
    reference has no bf16)."""
    from prophet_amd.stream import StreamingReducer
    N, B = 16, 256 << 20
    n = B // 2
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    host = []
    for k in range(N):
        gen.manual_seed(5000 + k)
        t = torch.empty(B, dtype=torch.uint8).pin_memory()
        t.view(torch.bfloat16).copy_(torch.randn(n, device=dev, generator=gen)
                                     .to(torch.bfloat16))
        host.append(t)
    out = torch.empty(B, dtype=torch.uint8).pin_memory()
    StreamingReducer(N, reducer=red).reduce(host, out, B, DType.BFLOAT16)
    # whole result vs torch's left fold on the device, chunk by chunk
    step = 32 << 20
    for o in range(0, n, step):
        e = min(n, o + step)
        acc = host[0].view(torch.bfloat16)[o:e].to(dev)
        for h in host[1:]:
            acc.add_(h.view(torch.bfloat16)[o:e].to(dev))
        assert torch.equal(acc.view(torch.int16).cpu(),
                           out.view(torch.bfloat16)[o:e].view(torch.int16)), f"chunk at {o}"
    # strided windows vs the restatement
    port = PortReducer(nthreads=4)
    W = 65_536
    for i in range(16):
        o = (i * (n - W)) // 15
        ins = [h.numpy()[2 * o: 2 * (o + W)].copy() for h in host]
        want = np.zeros(2 * W, np.uint8)
        port.sum_n(want, ins, 2 * W, DType.BFLOAT16)
        assert np.array_equal(out.numpy()[2 * o: 2 * (o + W)], want), f"window at {o}"
