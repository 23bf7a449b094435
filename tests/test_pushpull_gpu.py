"""End-to-end push_pull over the GPU-resident server: whole ResNet-50-shaped
gradient sets, partitioned and keyed like InitTensor/EnqueueTensor
(operations.cc:99-317), pushed in the Prophet PUSH scheduler's release groups
by 3 worker threads, folded on the GPU, pulled back in place.  Every worker's
every byte equals the oracle's left fold of that partition in the server's
recorded arrival order."""
import threading

import numpy as np
import pytest

from oracle.oracle import PortReducer
from prophet_amd.buckets import resnet50_param_sizes
from prophet_amd.dtypes import DType

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _grads(rank, it, sizes):
    rng = np.random.default_rng(1000 * it + rank)
    return {f"g{i}": rng.standard_normal(n, dtype=np.float32) for i, n in enumerate(sizes)}


@pytest.mark.parametrize("policy", [0, 1], ids=["fused", "incremental"])
def test_push_pull_iterations_prophet_order(policy):
    from prophet_amd.prophet import ProphetPushQueue, model_checkpoints
    from prophet_amd.pushpull import ServerFrontend, Worker
    from prophet_amd.server import PSServer
    assert torch.cuda.is_available()
    N, iters = 3, 2
    sizes = [max(1, n // 32) for n in resnet50_param_sizes()]        # 161 tensors, ~3 MB
    srv = PSServer(N, engine_lanes=4, policy=policy)
    fe = ServerFrontend(srv)
    workers = [Worker(r, fe, partition_bytes=64 << 10) for r in range(N)]
    data = {(r, it): _grads(r, it, sizes) for r in range(N) for it in range(iters + 1)}
    held = {(r, it): {k: v.copy() for k, v in data[(r, it)].items()}
            for r in range(N) for it in range(1, iters + 1)}
    bar = threading.Barrier(N + 1)
    errors = []

    def run(w):
        try:
            for name in data[(w.rank, 0)]:
                w.declare(name)
            for name, t in data[(w.rank, 0)].items():
                w.init_tensor(name, t, DType.FLOAT32)
            for it in range(1, iters + 1):
                q = ProphetPushQueue(batch_size=64, net_b=1000, credit=1 << 18,
                                     checkpoints=model_checkpoints(len(sizes)))
                w.push_pull_iteration(held[(w.rank, it)], scheduler=q)
                bar.wait(timeout=120)            # main thread reads arrival orders
                bar.wait(timeout=120)
        except Exception as e:  # surfaced below
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=run, args=(w,)) for w in workers]
    for t in ts:
        t.start()
    port = PortReducer(nthreads=4)
    ctx0 = workers[0].contexts
    for it in range(1, iters + 1):
        bar.wait(timeout=240)
        orders = {}
        for name, c in ctx0.items():
            for key, off, ln in c.parts:
                rounds, _, order = srv.key_info(key)
                assert rounds == it
                orders[key] = order
        bar.wait(timeout=120)
        for name, c in ctx0.items():
            for key, off, ln in c.parts:
                order = orders[key]
                assert sorted(order) == list(range(N))
                ins = [data[(r, it)][name].view(np.uint8)[off:off + ln].copy() for r in order]
                want = np.zeros(ln, np.uint8)
                port.sum_n(want, ins, ln, DType.FLOAT32)
                for r in range(N):
                    got = held[(r, it)][name].view(np.uint8)[off:off + ln]
                    assert np.array_equal(got, want), (it, name, key, r)
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    srv.close()


def test_push_pull_device_tensors():
    """Device tensors (BYTEPS_SERVER_DEVICE pushes and pulls): the in-place
    result equals torch's left fold in the recorded order."""
    from prophet_amd.pushpull import ServerFrontend, Worker
    from prophet_amd.server import PSServer
    N = 2
    dev = torch.device("cuda:0")
    srv = PSServer(N)
    fe = ServerFrontend(srv)
    ws = [Worker(r, fe, partition_bytes=1 << 20) for r in range(N)]
    gen = torch.Generator(device=dev)
    init = {r: torch.zeros(3_000_001, device=dev) for r in range(N)}
    grads = {}
    for r in range(N):
        gen.manual_seed(r)
        grads[r] = torch.randn(3_000_001, device=dev, generator=gen)
    orig = {r: grads[r].clone() for r in range(N)}

    def run(w):
        w.declare("w")
        w.init_tensor("w", init[w.rank], DType.FLOAT32)
        w.push_pull("w", grads[w.rank])
    ts = [threading.Thread(target=run, args=(w,)) for w in ws]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    torch.cuda.synchronize()
    c = ws[0].contexts["w"]
    assert len(c.parts) == 12                        # 12,000,004 B under a 1 MiB bound
    for key, off, ln in c.parts:
        order = srv.key_info(key)[2]
        a, b = off // 4, (off + ln) // 4
        ref = orig[order[0]][a:b].clone()
        ref.add_(orig[order[1]][a:b])
        for r in range(N):
            assert torch.equal(grads[r][a:b], ref), (key, r)
    srv.close()
