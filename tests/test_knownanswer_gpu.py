"""The reference's own known-answer test, restated on this build's whole
push_pull path: tests/test_mxnet.py:76-113 (test_byteps_push_pull_inplace).

Every rank declares the same 1-D/2-D/3-D tensors (17, 17x17, 17x17x17) of
uniform(-100, 100) values drawn with one seed (identical on every rank), cast
to int32 / int64 / float32 / float64, and push_pulls them in place; the result
must equal tensor * size within the reference's ladder — 0 when size <= 3 or
for integers, 1e-4 below 10 ranks, 5e-4 below 15 — compared exactly as the
reference does: max(result - tensor * size), signed, in the tensor's dtype.
Ranks are worker threads talking to the GPU-resident server through
pushpull.Worker (InitTensor keys, partitions, Cantor request word), tensors on
the device.  The bits are also checked
against the oracle's left fold of the same inputs, which is the stricter
parity bar."""
import itertools
import threading

import numpy as np
import pytest

from oracle.oracle import PortReducer
from prophet_amd.dtypes import DType

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]

DTYPES = {"int32": (DType.INT32, np.int32, torch.int32),
          "int64": (DType.INT64, np.int64, torch.int64),
          "float32": (DType.FLOAT32, np.float32, torch.float32),
          "float64": (DType.FLOAT64, np.float64, torch.float64)}
SHAPES = [(), (17,), (17, 17), (17, 17, 17)]


def _threshold(size, dtype):
    if size <= 3 or dtype in ("int32", "int64"):
        return 0.0
    if size < 10:
        return 1e-4
    if size < 15:
        return 5e-4
    return None                          # the reference stops checking (`break`)


@pytest.mark.parametrize("mode", ["sync", "async"])
@pytest.mark.parametrize("size", [2, 3, 8, 14])
def test_byteps_push_pull_inplace_known_answer(size, mode):
    from prophet_amd.pushpull import ServerFrontend, Worker
    from prophet_amd.server import PSServer
    srv = PSServer(size, engine_lanes=4)
    fe = ServerFrontend(srv)
    workers = [Worker(r, fe) for r in range(size)]
    cases = []
    for dtype, dim in itertools.product(DTYPES, [1, 2, 3]):
        # mx.random.seed(1234) on every rank: identical inputs
        base = np.random.default_rng(1234).uniform(-100, 100, SHAPES[dim])
        cases.append((f"tensor_{len(cases)}", dtype, base.astype(DTYPES[dtype][1])))
    tensors = {(r, name): torch.from_numpy(arr.copy()).cuda()
               for r in range(size) for name, _, arr in cases}
    torch.cuda.synchronize()
    errors = []

    def run(w):
        try:
            for name, dtype, _ in cases:
                w.declare(name)
            for name, dtype, _ in cases:
                w.init_tensor(name, tensors[(w.rank, name)], DTYPES[dtype][0])
            if mode == "sync":
                for name, dtype, _ in cases:
                    w.push_pull(name, tensors[(w.rank, name)])
            else:                   # push_pull_async + synchronize (byteps/torch/ops.py)
                hs = [w.push_pull_async(name, tensors[(w.rank, name)]) for name, _, _ in cases]
                for h in hs:
                    w.synchronize(h)
                w.close()
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=run, args=(w,)) for w in workers]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=180)
    assert not errors, errors
    port = PortReducer(nthreads=4)
    for name, dtype, arr in cases:
        multiplied = arr * DTYPES[dtype][1](size)          # in the tensor's dtype
        thr = _threshold(size, dtype)
        # the oracle: left fold of `size` identical pushes (server.cc:216-273)
        want = np.zeros(arr.nbytes, np.uint8)
        port.sum_n(want, [arr.view(np.uint8)] * size, arr.nbytes, DTYPES[dtype][0])
        for r in range(size):
            got = tensors[(r, name)].cpu().numpy()
            assert np.array_equal(got.view(np.uint8).ravel(), want), (name, dtype, r)
            if thr is not None:                      # test_mxnet.py:95, :112-113
                diff = float(np.max(got - multiplied))
                assert diff <= thr, (name, dtype, r, diff, thr)
    srv.close()


@pytest.mark.parametrize("size", [2, 3])
def test_byteps_broadcast(size):
    """tests/test_mxnet.py:116-158 on this build: every (dtype, dim, root rank)
    — tensor = ones * rank, broadcast from root_rank through push_pull with
    zeros on the non-root ranks (byteps/torch/__init__.py:264-272); the
    result equals ones * root_rank on every rank, bit for bit, and the source
    tensors are not modified."""
    from prophet_amd.pushpull import ServerFrontend, Worker
    from prophet_amd.server import PSServer
    srv = PSServer(size, engine_lanes=2)
    fe = ServerFrontend(srv)
    workers = [Worker(r, fe) for r in range(size)]
    cases = [(f"{len_}", dtype, dim, root)
             for len_, (dtype, dim, root) in enumerate(
                 itertools.product(DTYPES, [1, 2, 3], range(size)))]
    src = {(r, c[0]): (torch.ones(SHAPES[c[2]], device="cuda") * r).to(DTYPES[c[1]][2])
           for r in range(size) for c in cases}
    results, errors = {}, []

    def run(w):
        try:
            for name, dtype, dim, root in cases:
                w.declare(name)
                w.init_tensor(name, src[(w.rank, name)], DTYPES[dtype][0])
            for name, dtype, dim, root in cases:
                results[(w.rank, name)] = w.broadcast(name, src[(w.rank, name)], root)
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=run, args=(w,)) for w in workers]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=180)
    assert not errors, errors
    torch.cuda.synchronize()
    for name, dtype, dim, root in cases:
        want = (torch.ones(SHAPES[dim], device="cuda") * root).to(DTYPES[dtype][2])
        for r in range(size):
            assert torch.equal(results[(r, name)], want), (name, dtype, dim, root, r)
            mine = (torch.ones(SHAPES[dim], device="cuda") * r).to(DTYPES[dtype][2])
            assert torch.equal(src[(r, name)], mine), "broadcast modified its source"
    srv.close()
