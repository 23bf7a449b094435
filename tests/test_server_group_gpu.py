"""Key space over several server instances (byteps_server_group_*) on the GPU:
two instances on device 0 (both ordinals 0 — the routing, scatter and gather
are the same for distinct GPUs), fp32 and fp16, three rounds in random
arrival order from concurrent worker threads, whole-key hash and range split.
Each piece of each key must equal the oracle's left fold in the arrival order
ITS instance recorded (range pieces of one key may fold in different orders
when workers race; whole keys have one order, as in the reference)."""
import random
import threading
import time

import numpy as np
import pytest

from oracle.oracle import PortReducer
from prophet_amd import synth
from prophet_amd.dtypes import DType, elem_size

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]


def data(dt, n, worker, rnd, key):
    cls = "special" if dt == DType.FLOAT16 else "normal"
    return np.ascontiguousarray(synth.bucket(dt, n, worker, cls, 1000 * rnd + 37 * key)) \
        .view(np.uint8)


@pytest.mark.parametrize("batched", [False, True], ids=["single", "many"])
@pytest.mark.parametrize("split", ["hash", "range"])
@pytest.mark.parametrize("dt", [DType.FLOAT32, DType.FLOAT16], ids=lambda d: DType(d).name)
def test_group_rounds_bit_exact(dt, split, batched):
    from prophet_amd.server import PSServerGroup
    N, R = 4, 3
    es = elem_size(dt)
    sizes = [1, 100, 4096 + 7, 65_536 + 3, 1_000_003]          # elements per key
    keys = [(k << 16) + p for k, p in ((0, 0), (1, 0), (1, 1), (7, 2), (160, 0))]
    grp = PSServerGroup(N, devices=[0, 0], engine_lanes=2, split=split,
                        split_min_bytes=64 * 1024 if split == "range" else 0)
    routes = {k: grp.route(k, n * es) for k, n in zip(keys, sizes)}
    if split == "range":
        assert len(routes[keys[-1]]) == 2 and len(routes[keys[0]]) == 1
    else:
        assert all(len(r) == 1 for r in routes.values())
        assert {r[0][0] for r in routes.values()} == {0, 1}    # both instances used
    port = PortReducer(nthreads=4)
    bar = threading.Barrier(N + 1)
    errors, pulled = [], {}

    def worker(w):
        try:
            rng = random.Random(100 + w)
            for rnd in range(R + 1):
                order = list(range(len(keys)))
                if rnd > 0:
                    rng.shuffle(order)
                ins = {keys[j]: data(dt, sizes[j], w, rnd, j) for j in order}
                if batched:
                    grp.push_many([keys[j] for j in order], w, [ins[keys[j]] for j in order], dt)
                else:
                    for j in order:
                        time.sleep(rng.random() * 0.001)
                        grp.push(keys[j], w, ins[keys[j]], dt)
                outs = [np.zeros(n * es, np.uint8) for n in sizes]
                if rnd == 0:    # no pull after the init round (its store is not a
                    pulled[(w, rnd)] = outs     # finished push round, server.cc:175-199)
                    bar.wait()
                    bar.wait()
                    continue
                if batched:
                    grp.pull_many(keys, outs)
                else:
                    for k, o in zip(keys, outs):
                        grp.pull(k, o)
                pulled[(w, rnd)] = outs
                bar.wait()      # main thread checks this round
                bar.wait()
        except Exception as e:  # noqa: BLE001
            errors.append(e)
            bar.abort()
    ts = [threading.Thread(target=worker, args=(w,)) for w in range(N)]
    for t in ts:
        t.start()
    try:
        for rnd in range(R + 1):
            bar.wait()
            assert not errors, errors
            for j, (k, n) in enumerate(zip(keys, sizes)):
                ins = [data(dt, n, w, rnd, j) for w in range(N)]
                for inst, off, ln in routes[k]:
                    rounds, _, order = grp.instance(inst).key_info(k)
                    assert rounds == rnd, (k, inst, rounds, rnd)
                    if rnd == 0:
                        continue
                    want = np.zeros(ln, np.uint8)
                    port.sum_n(want, [ins[w][off:off + ln] for w in order], ln, dt)
                    for w in range(N):
                        assert np.array_equal(pulled[(w, rnd)][j][off:off + ln], want), \
                            (k, inst, w, rnd)
            bar.wait()
    finally:
        for t in ts:
            t.join(timeout=60)
        grp.close()
    assert not errors, errors


def test_group_device_buffers_and_instances():
    """Device-resident pushes and pulls through the group (D2D piece copies),
    and the pieces visible on their instances (instance(i).pull of a piece)."""
    from oracle.oracle import PortReducer
    from prophet_amd.server import PSServerGroup
    dt, N, n = DType.FLOAT32, 3, 2_000_001
    grp = PSServerGroup(N, devices=[0, 0, 0], split="range")
    key = (9 << 16) + 4
    pieces = grp.route(key, n * 4)
    assert len(pieces) == 3
    for rnd in range(3):
        ins = [data(dt, n, w, rnd, 9) for w in range(N)]
        dev = [torch.from_numpy(x).to("cuda:0") for x in ins]
        ts = [threading.Thread(target=grp.push, args=(key, w, dev[w], dt)) for w in range(N)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        if rnd == 0:       # init round: nothing to pull
            continue
        out = torch.zeros(n * 4, dtype=torch.uint8, device="cuda:0")
        grp.pull(key, out)
        got = out.cpu().numpy()
        for inst, off, ln in pieces:
            _, _, order = grp.instance(inst).key_info(key)
            want = np.zeros(ln, np.uint8)
            PortReducer(nthreads=4).sum_n(want, [ins[w][off:off + ln] for w in order], ln, dt)
            assert np.array_equal(got[off:off + ln], want), (rnd, inst)
            part = np.zeros(ln, np.uint8)
            grp.instance(inst).pull(key, part)
            assert np.array_equal(part, want)
        for w in range(N - 2):     # the round's remaining pulls (it re-arms after N)
            grp.pull(key, out)
    grp.close()
