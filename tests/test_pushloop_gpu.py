"""The native PUSH loop (byteps_prophet_loop_*): Prophet's scheduler feeding
the block queue from a library thread, as core_loops.cc's PUSH loop feeds the
network.  BASELINE config 3's shape — ResNet-50 fp16 gradients, 8 workers,
165 BytePS partitions in the 12 Prophet blocks — with the partitions arriving
from a feeder thread in backward order, at random small intervals, for three
back-to-back iterations; every iteration's output is bit-exact with torch's
own half-precision left fold (and that equals the oracle's fp16 rule, checked
on windows).  Also: a partition pushed twice, a missing partition (ETIMEOUT,
then the block queue's status clears), a schedule whose budgets cut blocks."""
import random
import threading
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]


def _setup(net_b=10**6, credit=1 << 30, n_workers=8, seed=0):
    from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes
    from prophet_amd.dtypes import DType
    from prophet_amd.prophet import ProphetPushQueue, PushTask, model_checkpoints
    from prophet_amd.reducer import GpuReducer
    dev = torch.device("cuda:0")
    red = GpuReducer(device=0)
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    toff = [0]
    for n in sizes:
        toff.append(toff[-1] + n)
    total = toff[-1]
    nparts = {}
    for p in parts:
        nparts[p.tensor] = nparts.get(p.tensor, 0) + 1
    table, block_of = [], []
    for b, blk in enumerate(prophet_blocks(len(sizes))):
        tset = set(blk)
        for p in parts:
            if p.tensor in tset:
                table.append(p)
                block_of.append(b)
    nb = max(block_of) + 1
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    w = [torch.randn(total // 2, device=dev, generator=gen).half().view(torch.uint8)
         for _ in range(n_workers)]
    out = torch.zeros(total, dtype=torch.uint8, device=dev)
    blocks = [[] for _ in range(nb)]
    for p, b in zip(table, block_of):
        o = toff[p.tensor] + p.offset
        blocks[b].append((out[o:o + p.len], [x[o:o + p.len] for x in w], p.len))
    bq = red.make_blockq(blocks, DType.FLOAT16)
    bq.config(wg_per_cu=0, timeout_s=1.0)
    q = ProphetPushQueue(batch_size=64, net_b=net_b, credit=credit,
                         checkpoints=model_checkpoints(len(sizes)))
    # arrivals: backward order (highest gradient first), handle = table index
    arrivals = sorted(range(len(table)), key=lambda i: (-table[i].tensor, table[i].part))
    tasks = [(PushTask(table[i].tensor, table[i].part, table[i].len, nparts[table[i].tensor],
                       (table[i].tensor << 16) + table[i].part), i) for i in arrivals]
    ref = w[0].view(torch.float16).clone()
    for x in w[1:]:
        ref.add_(x.view(torch.float16))
    return dict(red=red, bq=bq, q=q, block_of=block_of, tasks=tasks, out=out, ref=ref, w=w,
                nb=nb)


def _feed(loop, tasks, seed, skip=None):
    rng = random.Random(seed)
    for t, i in tasks:
        if i == skip:
            continue
        if rng.random() < 0.1:
            time.sleep(rng.random() * 0.0005)
        loop.push(t, i)


@pytest.mark.parametrize("host", [False, True], ids=["stream_release", "host_release"])
@pytest.mark.parametrize("inline", [False, True], ids=["thread", "inline"])
@pytest.mark.parametrize("net_b", [10**6, 1000], ids=["whole_blocks", "budget_cuts_blocks"])
def test_push_loop_iterations_exact(net_b, inline, host):
    """host: the loop releases complete blocks from the host (the pushes are
    resident before the iteration begins, BYTEPS_PROPHET_LOOP_HOST_RELEASE)."""
    from prophet_amd.prophet import PushLoop
    S = _setup(net_b=net_b)
    cons = S["bq"].stream()              # the library's consumer stream
    rel = torch.cuda.Stream()
    torch.cuda.synchronize()
    loop = PushLoop(S["q"], S["bq"], S["block_of"], release_stream=rel, inline=inline,
                    host_release=host)
    import gc
    gc.collect()      # inline: no GC-triggered hipFree may run inside an iteration
    for it in range(3):
        S["out"].zero_()
        torch.cuda.synchronize()
        loop.begin(cons)
        th = threading.Thread(target=_feed, args=(loop, S["tasks"], it))
        th.start()
        th.join()
        loop.end(timeout_s=10.0)
        torch.cuda.synchronize()
        S["bq"].status(cons)
        assert torch.equal(S["out"], S["ref"].view(torch.uint8)), f"iteration {it}"
    loop.close()
    # the fp16 rule of the oracle (cpu_reducer.cc:94-128) on two windows
    from oracle.oracle import PortReducer
    from prophet_amd.dtypes import DType
    port = PortReducer(nthreads=4)
    for a in (0, S["out"].numel() - (1 << 16)):
        ln = 1 << 16
        ins = [x[a:a + ln].cpu().numpy() for x in S["w"]]
        want = np.zeros(ln, np.uint8)
        port.sum_n(want, ins, ln, DType.FLOAT16)
        assert np.array_equal(S["out"][a:a + ln].cpu().numpy(), want)


@pytest.mark.parametrize("inline", [False, True], ids=["thread", "inline"])
def test_push_loop_push_many_exact(inline):
    """push_many: partitions that landed together in one call (one drain, the
    release groups ready together released as one kernel per run of blocks).
    Config 3's partitions in three batches per iteration (the last holds the
    rest), three iterations, bit-exact; a batch with a bad task is refused
    whole — none of its partitions counts as pushed."""
    from prophet_amd.prophet import PushLoop
    from prophet_amd.reducer import ReduceError
    S = _setup(seed=9)
    cons = S["bq"].stream()
    rel = torch.cuda.Stream()
    torch.cuda.synchronize()
    loop = PushLoop(S["q"], S["bq"], S["block_of"], release_stream=rel, inline=inline)
    tasks = S["tasks"]
    cuts = [0, 40, 41, len(tasks)]
    batches = [loop.make_batch([t for t, _ in tasks[a:b]], [i for _, i in tasks[a:b]])
               for a, b in zip(cuts, cuts[1:])]
    import gc
    gc.collect()
    for it in range(3):
        S["out"].zero_()
        torch.cuda.synchronize()
        loop.begin(cons)
        if it == 1:
            t0, i0 = tasks[0]
            with pytest.raises(ReduceError, match="twice"):
                loop.push_many([(t0, i0), (t0, i0)])
            with pytest.raises(ReduceError, match="outside the table"):
                loop.push_many([(t0, i0), (t0, 10_000)])
        c0 = loop.release_calls()
        for b in batches:
            loop.push_many(b)
        loop.end(timeout_s=10.0)
        # at most one release kernel per batch (per run of blocks it completed)
        assert 1 <= loop.release_calls() - c0 <= S["nb"]
        torch.cuda.synchronize()
        S["bq"].status(cons)
        assert torch.equal(S["out"], S["ref"].view(torch.uint8)), f"iteration {it}"
    loop.close()


def test_push_loop_errors_and_missing_partition():
    from prophet_amd.prophet import PushLoop
    from prophet_amd.reducer import ReduceError
    S = _setup(seed=3)
    cons = torch.cuda.Stream(priority=-100)
    rel = torch.cuda.Stream()
    loop = PushLoop(S["q"], S["bq"], S["block_of"], release_stream=rel)
    t0, i0 = S["tasks"][0]
    with pytest.raises(ReduceError, match="no iteration"):
        loop.push(t0, i0)
    loop.begin(cons)
    with pytest.raises(ReduceError, match="already begun"):
        loop.begin(cons)
    loop.push(t0, i0)
    with pytest.raises(ReduceError, match="twice"):
        loop.push(t0, i0)
    with pytest.raises(ReduceError, match="outside the table"):
        loop.push(t0, 10_000)
    # everything but the last partition of the last block: that block never
    # completes -> end() times out; the consumer gives up after its own 1-s
    # timeout and the block queue's status reports it once
    last = S["tasks"][-1][1]
    _feed(loop, S["tasks"][1:], 7, skip=last)
    with pytest.raises(ReduceError) as e:
        loop.end(timeout_s=0.5)
    assert e.value.code == -5                      # BYTEPS_REDUCE_ETIMEOUT
    loop.close()
    time.sleep(1.5)
    torch.cuda.synchronize()
    with pytest.raises(ReduceError):
        S["bq"].status(cons)
    S["bq"].status(cons)                           # reported once, then clear
    # free the block queue now (its destroy synchronises the device): left to
    # the garbage collector — `e` keeps this frame alive in a cycle — it could
    # run inside a later test's live iteration and stall an inline loop
    del e
    S["bq"].close()


@pytest.mark.parametrize("inline", [False, True], ids=["thread", "inline"])
def test_push_loop_empty_block_and_fifo_tasks(inline):
    """A table whose middle block has no partitions (released at begin), and a
    partition whose tensor does not match Z_keyword (a FIFO task, released
    only once no scheduled task is queued, scheduled_queue.cc:292-318; its
    index lies outside the scheduled model — a model gradient that is not
    scheduled would stall collection in the reference too): every block still
    folds, bit-exact, over two iterations."""
    from prophet_amd.dtypes import DType
    from prophet_amd.prophet import ProphetPushQueue, PushLoop, PushTask
    from prophet_amd.reducer import GpuReducer
    red = GpuReducer(device=0)
    dev = torch.device("cuda:0")
    N, n = 5, 70_001
    lens = [n, 3 * n, 2 * n + 7, n, 5 * n]    # elements per partition (fp32)
    grads = [3, 2, 1, 0, 77]                  # gradient of each partition
    fifo = [False, False, False, False, True]  # the last is not Prophet-scheduled
    block_of = [0, 0, 2, 2, 2]                # block 1 is empty
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    ins = [[torch.randn(L, device=dev, generator=gen) for L in lens] for _ in range(N)]
    outs = [torch.zeros(L, device=dev) for L in lens]
    blocks = [[], [], []]
    for i, L in enumerate(lens):
        blocks[block_of[i]].append((outs[i], [ins[k][i] for k in range(N)], L * 4))
    bq = red.make_blockq(blocks, DType.FLOAT32)
    bq.config(wg_per_cu=0, timeout_s=1.0)
    q = ProphetPushQueue(batch_size=64, net_b=10**6, credit=1 << 30, checkpoints=(-1, 1, 3),
                         backward_exec=(5, 5, 0))
    cons, rel = torch.cuda.Stream(priority=-100), torch.cuda.Stream()
    loop = PushLoop(q, bq, block_of, release_stream=rel, inline=inline)
    import gc
    gc.collect()      # inline: no GC-triggered hipFree may run inside an iteration
    for it in range(2):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        times = []
        t0 = time.perf_counter()
        loop.begin(cons)
        times.append(("begin", time.perf_counter() - t0))
        for i in range(len(lens)):
            t0 = time.perf_counter()
            loop.push(PushTask(grads[i], 0, lens[i] * 4, 1, grads[i] << 16,
                               scheduled=not fifo[i]), i)
            times.append((f"push{i}", time.perf_counter() - t0))
        t0 = time.perf_counter()
        loop.end(timeout_s=5.0)
        times.append(("end", time.perf_counter() - t0))
        torch.cuda.synchronize()
        try:
            bq.status(cons)
        except Exception as exc:
            raise AssertionError(f"iteration {it}: {exc}; host call times {times}; "
                                 f"block queue {bq.debug()}") from exc
        for i in range(len(lens)):
            ref = ins[0][i].clone()
            for k in range(1, N):
                ref.add_(ins[k][i])
            assert torch.equal(outs[i], ref), (it, i)
    loop.close()


def test_diagnosis_sequence_all_cases_pass():
    """The sequence that exposed the shared hardware queue (tools/
    pushloop_diag.py: a config-3 iteration, then small tables with one factor
    changed at a time; before the consumer had a queue of its own the 5th and
    9th cases timed out every time, profiles/r02_pushloop_diag_before.jsonl)
    runs clean, in a process of its own."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "pushloop_diag.py")],
                       capture_output=True, text=True, timeout=200, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    cases = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(cases) >= 12
    bad = [c["case"] for c in cases if '"status_ok": false' in json.dumps(c)
           or '"exact": false' in json.dumps(c)]
    assert not bad, bad


def test_push_loop_thread_keeps_releasing_while_pusher_frees():
    """Thread mode: the pushing thread may block on the device right after its
    last push — here it destroys a plan (hipFree synchronises the device)
    while the loop thread still has releases to issue.  The loop thread's
    launches are not held up by the blocked thread, so the consumer completes
    instead of waiting out its timeout.  The plan is made before the
    iteration begins: its table upload is a synchronous hipMemcpy, i.e.
    legacy NULL-stream work, which waits for the running consumer (a blocking
    stream) and holds back every stream sharing the NULL stream's hardware
    queue — the release stream among them, by the runtime's placement
    (include/bpsr/reduce.h: no NULL-stream work between a launch and its last
    release; this test once passed by placement alone)."""
    from prophet_amd.dtypes import DType
    from prophet_amd.prophet import PushLoop
    S = _setup(seed=5)
    red = S["red"]
    rel = torch.cuda.Stream()
    loop = PushLoop(S["q"], S["bq"], S["block_of"], release_stream=rel, inline=False)
    x, y, z = (torch.zeros(1 << 20, dtype=torch.uint8, device="cuda") for _ in range(3))
    for it in range(3):
        plan = red.make_plan([(x, [y, z], x.numel())], DType.UINT8)
        torch.cuda.synchronize()
        loop.begin()
        for t, i in S["tasks"]:
            loop.push(t, i)
        plan.close()                                  # hipFree while releases are pending
        loop.end(timeout_s=10.0)
        torch.cuda.synchronize()
        S["bq"].status()
        assert torch.equal(S["out"], S["ref"].view(torch.uint8)), it
    loop.close()
