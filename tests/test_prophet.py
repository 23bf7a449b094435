"""Prophet PUSH-queue release logic (scheduled_queue.cc:217-296, :362-371):
hand-worked small traces, budget carry-over, credit gating, and whole-iteration
properties on the ResNet-50 fp16 partition set (config 3)."""
import pytest

from prophet_amd.buckets import resnet50_param_sizes
from prophet_amd.prophet import (BACKWARD_EXEC, ProphetPushQueue, PushTask, backward_arrivals,
                                 model_checkpoints, release_groups)


def _q(exec_, credit=150, cps=(-1, 1, 3)):
    # batch 64 -> scale 1; Z_NET_B 1 -> B = 125 bytes per exec unit
    return ProphetPushQueue(batch_size=64, net_b=1, credit=credit, checkpoints=cps,
                            backward_exec=exec_)


def _arrivals(n=4, ln=100):
    return [PushTask(g, 0, ln) for g in range(n - 1, -1, -1)]


def _grads(groups):
    return [[t.grad for t in g] for g in groups]


def test_budget_releases_lowest_index_first():
    # block {3,2}: budget 250 -> 2 then 3; block {1,0} released under credit
    q = _q((2, 5, 0))
    assert _grads(release_groups(q, _arrivals())) == [[2, 3], [0, 1]]


def test_budget_leftover_stays_under_next_block():
    # budget 150 releases only gradient 2 (150 > 100, then 50 > 100 fails);
    # gradient 3 stays on the stack under 1 and 0 and goes last
    q = _q((1.2, 5, 0))
    assert _grads(release_groups(q, _arrivals())) == [[2], [0, 1, 3]]


def test_strict_budget_comparison():
    # dynamic_size > len is strict (scheduled_queue.cc:262): budget exactly
    # one task long releases nothing in that block
    q = _q((0.8, 5, 0))
    assert _grads(release_groups(q, _arrivals())) == [[0, 1, 2, 3]]


def test_credit_gates_after_gradient_zero():
    q = _q((2, 5, 0), credit=150)
    for t in _arrivals():
        q.add_task(t)
    got = []
    for _ in range(20):
        t = q.get_task()
        if t is not None:
            got.append(t.grad)
    # block 1 releases 2, 3 under budget; after gradient 0 is collected the
    # credit (150) admits one 100-byte task, then waits for report_finish
    assert got == [2, 3, 0]
    assert q.get_task() is None
    q.report_finish(100)
    assert q.get_task().grad == 1
    assert q.pending() == 0


def test_report_finish_only_counts_after_meetzero():
    q = _q((2, 5, 0), credit=150)
    q.report_finish(1000)                     # before _meetzero: ignored
    assert q._bps_credit == 150


def test_partitions_stack_per_gradient():
    # a 3-partition gradient pushes three stack slots; partitions leave in
    # arrival order (multiset keeps insertion order for equal priority)
    q = _q((100, 100, 0))
    arr = [PushTask(3, 0, 10, 1), PushTask(2, 0, 10, 3), PushTask(2, 1, 10, 3),
           PushTask(2, 2, 10, 3), PushTask(1, 0, 10, 1), PushTask(0, 0, 10, 1)]
    out = [(t.grad, t.part) for g in release_groups(q, arr) for t in g]
    assert out == [(2, 0), (2, 1), (2, 2), (3, 0), (0, 0), (1, 0)]


def test_state_resets_between_iterations():
    q = _q((2, 5, 0))
    a = _grads(release_groups(q, _arrivals()))
    b = _grads(release_groups(q, _arrivals()))
    assert a == b
    assert q._pointer == 2 and q._expected == 3 and not q._meetzero


@pytest.mark.parametrize("batch,net_b", [(64, 1), (256, 10), (64, 100)])
def test_resnet50_iteration_releases_every_partition_once(batch, net_b):
    sizes = [n * 2 for n in resnet50_param_sizes()]
    arr = backward_arrivals(sizes)
    q = ProphetPushQueue(batch_size=batch, net_b=net_b, credit=8 << 20,
                         checkpoints=model_checkpoints(len(sizes)))
    phased = release_groups(q, arr, with_phase=True)
    groups = [g for _, g in phased]
    flat = [t for g in groups for t in g]
    assert sorted(flat) == sorted(arr)
    assert len(flat) == len(set(flat)) == 165
    # budgeted blocks never release as many bytes as their budget
    budgets = [e * (batch // 64) * net_b * 125 for e in BACKWARD_EXEC]
    for ph, g in phased:
        if ph != "credit":
            assert sum(t.len for t in g) < budgets[ph]
    # the credit phase is last and starts at gradient 0
    assert phased[-1][0] == "credit" and groups[-1][0].grad == 0
    # a second iteration on the same queue reproduces the grouping
    assert [[(t.grad, t.part) for t in g] for g in release_groups(q, arr)] == \
        [[(t.grad, t.part) for t in g] for g in groups]


def test_huge_budget_releases_whole_blocks():
    sizes = [n * 2 for n in resnet50_param_sizes()]
    q = ProphetPushQueue(batch_size=64, net_b=10**9, credit=1 << 40,
                         checkpoints=model_checkpoints(len(sizes)))
    groups = release_groups(q, backward_arrivals(sizes))
    cps = model_checkpoints(len(sizes))
    want = [sorted(range(cps[i] + 1, cps[i + 1] + 1)) for i in range(len(cps) - 2, -1, -1)]
    assert [sorted({t.grad for t in g}) for g in groups] == want
    # inside a block the lowest index leaves first
    assert groups[0][0].grad == cps[-2] + 1
