"""bench.py on the GPU at N > 1, rehearsed on one GPU: ``--gpus 2`` starts two
rank processes (the launcher the driver's scaling run uses), both fold with
the HIP kernel on cuda:0, gloo carries the barrier and max-over-ranks (RCCL
refuses two ranks on one GPU), and the config-4 sharded fold runs at world
size 2 with its G=1 reference measured on rank 0, and the scatter and
local-reduce legs run over gloo with CUDA tensors.  One JSON line comes back."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_rehearsed_on_one_gpu():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-one-gpu",
           "--steps", "5", "--warmup", "2", "--bucket-mib", "16", "--no-cpu-baseline",
           "--scaling-elems", "4000037", "--e2e-bucket-mib", "16"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    e2e = line["e2e_cfg5"]
    assert "error" not in e2e, e2e
    assert e2e["exact_vs_torch_fold_windows"] is True and e2e["node_e2e_GiBps"] > 0
    assert line["n_gpus"] == 2 and len(line["config"]["devices"]) == 2
    assert "rehearsal" in line["device"]
    assert line["check_vs_torch_fold"] is True
    assert line["roofline"]["kernel_ms"] > 0
    sc = line["scaling_cfg4"]
    assert sc["exact_vs_torch_fold"] is True, sc
    assert sum(sc["shard_elems"]) == 4000037 and len(sc["shard_elems"]) == 2
    assert sc["g1_fold_ms"] > 0 and sc["per_gpu_fold_ms"] > 0
    # the N > 1 exchange legs' code on one GPU: gloo moves the CUDA tensors
    assert sc["scatter"]["exact_vs_torch_fold"] is True, sc["scatter"]
    lr = line["local_reduce"]
    assert "error" not in lr, lr
    assert lr["exact_vs_rank_order_fold"] is True
    srv = line["server_cfg1"]          # one PS server per rank, host-resident rounds
    assert "error" not in srv, srv
    assert srv["exact_vs_torch_sum"] is True and srv["node_GiBps"] > 0


def test_bench_one_gpu_line_has_every_object():
    """The N = 1 line the driver records: headline fold checked, the config-4
    scaling object and the config-3 block-queue object present and exact (a
    leg that raised would carry an "error" field instead)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2",
           "--bucket-mib", "16", "--no-cpu-baseline", "--scaling-elems", "4000037",
           "--e2e-bucket-mib", "16"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["check_vs_torch_fold"] is True
    assert "device" not in line                      # a measurement, not a self-test
    blk = line["roofline"]["kernel_ms_blocks"]       # the spread object
    assert 0 < blk["min"] <= blk["median"] <= blk["max"]
    assert blk["median"] < 3 * line["roofline"]["kernel_ms"]
    assert line["scaling_cfg4"]["exact_vs_torch_fold"] is True
    f16 = line["fp16"]
    assert "error" not in f16, f16
    assert f16["exact_vs_torch_fold"] is True and 0 < f16["frac_of_roofline"] < 1
    c3 = line["cfg3_blockq"]
    assert "error" not in c3, c3
    assert c3["exact_vs_torch_fold"] is True
    for k in ("live", "pre_released", "live_no_overlap", "pre_released_no_overlap",
              "live_host_releases", "live_per_block"):
        assert 0 < c3[k]["frac_of_roofline"] < 1, k
    assert "overlap" in c3 and c3["live"]["release_kernels_per_iter"] > 0
    assert line["scaling"] == "weak" and "no collective" in line["scaling_note"]
    s3 = line["server_cfg3"]             # config 3's keys through the server, two ways
    assert "error" not in s3, s3
    for k in ("launch", "device_releases"):
        assert s3[k]["exact_vs_torch_fold_in_recorded_order"] is True, s3[k]
        assert 0 < s3[k]["frac_of_roofline"] < 1
    assert s3["device_releases"]["consumer_launches_per_round"] >= 1
    assert s3["launch"]["consumer_launches_per_round"] == 0
    e2e = line["e2e_cfg5"]
    assert "error" not in e2e, e2e
    assert e2e["exact_vs_torch_fold_windows"] is True and e2e["pcie_inclusive"] is True
    srv = line["server_cfg1"]
    assert "error" not in srv, srv
    assert srv["exact_vs_torch_sum"] is True and srv["node_GiBps"] > 0
    assert srv["pull"].startswith("host_view") and srv["copying_pulls"]["node_GiBps"] > 0
    # the link measured in the same run, and each host-resident object's share of it
    link = line["pcie"]
    assert "error" not in link, link
    assert link["h2d_GBps"] > 1 and link["d2h_GBps"] > 1 and link["bidir_GBps"] > 1
    for obj in (srv, srv["copying_pulls"], e2e):
        assert 0 < obj["frac_of_link"] < 1.5 and 0 < obj["frac_of_h2d"] < 1.5, obj
        assert obj["link_bound_ms"] > 0


def test_server_group_leg_matches_oracle():
    """The config-1 server-group object's rounds, checked against the oracle:
    the same group calls on fresh data, every worker's pull equals the oracle's
    fold of the pushes in the arrival order the instance recorded."""
    import threading
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from oracle.oracle import PortReducer
    from prophet_amd.buckets import partition_tensor
    from prophet_amd.dtypes import DType
    from prophet_amd.server import PSServerGroup
    N, B = 2, 8 << 20
    parts = [(p.key, p.offset, p.len) for p in partition_tensor(0, B, bound=1 << 20)]
    keys = [k for k, _, _ in parts]
    grp = PSServerGroup(N, devices=[0], split="hash")
    host = [torch.randn(B // 4).pin_memory() for _ in range(N)]
    outs = [torch.zeros(B, dtype=torch.uint8).pin_memory() for _ in range(N)]
    for rnd in range(3):
        ts = [threading.Thread(target=lambda w=w: (
            grp.push_many(keys, w, [host[w].view(torch.uint8)[o:o + ln] for _, o, ln in parts],
                          DType.FLOAT32),
            rnd and grp.pull_many(keys, [outs[w][o:o + ln] for _, o, ln in parts])))
              for w in range(N)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
    port = PortReducer(nthreads=4)
    for k, o, ln in parts:
        order = grp.instance(0).key_info(k)[2]
        want = np.zeros(ln, np.uint8)
        port.sum_n(want, [host[w].view(torch.uint8)[o:o + ln].numpy() for w in order], ln,
                   DType.FLOAT32)
        for w in range(N):
            assert np.array_equal(outs[w][o:o + ln].numpy(), want), (k, w)
    grp.close()


def _lr_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        r = bench.local_reduce_leg(torch.device("cuda", 0), world, rank, reps=1,
                                   n_elems=1_000_003)
        q.put((rank, r))
        dist.destroy_process_group()
    except Exception as e:  # reported to the parent
        q.put((rank, {"error": repr(e)}))


def test_local_reduce_leg_two_gloo_ranks_on_one_gpu():
    """The N > 1 ``local_reduce`` object's code path on one GPU: two gloo
    ranks (CUDA tensors through gloo's P2P), each folding its owned slice with
    the HIP fold in rank order; windows bit-exact against the rank-order left
    fold of both regenerated vectors (timings here are not measurements)."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_lr_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert "error" not in out[r], out[r]
        assert out[r]["exact_vs_rank_order_fold"] is True


_RCCL_LEGS = r'''
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["BPSR_ROOT"])
import bench
from oracle.oracle import PortReducer
from prophet_amd.dtypes import DType
from prophet_amd.shard import ShardedReducer
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
dist.barrier()
comm, how = bench.shard_comm(dev)
rccl = bench.rccl_object(dev, comm, 1, 0)
E = 1_000_003
sc = bench.scatter_leg(dev, 1, 0, 8, reps=2, n_elems=E, comm=comm)
lr = bench.local_reduce_leg(dev, 1, 0, reps=2, n_elems=E, comm=comm)
# the same call, checked against the oracle's left fold of the 8 pushes
g = torch.Generator(device=dev)
g.manual_seed(11)
pushes = [torch.randn(E, device=dev, generator=g) for _ in range(8)]
recv = [torch.empty(E, device=dev) for _ in range(8)]
owned = torch.empty(E, device=dev)
ShardedReducer(E, comm=comm).scatter_reduce(0, pushes, recv, owned)
torch.cuda.synchronize()
want = np.zeros(E * 4, np.uint8)
PortReducer(nthreads=4).sum_n(want, [p.cpu().numpy().view(np.uint8) for p in pushes], E * 4,
                              DType.FLOAT32)
oracle_ok = bool(np.array_equal(owned.cpu().numpy().view(np.uint8), want))
comm.close()
dist.destroy_process_group()
print(json.dumps({"how": how, "scatter": sc, "local_reduce": lr, "oracle_ok": oracle_ok,
                  "rccl": rccl}))
'''


def test_exchange_legs_through_shard_abi_on_rccl_world1():
    """The N > 1 bench legs as the driver's multi-GPU run takes them, at world
    1 on this box: the communicator comes from the torch process group
    (bench.shard_comm), every exchange is a byteps_shard_* call over RCCL
    (transport "rccl-shard-abi"), and both legs' results are exact; the same
    scatter_reduce call equals the oracle's left fold bit for bit; the
    line's ``rccl`` object reports a world-1 communicator on the bound GPU."""
    env = dict(os.environ, BPSR_ROOT=ROOT, MASTER_ADDR="127.0.0.1")
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    env["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _RCCL_LEGS], env=env, capture_output=True,
                       text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert "RCCL" in out["how"] or "NCCL" in out["how"], out["how"]
    sc, lr = out["scatter"], out["local_reduce"]
    assert sc["transport"] == lr["transport"] == "rccl-shard-abi"
    assert sc["exact_vs_torch_fold"] is True and sc["scatter_fold_ms"] > 0
    assert lr["exact_vs_rank_order_fold"] is True and lr["allreduce_ms"] > 0
    assert out["oracle_ok"] is True
    # the line's rccl object: the communicator RCCL made has world 1, this
    # rank, the bound device; no problems
    rc = out["rccl"]
    assert rc["world"] == 1 and rc["problems"] == [], rc
    v = rc["ranks"][0]
    assert (v["comm_world"], v["comm_rank"], v["comm_device"], v["device"]) == (1, 0, 0, 0), v
    assert v["rccl_version"] > 20000 and v["device_count"] >= 1 and v["pci_bus_id"]
