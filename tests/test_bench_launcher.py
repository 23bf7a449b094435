"""bench.py's multi-rank launcher and its config-4 scaling object, on CPU.

``python bench.py --gpus N`` with no WORLD_SIZE starts N rank processes itself
(before anything touches a GPU) and exactly one JSON line comes back with
``n_gpus == N``.  ``--device cpu`` swaps the HIP fold for torch's CPU add and
RCCL for gloo, so the launcher, the barrier / max-over-ranks timing, the
config-4 sharded fold and the scatter + all-gather leg all run here; the line
says it is not a measurement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(n, extra=()):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", str(n),
           "--steps", "2", "--warmup", "1", "--workers", "3", "--bucket-mib", "0.0625",
           "--sets", "2", "--no-cpu-baseline", "--scaling-elems", "10007", *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    # stdout is exactly the one JSON line: library chatter (gloo's connection
    # notes on rank 0) is routed to stderr
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout
    return json.loads(r.stdout)


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_launcher_one_line_n_ranks(n):
    line = _run_bench(n)
    assert line["n_gpus"] == n
    assert line["config"]["parallelism"] == f"key-space shard x{n}"
    assert len(line["config"]["devices"]) == n
    assert line["check_vs_torch_fold"] is True
    assert "NOT a measurement" in line["device"]
    pl = line["roofline"]["kernel_ms_blocks"]   # median and min
    assert 0 < pl["min"] <= pl["median"] <= pl["max"] and pl["blocks"] == 5
    # the config-1 server-group object is in every line (it needs the GPU: on
    # the CPU self-test it says so rather than disappearing)
    assert "skipped" in line["server_cfg1"] and "skipped" in line["pcie"]
    sc = line["scaling_cfg4"]
    assert sc["exact_vs_torch_fold"] is True
    assert len(sc["shard_elems"]) == n and sum(sc["shard_elems"]) == 10007
    assert sc["per_gpu_fold_ms"] > 0 and sc["g1_fold_ms"] > 0
    assert sc["strong_efficiency"] is not None
    if n == 1:
        assert sc["g1_fold_ms"] == sc["per_gpu_fold_ms"] and "scatter" not in sc
    else:
        assert sc["scatter"]["exact_vs_torch_fold"] is True
        assert sc["scatter"]["scatter_fold_ms"] > 0
        lr = line["local_reduce"]
        assert "error" not in lr, lr
        assert lr["exact_vs_rank_order_fold"] is True and lr["allreduce_ms"] > 0
        # the CPU self-test moves slices with torch P2P over gloo
        assert sc["scatter"]["transport"] == lr["transport"] == "torch-p2p"
        assert "shard_comm" not in line
        assert line["rccl"] == {"transport": "gloo, no RCCL", "world": n}
    if n == 1:
        assert "rccl" not in line


def test_exchange_transport_rule():
    """N > 1 on GPUs (one rank per GPU): the scatter and local-reduce legs go
    through byteps_shard_* over RCCL (the code core_loops.cc binds); a
    one-GPU rehearsal and the CPU self-test use torch P2P."""
    sys.path.insert(0, ROOT)
    import bench
    for n in (2, 4, 8):
        assert bench.uses_shard_abi(n, cuda=True, rehearse=False)
        assert not bench.uses_shard_abi(n, cuda=True, rehearse=True)
        assert not bench.uses_shard_abi(n, cuda=False, rehearse=False)
    assert not bench.uses_shard_abi(1, cuda=True, rehearse=False)
    assert bench._transport(object()) == "rccl-shard-abi"
    assert bench._transport(None) == "torch-p2p"


def test_rccl_problems_rule():
    """The N > 1 line's ``rccl`` check (bench.rccl_problems): a communicator
    of N ranks on N distinct GPUs passes; a wrong world, a rank mismatch, a
    communicator on another device than the rank bound, two ranks on one GPU
    and mixed RCCL versions are each reported."""
    sys.path.insert(0, ROOT)
    import bench

    def views(n, over=None):
        vs = [{"rank": r, "comm_world": n, "comm_rank": r, "comm_device": r, "device": r,
               "pci_bus_id": f"0000:{0x05 + 0x10 * r:02x}:00", "rccl_version": 22707,
               "device_count": n} for r in range(n)]
        for (r, k), v in (over or {}).items():
            vs[r][k] = v
        return vs
    for n in (2, 4, 8):
        assert bench.rccl_problems(views(n), n) == []
    assert bench.rccl_problems(views(8), 4)                       # 8 views, WORLD_SIZE 4
    bad = {(1, "comm_world"): 1, (2, "comm_rank"): 5, (3, "comm_device"): 0,
           (4, "rccl_version"): 22500}
    for k, v in bad.items():
        p = bench.rccl_problems(views(8, {k: v}), 8)
        assert len(p) == 1, (k, p)
    shared = views(8, {(5, "pci_bus_id"): "0000:05:00", (5, "device"): 0,
                       (5, "comm_device"): 0})
    assert any("share a GPU" in s for s in bench.rccl_problems(shared, 8))


def test_link_bound_model():
    """bench.link_bound_s: H2D and D2H share the measured both-ways rate while
    both run, the rest goes one way; link_fracs reports the object's time
    against that bound and its H2D rate against the one-way rate."""
    sys.path.insert(0, ROOT)
    import bench
    L = {"h2d_GBps": 50.0, "d2h_GBps": 40.0, "bidir_GBps": 80.0}
    assert abs(bench.link_bound_s(100e9, 0, L) - 2.0) < 1e-12          # one way, H2D
    assert abs(bench.link_bound_s(0, 80e9, L) - 2.0) < 1e-12           # one way, D2H
    assert abs(bench.link_bound_s(80e9, 80e9, L) - 2.0) < 1e-12        # both: 40 + 40
    assert abs(bench.link_bound_s(120e9, 40e9, L) - (1.0 + 80e9 / 50e9)) < 1e-12
    f = bench.link_fracs(120e9, 40e9, 5.2, L)
    assert f["frac_of_link"] == round(2.6 / 5.2, 4) and f["link_bound_ms"] == 2600.0
    assert f["frac_of_h2d"] == round(120e9 / 5.2 / 50e9, 4)
    assert bench.link_fracs(1, 1, 1.0, None) == {}


def test_rccl_check_failure_fails_the_run():
    """Every rank of a world-2 run whose communicator views say 'two ranks on
    one GPU' (test hook) exits RCCL_EXIT; rank 0 still prints the line, with
    the gathered views, the problem and an "error" field."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BPSR_BENCH_TEST_RCCL"] = "shared_device"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--workers", "3", "--bucket-mib", "0.0625",
           "--sets", "2", "--no-cpu-baseline", "--scaling-elems", "10007"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    sys.path.insert(0, ROOT)
    import bench
    assert r.returncode == bench.RCCL_EXIT, r.stderr[-3000:]
    line = json.loads(r.stdout)
    rc = line["rccl"]
    assert rc["world"] == 2 and len(rc["ranks"]) == 2
    assert any("share a GPU" in p for p in rc["problems"])
    assert line["error"].startswith("rccl:")


def test_torchrun_launch_one_line():
    """The driver's own multi-GPU form: ``python -m torch.distributed.run
    --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P
    bench.py --gpus N`` (ranks from the environment, no self-launch)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "2",
           "--warmup", "1", "--workers", "3", "--bucket-mib", "0.0625", "--sets", "2",
           "--no-cpu-baseline", "--scaling-elems", "10007"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and len(line["config"]["devices"]) == 2
    assert line["scaling_cfg4"]["scatter"]["exact_vs_torch_fold"] is True


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_stalled_collective_fails_loudly(launcher):
    """A leg that never returns (test hook: the scatter leg sleeps, as a stuck
    RCCL call would) trips the watchdog: the headline line still comes out,
    carrying ``error``, and the run exits NON-zero (every rank exits 3; the
    self-launcher and torch.distributed.run relay it)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BPSR_BENCH_TEST_STALL="scatter", BPSR_BENCH_WATCHDOG_S="8")
    args = [os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2", "--steps", "2",
            "--warmup", "1", "--workers", "3", "--bucket-mib", "0.0625", "--sets", "2",
            "--no-cpu-baseline", "--scaling-elems", "10007"]
    if launcher == "self":
        cmd = [sys.executable] + args
    else:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               "2", "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert "scatter" in line["error"] and "still running" in line["error"]
    assert line["n_gpus"] == 2 and line["value"] > 0


def test_launcher_failing_rank_fails_the_run():
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
           "--mode", "accum", "--no-cpu-baseline"]   # cpu self-test refuses accum mode
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_traffic_quoted_only_for_same_kernel_sources(tmp_path, monkeypatch):
    import bench
    bid = bench.kernel_build_id()
    wl = "8-way f32 left-fold sum of one 256 MiB bucket per GPU"
    rec = {"workload": wl, "kernel_build": bid, "session": "sX", "hbm_bytes_per_launch": 123.0}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    t, src = bench.pmc_traffic(wl)
    assert t == 123.0 and src["session"] == "sX"
    rec["kernel_build"] = "0" * 16
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    t, src = bench.pmc_traffic(wl)
    assert t is None and "changed" in src["status"]
    t, src = bench.pmc_traffic("other workload")
    assert t is None


def test_pmc_tool_counts_the_headline_kernel_only(tmp_path):
    """tools/pmc_traffic.py sums each dispatch's counter over the headline
    kernel only: other fold instantiations in the same pass (the bench line's
    fp16, config-3/4/5 objects) must not enter the median."""
    import csv
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic
    d = tmp_path / "write_size"
    d.mkdir()
    rows = []
    for i in range(5):   # headline dispatches, counter split over two rows each
        for part in (100.0, 28.0):
            rows.append({"Dispatch_Id": str(i), "Kernel_Name":
                         "void bpsr::fold_kernel<bpsr::OpF32, 2, 1, 8>(bpsr::FoldArgs)",
                         "Counter_Name": "WRITE_SIZE", "Counter_Value": str(part)})
    for i in range(5, 30):   # another fold in the same pass
        rows.append({"Dispatch_Id": str(i), "Kernel_Name":
                     "void bpsr::fold_kernel<bpsr::OpBF16, 4, 2, 16>(bpsr::FoldArgs)",
                     "Counter_Name": "WRITE_SIZE", "Counter_Value": "7"})
    with open(d / "x_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    vals = pmc_traffic.collect("WRITE_SIZE", str(d))
    assert sorted(vals) == [128.0] * 5
