#!/usr/bin/env python3
"""HBM traffic per launch of the fold kernel from rocprofv3 PMC counters.

Two separate counter passes over the same bench command (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950: TCC has 4 slots, FETCH_SIZE costs 3,
WRITE_SIZE 2 — MI355X_MICROARCH.md "rocprofv3 PMC slots").  Corrections per
MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports exactly half of a wide
coalesced streaming read on gfx950, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores.

Writes <out>/pmc_traffic.json and, with --commit, profiles/pmc_traffic.json
(read by bench.py for roofline.traffic).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the headline kernel only: other fold instantiations in the same run (the
# bench line's fp16, config-3/4/5 objects, when not disabled) must not enter
# the median
KERNEL_KEY = "fold_kernel<bpsr::OpF32, 2, 1, 8>"
KERNEL = None   # --kernel


def run_pass(counter: str, outdir: str, bench_args: list[str]) -> tuple[list[float], dict]:
    d = os.path.join(outdir, counter.lower())
    shutil.rmtree(d, ignore_errors=True)
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv",
           "-d", d, "-o", counter.lower(), "--", sys.executable,
           os.path.join(ROOT, "bench.py")] + bench_args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    bench_line = {}
    for line in r.stdout.splitlines():
        if line.startswith("{") and '"metric"' in line:
            bench_line = json.loads(line)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 pass {counter} failed rc={r.returncode}\n{r.stderr[-3000:]}")
    with open(os.path.join(d, "bench_line.json"), "w") as fh:
        json.dump(bench_line, fh)
    return collect(counter, d, KERNEL), bench_line


def collect(counter: str, d: str, kernel: str | None = None) -> list[float]:
    """Per-dispatch counter sums of the headline kernel (or ``kernel``) from a
    pass's CSVs."""
    kname = kernel or KERNEL_KEY
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kname not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    p.add_argument("--commit", action="store_true")
    p.add_argument("--session", default=os.environ.get("BPSR_SESSION", ""),
                   help="session tag recorded with the numbers (bench line traffic_source)")
    p.add_argument("--kernel", default=None,
                   help="kernel-name substring to count (default: the headline kernel)")
    p.add_argument("--reaggregate", action="store_true",
                   help="re-read the passes already under --out (no profiling run)")
    p.add_argument("bench_args", nargs="*",
                   default=["--steps", "12", "--warmup", "2", "--no-cpu-baseline",
                            "--no-scaling", "--no-cfg3", "--no-fp16", "--no-e2e"])
    a = p.parse_args()
    global KERNEL
    KERNEL = a.kernel
    os.makedirs(a.out, exist_ok=True)
    if a.reaggregate:
        fetch = collect("FETCH_SIZE", os.path.join(a.out, "fetch_size"), KERNEL)
        write = collect("WRITE_SIZE", os.path.join(a.out, "write_size"), KERNEL)
        bl = {}
        blf = os.path.join(a.out, "fetch_size", "bench_line.json")
        if os.path.exists(blf):
            with open(blf) as fh:
                bl = json.load(fh)
    else:
        fetch, bl = run_pass("FETCH_SIZE", a.out, a.bench_args)
        write, _ = run_pass("WRITE_SIZE", a.out, a.bench_args)
    cfg = bl.get("config", {})
    sys.path.insert(0, ROOT)
    import bench
    res = {
        "workload": cfg.get("workload"),
        "session": a.session or None,
        "kernel_build": bench.kernel_build_id(),
        "kernel": KERNEL or KERNEL_KEY,
        "dispatches": [len(fetch), len(write)],
        "FETCH_SIZE_KiB_median": statistics.median(fetch) if fetch else None,
        "WRITE_SIZE_KiB_median": statistics.median(write) if write else None,
        "read_bytes_per_launch": 2 * 1024 * statistics.median(fetch) if fetch else None,
        "write_bytes_per_launch": 1024 * statistics.median(write) if write else None,
        "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of wide streaming "
                      "reads), write = WRITE_SIZE x 1024 (MI355X_MICROARCH.md §HBM)",
        "alg_bytes_per_launch": (bl.get("roofline") or {}).get("alg_bytes_per_launch"),
    }
    if fetch and write:
        res["hbm_bytes_per_launch"] = res["read_bytes_per_launch"] + res["write_bytes_per_launch"]
        if res["alg_bytes_per_launch"]:
            res["traffic_over_alg"] = res["hbm_bytes_per_launch"] / res["alg_bytes_per_launch"]
    with open(os.path.join(a.out, "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    if a.commit:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
