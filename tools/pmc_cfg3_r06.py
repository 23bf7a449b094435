#!/usr/bin/env python3
"""HBM traffic per launch of config 3's round-5/6 consumers from rocprofv3 PMC
counters (missing 3):

  blockq_gate_kernel   the block queue's dispatch-ordered consumer as it runs
                       since round 5 — overlapped launches on two consumer
                       queues, the dispatch-sequence counting, the arena
                       layout; every iteration released before its launch
                       (tools/dbg/cfg3_pre_released.py)
  blockq_key_kernel    the PS server's keyed consumer (device releases):
                       config 3's 165 keys x 8 workers through the server,
                       host releases forwarded by the helper workgroup
                       (tools/dbg/server_cfg3_once.py, bench.server_cfg3_leg)

Two passes per driver, FETCH_SIZE then WRITE_SIZE (they cannot share a pass
on gfx950), each its own rocprofv3 run with --kernel-trace only; corrections
of MI355X_MICROARCH.md §HBM: read bytes = 2 x FETCH_SIZE KiB, write bytes =
WRITE_SIZE KiB.  Algorithmic bytes per launch: 8 reads + 1 write of
51,114,064 B.  Writes <out>/pmc_cfg3_r06.json and prints it.
    python tools/pmc_cfg3_r06.py [outdir]"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BYTES = 51_114_064
N = 8
DRIVERS = {
    "blockq_gate_kernel": [sys.executable, os.path.join(ROOT, "tools", "dbg", "cfg3_pre_released.py"),
                           "40"],
    "blockq_key_kernel": [sys.executable, os.path.join(ROOT, "tools", "dbg", "server_cfg3_once.py"),
                          "--reps", "1"],
}


def run_pass(kernel: str, counter: str, outdir: str):
    d = os.path.join(outdir, kernel, counter.lower())
    shutil.rmtree(d, ignore_errors=True)
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", counter, "--kernel-trace",
           "--output-format", "csv", "-d", d, "-o", counter.lower(), "--"] + DRIVERS[kernel]
    os.makedirs(d, exist_ok=True)
    print(f"pass {kernel} {counter}: start", file=sys.stderr, flush=True)
    # the driver's output goes to files under outdir as it runs (progress)
    with open(os.path.join(d, "stdout.txt"), "w") as fo, open(os.path.join(d, "stderr.txt"), "w") as fe:
        r = subprocess.run(cmd, stdout=fo, stderr=fe, text=True)
    with open(os.path.join(d, "stdout.txt")) as fo:
        r.stdout = fo.read()
    print(f"pass {kernel} {counter}: rc {r.returncode}", file=sys.stderr, flush=True)
    # rocprofv3 can fault in its own exit after writing its files
    # (profiles/r06s06_exit_fault_frames.txt): judge by the files
    vals: dict = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return list(vals.values()), r.returncode, lines


def main(outdir=os.path.join(ROOT, "gpurun_out", "pmc_cfg3_r06")):
    os.makedirs(outdir, exist_ok=True)
    res = {"config": "cfg3 ResNet-50 fp16, 8 workers, 165 partitions (12 blocks / 165 keys)",
           "alg_read_bytes": N * BYTES, "alg_write_bytes": BYTES,
           "corrections": "read = 2 x FETCH_SIZE KiB (gfx950 tallies 128-B streaming reads "
                          "at 64 B), write = WRITE_SIZE KiB (MI355X_MICROARCH.md)",
           "kernels": {}}
    for k in DRIVERS:
        fetch, rc1, l1 = run_pass(k, "FETCH_SIZE", outdir)
        write, rc2, l2 = run_pass(k, "WRITE_SIZE", outdir)
        ent = {"driver": " ".join(os.path.relpath(x, ROOT) if x.startswith(ROOT) else x
                                  for x in DRIVERS[k][1:]),
               "rocprofv3_rc": [rc1, rc2], "driver_lines": l1 + l2}
        if not fetch or not write:
            ent["error"] = "no dispatches counted"
        else:
            rd = statistics.median(fetch) * 1024 * 2
            wr = statistics.median(write) * 1024
            ent.update({"dispatches": [len(fetch), len(write)],
                        "read_bytes_median": rd, "write_bytes_median": wr,
                        "read_over_alg": round(rd / (N * BYTES), 5),
                        "write_over_alg": round(wr / BYTES, 5),
                        "traffic_over_alg": round((rd + wr) / ((N + 1) * BYTES), 5)})
        res["kernels"][k] = ent
    with open(os.path.join(outdir, "pmc_cfg3_r06.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
