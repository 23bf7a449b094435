#!/usr/bin/env python3
"""HBM traffic per launch of config 3's kernels from rocprofv3 PMC counters.

tools/cfg3_native (C++, no Python in the loop) runs ResNet-50 fp16, 8 workers,
165 partitions in 12 Prophet blocks: the block-queue consumer
(``blockq_gate_kernel``, every block released before its launch — a PMC pass
serialises dispatches, so a live release could never reach a running
consumer) and one plan over all partitions (``batched_kernel``).  Two counter
passes, FETCH_SIZE then WRITE_SIZE (they cannot share a pass on gfx950), with
the corrections of MI355X_MICROARCH.md §HBM: read bytes = 2 x FETCH_SIZE KiB,
write bytes = WRITE_SIZE KiB.  Algorithmic bytes per iteration: 8 reads + 1
write of 51,114,064 B.  Writes one JSON summary to stdout and <out>/pmc_cfg3.json.
"""
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
KERNELS = ("blockq_gate_kernel", "batched_kernel")
BYTES = 51_114_064
N = 8


def run_pass(counter: str, outdir: str) -> dict:
    d = os.path.join(outdir, counter.lower())
    shutil.rmtree(d, ignore_errors=True)
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv",
           "-d", d, "-o", counter.lower(), "--",
           os.path.join(ROOT, "tools", "cfg3_native"),
           os.path.join(ROOT, "tools", "cfg3_resnet50_table.txt"), "20", "1", "",
           "plan_all,pre_released"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)  # SIGKILL on expiry
    if r.returncode != 0:
        raise SystemExit(f"pass {counter} rc={r.returncode}\n{r.stderr[-3000:]}")
    vals: dict = {k: {} for k in KERNELS}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for k in KERNELS:
                    if k in name:
                        key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                        vals[k][key] = vals[k].get(key, 0.0) + float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in vals.items()}, r.stdout


def main(outdir=os.path.join(ROOT, "gpurun_out", "pmc_cfg3")):
    os.makedirs(outdir, exist_ok=True)
    fetch, out1 = run_pass("FETCH_SIZE", outdir)
    write, out2 = run_pass("WRITE_SIZE", outdir)
    res = {"config": "cfg3 ResNet-50 fp16, 8 workers, 165 partitions, 12 blocks",
           "driver": "tools/cfg3_native (variants plan_all_partitions_no_blocks, "
                     "blockq_pre_released; 20 iterations after 30 warm-up, 3 rotated sets)",
           "alg_read_bytes": N * BYTES, "alg_write_bytes": BYTES,
           "corrections": "read = 2 x FETCH_SIZE KiB (gfx950 tallies 128-B streaming reads "
                          "at 64 B), write = WRITE_SIZE KiB (MI355X_MICROARCH.md)",
           "kernels": {}}
    for k in KERNELS:
        if not fetch[k] or not write[k]:
            res["kernels"][k] = {"error": "no dispatches counted"}
            continue
        rd = statistics.median(fetch[k]) * 1024 * 2
        wr = statistics.median(write[k]) * 1024
        res["kernels"][k] = {
            "dispatches": [len(fetch[k]), len(write[k])],
            "read_bytes_median": rd, "write_bytes_median": wr,
            "read_over_alg": round(rd / (N * BYTES), 5),
            "write_over_alg": round(wr / BYTES, 5),
            "traffic_over_alg": round((rd + wr) / ((N + 1) * BYTES), 5),
        }
    res["driver_lines"] = [json.loads(x) for x in (out1 + out2).splitlines() if x.startswith("{")]
    with open(os.path.join(outdir, "pmc_cfg3.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "driver_lines"}))


if __name__ == "__main__":
    main(*sys.argv[1:])
