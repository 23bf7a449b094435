#!/usr/bin/env python3
"""Write BASELINE config 3's bucket table for the native drivers
(tools/cfg3_native.cpp): ResNet-50 fp16 gradients (torchvision layout, 161
tensors), BytePS partitions (operations.cc:99-136, 4,096,000-B bound), grouped
into the 12 Prophet blocks (scheduled_queue.h:78-79, last checkpoint extended
to index 160), blocks in release order.  Byte offsets are into one worker's
whole gradient vector (tensor order), as tools/bench_configs.py lays it out.

Format: "total_bytes nparts nblocks", then nparts lines "offset len", then one
line of nblocks block ends (cumulative partition counts).

A second file (``..._tasks.txt``) feeds the native Prophet scheduler
(include/bpsr/prophet.h) in the same driver: "ncheckpoints" and the
checkpoints, then per partition in table order "grad part total_partnum len"."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from prophet_amd.buckets import partition_all, prophet_blocks, resnet50_param_sizes  # noqa: E402


def main(path=os.path.join(ROOT, "tools", "cfg3_resnet50_table.txt")):
    from prophet_amd.prophet import model_checkpoints
    sizes = [n * 2 for n in resnet50_param_sizes()]
    parts = partition_all(sizes)
    nparts = {}
    for p in parts:
        nparts[p.tensor] = nparts.get(p.tensor, 0) + 1
    tasks = []
    toff = [0]
    for n in sizes:
        toff.append(toff[-1] + n)
    rows, ends = [], []
    for blk in prophet_blocks(len(sizes)):
        tset = set(blk)
        for p in parts:
            if p.tensor in tset:
                rows.append((toff[p.tensor] + p.offset, p.len))
                tasks.append((p.tensor, p.part, nparts[p.tensor], p.len))
        ends.append(len(rows))
    with open(path, "w") as f:
        f.write(f"{toff[-1]} {len(rows)} {len(ends)}\n")
        for o, ln in rows:
            f.write(f"{o} {ln}\n")
        f.write(" ".join(map(str, ends)) + "\n")
    cps = model_checkpoints(len(sizes))
    with open(path.replace("_table.txt", "_tasks.txt"), "w") as f:
        f.write(f"{len(cps)} " + " ".join(map(str, cps)) + "\n")
        for t in tasks:
            f.write(" ".join(map(str, t)) + "\n")
    print(path, toff[-1], len(rows), len(ends))


if __name__ == "__main__":
    main(*sys.argv[1:])
