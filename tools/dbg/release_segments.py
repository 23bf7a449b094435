"""Probe analysis (not product code), round 6: per segment of a rocprofv3
kernel trace (segments split at > 20 ms with no kernel), the block queue's
release kernels — count, median and p90 duration, the (hardware queue,
stream) pairs they ran on — and the consumers' median duration.  The form of
profiles/r05s34_ctx_release_queues.txt, for the VERDICT round-5 check "every
segment's release median within 2x of 5 us".
Usage: python tools/dbg/release_segments.py <kernel_trace.csv> [gap_ms=20]"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    gap_ns = float(sys.argv[2] if len(sys.argv) > 2 else 20) * 1e6
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    rows.sort()
    segs, cur, last_end = [], [], None
    for row in rows:
        if last_end is not None and row[0] - last_end > gap_ns and cur:
            segs.append(cur)
            cur = []
        cur.append(row)
        last_end = row[1] if last_end is None else max(last_end, row[1])
    if cur:
        segs.append(cur)
    for i, seg in enumerate(segs):
        rel = [(e - s) / 1e3 for s, e, n, q, st in seg if "blockq_release" in n]
        cons = [(e - s) / 1e3 for s, e, n, q, st in seg if "blockq_gate_kernel" in n]
        if not rel:
            continue
        qs = sorted({(q, st) for s, e, n, q, st in seg if "blockq_release" in n})
        rel.sort()
        print(f"segment {i}: {len(rel)} releases, median {statistics.median(rel):.1f} us, "
              f"p90 {rel[int(0.9 * (len(rel) - 1))]:.1f} us, queues (hw, stream) {qs}, "
              f"consumer median {statistics.median(cons) if cons else float('nan'):.1f} us")


if __name__ == "__main__":
    main()
