"""Probe (not product code): from a rocprofv3 --kernel-trace CSV, the keyed
consumer's per-epoch duration and the gap to the next epoch's consumer.
    python tools/dbg/keyed_trace_gaps.py <kernel_trace.csv>"""
import csv
import statistics
import sys


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "blockq_key_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    dur = [(e - s) / 1e3 for s, e in rows]
    gaps = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    per = [(rows[i + 1][1] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    q = lambda v: (round(statistics.median(v), 1), round(min(v), 1), round(max(v), 1)) if v else None
    print({"consumers": len(rows), "duration_us_med_min_max": q(dur),
           "gap_to_next_us": q(gaps), "end_to_end_us": q(per)})


if __name__ == "__main__":
    main(sys.argv[1])
