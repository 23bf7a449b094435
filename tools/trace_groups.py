#!/usr/bin/env python3
"""Per-launch duration and inter-launch gap of repeated launch sequences in a
rocprofv3 kernel-trace CSV (e.g. the 12 block plans of cfg3 replayed from a
hipGraph).  usage: trace_groups.py TRACE.csv [kernel-substring] [group-size]"""
import csv
import statistics as st
import sys


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "batched_kernel"
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], []
    for r in rows:
        if key in r["Kernel_Name"]:
            cur.append(r)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    for run in runs:
        if len(run) < 5 * G:
            continue
        its = [run[i:i + G] for i in range(0, len(run) // G * G, G)]
        t = lambda r, a: int(r[a]) / 1e3
        durs = [st.median(t(it[k], "End_Timestamp") - t(it[k], "Start_Timestamp") for it in its)
                for k in range(G)]
        gaps = [st.median(t(it[k + 1], "Start_Timestamp") - t(it[k], "End_Timestamp") for it in its)
                for k in range(G - 1)]
        tot = st.median(t(it[-1], "End_Timestamp") - t(it[0], "Start_Timestamp") for it in its)
        grids = [int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) for r in its[0]]
        print(f"iters {len(its)} grids {grids}")
        print(f"  durs {[round(d, 1) for d in durs]} sum {sum(durs):.1f}")
        print(f"  gaps {[round(g, 2) for g in gaps]} sum {sum(gaps):.1f} total {tot:.1f}")


if __name__ == "__main__":
    main()
