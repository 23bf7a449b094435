#!/usr/bin/env python3
"""Idle stretches of a rocprofv3 kernel + memory-copy trace (csv output):
merge every kernel dispatch and copy into busy intervals and list the gaps
longer than --min-us, plus per-direction copy rates and busy fractions over
the traced window's last --window-ms.  Not product code."""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kind = "h2d" if "HOST_TO_DEVICE" in r["Direction"] else (
                "d2h" if "DEVICE_TO_HOST" in r["Direction"] else "d2d")
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "k:" + r["Kernel_Name"].split("<")[0].split("::")[-1]))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=50.0)
    ap.add_argument("--window-ms", type=float, default=0.0, help="0 = whole trace")
    a = ap.parse_args()
    ev = load(a.dir)
    t_end = max(e for _, e, _ in ev)
    t_lo = t_end - a.window_ms * 1e6 if a.window_ms else ev[0][0]
    ev = [x for x in ev if x[1] > t_lo]
    gaps, busy, cur_s, cur_e = [], 0, None, None
    for s, e, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                if (s - cur_e) / 1e3 >= a.min_us:
                    gaps.append(((cur_e - t_lo) / 1e3, (s - cur_e) / 1e3))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - max(t_lo, ev[0][0])
    by = {}
    for s, e, k in ev:
        d = by.setdefault(k, [0, 0])
        d[0] += 1
        d[1] += e - s
    print(json.dumps({"span_ms": round(span / 1e6, 3), "busy_frac": round(busy / span, 3),
                      "gaps_over_min": len(gaps), "gap_ms_total": round(sum(g for _, g in gaps) / 1e3, 3),
                      "largest_gaps_us": sorted((round(g, 1) for _, g in gaps), reverse=True)[:12],
                      "by_kind": {k: {"n": v[0], "mean_us": round(v[1] / v[0] / 1e3, 1)}
                                  for k, v in by.items()}}))


if __name__ == "__main__":
    main()
