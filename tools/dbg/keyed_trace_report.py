"""Probe (not product code): read a keyed-consumer stamp dump written by the
BPSR_KEYED_TRACE build (tools/dbg/build_keyed_trace_lib.sh) and summarise
where each epoch's time goes.  Times in microseconds from the epoch's first
forwarded release (the helper's first store of a host release word).
    python tools/dbg/keyed_trace_report.py <dump.bin>"""
import statistics
import struct
import sys

import numpy as np


def main(path):
    raw = open(path, "rb").read()
    ep, slots, per, tiles, nkeys, khz = struct.unpack_from("<6Q", raw, 0)
    off = 48
    bf = np.frombuffer(raw, np.uint32, nkeys + 1, off)
    off += 4 * (nkeys + 1)
    buf = np.frombuffer(raw, np.uint64, per * slots, off).reshape(slots, per)
    us = 1e3 / khz  # ticks -> us
    tile_key = np.repeat(np.arange(nkeys), np.diff(bf.astype(np.int64)))
    rows = []
    for s in range(slots):
        e = int(ep) - ((int(ep) - s) % slots)  # epoch held in slot s (the latest ones)
        t = buf[s, : 4 * tiles].reshape(tiles, 4).astype(np.int64)
        fw = buf[s, 4 * tiles: 4 * tiles + nkeys].astype(np.int64)
        if (t == 0).any() or (fw == 0).any():
            continue
        f0 = fw.min()
        rel = lambda x: (x - f0) * us
        start, seen, folded, counted = (rel(t[:, k]) for k in range(4))
        fwd = rel(fw)
        wait = seen - np.maximum(start, fwd[tile_key])     # seen after max(start, forward)
        rows.append({
            "epoch": e,
            "span_us": round(float(counted.max()), 1),
            "first_tile_start_us": round(float(start.min()), 1),
            "forward_last_us": round(float(fwd.max()), 1),
            "tile_fold_us_med": round(float(np.median(folded - seen)), 2),
            "tile_count_us_med": round(float(np.median(counted - folded)), 2),
            "tile_seen_lag_us_med": round(float(np.median(wait)), 2),
            "tile_seen_lag_us_p90": round(float(np.percentile(wait, 90)), 2),
            "tiles_started_before_forward": int((start < fwd[tile_key]).sum()),
            "last_tile_start_us": round(float(start.max()), 1),
        })
    rows.sort(key=lambda r: r["epoch"])
    for r in rows[-6:]:
        print(r)
    if rows:
        keys = [k for k in rows[0] if k != "epoch"]
        print({"epochs": len(rows), **{k: round(statistics.median(r[k] for r in rows), 2) for k in keys}})


if __name__ == "__main__":
    main(sys.argv[1])
