#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace run: the last N dispatches, in start order, in us from the
first one shown (kernel, start, end, duration, grid, queue).

    python tools/trace_timeline.py DIR [--last 40] [--only spmm,hub,delay]
"""
import argparse
import csv
import glob
import os


def short(name):
    for key, s in (("k_spmm_hub", "hub"), ("k_dispatch_delay", "delay"), ("k_gather_rows", "pack"),
                   ("k_spmm", "spmm"), ("k_cheby", "cheby")):
        if key in name:
            return s
    return name.split("(")[0].split("<")[0][-24:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--only", default=None, help="comma list of short names (spmm, hub, delay, pack, cheby) to keep")
    a = ap.parse_args()
    keep = set(a.only.split(",")) if a.only else None
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Queue_Id", "")))
    rows.sort()
    if keep is not None:
        rows = [r for r in rows if short(r[2]) in keep]
    rows = rows[-a.last:]
    t0 = rows[0][0] if rows else 0
    for s, e, name, grid, q in rows:
        print(f"{short(name):6s} start {(s - t0) / 1e3:10.1f} end {(e - t0) / 1e3:10.1f} dur {(e - s) / 1e3:9.1f} "
              f"grid {grid:>10s} q {q}")


if __name__ == "__main__":
    main()
