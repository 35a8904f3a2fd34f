#!/usr/bin/env python3
"""Sums of one rocprofv3 --pmc counter per kernel family (k_spmm, k_spmm_hub, k_gather_rows, ...)
over a run: total, dispatches, and total per dispatch of a reference family (e.g. per hub launch =
per hop of the halo probe).

    python tools/pmc_sum.py DIR COUNTER [--per hub]
"""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_timeline import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("counter")
    ap.add_argument("--per", default="hub")
    ap.add_argument("--cycle", type=int, default=0,
                    help="also average the k_spmm dispatches by position in a cycle of this many (one hop's "
                         "launches, in dispatch order)")
    a = ap.parse_args()
    vals, disp, spmm = {}, {}, {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != a.counter:
                    continue
                k = short(r.get("Kernel_Name", ""))
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
                disp.setdefault(k, set()).add((f, r.get("Dispatch_Id")))
                if k == "spmm":
                    key = (f, int(r.get("Dispatch_Id", 0)))
                    spmm[key] = spmm.get(key, 0.0) + float(r["Counter_Value"])
    n = len(disp.get(a.per, ())) or 1
    out = {"counter": a.counter, "per": a.per, "units": n,
           "families": {k: {"total": v, "dispatches": len(disp[k]), "per_unit": v / n} for k, v in vals.items()}}
    if a.cycle > 0 and spmm:
        seq = [v for _, v in sorted(spmm.items())]
        seq = seq[len(seq) % a.cycle:]                      # whole cycles, the last ones
        out["spmm_by_position"] = [sum(seq[i::a.cycle]) / max(1, len(seq[i::a.cycle])) for i in range(a.cycle)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
