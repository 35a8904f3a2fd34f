#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of tools/spmm_probe.py into per-launch
HBM traffic of the SpMM kernel, calibrated on the identity-operator run.

    python tools/pmc_traffic.py --fetch DIR --write DIR --cal-fetch DIR --cal-write DIR \
        --probe probe.json --cal-probe cal.json --out profiles/pmc_products.json

Calibration: the identity run moves a known byte count (x_read + index reads, y_write) with the
same kernel; scale = known / counted.  traffic = fetch * scale_r + write * scale_w (bytes/launch).
"""
import argparse
import csv
import glob
import json
import os


def per_launch(d, counter, kernel_sub="k_spmm"):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_sub} under {d}")
    v = sorted(vals.values())
    return v[len(v) // 2] * 1024.0, len(v)        # FETCH_SIZE / WRITE_SIZE are in KiB


def main():
    ap = argparse.ArgumentParser()
    for k in ("fetch", "write", "cal_fetch", "cal_write", "probe", "cal_probe", "out"):
        ap.add_argument("--" + k.replace("_", "-"), required=True)
    a = ap.parse_args()
    probe = json.load(open(a.probe))
    cal = json.load(open(a.cal_probe))
    f_raw, nf = per_launch(a.fetch, "FETCH_SIZE")
    w_raw, nw = per_launch(a.write, "WRITE_SIZE")
    cf_raw, _ = per_launch(a.cal_fetch, "FETCH_SIZE")
    cw_raw, _ = per_launch(a.cal_write, "WRITE_SIZE")
    known_r = cal["x_read_bytes"] + cal["index_bytes"]
    known_w = cal["y_write_bytes"]
    sr, sw = known_r / cf_raw, known_w / cw_raw
    rec = {
        "config": probe["config"], "kernel": "k_spmm (one hop)",
        "fetch_size_raw_bytes": f_raw, "write_size_raw_bytes": w_raw, "launches": [nf, nw],
        "calibration": {"identity_n": cal["n"], "d": cal["d"], "known_read": known_r, "known_write": known_w,
                        "fetch_counted": cf_raw, "write_counted": cw_raw,
                        "read_scale": sr, "write_scale": sw},
        "hbm_read_bytes_per_launch": f_raw * sr, "hbm_write_bytes_per_launch": w_raw * sw,
        "hbm_bytes_per_launch": f_raw * sr + w_raw * sw,
        "algorithmic_bytes_per_launch": probe["algorithmic_bytes"],
        "compulsory_bytes_per_launch": probe["compulsory_bytes"],
    }
    rec["traffic_over_compulsory"] = rec["hbm_bytes_per_launch"] / probe["compulsory_bytes"]
    rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / probe["algorithmic_bytes"]
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
