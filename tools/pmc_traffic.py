#!/usr/bin/env python3
"""Per-hop HBM traffic of the SpMM kernel from rocprofv3 --pmc runs of tools/spmm_probe.py (a hop
is one launch, or one per column block; the "_per_hop" keys hold the sums over a hop's launches;
the bytes are L2 -> fabric bytes, Infinity-Cache hits included, not DRAM bytes).

    python tools/pmc_traffic.py --fetch DIR --write DIR [--hits DIR] --probe probe.json --out OUT.json

traffic = 2 * FETCH_SIZE + WRITE_SIZE  (MI355X_MICROARCH.md, HBM: on gfx950 FETCH_SIZE reports
exactly half the bytes of wide coalesced reads -- our gathers are whole 512-byte rows read 8 or 16
bytes per lane; WRITE_SIZE is exact for wide stores).  Cross-check: TCC_MISS_sum * 128 B (L2
misses, 128-byte lines), recorded beside it when a TCC_HIT/TCC_MISS run is given.  FETCH_SIZE
counts every L2 miss served by the fabric, so Infinity-Cache hits are included (an upper bound on
DRAM bytes).
"""
import argparse
import csv
import glob
import json
import os


def per_launch(d, counters, kernel_sub="k_spmm<", hops=None):
    """Median over the main k_spmm dispatches (hub workgroups excluded) of each counter, or with
    `hops`, the sum over all of them divided by the hop count (column-blocked hops are several
    launches).  Returns {counter: (value, dispatches)}."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row.get("Kernel_Name", "") or "k_spmm_hub" in row.get("Kernel_Name", ""):
                    continue
                name = row.get("Counter_Name")
                if name not in counters:
                    continue
                key = (name, f, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for c in counters:
        v = sorted(x for (n, _, _), x in vals.items() if n == c)
        if not v:
            raise SystemExit(f"no {c} rows for {kernel_sub} under {d}")
        out[c] = (sum(v) / hops if hops else v[len(v) // 2], len(v))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--hits")
    ap.add_argument("--probe", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    probe = json.load(open(a.probe))
    hops = probe["reps"]
    f = per_launch(a.fetch, ["FETCH_SIZE"], hops=hops)["FETCH_SIZE"]
    w = per_launch(a.write, ["WRITE_SIZE"], hops=hops)["WRITE_SIZE"]
    B = probe.get("launches_per_hop", 1)
    rec = {"config": probe["config"], "kernel": f"k_spmm (one hop: {B} launch{'es' if B > 1 else ''}, "
                                               "hub workgroups excluded)", "n_heavy": probe.get("n_heavy"),
           "launches": f[1], "launches_per_hop": B,
           "fetch_size_kib": f[0], "write_size_kib": w[0],
           "hbm_read_bytes_per_hop": 2.0 * f[0] * 1024, "hbm_write_bytes_per_hop": w[0] * 1024}
    rec["hbm_bytes_per_hop"] = rec["hbm_read_bytes_per_hop"] + rec["hbm_write_bytes_per_hop"]
    if a.hits:
        h = per_launch(a.hits, ["TCC_HIT_sum", "TCC_MISS_sum"], hops=hops)
        hit, miss = h["TCC_HIT_sum"][0], h["TCC_MISS_sum"][0]
        rec["l2_hit_rate"] = hit / (hit + miss)
        rec["l2_miss_bytes_per_hop"] = miss * 128.0
    rec["algorithmic_bytes_per_hop"] = probe["algorithmic_bytes"]
    rec["compulsory_bytes_per_hop"] = probe["compulsory_bytes"]
    rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_hop"] / probe["algorithmic_bytes"]
    rec["traffic_over_compulsory"] = rec["hbm_bytes_per_hop"] / probe["compulsory_bytes"]
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
