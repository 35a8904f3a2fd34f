#!/usr/bin/env python3
"""In-process A/B of SpMM schedule variants on one graph (interleaved rounds, cdna guide rule 24).
Prints per-variant median / min kernel ms and the implied no-reuse roofline fraction."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from srgnn import graphs, roofline, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--thresholds", default="32:-1,32:4096,32:16384,32:65536",
                help="comma list of heavy:hub thresholds (-1 disables a group)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--nt", action="store_true")
ap.add_argument("--n", type=int, default=None)
ap.add_argument("--bigbuf", type=int, default=0, help="X, Y as slices of one (bigbuf, n, d) buffer")
ap.add_argument("--n-edges", type=int, default=None)
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build(a.config, dev, n=a.n, n_edges=a.n_edges)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
if a.bigbuf:
    big = torch.empty((a.bigbuf, n, d), dtype=torch.float32, device=dev)
    big[0].copy_(X)
    X, Y = big[0], big[1]
variants = {}
for spec in a.thresholds.split(","):
    parts = spec.split(":")
    h = int(parts[0])
    hub = int(parts[1]) if len(parts) > 1 else -1
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=h, hub_threshold=hub, device=dev)
    variants[f"thr={spec}"] = (A, False)
    if a.nt:
        variants[f"thr={spec},nt"] = (A, True)
ref = None
times = {k: [] for k in variants}
for r in range(a.rounds):
    for k, (A, nt) in variants.items():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        spmm(A, X, out=Y, nt_store=nt)
        e.record()
        torch.cuda.synchronize()
        times[k].append(s.elapsed_time(e))
        if r == 0:
            if ref is None:
                ref = Y.clone()
            else:
                assert torch.equal(ref, Y), f"{k} changed the result"
b = roofline.bytes_no_reuse(n, ix.numel(), d)
out = {}
for k, v in times.items():
    med = float(np.median(v[1:] if len(v) > 1 else v))
    out[k] = {"median_ms": med, "min_ms": float(min(v)), "all_ms": [round(t, 3) for t in v],
              "n_heavy": variants[k][0].n_heavy,
              "n_hub": variants[k][0].n_hub,
              "frac": b / (med * 1e-3) / 1e9 / roofline.MI355X_HBM_PEAK_GBS}
print(json.dumps({"config": a.config, "n": n, "nnz": int(ix.numel()), "d": d, "variants": out}, indent=1))
