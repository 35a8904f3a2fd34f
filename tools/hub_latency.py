#!/usr/bin/env python3
"""Latency of the longest rows alone: an operator made of only the top-R rows of the products-shaped
graph, through the slice path vs the hub path.  This is the tail that bounds multi-GPU hops."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402

dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build("products", dev)
X = synth.uniform_features_t(n, d, device=dev)
deg = ip[1:] - ip[:-1]
out = {}
for R in (1, 8, 64, 512):
    top = torch.sort(deg, descending=True).indices[:R]
    top = torch.sort(top).values
    sub_deg = deg[top]
    sub_ip = torch.zeros(R + 1, dtype=torch.int64, device=dev)
    sub_ip[1:] = torch.cumsum(sub_deg, 0)
    sel = torch.cat([torch.arange(int(ip[r]), int(ip[r + 1]), device=dev) for r in top.tolist()])
    sub_ix, sub_v = ix[sel], vals[sel]
    res = {}
    ref = None
    for name, (h, u) in {"slice": (0, -1), "hub": (0, 0), "row": (-1, -1)}.items():
        A = DeviceCSR.from_tensors(sub_ip, sub_ix, sub_v, n_cols=n, heavy_threshold=h, hub_threshold=u, device=dev)
        Y = torch.empty((R, d), device=dev)
        ts = []
        for _ in range(4):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(); spmm(A, X, out=Y); e.record(); torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        if ref is None:
            ref = Y.clone()
        assert torch.equal(ref, Y), name
        res[name] = float(np.median(ts[1:]))
    out[f"top{R}"] = {"max_deg": int(sub_deg.max()), "nnz": int(sub_deg.sum()), "ms": res}
print(json.dumps(out, indent=1))
