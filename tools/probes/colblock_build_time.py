#!/usr/bin/env python3
"""Time DeviceCSR.column_blocks(2) (the one-off cut of an operator into column blocks) against the
per-hop gain, on the products-shaped graph.  Prints one JSON object."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "scalable-roubust-gnn_amd"))
import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import auto_col_blocks, hop  # noqa: E402

dev = torch.device("cuda", 0)
ip, ix, vals, n, d, K = graphs.build("products", dev)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
res = {}
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
B_auto = auto_col_blocks(A, d, hops=1 << 30)
res["B_auto"] = B_auto
for rep in range(3):
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A.column_blocks(B_auto)
    torch.cuda.synchronize()
    res.setdefault("build_ms", []).append((time.perf_counter() - t0) * 1e3)
for B in sorted({1, 2, B_auto}):
    hop(A, X, Y, col_blocks=B)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        hop(A, X, Y, col_blocks=B)
    ev[1].record()
    torch.cuda.synchronize()
    res[f"hop_ms_B{B}"] = ev[0].elapsed_time(ev[1]) / 10
print(json.dumps(res))
