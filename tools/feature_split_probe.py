#!/usr/bin/env python3
"""Hop time of the products-shaped SpMM with the panel's FEATURE columns split into F sub-panels
(each a strided view of X and Y, one hop per sub-panel), times B column blocks per sub-panel hop.

Every output element is its own fma chain over the row's entries in CSR order (matmul.c:26-39), so
a feature split is bitwise the one-panel hop; it trades F reads of the operator's index / value
arrays for a gathered row of 4d/F bytes, i.e. F times as many X rows per MiB of L2.  Prints one JSON
line per (F, B) with the median hop time and a bitwise check against the F = 1 hop."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import column_blocks_for, hop  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--splits", default="1,2,4")
ap.add_argument("--col-blocks", default="1,2,4,8")
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, K = graphs.build(a.config, dev)
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
want = None
for B in [int(b) for b in a.col_blocks.split(",")]:
    if B > 1:
        column_blocks_for(A, B, hops=1 << 20)
    for F in [int(f) for f in a.splits.split(",")]:
        w = d // F

        def run():
            for f in range(F):
                hop(A, X[:, f * w:(f + 1) * w], Y[:, f * w:(f + 1) * w], col_blocks=B)
        run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
        for r in range(a.reps):
            ev[2 * r].record()
            run()
            ev[2 * r + 1].record()
        torch.cuda.synchronize()
        ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
        if want is None:
            want = Y.clone()
        same = bool(torch.equal(Y, want))
        print(json.dumps({"config": a.config, "F": F, "B": B, "sub_panel_d": w, "hop_ms": ms[len(ms) // 2],
                          "hop_ms_min": ms[0], "bitwise_vs_first": same}), flush=True)
    A._blocks.clear() if hasattr(A, "_blocks") else None
