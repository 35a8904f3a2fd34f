#!/usr/bin/env python3
"""Probe: the fp32 hop with more whole hub rows (SRG_PLAN_WHOLE_HUBS at an explicit length) against the
planner's automatic rule (rows > max(2048, nnz / 1024)), products-shaped, d = 128, compact plans as the
bench builds them.  Each variant's hop is checked bitwise against the default plan's."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.plan import NativePlan  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "products"
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build(cfg, dev)
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
ref = None
for ht in (None, 65536, 32768, 16384, 8192):
    P = NativePlan(A, d, 1 << 20, hub_threshold=ht)
    P.hop(X, Y, d)
    torch.cuda.synchronize()
    if ref is None:
        ref = Y.clone()
    same = bool(torch.equal(Y, ref))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        P.hop(X, Y, d)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"hub_threshold": ht, "col_blocks": P.col_blocks, "n_launch": P.n_launch,
                      "hub_rows_whole": P.hub_rows_whole, "compact": P.compact, "ms_per_hop": e0.elapsed_time(e1) / 10,
                      "bitwise_vs_auto": same}), flush=True)
    P.close()
