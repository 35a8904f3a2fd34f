#!/usr/bin/env python3
"""Where one hop's time goes: the full hop against operators made of one row group only (hub rows,
slice-wave rows, row-wave rows), each launched alone with the default schedule, plus the empty
launch overhead.  Row groups follow srgnn.csr.make_schedule.  Prints one JSON object.

    python tools/hop_breakdown.py --config arxiv [--reps 50]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR, auto_hub_threshold  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="arxiv")
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build(a.config, dev)
X = synth.uniform_features_t(n, d, device=dev)
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
HUB_T = auto_hub_threshold(A.nnz)     # the full operator's split, kept for the subsets


def timed(op, rows_out):
    Y = torch.empty((rows_out, d), device=dev)
    for _ in range(3):
        spmm(op, X, out=Y)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.reps):
        spmm(op, X, out=Y)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / a.reps


def subset(rows):
    rows = torch.sort(rows).values
    deg = ip[rows + 1] - ip[rows]
    sip = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=dev)
    sip[1:] = torch.cumsum(deg, 0)
    starts = torch.repeat_interleave(ip[rows], deg)
    offs = torch.arange(int(sip[-1]), device=dev) - torch.repeat_interleave(sip[:-1], deg)
    sel = starts + offs
    return (DeviceCSR.from_tensors(sip, ix[sel], vals[sel], n_cols=n, device=dev, hub_threshold=HUB_T),
            rows.numel(), int(deg.sum()))


order = A.order.to(torch.int64)
groups = {"hub": order[: A.n_hub], "slice": order[A.n_hub: A.n_hub + A.n_heavy],
          "row": order[A.n_hub + A.n_heavy:]}
out = {"config": a.config, "n": n, "nnz": A.nnz, "d": d, "n_hub": A.n_hub, "n_heavy": A.n_heavy,
       "env": {k: v for k, v in os.environ.items() if k.startswith("SRGNN_")}, "full_ms": timed(A, n)}
Yf = torch.empty((n, d), device=dev)
spmm(A, X, out=Yf)
torch.cuda.synchronize()
out["full_sha256"] = __import__("hashlib").sha256(Yf.cpu().numpy().tobytes()).hexdigest()[:16]
del Yf
for name, rows in groups.items():
    if rows.numel() == 0:
        continue
    op, r, z = subset(rows)
    out[f"{name}_rows"] = r
    out[f"{name}_nnz"] = z
    out[f"{name}_ms"] = timed(op, r)
empty = DeviceCSR.from_tensors(torch.zeros(2, dtype=torch.int64, device=dev), ix[:0], vals[:0], n_cols=n, device=dev)
out["empty_launch_ms"] = timed(empty, 1)
print(json.dumps(out))
