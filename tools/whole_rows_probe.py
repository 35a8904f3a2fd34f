#!/usr/bin/env python3
"""Probe: the launch of block 0's whole rows (the short rows a column-blocked hop computes in one
piece, DeviceCSR.split_whole()[1]) timed alone, next to one cut-span launch of the same hop (the
packed-row geometry is a compile-time constant of the library since round 5; round 3 swept it through
environment knobs).  Prints one JSON line.

    python tools/whole_rows_probe.py [--config products] [--reps 20]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--u2", type=int, default=0, help="pass SRG_SPMM_PACKED_U2 to the whole-row launch")
ap.add_argument("--natural", action="store_true", help="whole rows in row order (no length sort)")
ap.add_argument("--check", action="store_true", help="the launches together == hop(), bitwise")
ap.add_argument("--sched", action="store_true", help="entries copied out in schedule order (DeviceCSR.schedule_ordered)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build(a.config, dev)
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
blocks = A.compact_column_blocks(4)   # the probe's fixed layout: four blocks
cut, whole = blocks[0].split_whole()
if a.natural:
    whole.order = torch.sort(whole.order).values.contiguous()
    whole.n_heavy = 0
if a.sched:
    whole = whole.schedule_ordered()
    cut = cut.schedule_ordered()
    blocks = [blocks[0]] + [b.schedule_ordered() for b in blocks[1:]]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / a.reps


res = {"config": a.config, "env": {k: v for k, v in os.environ.items() if k.startswith("SRGNN_")},
       "u2": a.u2, "natural": a.natural, "sched": a.sched,
       "whole_rows": whole.n_rows, "whole_nnz": int(((whole.row_end if whole.is_span else whole.indptr[1:])
                                                      - whole.indptr[: whole.out_rows])[whole.order.long()].sum()),
       "ms_whole": timed(lambda: spmm(whole, X, out=Y, packed_u2=bool(a.u2))),
       "ms_block1": timed(lambda: spmm(blocks[1], X, out=Y, accumulate=True, packed_u2=True)),
       "ms_cut0": timed(lambda: spmm(cut, X, out=Y, packed_u2=True))}
if a.check:
    from srgnn.spmm import hop
    ref = hop(A, X, torch.empty_like(X), col_blocks=4)
    Y2 = torch.empty_like(X)
    spmm(cut, X, out=Y2, packed_u2=True)
    spmm(whole, X, out=Y2, packed_u2=True)
    for b in blocks[1:]:
        spmm(b, X, out=Y2, accumulate=True, packed_u2=True)
    torch.cuda.synchronize()
    res["bitwise_equal_to_hop"] = bool(torch.equal(ref, Y2))
print(json.dumps(res))
