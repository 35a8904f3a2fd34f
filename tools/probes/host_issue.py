#!/usr/bin/env python3
"""Host cost of issuing one halo-exchange hop (rank 0 of P virtual ranks, products-shaped graph):
the CPU time of HaloPartitionedOperator.compute + the per-group packs, issued back to back without
synchronising, against the GPU time of the same work.  The collectives are not included (no
process group here).  Prints one JSON object."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "scalable-roubust-gnn_amd"))
import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.dist import HaloPartitionedOperator  # noqa: E402
from srgnn.spmm import gather_rows  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, K = graphs.build("products", dev)
x = synth.uniform_features_t(n, d, device=dev)
op = HaloPartitionedOperator(ip, ix, vals, n, chunks=6, device=dev, rank=0, world=P)
src = op.new_panel(d)
src[: op.rows].copy_(x[op.r0:op.r1])
dst = op.new_panel(d)


def hop():
    op.compute(src, dst)
    for g in range(op.n_groups):
        if op.send_cat[g].numel():
            gather_rows(dst[: op.rows], op.send_cat[g])


for _ in range(3):
    hop()
torch.cuda.synchronize()
reps = 20
t0 = time.perf_counter()
for _ in range(reps):
    hop()
t_issue = (time.perf_counter() - t0) / reps
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / reps
print(json.dumps({"P": P, "groups": op.n_groups, "host_issue_ms_per_hop": t_issue * 1e3,
                  "wall_ms_per_hop": t_all * 1e3}))
