#!/usr/bin/env python3
"""Check of the C-ABI communicator path on a multi-GPU node (one process, every visible GPU):
srg_comm_init_all + srg_dist_propagate_khop_f32 over P nnz-balanced row blocks, compared bitwise with
the one-GPU K-hop propagate, and timed per hop.  Prints one JSON line.

    python tools/comm_capi_check.py [--config products] [--gpus P] [--k 4]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))
import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.comm import Comm  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.dist import balanced_row_starts  # noqa: E402
from srgnn.spmm import propagate  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--gpus", type=int, default=torch.cuda.device_count())
ap.add_argument("--k", type=int, default=4)
a = ap.parse_args()
P = a.gpus
ip, ix, vals, n, d, _ = graphs.build(a.config, torch.device("cuda", 0))
X = synth.uniform_features_t(n, d, device=torch.device("cuda", 0))
starts = [int(s) for s in balanced_row_starts(ip, P)]
blocks, xs = [], []
for r in range(P):
    dev = torch.device("cuda", r)
    b0, b1 = int(ip[starts[r]]), int(ip[starts[r + 1]])
    bip = (ip[starts[r]:starts[r + 1] + 1] - b0).to(dev)
    blocks.append(DeviceCSR.from_tensors(bip, ix[b0:b1].to(dev), vals[b0:b1].to(dev), n_cols=n, device=dev))
    xs.append(X[starts[r]:starts[r + 1]].to(dev).contiguous())
comm = Comm.init_all(list(range(P)))
comm.propagate(blocks, starts, xs, 1)          # warm-up
t0 = time.perf_counter()
out = comm.propagate(blocks, starts, xs, a.k)
dt = time.perf_counter() - t0
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda:0")
want = propagate(A, X, a.k)
ok = all(torch.equal(out[r][k].to("cuda:0"), want[k][starts[r]:starts[r + 1]])
         for r in range(P) for k in range(a.k + 1))
comm.destroy()
print(json.dumps({"config": a.config, "gpus": P, "K": a.k, "bitwise_equal_one_gpu": ok,
                  "ms_per_hop": dt / a.k * 1e3, "row_starts": starts}))
sys.exit(0 if ok else 1)
