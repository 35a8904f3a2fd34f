#!/usr/bin/env python3
"""End-to-end time of the reference API on the GPU path ("report the end-to-end
API time separately"): SymLaplacianGraphOp(K).propagate(adj, X) from a host scipy adjacency and a
host numpy feature matrix to the list of K+1 host tensors, and the fused SGC-style
propagate_aggregate(adj, X, LastMessageOp()).  Stages are timed separately in extra runs:
construct_adj on the device vs the reference's host scipy construct_adj (same code as
operators/utils.py:81-93), and the hop loop alone.

    python tools/e2e_api.py [--config arxiv] [--reps 3]     -> one JSON line
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from srgnn import synth  # noqa: E402


def timed(fn, reps):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        del out
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="arxiv", choices=sorted(synth.CONFIGS))
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    cfg = synth.CONFIGS[a.config]
    n, m, d, K = cfg["n"], cfg["n_edges"], cfg["d"], cfg["k"]
    u, v = synth.rmat_undirected_t(n, m, device="cuda")
    u, v = u.cpu().numpy(), v.cpu().numpy()
    adj = sp.csr_matrix((np.ones(2 * m), (np.r_[u, v], np.r_[v, u])), shape=(n, n))
    X = synth.uniform_features_t(n, d, device="cuda").cpu().numpy()
    from operators.graph_operator.symmetrical_simgraph_laplacian_operator import SymLaplacianGraphOp
    from operators.message_operator.last_message_op import LastMessageOp
    from operators.utils import adj_to_symmetric_norm
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import propagate
    op = SymLaplacianGraphOp(K, r=0.5)
    dev = torch.device("cuda", 0)
    op.propagate(adj, X)                       # warm-up (library load, allocator)
    res = {"config": a.config, "n": n, "nnz_adj": int(adj.nnz), "d": d, "K": K, "reps": a.reps}
    res["propagate_e2e_s"] = timed(lambda: op.propagate(adj, X), a.reps)
    res["propagate_aggregate_last_e2e_s"] = timed(lambda: op.propagate_aggregate(adj, X, LastMessageOp()), a.reps)
    res["construct_adj_device_s"] = timed(lambda: op.construct_adj_device(adj, dev), a.reps)
    t0 = time.perf_counter()
    host = adj_to_symmetric_norm(adj.tocoo(), 0.5).tocsr()
    res["construct_adj_host_scipy_s"] = time.perf_counter() - t0
    ip, ix, v64 = op.construct_adj_device(adj, dev)
    assert np.array_equal(v64.cpu().numpy(), host.data) and np.array_equal(ix.cpu().numpy(), host.indices)
    A = DeviceCSR.from_tensors(ip, ix, v64.to(torch.float32), n_cols=n, device=dev)
    Xd = torch.from_numpy(X).to(dev)
    res["hops_device_s"] = timed(lambda: propagate(A, Xd, K), a.reps)
    res["h2d_feature_s"] = timed(lambda: torch.from_numpy(X).to(dev), a.reps)
    res["note"] = ("propagate_e2e = construct_adj (device) + H2D of X + K hops + D2H of K panels into "
                   "pinned host tensors; construct_adj_host_scipy is the reference's own host step; "
                   "results checked equal (fp64 A-hat)")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
