#!/usr/bin/env python3
"""Stage times of construct_adj on the device (srgnn.construct.sym_norm) for a products-shaped host CSR."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from srgnn import construct as C, synth  # noqa: E402

cfg = synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "products"]
n, m = cfg["n"], cfg["n_edges"]
u, v = synth.rmat_undirected_t(n, m, device="cuda")
u, v = u.cpu().numpy(), v.cpu().numpy()
adj = sp.csr_matrix((np.ones(2 * m), (np.r_[u, v], np.r_[v, u])), shape=(n, n))
dev = torch.device("cuda", 0)
C.sym_norm(adj.indptr, adj.indices, adj.data, n, 0.5, device=dev)   # warm-up
T = {}


def t(name, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    T[name] = time.perf_counter() - t0
    return r


ip = t("h2d_indptr", lambda: torch.as_tensor(adj.indptr.astype(np.int64)).to(dev))
ix = t("h2d_indices", lambda: torch.as_tensor(adj.indices).to(dev, torch.int64))
vv = t("h2d_data", lambda: torch.as_tensor(adj.data).to(dev, torch.float64))
rows = t("rows", lambda: torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1]))
diag = torch.arange(n, device=dev)
key = t("key", lambda: torch.cat([rows, diag]) * n + torch.cat([ix, diag]))
srt = t("sort1", lambda: torch.sort(key, stable=True))
T["total_sym_norm"] = t("total", lambda: C.sym_norm(adj.indptr, adj.indices, adj.data, n, 0.5, device=dev)) and T["total"]
print(json.dumps({k: round(x * 1e3, 2) for k, x in T.items()}))
