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


ip = t("h2d_indptr", lambda: torch.as_tensor(adj.indptr).to(dev).to(torch.int64))
ix = t("h2d_indices", lambda: torch.as_tensor(adj.indices).to(dev).to(torch.int64))
vv = t("h2d_data", lambda: torch.as_tensor(adj.data).to(dev).to(torch.float64))
rows = t("rows", lambda: torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1]))
diag = torch.arange(n, device=dev)
r2, c2, v2 = t("canonical_sum(A+I)", lambda: C.canonical_sum(torch.cat([rows, diag]), torch.cat([ix, diag]),
                                                              torch.cat([vv, torch.ones(n, dtype=torch.float64, device=dev)]),
                                                              n, C.segment_sum_device))
deg = t("degree_segsum", lambda: C.segment_sum_device(C._indptr(r2, n), v2))
left, right = t("degree_powers(host)", lambda: C.degree_powers(deg.cpu().numpy(), 0.5))
lt, rt = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
st = t("scale", lambda: (v2 * lt[c2]) * rt[r2])
key = t("transpose_key", lambda: c2 * n + r2)
srt = t("transpose_sort", lambda: torch.sort(key))
T["total_sym_norm"] = t("total", lambda: C.sym_norm(adj.indptr, adj.indices, adj.data, n, 0.5, device=dev)) and T["total"]
print(json.dumps({k: round(x * 1e3, 2) for k, x in T.items()}))
