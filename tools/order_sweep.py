#!/usr/bin/env python3
"""Locality experiment: the same Â, X and kernel under different row schedules (which rows run
concurrently).  Results must be bitwise identical; only time changes.  Interleaved rounds."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from srgnn import graphs, roofline, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--thr", type=int, default=32)
ap.add_argument("--rcm", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build(a.config, dev)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
deg = ip[1:] - ip[:-1]
heavy = deg > a.thr
nh = int(heavy.sum())


def make(order_key_heavy, order_key_light):
    """order = heavy rows sorted by key_h, then light rows sorted by key_l (stable)."""
    hv = torch.nonzero(heavy).flatten()
    lv = torch.nonzero(~heavy).flatten()
    hv = hv[torch.sort(order_key_heavy[hv], stable=True).indices]
    lv = lv[torch.sort(order_key_light[lv], stable=True).indices]
    order = torch.cat([hv, lv]).to(torch.int32).contiguous()
    return DeviceCSR(ip, ix, vals, n, n, order, nh)


rid = torch.arange(n, device=dev)
perm = synth.relabel_permutation_t(n, synth.RMAT_SEED, dev)   # new_id[old]
old_of_new = torch.empty_like(perm)
old_of_new[perm] = rid
V = {
    "deg_desc": make(-deg, -deg),
    "deg_desc_heavy+natural_light": make(-deg, rid),
    "natural": make(rid, rid),
    "rmat_id": make(old_of_new, old_of_new),
    "deg_desc_heavy+rmat_id_light": make(-deg, old_of_new),
}
if a.rcm:
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    t = time.time()
    m = sp.csr_matrix((np.ones(ix.numel(), np.int8), ix.cpu().numpy(), ip.cpu().numpy()), shape=(n, n))
    rc = torch.from_numpy(reverse_cuthill_mckee(m, symmetric_mode=True).astype(np.int64)).to(dev)
    pos = torch.empty_like(rc)
    pos[rc] = rid
    print("rcm", time.time() - t, "s", file=sys.stderr)
    V["rcm"] = make(pos, pos)
    V["deg_desc_heavy+rcm_light"] = make(-deg, pos)
times = {k: [] for k in V}
ref = None
for r in range(a.rounds):
    for k, A in V.items():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        spmm(A, X, out=Y)
        e.record()
        torch.cuda.synchronize()
        times[k].append(s.elapsed_time(e))
        if r == 0:
            if ref is None:
                ref = Y.clone()
            else:
                assert torch.equal(ref, Y), k
b = roofline.bytes_no_reuse(n, ix.numel(), d)
print(json.dumps({k: {"median_ms": float(np.median(v[1:])), "min_ms": float(min(v)),
                      "frac": b / (float(np.median(v[1:])) * 1e-3) / 8e12} for k, v in times.items()}, indent=1))
