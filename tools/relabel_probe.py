#!/usr/bin/env python3
"""Probe: does the X row layout matter?  One hop of the products-shaped graph as generated (random
relabelling) against the same graph relabelled so that rows are numbered by decreasing degree
(the hot X rows contiguous at the front).  Each row keeps its entries in their original order, so
the hop is the same fma chains (checked bitwise after undoing the permutation).

    python tools/relabel_probe.py [--config products] [--reps 10]   -> JSON
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402


def relabel(ip, ix, vals, perm_new2old):
    """Rows and columns renumbered: new row i = old row perm[i]; entries keep their order."""
    n = perm_new2old.numel()
    old2new = torch.empty_like(perm_new2old)
    old2new[perm_new2old] = torch.arange(n, device=ip.device)
    deg = ip[1:] - ip[:-1]
    ndeg = deg[perm_new2old]
    nip = torch.zeros(n + 1, dtype=torch.int64, device=ip.device)
    torch.cumsum(ndeg, 0, out=nip[1:])
    starts = torch.repeat_interleave(ip[:-1][perm_new2old], ndeg)
    first = torch.repeat_interleave(nip[:-1], ndeg)
    pos = starts + (torch.arange(int(nip[-1]), device=ip.device) - first)
    nix = old2new[ix[pos].long()].to(torch.int32)
    return nip, nix, vals[pos], old2new


def time_hop(A, X, Y, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    spmm(A, X, out=Y)
    for r in range(reps):
        ev[2 * r].record()
        spmm(A, X, out=Y)
        ev[2 * r + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps))
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev)
    x = synth.uniform_features_t(n, d, device=dev)
    out = {"config": a.config, "n": n, "nnz": int(ix.numel()), "d": d}
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
    Y = torch.empty_like(x)
    out["ms_generated"] = time_hop(A, x, Y, a.reps)
    deg = ip[1:] - ip[:-1]
    perm = torch.sort(deg, descending=True, stable=True).indices
    nip, nix, nv, old2new = relabel(ip, ix, vals, perm)
    B = DeviceCSR.from_tensors(nip, nix, nv, n_cols=n, device=dev)
    xp = x[perm].contiguous()
    Yp = torch.empty_like(xp)
    out["ms_degree_relabelled"] = time_hop(B, xp, Yp, a.reps)
    out["bitwise_equal"] = bool(torch.equal(Yp[old2new], Y))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
