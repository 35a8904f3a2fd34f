#!/usr/bin/env python3
"""Probe: exact column-blocked hop ("locality").

Â's column ids are sorted within each row (utils.py:81-93 builds Â as a canonical transpose), so a
row's fma chain can be cut at column-block boundaries and continued: pass 0 runs the entries with
column ids in block 0 from +0.0f, pass b > 0 runs block b's entries with ACCUMULATE, i.e. starting
from the fp32 value pass b-1 stored.  The chain is the same sequence of fmas, so Y is bitwise the
one-pass hop (checked here).  Each pass gathers only from an X slice of n/B rows, which fits the
Infinity Cache once B is large enough; the price is one extra read + write of Y per extra pass.

    python tools/colblock_probe.py [--config products] [--blocks 1,2,3,4,5,6,8] [--reps 7]  -> JSON

A block count may repeat (--blocks 1,2,1,2): ms_per_hop keeps one median per occurrence.
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


def column_blocks(ip, ix, vals, n, B):
    """B CSRs over the same rows: block b holds each row's entries with ids in [b n/B, (b+1) n/B),
    in their stored order."""
    deg = ip[1:] - ip[:-1]
    row = torch.repeat_interleave(torch.arange(n, device=ip.device), deg)
    blk = (ix.long() * B) // n
    out = []
    for b in range(B):
        m = blk == b
        cnt = torch.bincount(row[m], minlength=n)
        bip = torch.zeros(n + 1, dtype=torch.int64, device=ip.device)
        torch.cumsum(cnt, 0, out=bip[1:])
        out.append(DeviceCSR.from_tensors(bip, ix[m], vals[m], n_cols=n, device=ip.device))
        del m, cnt
    del row, blk
    return out


def run_blocks(As, X, Y):
    spmm(As[0], X, out=Y)
    for A in As[1:]:
        spmm(A, X, out=Y, accumulate=True)


def time_blocks(As, X, Y, reps):
    run_blocks(As, X, Y)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for r in range(reps):
        ev[2 * r].record()
        run_blocks(As, X, Y)
        ev[2 * r + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps))
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--blocks", default="1,2,3,4,5,6,8")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev)
    x = synth.uniform_features_t(n, d, device=dev)
    res = {"config": a.config, "n": n, "nnz": int(ix.numel()), "d": d, "ms_per_hop": {}, "bitwise_equal": {}}
    Y1 = torch.empty_like(x)
    Y = torch.empty_like(x)
    for B in [int(s) for s in a.blocks.split(",")]:
        As = column_blocks(ip, ix, vals, n, B)
        res["ms_per_hop"].setdefault(B, []).append(time_blocks(As, x, Y if B > 1 else Y1, a.reps))
        if B > 1:
            res["bitwise_equal"][B] = bool(torch.equal(Y, Y1))
        del As
        torch.cuda.empty_cache()
        print(json.dumps({"B": B, "ms": res["ms_per_hop"][B][-1], "eq": res["bitwise_equal"].get(B)}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
