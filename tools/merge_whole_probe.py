#!/usr/bin/env python3
"""Probe: the whole rows of a column-blocked hop (rows of <= BLOCK_WHOLE_MAX entries, computed whole in
a launch of their own) spread over the B block launches instead -- part b (every B-th row of their
schedule) runs in block b's launch with per-row accumulation (srg_spmm_span_rowacc_f32: a span that
starts at its row's first entry starts from +0.0f), so the latency-bound short rows run beside the
bandwidth-bound spans and the hop has one launch less.  The hub rows' spans run as before, chained
on the library's side stream.  Bitwise the default hop (checked).  Span blocks (no compact copies).

    python tools/merge_whole_probe.py [--config products] [--hops 20]     -> one JSON line
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import _lib, graphs, synth  # noqa: E402
from srgnn import spmm as S  # noqa: E402
from srgnn.csr import DeviceCSR, auto_heavy_threshold, BLOCK_HEAVY_PER  # noqa: E402


def merged_plan(A: DeviceCSR, B: int, d: int):
    blocks = S.column_blocks_for(A, B, hops=1)
    cut0, whole = blocks[0].split_whole()
    ip = A.indptr
    wrows = whole.order.to(torch.int64)
    launches = []
    for b in range(B):
        blk = cut0 if b == 0 else blocks[b]
        own = blk.order.to(torch.int64)
        hub = own[: blk.n_hub]
        rest = own[blk.n_hub:]
        part = wrows[b::B]
        beg = blk.indptr.clone()
        end = blk.row_end.clone()
        beg[part] = ip[part]
        end[part] = ip[part + 1]
        rows = torch.cat([rest, part])
        lens = end[rows] - beg[rows]
        srt = torch.sort(lens, descending=True, stable=True)
        order = rows[srt.indices].to(torch.int32).contiguous()
        heavy_t = max(96, int(lens.sum()) // BLOCK_HEAVY_PER)
        n_heavy = int((srt.values > heavy_t).sum())
        hubv = None
        if hub.numel():
            hubv = DeviceCSR(blk.indptr, A.indices, A.values, int(hub.numel()), A.n_cols, hub.to(torch.int32).contiguous(),
                             0, int(hub.numel()), None, row_end=blk.row_end, row_space=A.n_rows)
        launches.append((hubv, beg, end, order, n_heavy))
    return launches


def merged_hop(A, launches, X, Y):
    d = X.shape[1]
    st = _lib.stream(X.device)
    forked = False
    for b, (hubv, beg, end, order, n_heavy) in enumerate(launches):
        if hubv is not None:
            S.spmm(hubv, X, out=Y, accumulate=b > 0, hub_nojoin=True, hub_continue=forked)
            forked = True
        _lib.call(X.device, "srg_spmm_span_rowacc_f32", beg.data_ptr(), end.data_ptr(), A.indptr.data_ptr(),
                  A.indices.data_ptr(), A.values.data_ptr(), int(order.numel()), order.data_ptr(), n_heavy,
                  X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), d,
                  _lib.SRG_SPMM_PACKED_U2 if d >= 128 else 0, st)
    if forked:
        _lib.call(X.device, "srg_hub_join", st)


def timed(fn, hops):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(hops):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / hops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--hops", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=6)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev)
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
    X = synth.uniform_features_t(n, d, device=dev)
    B = a.blocks
    Y0 = torch.empty_like(X)
    Y1 = torch.empty_like(X)
    launches = merged_plan(A, B, d)
    out = {"config": a.config, "blocks": B}
    for rep in range(3):
        out.setdefault("default_ms", []).append(timed(lambda: S.hop(A, X, Y0, col_blocks=B), a.hops))
        out.setdefault("merged_ms", []).append(timed(lambda: merged_hop(A, launches, X, Y1), a.hops))
    out["bitwise_equal"] = bool(torch.equal(Y0, Y1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
