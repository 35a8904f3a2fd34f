#!/usr/bin/env python3
"""Probe: the LDS-DMA light-row stream (srg_stream.hip) against k_spmm's packed light rows, launch by
launch of the bench's hop layout, bitwise and timed.  For every launch of the hop plan (compact
column blocks in launch order) it times
  * old_light: k_spmm over the launch's light rows only (the plan loop, slot spans),
  * stream:    k_stream over the same rows,
  * old_full:  the whole launch (hub + slice waves + light rows), and heavy: the hub + slice rows alone,
checks that heavy + stream leaves the output panel bitwise equal to the whole launch after every
launch, and times the whole hop both ways.  Prints one JSON line.

    python tools/stream_probe.py [--config products] [--reps 20] [--wave-entries 512]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import _lib, graphs, spmm, stream, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--wave-entries", type=int, default=stream.WAVE_ENTRIES)
ap.add_argument("--d", type=int, default=None)
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, vals, n, d, _ = graphs.build(a.config, dev)
d = a.d or d
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
X = synth.uniform_features_t(n, d, device=dev).view(n, d)
B = spmm.prepare(A, d, hops=100)
plan, join = spmm._hop_plan(A, d, B)
HUBF = _lib.SRG_SPMM_HUB_NOJOIN | _lib.SRG_SPMM_HUB_CONTINUE


def timed(fn, reps=a.reps):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def run_plan(p, Xin, Y, join_hub=1):
    arr = (ctypes.c_void_p * 2)(Xin.data_ptr(), Y.data_ptr())
    _lib.call(dev, "srg_propagate_plan_f32", spmm._plan_array(p, d), len(p), join_hub, arr, Xin.stride(0), d, 1,
              _lib.stream(dev))


def view(Ab, lo, hi, n_hub, n_heavy):
    """Ab's schedule slots [lo, hi) as a span operator over the same arrays."""
    return DeviceCSR(Ab.indptr, Ab.indices, Ab.values, hi - lo, Ab.n_cols, Ab.order[lo:hi].contiguous(), n_heavy,
                     n_hub, None, row_end=Ab.row_end, row_space=Ab.out_rows)


Yold = torch.randn_like(X)
Ynew = Yold.clone()
launches, t_new_parts = [], []
for Ab, f, kind in plan:
    f = f & ~HUBF
    acc = bool(f & _lib.SRG_SPMM_ACCUMULATE)
    nh, nv = Ab.n_hub, Ab.heavy(d)
    lo = nh + nv
    light = view(Ab, lo, Ab.n_rows, 0, 0)
    heavy = view(Ab, 0, lo, nh, nv) if lo else None
    L = stream.build(Ab.order[lo:], Ab.indptr, Ab.row_end, Ab.indices, Ab.values, acc, a.wave_entries)
    run_plan([(Ab, f, "plain")], X, Yold)
    if heavy is not None:
        run_plan([(heavy, f, "plain")], X, Ynew)
    stream.run(L, X, Ynew)
    torch.cuda.synchronize()
    same = bool(torch.equal(Yold, Ynew))
    scratch = Yold.clone()
    rec = {"rows": Ab.n_rows, "hub": nh, "heavy": nv, "light": Ab.n_rows - lo, "light_entries": L.entries - (
        (Ab.n_rows - lo) if acc else 0), "stream_entries": L.entries, "waves": L.waves, "acc": acc,
        "bitwise": same,
        "ms_old_full": timed(lambda: run_plan([(Ab, f, "plain")], X, scratch)),
        "ms_old_light": timed(lambda: run_plan([(light, f, "plain")], X, scratch)),
        "ms_heavy": timed(lambda: run_plan([(heavy, f, "plain")], X, scratch)) if heavy is not None else 0.0,
        "ms_stream": timed(lambda: stream.run(L, X, scratch))}
    launches.append(rec)
    t_new_parts.append((heavy, f, L))
    del scratch


def new_hop(Y):
    for heavy, f, L in t_new_parts:
        if heavy is not None:
            run_plan([(heavy, f, "plain")], X, Y)
        stream.run(L, X, Y)


Yh = torch.empty_like(X)
ms_hop_old = timed(lambda: spmm.hop(A, X, Yh, col_blocks=B))
ms_hop_new = timed(lambda: new_hop(Yh))
ref = spmm.hop(A, X, torch.empty_like(X), col_blocks=B)
Yn = torch.empty_like(X)
new_hop(Yn)
torch.cuda.synchronize()
print(json.dumps({"config": a.config, "d": d, "col_blocks": B, "wave_entries": a.wave_entries,
                  "hop_bitwise": bool(torch.equal(ref, Yn)), "ms_hop_old": ms_hop_old, "ms_hop_new_serial": ms_hop_new,
                  "all_launches_bitwise": all(r["bitwise"] for r in launches), "launches": launches}))
