#!/usr/bin/env python3
"""Probe: the fp64 filter bank's per-rank compute over the halo partition (HaloWaveletFilter dtype=float64),
every rank's share built and timed on ONE GPU in turn -- what a P-GPU run's order would take before its
exchange, against the one-GPU blocked step.  One STEP order (F T_k - T_{k-1}, both scales' R updated) per
rank, HIP events over `reps` orders on random panels.  Timing only (the partition's parity is tested in
tests/test_wavelet_gpu.py::test_halo_wavelet_f64_virtual_ranks_bitwise).

  tools/probes/halo_cheby64_ranks.py [config=products] [P=8] [d=config's or --d] [reps=5]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import _lib, graphs  # noqa: E402
from srgnn import wavelet as W  # noqa: E402
from srgnn.dist import HaloWaveletFilter  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--d", type=int, default=None)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--chunks", type=int, default=0,
                help="time the GPU ranks' overlapped order: one launch per exchange group of a C-chunk halo plan "
                     "(no exchange); 0: one launch per order")
ap.add_argument("--blocks", type=int, default=1,
                help="each rank's fp64 column blocks (1: one launch per order, 0: the planner's rule)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
ip, ix, lv, n, d, lmax = graphs.build_laplacian(a.config, dev, d=a.d)
taus = [-0.5, 0.5]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = {"config": a.config, "n": n, "nnz": int(ix.numel()), "d": d, "world": a.world, "chunks": a.chunks or None,
       "ranks": []}
# the one-GPU blocked step for scale
one = W.HeatWaveletFilter.from_device(ip, ix, lv, n, taus, order=3, lmax=lmax, dtype=torch.float64)
S = torch.rand((n, d), dtype=torch.float64, device=dev)
To, Tn = torch.rand_like(S), torch.empty_like(S)
R = torch.zeros((2, n, d), dtype=torch.float64, device=dev)
out["one_gpu_ms"] = timed(lambda: one.order_step(one.fvals, S, To, Tn, _lib.SRG_CHEBY_STEP, None, one.coeffs[:, 2], R),
                          a.reps)
P = one._plan64(d)
out["one_gpu_col_blocks"] = P.col_blocks if P is not None else 1
one.drop_layouts()
del one, S, To, Tn, R
torch.cuda.empty_cache()
for q in range(a.world):
    f = HaloWaveletFilter(ip, ix, lv, n, taus, order=3, lmax=lmax, device=dev, rank=q, world=a.world,
                          dtype=torch.float64, **({"chunks": a.chunks} if a.chunks else {}))
    f.col_blocks64 = a.blocks or None
    m = f.rows + f.opL.halo
    Tc = torch.rand((m, d), dtype=torch.float64, device=dev)
    To, Tn = torch.rand_like(Tc), torch.empty_like(Tc)
    Pq = f._plan64(d)
    R = torch.zeros((2, m if Pq is not None else f.rows, d), dtype=torch.float64, device=dev)
    extra = {}
    if a.chunks:
        # the halo plan's exchange groups as launches (hub group, then each chunk's other rows), each timed
        def order():   # as the GPU ranks run it: hub group unjoined, the chunks beside it, the join
            f._order64_overlapped("F", Tc, To, Tn, _lib.SRG_CHEBY_STEP, None, f.coeffs[:, 2], R, exchange=False)
        extra["group_ms"] = [timed(lambda sc=sc: f._order64("F", Tc, To, Tn, _lib.SRG_CHEBY_STEP, None, f.coeffs[:, 2], R,
                                                             sched=sc), a.reps) for _, sc in f._sched64_groups]
        extra["group_rows"] = [int(o.numel()) for _, (o, _) in f._sched64_groups]
        extra["group_hubs"] = [h for _, (_, h) in f._sched64_groups]
        extra["one_launch_ms"] = timed(lambda: f._order64("F", Tc, To, Tn, _lib.SRG_CHEBY_STEP, None, f.coeffs[:, 2], R),
                                       a.reps)
    else:
        def order():
            f._order64("F", Tc, To, Tn, _lib.SRG_CHEBY_STEP, None, f.coeffs[:, 2], R)
    ms = timed(order, a.reps)
    out["ranks"].append({"rank": q, "rows": f.rows, "halo": f.opL.halo, "nnz": f.opL.nnz_local,
                         "hub_rows": f._n_hub64, "col_blocks": Pq.col_blocks if Pq is not None else 1,
                         "ms_per_order": ms, **extra})
    print(json.dumps(out["ranks"][-1]), flush=True)
    f.drop_layouts()
    del f, Tc, To, Tn, R, Pq
    torch.cuda.empty_cache()
mx = max(r["ms_per_order"] for r in out["ranks"])
out["max_rank_ms"] = mx
out["compute_speedup_vs_one_gpu"] = out["one_gpu_ms"] / mx
print(json.dumps(out), flush=True)
