#!/usr/bin/env python3
"""Probe: where the fp64 Chebyshev STEP's time goes (srg_cheby_step_f64, products-shaped, d = 128).

Times, with HIP events around `reps` launches each:
  full      the step over every row (bench.py --op wavelet --dtype f64's launch),
  top<k>    the k longest rows alone (a launch over order[:k]: their chains' latency, nothing beside),
  rest<k>   every other row (order[k:]),
  cb<B>     the step over B column-block CSRs of F, one launch each (INIT mode, 1 scale: the same
            row-wave gather per block with only X's column range touched; the epilogue's panel passes
            repeat per block, so this over-counts them) -- what column locality would buy.
  hub<h>    srg_cheby_step_hub_f64 with the h longest rows as hub workgroups beside the row waves,
  --plan    the blocked steps (srg_plan_cheby_step_f64) over B column blocks and hub thresholds, each
            checked bitwise against the one-launch step.
Results are not combined with the oracle (timing only).
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import _lib, graphs, synth  # noqa: E402
from srgnn import wavelet as W  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "products"
reps = 3
dev = torch.device("cuda", 0)
def _arg(name, default=None):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


d_arg = _arg("--d")
ip, ix, lv, n, d, lmax = graphs.build_laplacian(cfg, dev, d=int(d_arg) if d_arg else None)
filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float64)
S = synth.uniform_features_t(n, d, device=dev).to(torch.float64)
R = torch.zeros((2, n, d), dtype=torch.float64, device=dev)
To, Tn = torch.zeros_like(S), torch.empty_like(S)
coef = (ctypes.c_double * 2)(*[float(c) for c in filt.coeffs[:, 2]])
coef1 = (ctypes.c_double * 1)(1.0)
deg = (filt.indptr[1:] - filt.indptr[:-1])
order = filt.order


def step(indptr, indices, vals, order_t, rows, mode=_lib.SRG_CHEBY_STEP, ns=2):
    c = coef if ns == 2 else coef1
    _lib.call(dev, "srg_cheby_step_f64", indptr.data_ptr(), indices.data_ptr(), vals.data_ptr(), rows,
              order_t.data_ptr(), S.data_ptr(), To.data_ptr(), Tn.data_ptr(), d, d, mode, filt.a1, filt.a2,
              c if mode == _lib.SRG_CHEBY_INIT else None, c, ns, R.data_ptr(), n * d, _lib.stream(dev))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = {"config": cfg, "n": n, "nnz": int(ix.numel()), "d": d,
       "top_degrees": [int(x) for x in deg[order[:4].long()].tolist()]}
if "--no-ref" not in sys.argv:
    out["full_ms"] = timed(lambda: step(filt.indptr, filt.indices, filt.fvals, order, n))
out["n_hub_auto"] = filt.n_hub


def step_hub(h):
    _lib.call(dev, "srg_cheby_step_hub_f64", filt.indptr.data_ptr(), filt.indices.data_ptr(), filt.fvals.data_ptr(), n,
              order.data_ptr(), h, S.data_ptr(), To.data_ptr(), Tn.data_ptr(), d, d, _lib.SRG_CHEBY_STEP, filt.a1,
              filt.a2, None, coef, 2, R.data_ptr(), n * d, _lib.stream(dev))


if "--plan" in sys.argv:
    # the blocked steps (srg_plan_cheby_step_f64 through HeatWaveletFilter.order_step), bitwise against the
    # one-launch step with the automatic hub rows
    import time
    ref = "--no-ref" not in sys.argv
    if ref:
        R.zero_()
        step_hub(filt.n_hub)
        torch.cuda.synchronize()
        ref_T, ref_R = Tn.clone(), R.clone()
    cf = filt.coeffs[:, 2]
    configs = ((0, None), (16, None), (16, 32768), (16, 16384), (24, 16384), (16, 12288), (32, 16384))
    if _arg("--configs"):    # B:hub[:whole],... (hub empty: the fp64 rule; whole: block 0's whole-row limit)
        configs = tuple(tuple(int(x) if x else None for x in (c.split(":") + [""])[:3])
                        for c in _arg("--configs").split(","))
    for cfg_ in configs:
        B, ht, wm = (tuple(cfg_) + (None,))[:3]
        filt.col_blocks64, filt.hub64_threshold, filt.whole64_max = (B or None), ht, wm
        t0 = time.perf_counter()
        P = filt._plan64(d)
        torch.cuda.synchronize()
        tb = time.perf_counter() - t0
        R.zero_()
        filt.order_step(filt.fvals, S, To, Tn, _lib.SRG_CHEBY_STEP, None, cf, R)
        torch.cuda.synchronize()
        same = bool(torch.equal(Tn, ref_T) and torch.equal(R, ref_R)) if ref else None
        ms = timed(lambda: filt.order_step(filt.fvals, S, To, Tn, _lib.SRG_CHEBY_STEP, None, cf, R))
        print(json.dumps({"col_blocks": P.col_blocks if P else 1,
                          "hub64_threshold": ht, "whole_max": wm,
                          "hub_rows_whole": P.hub_rows_whole if P else filt.n_hub, "launches": P.n_launch if P else 1,
                          "plan_mb": (P.device_bytes >> 20) if P else 0, "build_s": round(tb, 3), "step_ms": ms,
                          "bitwise_vs_one_launch": same}), flush=True)
        filt.drop_layouts()
    sys.exit(0)
for h in (1, 4, 16, 64, 256, 1024):
    out[f"hub{h}_ms"] = timed(lambda: step_hub(h))
print(json.dumps(out), flush=True)
if "--hub-only" in sys.argv:
    sys.exit(0)
for k in (1, 16, 4096):
    out[f"top{k}_ms"] = timed(lambda: step(filt.indptr, filt.indices, filt.fvals, order[:k], k))
    rest = order[k:].contiguous()
    out[f"rest{k}_ms"] = timed(lambda: step(filt.indptr, filt.indices, filt.fvals, rest, n - k))
print(json.dumps(out), flush=True)

# column-block CSRs of F (every row, its entries in [lo, hi)); timing only
rows = torch.repeat_interleave(torch.arange(n, device=dev), deg)
# the epilogue alone: an operator with no entries (every row's gather is empty)
zip_ = torch.zeros(n + 1, dtype=torch.int64, device=dev)
out["epilogue_init1_ms"] = timed(lambda: step(zip_, filt.indices, filt.fvals, order, n, _lib.SRG_CHEBY_INIT, 1))
for B in (2, 4, 8, 16):
    t = 0.0
    t1 = timed(lambda: step(filt.indptr, filt.indices, filt.fvals, order, n, _lib.SRG_CHEBY_INIT, 1))
    for b in range(B):
        lo, hi = b * n // B, (b + 1) * n // B
        m = (filt.indices >= lo) & (filt.indices < hi)
        bip = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        bip[1:] = torch.cumsum(torch.bincount(rows[m], minlength=n), 0)
        bix, bv = filt.indices[m].contiguous(), filt.fvals[m].contiguous()
        t += timed(lambda: step(bip, bix, bv, order, n, _lib.SRG_CHEBY_INIT, 1))
        del m, bip, bix, bv
    out[f"cb{B}_ms"] = t
    out["full_init1_ms"] = t1
    print(json.dumps({"B": B, "sum_ms": t, "gather_est_ms": t - B * out["epilogue_init1_ms"],
                      "full_init_1scale_ms": t1, "full_gather_est_ms": t1 - out["epilogue_init1_ms"]}), flush=True)
print(json.dumps(out), flush=True)
