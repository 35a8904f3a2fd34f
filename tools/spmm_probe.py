#!/usr/bin/env python3
"""Workload for rocprofv3 counter runs: R single-hop SpMM launches on a benchmark graph.

  --identity   calibration: Â = I on an [N, d] panel larger than the Infinity Cache, so every
               launch reads exactly N*4d bytes of X (+ index arrays) and writes N*4d bytes of Y
               with the SAME kernel and access widths as the real hop -> FETCH_SIZE / WRITE_SIZE
               scale factors for this access pattern (MI355X_MICROARCH.md: FETCH_SIZE under-counts
               wide reads on gfx950; calibrate on a known byte count).
  --permutation  calibration on gathers: Â = a random permutation matrix with the config's N (one
               nonzero per row, a random column, every column once), so every launch gathers each
               X row exactly once as a random whole-row read -- the hop kernel's access pattern with
               no reuse and known bytes (N*4d read, N*4d written, plus ids, values, pointers).
Prints one JSON line with the launch geometry and algorithmic bytes.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, roofline, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import hop, launches_per_hop, prepare  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="products")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--identity", action="store_true")
ap.add_argument("--permutation", action="store_true")
ap.add_argument("--heavy-threshold", type=int, default=None)
ap.add_argument("--col-blocks", type=int, default=None, help="column blocks per hop (default: auto_col_blocks)")
ap.add_argument("--d", type=int, default=None, help="panel width (default: the config's)")
ap.add_argument("--hops", type=int, default=1 << 30,
                help="hops the operator serves (bench.py: K x (steps + warmup)); picks spans or compact blocks")
ap.add_argument("--op", default="khop", choices=["khop", "wavelet", "wavelet64"],
                help="wavelet: the Chebyshev STEP operator F = (2/a1)(L - a2 I) of the config's Laplacian "
                     "on a --col-block wide panel (bench.py --op wavelet's SpMM launches)")
ap.add_argument("--col-block", type=int, default=None,
                help="wavelet: column block width (default: bench.py's rule, the widest whose work panels fit)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
if a.op == "wavelet64":
    # bench.py --op wavelet --dtype f64's roofline step: one fp64 Chebyshev STEP order (HeatWaveletFilter.
    # order_step: srg_plan_cheby_step_f64 over the column-blocked plan, or one srg_cheby_step_hub_f64 launch)
    # over the block width bench.py picks (the widest whose five fp64 panels fit), `reps` times
    from srgnn import _lib
    from srgnn import wavelet as W
    ip, ix, lv, n, d, lmax = graphs.build_laplacian(a.config, dev, d=a.d)
    filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float64,
                                           heavy_threshold=a.heavy_threshold)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    cb = a.col_block or d
    while not a.col_block and cb > 1 and 5 * n * cb * 8 > free - 4 * 2 ** 30:
        cb //= 2
    S = synth.uniform_features_t(n, cb, device=dev).to(torch.float64)
    R = torch.zeros((2, n, cb), dtype=torch.float64, device=dev)
    To, Tn = torch.zeros_like(S), torch.empty_like(S)
    P = filt._plan64(cb)          # the blocked layout bench.py's steps run (None: one launch per order)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        filt.order_step(filt.fvals, S, To, Tn, _lib.SRG_CHEBY_STEP, None, filt.coeffs[:, 2], R)
    torch.cuda.synchronize()
    nnz = int(ix.numel())
    print(json.dumps({"config": a.config, "op": "wavelet64", "n": n, "nnz": nnz, "d": cb, "reps": a.reps,
                      "launches_per_hop": P.n_launch if P else 1, "column_blocks": P.col_blocks if P else 1,
                      "n_heavy": filt.n_heavy, "n_hub": P.hub_rows_whole if P else filt.n_hub,
                      "algorithmic_bytes": roofline.cheby_step_bytes_no_reuse_f64(n, nnz, cb, 2),
                      "compulsory_bytes": roofline.cheby_step_bytes_compulsory_f64(n, nnz, cb, 2)}))
    sys.exit(0)
if a.op == "wavelet":
    from srgnn import wavelet as W
    ip, ix, lv, n, d, lmax = graphs.build_laplacian(a.config, dev, d=a.d)
    filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float32,
                                           heavy_threshold=a.heavy_threshold)
    S = synth.uniform_features_t(n, d, device=dev)
    R = torch.empty((2, n, d), dtype=torch.float32, device=dev)     # resident as in bench.py
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    cb = a.col_block or d
    while not a.col_block and cb > 8 and filt.work_panels() * n * cb * 4 > free - 2 ** 30:
        cb //= 2
    d = cb
    B = filt.prepare_column_blocks(d, hops=a.hops)
    A = filt._csr(filt.fvals)
    X = S[:, :d]
    Y = torch.empty((n, d), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        hop(A, X, Y, col_blocks=B)
    torch.cuda.synchronize()
    nnz = A.nnz
    print(json.dumps({"config": a.config, "op": "wavelet", "n": n, "nnz": nnz, "d": d, "reps": a.reps,
                      "launches_per_hop": launches_per_hop(A, B, d), "column_blocks": B, "n_heavy": A.n_heavy, "n_hub": A.n_hub,
                      "algorithmic_bytes": roofline.bytes_no_reuse(n, nnz, d),
                      "compulsory_bytes": roofline.bytes_compulsory(n, nnz, d)}))
    sys.exit(0)
if a.identity:
    d = a.d or 128
    n = (1 << 31) // (4 * d)              # 2 GiB panel (> 256 MiB Infinity Cache)
    ip = torch.arange(n + 1, dtype=torch.int64, device=dev)
    ix = torch.arange(n, dtype=torch.int32, device=dev)
    vals = torch.ones(n, dtype=torch.float32, device=dev)
elif a.permutation:
    n = synth.CONFIGS[a.config]["n"]
    d = a.d or synth.CONFIGS[a.config]["d"]
    ip = torch.arange(n + 1, dtype=torch.int64, device=dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    ix = torch.randperm(n, generator=g).to(dev, torch.int32)
    vals = torch.ones(n, dtype=torch.float32, device=dev)
else:
    ip, ix, vals, n, d, _ = graphs.build(a.config, dev, d=a.d)
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=a.heavy_threshold, device=dev)
X = synth.uniform_features_t(n, d, device=dev)
Y = torch.empty_like(X)
# the probe stands for a long run of hops (bench.py's operator serves every step): the panel rule alone
if a.identity or a.permutation:
    B = 1
else:
    B = prepare(A, d, a.hops, a.col_blocks)   # as bench.py: blocks, or a launch-ordered copy for long runs
torch.cuda.synchronize()
for _ in range(a.reps):
    hop(A, X, Y, col_blocks=B)      # one hop = B k_spmm launches (column blocks), same bits
torch.cuda.synchronize()
nnz = A.nnz
print(json.dumps({"config": "identity" if a.identity else (f"permutation-{a.config}" if a.permutation else a.config), "n": n, "nnz": nnz, "d": d,
                  "reps": a.reps, "launches_per_hop": launches_per_hop(A, B, d), "column_blocks": B,
                  "n_heavy": A.n_heavy, "n_hub": A.n_hub,
                  "algorithmic_bytes": roofline.bytes_no_reuse(n, nnz, d),
                  "compulsory_bytes": roofline.bytes_compulsory(n, nnz, d),
                  "x_read_bytes": n * 4 * d, "y_write_bytes": n * 4 * d,
                  "index_bytes": nnz * 8 + (n + 1) * 8}))
