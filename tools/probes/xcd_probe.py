#!/usr/bin/env python3
"""Probe: one column block per XCD (tools/probes/xcd_probe.hip) against the sequential blocked hop.

Every row of the products-shaped Â is cut into 8 column blocks (compact CSRs, hub rows left out).
Times, on the same persistent kernel and the same work items:
  seq   8 launches, block b on every XCD (the sequential B = 8 hop, without its Y round trip),
  xcd   1 launch, XCD x works on block x only (each L2 caches one eighth of X's rows),
  mix   1 launch, every XCD works on every block (same concurrency as xcd, no L2 partition),
and the library's own B = 8 and B = 4 hops for scale.  Results are not combined (throughput only).
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))

import torch  # noqa: E402

from srgnn import csr as _csr, graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import hop  # noqa: E402



B = 8
LR = 4
dev = torch.device("cuda", 0)
lib = ctypes.CDLL(os.path.join(HERE, "tools", "probes", "_build", "libxcd_probe.so"))
lib.xprobe_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]

cfg = sys.argv[1] if len(sys.argv) > 1 else "products"
ip, ix, vals, n, d, _ = graphs.build(cfg, dev)
A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
X = synth.uniform_features_t(n, d, device=dev)
import plan_layout_ref as R  # noqa: E402  (tests/: the torch restatement of the layout)
blocks = R.compact_column_blocks(A, B, whole_max=0)   # every row cut (the probe's round-2 setting)
n_slices = d // 32
desc, Ys, info = [], [], []
for blk in blocks:
    nh = blk.n_hub
    order = blk.order[nh:].contiguous()
    n_rows = blk.n_rows - nh
    n_heavy = blk.n_heavy
    nb_heavy = (n_heavy * n_slices + 3) // 4
    n_light = n_rows - n_heavy
    n_blocks = nb_heavy + (n_light + 4 * LR - 1) // (4 * LR)
    Y = torch.empty((n, d), dtype=torch.float32, device=dev)
    Ys.append((Y, order))
    desc.append([blk.indptr.data_ptr(), blk.indices.data_ptr(), blk.values.data_ptr(), order.data_ptr(),
                 Y.data_ptr(), n_rows, n_heavy, nb_heavy, n_blocks])
    info.append({"nnz": blk.nnz, "n_hub": nh, "n_heavy": n_heavy, "n_rows": n_rows, "n_blocks": n_blocks})
D = torch.tensor(desc, dtype=torch.int64, device=dev)
ctr = torch.zeros(B, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev)


def run(mode, grid, xlog=None):
    ctr.zero_()
    if mode == 1:
        for b in range(B):
            rc = lib.xprobe_run(D.data_ptr(), 1, b, ctr.data_ptr(), None, grid, n_slices, X.data_ptr(), d, d,
                                s.cuda_stream)
            assert rc == 0
    else:
        rc = lib.xprobe_run(D.data_ptr(), mode, 0, ctr.data_ptr(), xlog.data_ptr() if xlog is not None else None,
                            grid, n_slices, X.data_ptr(), d, d, s.cuda_stream)
        assert rc == 0


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(reps):
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return min(out), sorted(out)[len(out) // 2]


res = {"config": cfg, "n": n, "nnz": A.nnz, "d": d, "blocks": info}
xlog = torch.full((2048,), -1, dtype=torch.int32, device=dev)
run(0, 2048, xlog)
torch.cuda.synchronize()
res["xcc_histogram_mode0"] = torch.bincount(xlog.to(torch.int64), minlength=8).tolist()
res["xcc_of_block_0_15"] = xlog[:16].tolist()
for grid in (1024, 2048, 4096):
    for name, mode in (("seq", 1), ("xcd", 0), ("mix", 2)):
        res[f"{name}_grid{grid}_ms"] = timed(lambda: run(mode, grid))
Yl = torch.empty_like(X)
for Bl in (8, 4):
    res[f"library_hop_B{Bl}_ms"] = timed(lambda: hop(A, X, Yl, col_blocks=Bl))
res["library_hop_B1_ms"] = timed(lambda: hop(A, X, Yl, col_blocks=1))
print(json.dumps(res))
