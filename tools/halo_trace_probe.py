#!/usr/bin/env python3
"""Probe for rocprofv3 --kernel-trace: one virtual rank's hop launch (op.compute) repeated, so the
trace shows when the hub group's workgroups run relative to the row chunks.

    rocprofv3 --kernel-trace -d DIR -o t --output-format csv -- python3 tools/halo_trace_probe.py --world 8 --rank 1
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs  # noqa: E402
from srgnn.dist import HaloPartitionedOperator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev)
    op = HaloPartitionedOperator(ip, ix, vals, n, chunks=a.chunks, device=dev, rank=a.rank, world=a.world)
    del ip, ix, vals
    src = op.new_panel(d)
    src.uniform_(-1, 1)
    dst = op.new_panel(d)
    for _ in range(a.reps):
        op.compute(src, dst)
        torch.cuda.synchronize()
    import time
    # host issue cost of one hop's launches (no sync: the GPU queue absorbs them) vs GPU time
    t0 = time.perf_counter()
    for _ in range(a.reps):
        op.compute(src, dst)
    t_issue = (time.perf_counter() - t0) / a.reps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        op.compute(src, dst)
    torch.cuda.synchronize()
    t_total = (time.perf_counter() - t0) / a.reps
    t0 = time.perf_counter()
    for _ in range(a.reps):
        op.hop(src, dst, exchange=False)
    t_hop_issue = (time.perf_counter() - t0) / a.reps
    torch.cuda.synchronize()
    print(f"rank {a.rank}/{a.world}: hub rows {op.views[op.C][1]} (workgroup rows {op.views[op.C][3]}), "
          f"ghosts {op.n_ghost}; host issue {t_issue * 1e3:.3f} ms per compute(), "
          f"{t_hop_issue * 1e3:.3f} ms per hop(exchange=False); wall {t_total * 1e3:.3f} ms per compute()", flush=True)


if __name__ == "__main__":
    main()
