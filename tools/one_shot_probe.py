#!/usr/bin/env python3
"""The reference's call pattern -- ONE propagate(K) on a freshly built operator -- under the layouts a
short run can take: span column blocks (the default below spmm.MIN_HOPS_TO_COMPACT hops) or compact
copies in launch order (what a long run gets), with the layout's cost inside the bracket.  HIP events:
operator build, column cut + layout, the K hops.

    python tools/one_shot_probe.py [--config products] [--reps 3]      -> one JSON line
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, spmm as S, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402


def one(ip, ix, vals, n, X, K, compact_min):
    S.MIN_HOPS_TO_COMPACT = compact_min
    dev = X.device
    st = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(st)
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
    ev[1].record(st)
    B = S.auto_col_blocks(A, X.shape[1], hops=K)
    if B > 1:
        S.column_blocks_for(A, B, hops=K)
    ev[2].record(st)
    out = S.propagate(A, X, K, col_blocks=B)
    ev[3].record(st)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    res = {"compact_min_hops": compact_min, "column_blocks": B, "compact": bool(A._blocks.get(("compact", B))),
           "ms_total": wall * 1e3, "ms_build": ev[0].elapsed_time(ev[1]), "ms_layout": ev[1].elapsed_time(ev[2]),
           "ms_hops": ev[2].elapsed_time(ev[3]), "ms_per_hop": ev[2].elapsed_time(ev[3]) / K}
    del out, A
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev)
    X = synth.uniform_features_t(n, d, device=dev)
    default = S.MIN_HOPS_TO_COMPACT
    one(ip, ix, vals, n, X, K, default)               # warm: allocator, code objects
    runs = []
    for _ in range(a.reps):
        for cm in (default, 1):
            runs.append(one(ip, ix, vals, n, X, K, cm))
            print(json.dumps(runs[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"config": a.config, "K": K, "runs": runs}))


if __name__ == "__main__":
    main()
