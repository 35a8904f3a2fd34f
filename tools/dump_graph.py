"""Writes a benchmark graph (srgnn.graphs.build, the bench's synthetic workloads) as a raw CSR file for the
plain-C hosts (examples/plan_propagate.c):

    8 bytes "SRGCSR1\\0", int64 n, int64 nnz, int64 indptr[n + 1], int32 indices[nnz], float32 values[nnz]

    python tools/dump_graph.py --config products --out /tmp/products.csr
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scalable-roubust-gnn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from srgnn import graphs
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    ip, ix, v, n, d, k = graphs.build(a.config, dev)
    with open(a.out, "wb") as f:
        f.write(b"SRGCSR1\0")
        f.write(np.array([n, ix.numel()], dtype=np.int64).tobytes())
        for t in (ip, ix, v):
            f.write(t.cpu().numpy().tobytes())
    print(f"{a.config}: n={n} nnz={ix.numel()} d={d} K={k} -> {a.out}")


if __name__ == "__main__":
    main()
