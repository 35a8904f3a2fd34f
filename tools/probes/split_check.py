"""Bitwise check of the halo layout with automatic hub thresholds (virtual ranks, real kernels)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "scalable-roubust-gnn_amd"))
import torch  # noqa: E402
from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.dist import simulate_halo_propagate  # noqa: E402
from srgnn.spmm import propagate  # noqa: E402

dev = torch.device("cuda", 0)
ip, ix, vals, n, d, K = graphs.build("arxiv", dev)
x = synth.uniform_features_t(n, d, device=dev)
want = propagate(DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev), x, 3)
for P in (2, 4, 8):
    got = simulate_halo_propagate(ip, ix, vals, n, x, 3, P, chunks=6, device=dev)
    print(P, all(torch.equal(got[k], want[k]) for k in range(4)), flush=True)
