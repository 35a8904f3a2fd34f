"""Probe (round 5): a small operator's 10-hop plan call repeated 200 times on a non-null stream, timed
per call, for library builds with and without SRG_PLAN_GRAPHS (the K-hop loop replayed as a HIP graph
from the second identical call).  Checks the bits stay the same."""
import os, sys, time
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "scalable-roubust-gnn_amd"))
import numpy as np, torch
from srgnn.csr import DeviceCSR
from srgnn.plan import NativePlan
rng = np.random.default_rng(0)
n = 4000
deg = np.minimum(rng.zipf(1.9, n), 800).astype(np.int64); deg[3] = 3000
ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) for k in deg]).astype(np.int32)
A = DeviceCSR.from_tensors(ip, ix, rng.standard_normal(ix.size).astype(np.float32), n_cols=n, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)                 # a capturable stream (the null stream is not)
for d, B in ((128, 1), (128, 4)):
    P = NativePlan(A, d, hops=10, col_blocks=B)
    X = torch.randn(n, d, device="cuda")
    panels = [X] + [torch.empty_like(X) for _ in range(10)]
    for _ in range(3):
        P.propagate(panels, d, d, 10)
    torch.cuda.synchronize()
    ref = [p.clone() for p in panels]
    t0 = time.perf_counter()
    for _ in range(200):
        P.propagate(panels, d, d, 10)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 200
    ok = all(torch.equal(a, b) for a, b in zip(ref, panels))
    t0 = time.perf_counter()
    for _ in range(20):
        P.propagate(panels, d, d, 10)
    host = (time.perf_counter() - t0) / 20          # host enqueue cost per call (the GPU runs behind)
    torch.cuda.synchronize()
    print(os.environ.get("SRGNN_HIP_LIB", "default").split("/")[-1], f"d={d} B={B} launches={P.n_launch}: {dt*1e3:.3f} ms per 10-hop call, host enqueue {host*1e3:.3f} ms, same bits {ok}", flush=True)
