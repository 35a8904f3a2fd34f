#!/usr/bin/env python3
"""Multi-rank rehearsal of the distributed path over the real RCCL ("nccl") backend.

Launched by torchrun with P ranks, one per GPU (LOCAL_RANK).  It needs P GPUs: RCCL refuses two
ranks on one card ("Duplicate GPU detected", seen on the one-GPU box), so on one GPU the N > 1 path
is covered by the gloo tests and the virtual-rank GPU tests instead.  Every rank checks its rows of
  * HaloPartitionedOperator.propagate (asynchronous all_to_all_single per group; ghost rows
    off, automatic and forced),
  * RowPartitionedOperator.propagate (all_gather_into_tensor),
  * HaloWaveletFilter.apply,
bitwise against the single-GPU kernels (propagate on the whole graph / the virtual-rank wavelet
simulation, itself bitwise equal to one GPU), and rank 0 prints one JSON line.

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_rehearsal.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.dist import (HaloPartitionedOperator, HaloWaveletFilter, RowPartitionedOperator,  # noqa: E402
                        simulate_halo_wavelet)
from srgnn.spmm import propagate  # noqa: E402


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SRGNN_DIST_BACKEND=gloo: a dry run of this script with ranks sharing the GPUs there are
    # (gloo through the host; RCCL refuses two ranks on one GPU)
    backend = os.environ.get("SRGNN_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    n, e, d, K = 60000, 700000, 64, 4
    ip, ix, vals, n, d, _ = graphs.build("arxiv", dev, n=n, n_edges=e, d=d)
    X = synth.uniform_features_t(n, d, device=dev)
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev)
    ref = propagate(A, X, K)
    res = {"world": world, "n": n, "nnz": int(ix.numel()), "d": d, "K": K}
    ok = True
    # ghost rows off / auto cap / forced cap; hop 0's halo exchanged or gathered from the whole X
    for chunks, ghost, whole in ((1, 0, False), (4, None, False), (4, 16, False), (4, None, True)):
        t0 = time.perf_counter()
        op = HaloPartitionedOperator(ip, ix, vals, n, chunks=chunks, device=dev, ghost_max_degree=ghost)
        panels = [op.new_panel(d) for _ in range(K + 1)]
        panels[0][: op.rows].copy_(X[op.r0:op.r1])
        for _ in range(2):                     # twice: the second run reuses streams and buffers
            op.propagate(panels[0], K, panels=panels, x_full=X if whole else None)
        torch.cuda.synchronize()
        good = all(torch.equal(panels[k][: op.rows], ref[k][op.r0:op.r1]) for k in range(K + 1))
        key = f"halo_chunks{chunks}_ghost{op.ghost_max_degree}" + ("auto" if ghost is None else "") + \
            ("_wholeX" if whole else "")
        res[key] = bool(good)
        res[key + "_s"] = time.perf_counter() - t0
        ok &= good
    op = RowPartitionedOperator(ip, ix, vals, n, device=dev)
    x_loc = op.new_panel(d)
    x_loc[: op.rows].copy_(X[op.r0:op.r1])
    out = op.propagate(x_loc, K, panels=[x_loc] + [op.new_panel(d) for _ in range(K)])
    torch.cuda.synchronize()
    good = all(torch.equal(out[k][: op.rows], ref[k][op.r0:op.r1]) for k in range(K + 1))
    res["allgather"] = bool(good)
    ok &= good
    lip, lix, lv, n2, _, lmax = graphs.build_laplacian("arxiv", dev, n=n, n_edges=e, d=d)
    S = synth.uniform_features_t(n2, d, seed=synth.FEATURE_SEED + 1, device=dev)
    f = HaloWaveletFilter(lip, lix, lv, n2, [-0.5, 0.5], order=3, lmax=lmax, chunks=2, device=dev)
    R = f.apply(S[f.r0:f.r1].contiguous())
    want = simulate_halo_wavelet(lip, lix, lv, n2, S, [-0.5, 0.5], 3, lmax, world=world, chunks=2, device=dev)
    torch.cuda.synchronize()
    good = torch.equal(R, want[:, f.r0:f.r1])
    res["wavelet"] = bool(good)
    ok &= good
    flag = torch.tensor([1 if ok else 0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    res["all_ranks_ok"] = bool(flag.item())
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if res["all_ranks_ok"] else 1)


if __name__ == "__main__":
    main()
