"""The multi-GPU hop path on GPU ranks, rehearsed on ONE GPU: 2-3 processes share cuda:0 and talk
over gloo (RCCL refuses two ranks on one GPU; gloo moves CUDA tensors through the host).  Every
rank runs HaloPartitionedOperator.propagate exactly as on a multi-GPU node -- the hub fork without
join, the packs and the asynchronous all_to_all per group, ghost rows, hop 0 exchanged or gathered
from the whole X -- and its rows of every hop must be bitwise the single-GPU propagation."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    """A fresh file:// rendezvous for the ranks' process group: no TCP port to pick and then race
    for (a port probed free here was once taken before rank 0 listened on it: EADDRINUSE)."""
    fd, path = tempfile.mkstemp(prefix="srgnn_pg_")
    os.close(fd)
    os.unlink(path)
    return path


def _worker(rank, world, port, out_path, ghost, whole_x, chunks, cb=None, fast=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "scalable-roubust-gnn_amd")]
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.dist import HaloPartitionedOperator
    from srgnn.normalize import sym_norm_binary
    from srgnn.spmm import propagate
    dev = torch.device("cuda", 0)
    n, K = 30000, 4
    u, v = synth.rmat_undirected_t(n, 240000, seed=31, device=dev)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 64, device=dev)
    want = propagate(DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev), x, K)
    op = HaloPartitionedOperator(ip, ix, vals, n, chunks=chunks, hub_threshold=400, device=dev,
                                 ghost_max_degree=ghost, col_blocks=cb, fast=fast)
    ok = op.views[op.C][1] > 0 and (ghost is None or (op.n_ghost > 0) == (ghost > 0))
    panels = [op.new_panel(64) for _ in range(K + 1)]
    panels[0][: op.rows].copy_(x[op.r0:op.r1])
    for _ in range(2):                          # twice: buffers and the hub side stream reused
        op.propagate(panels[0], K, panels=panels, x_full=x if whole_x else None)
    torch.cuda.synchronize()
    if cb:
        ok = ok and op.chunk_blocks(64) is not None
    if fast:        # hub rows re-associated (tolerance mode): within 1e-5 normwise per row, others exact
        ok = ok and all(bool(((panels[k][: op.rows] - want[k][op.r0:op.r1]).norm(dim=1)
                              <= 1e-5 * want[k][op.r0:op.r1].norm(dim=1)).all()) for k in range(K + 1))
    else:
        ok = ok and all(torch.equal(panels[k][: op.rows], want[k][op.r0:op.r1]) for k in range(K + 1))
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    if rank == 0:
        np.save(out_path, np.array(flags))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,ghost,whole_x,chunks,cb,fast", [(2, None, False, 3, None, False), (3, 0, False, 2, None, False),
                                                                 (2, 16, True, 4, None, False), (3, None, True, 6, None, False),
                                                                 (2, None, True, 3, 2, False), (3, 0, False, 4, 4, False),
                                                                 (2, None, True, 3, None, True)])
def test_halo_hop_on_gpu_ranks_bitwise(tmp_path, world, ghost, whole_x, chunks, cb, fast):
    """Column blocks in the row chunks (cb) stay bitwise; FAST (hub group re-associated) within 1e-5."""
    out = str(tmp_path / "flags.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, ghost, whole_x, chunks, cb, fast), nprocs=world, join=True)
    flags = np.load(out)
    assert flags.all(), f"ranks disagree with one GPU: {flags.tolist()}"


def _wavelet_worker(rank, world, port, out_path, chunks, f64=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "scalable-roubust-gnn_amd")]
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    from srgnn import graphs, synth
    from srgnn.dist import HaloWaveletFilter, simulate_halo_wavelet
    dev = torch.device("cuda", 0)
    lip, lix, lv, n, _, lmax = graphs.build_laplacian("arxiv", dev, n=20000, n_edges=160000, d=48)
    S = synth.uniform_features_t(n, 48, seed=9, device=dev)
    taus = [-0.5, 0.5]
    dt = torch.float64 if f64 else torch.float32
    S = S.to(dt)
    f = HaloWaveletFilter(lip, lix, lv, n, taus, order=4 if f64 else 3, lmax=lmax, chunks=chunks, hub_threshold=300,
                          device=dev, dtype=dt)
    R = f.apply(S[f.r0:f.r1].contiguous())              # orders overlapped with their exchange
    want = simulate_halo_wavelet(lip, lix, lv, n, S, taus, 4 if f64 else 3, lmax, world=world, chunks=chunks,
                                 hub_threshold=300, device=dev, dtype=dt)
    torch.cuda.synchronize()
    ok = bool(f.opL.views[f.opL.C][1] > 0) and R.dtype == dt and torch.equal(R, want[:, f.r0:f.r1])
    if f64:
        # the overlapped path ran (one launch per exchange group, sent right after), with hub rows in it, and
        # the groups' launches cover every own row once
        rows = torch.cat([o for _, (o, _) in f._sched64_groups]).to(torch.int64)
        ok = (ok and f._overlap64(48) and f._sched64_groups[0][1][1] >= f._n_hub64 > 0
              and torch.equal(torch.sort(rows).values, torch.arange(f.rows, device=dev)))
    flags = [None] * world
    dist.all_gather_object(flags, ok)
    if rank == 0:
        np.save(out_path, np.array(flags))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks,f64", [(2, 3, False), (3, 2, False), (2, 3, True), (3, 4, True)])
def test_halo_wavelet_on_gpu_ranks_bitwise(tmp_path, world, chunks, f64):
    """HaloWaveletFilter.apply on GPU ranks (each Chebyshev order's exchange overlapped chunk by
    chunk, the recurrence applied per chunk range before its rows are sent; fp64: one fused launch per
    exchange group, the hub group first) equals the virtual-rank simulation, itself bitwise one GPU."""
    out = str(tmp_path / "flags.npy")
    mp.spawn(_wavelet_worker, args=(world, _free_port(), out, chunks, f64), nprocs=world, join=True)
    flags = np.load(out)
    assert flags.all(), f"ranks disagree: {flags.tolist()}"
