"""The C-ABI halo hop loop (srg_halo_propagate_f32) on the GPU: the C planner's shares of P virtual
ranks on one MI355X, exchanging through the loopback transport (device copies laid out exactly as
the RCCL grouped send / receive lays them: per group, peers ascending), run every rank's kernels,
packs, groups and offsets; each rank's own rows of every hop are bitwise the one-GPU hops.  One
real RCCL rank (srg_comm_init_all / init_rank) runs the same loop.  Several RCCL ranks need a
multi-GPU node (tools/rccl_rehearsal.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(n=20000, e=200000, d=64, seed=5):
    from srgnn import synth
    from srgnn.normalize import sym_norm_binary
    u, v = synth.rmat_undirected_t(n, e, seed=seed, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    X = synth.uniform_features_t(n, d, device="cuda")
    return ip, ix, vals, X, n


def _one_gpu(ip, ix, vals, X, n, K):
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import propagate
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
    return propagate(A, X, K, col_blocks=1)


@pytest.mark.parametrize("world,chunks,ghost,x_filled,hub", [(2, 3, 0, True, 64), (3, 4, 8, False, 64),
                                                             (8, 6, 2, True, None), (8, 6, 2, False, 256),
                                                             (4, 2, 16, False, None), (1, 2, 0, False, 64)])
def test_loopback_ranks_bitwise_equal_one_gpu(world, chunks, ghost, x_filled, hub):
    from srgnn import _lib
    from srgnn.comm import HaloPlan, HaloShare, halo_propagate, loopback
    ip, ix, vals, X, n = _graph()
    d, K = X.shape[1], 4
    want = _one_gpu(ip, ix, vals, X, n, K)
    ipn, ixn, vn = ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy()
    plans = [HaloPlan(ipn, ixn, n, world, r, chunks=chunks, ghost_max_degree=ghost,
                      hub_threshold=_lib.SRG_HALO_AUTO if hub is None else hub) for r in range(world)]
    assert world == 1 or sum(p.info["hub_rows"] for p in plans) > 0
    shares = [HaloShare(p, vn, 0, d) for p in plans]
    panels = [[s.new_panel(d) for _ in range(K + 1)] for s in shares]
    for s, ps in zip(shares, panels):
        if x_filled:
            s.fill_x_halo(X, ps[0])
        else:
            ps[0][: s.rows].copy_(X[s.plan.info["row0"]:s.plan.info["row0"] + s.rows])
    comm = loopback(world, 0)
    streams = [torch.cuda.Stream() for _ in range(world)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    try:
        halo_propagate(comm, shares, panels, K, x_halo_filled=x_filled, streams=[st.cuda_stream for st in streams])
        torch.cuda.synchronize()
        for k in range(K + 1):
            got = torch.cat([ps[k][: s.rows] for s, ps in zip(shares, panels)])
            assert torch.equal(got, want[k]), f"hop {k}"
        # the halo rows of hop K-1 (the last exchanged panel) equal the owners' rows
        for s, ps in zip(shares, panels):
            ids = torch.from_numpy(s.plan.array(_lib.SRG_HALO_HALO_IDS)).cuda()
            if ids.numel():
                assert torch.equal(ps[K - 1][s.rows:s.rows + s.halo], want[K - 1][ids])
    finally:
        comm.destroy()
        for s in shares:
            s.destroy()


@pytest.mark.parametrize("world,chunks,ghost,blocks,d", [(2, 3, 0, 2, 64), (4, 3, 2, 3, 128), (8, 6, 0, 8, 256),
                                                        (3, 2, 8, 5, 32), (1, 2, 0, 4, 128)])
def test_loopback_ranks_column_blocks_bitwise(world, chunks, ghost, blocks, d):
    """srg_halo_share_col_blocks: every row chunk in `blocks` column-block span launches (rows of
    <= 32 entries whole in block 0, later blocks continuing the chains) -- bitwise the one-GPU hops,
    and the same after switching the share back to unblocked."""
    from srgnn.comm import HaloPlan, HaloShare, halo_propagate, loopback
    ip, ix, vals, X, n = _graph(n=30000, e=400000, d=d, seed=9)
    K = 3
    want = _one_gpu(ip, ix, vals, X, n, K)
    ipn, ixn, vn = ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy()
    plans = [HaloPlan(ipn, ixn, n, world, r, chunks=chunks, ghost_max_degree=ghost, hub_threshold=128)
             for r in range(world)]
    shares = [HaloShare(p, vn, 0, d).col_blocks(blocks) for p in plans]
    comm = loopback(world, 0)
    try:
        for nb in (blocks, 1):
            for s in shares:
                s.col_blocks(nb)
            panels = [[s.new_panel(d) for _ in range(K + 1)] for s in shares]
            for s, ps in zip(shares, panels):
                s.fill_x_halo(X, ps[0])
            halo_propagate(comm, shares, panels, K, x_halo_filled=True)
            torch.cuda.synchronize()
            for k in range(K + 1):
                got = torch.cat([ps[k][: s.rows] for s, ps in zip(shares, panels)])
                assert torch.equal(got, want[k]), f"blocks {nb} hop {k}"
    finally:
        comm.destroy()
        for s in shares:
            s.destroy()


def test_one_rccl_rank_runs_the_halo_loop():
    from srgnn.comm import Comm, HaloPlan, HaloShare, halo_propagate, unique_id
    ip, ix, vals, X, n = _graph(n=6000, e=60000)
    d, K = X.shape[1], 3
    want = _one_gpu(ip, ix, vals, X, n, K)
    pl = HaloPlan(ip.cpu().numpy(), ix.cpu().numpy(), n, 1, 0, chunks=3, hub_threshold=64)
    sh = HaloShare(pl, vals.cpu().numpy(), 0, d)
    panels = [sh.new_panel(d) for _ in range(K + 1)]
    panels[0].copy_(X)
    for how in ("init_all", "init_rank"):
        comm = Comm.init_all([0]) if how == "init_all" else Comm.init_rank(1, unique_id(), 0, 0)
        try:
            halo_propagate(comm, [sh], [panels], K)
            torch.cuda.synchronize()
            for k in range(K + 1):
                assert torch.equal(panels[k], want[k]), f"{how} hop {k}"
        finally:
            comm.destroy()
    sh.destroy()


def test_halo_entry_argument_checks():
    from srgnn import _lib
    from srgnn.comm import HaloPlan, HaloShare, halo_propagate, loopback
    ip, ix, vals, X, n = _graph(n=3000, e=20000, d=16)
    ipn, ixn, vn = ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy()
    plans = [HaloPlan(ipn, ixn, n, 2, r, chunks=2) for r in range(2)]
    shares = [HaloShare(p, vn, 0, 16) for p in plans]
    comm = loopback(2, 0)
    try:
        panels = [[s.new_panel(16) for _ in range(3)] for s in shares]
        with pytest.raises(_lib.SrgError, match="shares for"):
            halo_propagate(comm, shares[:1], panels[:1], 2)
        with pytest.raises(_lib.SrgError, match="rank"):
            halo_propagate(comm, shares[::-1], panels[::-1], 2)
        # the Python wrapper checks what the C side trusts: panel count, shape, dtype,
        # layout and device of every panel
        with pytest.raises(ValueError, match="panels needed"):
            halo_propagate(comm, shares, [ps[:2] for ps in panels], 2)
        with pytest.raises(ValueError, match="panel list per share"):
            halo_propagate(comm, shares, panels[:1], 2)
        strided = [[torch.zeros((s.rows + s.halo, 32), device="cuda")[:, :16] for _ in range(3)] for s in shares]
        with pytest.raises(ValueError, match="contiguous"):
            halo_propagate(comm, shares, strided, 2)
        short = [[torch.zeros((s.rows, 16), device="cuda") for _ in range(3)] for s in shares]
        with pytest.raises(ValueError, match="contiguous float32"):
            halo_propagate(comm, shares, short, 2)
        f64 = [[torch.zeros((s.rows + s.halo, 16), device="cuda", dtype=torch.float64) for _ in range(3)]
               for s in shares]
        with pytest.raises(ValueError, match="float32"):
            halo_propagate(comm, shares, f64, 2)
        with pytest.raises(ValueError, match="panel0"):
            shares[0].fill_x_halo(X, panels[0][0][:, :8])
        with pytest.raises(ValueError, match="global CSR"):
            HaloShare(plans[0], vn[:-1], 0, 16)
        wide = [[torch.zeros((s.rows + s.halo, 32), device="cuda") for _ in range(3)] for s in shares]
        with pytest.raises(_lib.SrgError, match="d_max"):
            halo_propagate(comm, shares, wide, 2)
        for bad in (0, 65, -2):
            with pytest.raises(_lib.SrgError, match="n_blocks"):
                shares[0].col_blocks(bad)
        # a loopback communicator is not an RCCL one
        from srgnn.comm import Comm
        from srgnn.csr import DeviceCSR
        A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
        with pytest.raises(_lib.SrgError, match="loopback"):
            Comm(comm._h, [0, 0]).propagate([A, A], [0, n // 2, n], [X[: n // 2], X[n // 2:]], 1)
    finally:
        comm.destroy()
        for s in shares:
            s.destroy()
