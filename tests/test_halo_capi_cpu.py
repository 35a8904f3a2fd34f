"""The halo planner (srg_halo_plan_build, include/srgnn_hip.h) on the CPU: it builds rank p's share of
the halo-exchange partition from the global CSR, for C / C++ hosts and for the Python package's
srgnn.dist.HaloPartitionedOperator alike.  Every array of its plan is compared with the torch
restatement of the same plan (tests/halo_plan_ref.py, the planner the package ran before round 5): row
blocks, local CSR (remapped columns), schedules and their slice / hub counts, receive and send lists
per group, ghost rows and their sends, halo ids, and the automatic ghost cap of the link-rate cost
model.  Host-only entry: no device needed."""
import numpy as np
import pytest
import torch


def _graph(n=1500, e=9000, seed=12):
    from srgnn import synth
    from srgnn.normalize import sym_norm_binary
    u, v = synth.rmat_undirected_t(n, e, seed=seed)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    return ip, ix, vals, n


def _python_share(ip, ix, vals, n, world, rank, chunks, hub, ghost, link_bps=64e9):
    from halo_plan_ref import PyHaloPlan
    return PyHaloPlan(ip, ix, n, world, rank, chunks=chunks, hub_threshold=hub, ghost_max_degree=ghost,
                      link_bps=link_bps)


@pytest.mark.parametrize("world,chunks,hub,ghost,link", [(2, 3, 60, 0, 0), (3, 2, 60, 8, 0), (8, 6, None, 2, 0),
                                                        (4, 4, 40, 16, 0), (1, 2, None, 0, 0),
                                                        (4, 3, 60, None, 64e9), (4, 3, 60, None, 1e3),
                                                        (8, 6, None, None, 2e4), (3, 2, None, None, 1e30)])
def test_c_planner_equals_python_plan(world, chunks, hub, ghost, link):
    from srgnn import _lib
    from srgnn.comm import HaloPlan
    ip, ix, vals, n = _graph()
    caps = set()
    for rank in range(world):
        op = _python_share(ip, ix, vals, n, world, rank, chunks, hub, ghost, link_bps=link or 64e9)
        pl = HaloPlan(ip.numpy(), ix.numpy(), n, world, rank, chunks=chunks,
                      hub_threshold=_lib.SRG_HALO_AUTO if hub is None else hub,
                      ghost_max_degree=_lib.SRG_HALO_AUTO if ghost is None else ghost, link_bps=link)
        assert pl.info["ghost_max_degree"] == op.ghost_max_degree
        caps.add(op.ghost_max_degree)
        info = pl.info
        assert (info["row0"], info["n_rows"], info["n_recv"], info["n_ghost"], info["halo"]) == \
            (op.r0, op.rows, op.n_recv, op.n_ghost, op.halo)
        assert info["n_groups"] == op.n_groups and info["hub_rows"] == op.views[op.C][1]
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_STARTS), op.starts)
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_LOCAL_INDPTR), op._lip.numpy())
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_LOCAL_INDICES), op._lix.numpy())
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_GHOST_POSITIONS), op._ghost_pos.numpy())
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_HALO_IDS), op.halo_ids().numpy())
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_GROUP_OFFSETS), op.group_offsets)
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_CHUNK_RANGES)[1:],
                                      [b for _, b in op.chunk_ranges])
        for g in range(op.n_groups):
            np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_RECV_COUNTS, g), op.recv_counts[g])
            np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_SEND_COUNTS, g), op.send_counts[g])
            np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_SEND_ROWS, g), op.send_cat[g].numpy())
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_GHOST_SEND), op.ghost_send_cat.numpy())
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_GHOST_SEND_COUNTS), op.ghost_send_counts)
        np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_GHOST_RECV_COUNTS), op.ghost_recv_counts)
        for v, (order, n_g, n_heavy, n_hub) in enumerate(op.views + [op.ghost_view]):
            np.testing.assert_array_equal(pl.array(_lib.SRG_HALO_VIEW_ORDER, v), order.numpy(), err_msg=f"view {v}")
            meta = pl.array(_lib.SRG_HALO_VIEW_META, v)
            assert (meta[0], meta[1], meta[2]) == (n_g, n_hub, n_heavy), f"view {v}"
            if op.narrow[v] is not None:
                assert meta[3] == op.narrow[v], f"view {v}"
        pl.destroy()
    assert len(caps) == 1                    # every rank derives the same cap
    if ghost is None and link >= 1e30:
        assert caps == {0}                   # free links: nothing is worth computing twice
    if ghost is None and link <= 1e3:
        assert caps.pop() > 0                # slow links: ghosts


def test_c_planner_argument_checks():
    from srgnn import _lib
    from srgnn.comm import HaloPlan
    ip, ix, vals, n = _graph(n=300, e=1500)
    with pytest.raises(_lib.SrgError, match="rank"):
        HaloPlan(ip.numpy(), ix.numpy(), n, 2, 2)
    with pytest.raises(_lib.SrgError, match="chunks"):
        HaloPlan(ip.numpy(), ix.numpy(), n, 2, 0, chunks=0)
    bad = ix.numpy().copy()
    bad[7] = n
    with pytest.raises(_lib.SrgError, match="outside"):
        HaloPlan(ip.numpy(), bad, n, 2, 0)
    ipb = ip.numpy().copy()
    ipb[5] = ipb[6] + 1
    with pytest.raises(_lib.SrgError, match="decreases"):
        HaloPlan(ipb, ix.numpy(), n, 2, 0)
    # no hub rows at all
    pl = HaloPlan(ip.numpy(), ix.numpy(), n, 3, 1, chunks=2, hub_threshold=_lib.SRG_HALO_NONE)
    assert pl.info["hub_rows"] == 0
    # array sizes are checked before the planner reads them (short arrays were host over-reads)
    with pytest.raises(ValueError, match="n \\+ 1"):
        HaloPlan(ip.numpy()[:-1], ix.numpy(), n, 2, 0)
    with pytest.raises(ValueError, match="indices must have"):
        HaloPlan(ip.numpy(), ix.numpy()[:-3], n, 2, 0)
