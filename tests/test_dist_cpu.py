"""Row-partitioned multi-rank propagation on CPU ranks (gloo, world_size 2 and 3).

The exchange / partition / column-remap logic of srgnn.dist runs exactly as on GPUs; only the
local product is the oracle (injected), so the test checks that the partitioned result is
BITWISE equal to the single-process propagation."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    """A fresh file:// rendezvous for the ranks' process group: no TCP port to pick and then race
    for (a port probed free here was once taken before rank 0 listened on it: EADDRINUSE)."""
    fd, path = tempfile.mkstemp(prefix="srgnn_pg_")
    os.close(fd)
    os.unlink(path)
    return path


def _graph():
    from srgnn import synth
    from srgnn.normalize import sym_norm_binary
    n = 1500
    u, v = synth.rmat_undirected_t(n, 9000, seed=12)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 48, seed=3)
    return ip, ix, vals, x, n


def _worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "scalable-roubust-gnn_amd"), repo]
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    from oracle import oracle as O
    from srgnn.dist import RowPartitionedOperator

    def local_spmm(A, X, out):
        ip, ix, vv = A
        out.copy_(torch.from_numpy(O.spmm(ip.numpy(), ix.numpy(), vv.numpy(), X.numpy())))

    ip, ix, vals, x, n = _graph()
    op = RowPartitionedOperator(ip, ix, vals, n, local_spmm=local_spmm, device="cpu")
    panels = op.propagate(x[op.r0:op.r1], 3)
    # gather every rank's valid rows of the last hop
    full = [torch.zeros((op.max_rows, x.shape[1])) for _ in range(world)]
    dist.all_gather(full, panels[3])
    if rank == 0:
        res = torch.cat([full[p][: op.starts[p + 1] - op.starts[p]] for p in range(world)])
        np.save(out_path, res.numpy())
        np.save(out_path + ".starts.npy", np.array(op.starts))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_propagation_bitwise_equals_single(tmp_path, oracle_mod, world):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    ip, ix, vals, x, n = _graph()
    want = oracle_mod.propagate(ip.numpy(), ix.numpy(), vals.numpy(), x.numpy(), 3)[3]
    got = np.load(out)
    np.testing.assert_array_equal(got, want)
    starts = np.load(out + ".starts.npy")
    per = [int(ip[starts[p + 1]] - ip[starts[p]]) for p in range(world)]
    assert max(per) - min(per) <= int((ip[1:] - ip[:-1]).max())   # nnz-balanced blocks


def test_balanced_row_starts_and_remap():
    from srgnn.dist import balanced_row_starts, remap_columns
    ip = torch.tensor([0, 5, 5, 6, 20, 21, 30])
    s = balanced_row_starts(ip, 3)
    assert s[0] == 0 and s[-1] == 6 and all(a <= b for a, b in zip(s, s[1:]))
    cols = torch.tensor([0, 1, 2, 3, 4, 5], dtype=torch.int32)
    m = remap_columns(cols, [0, 2, 4, 6], 3)
    assert m.tolist() == [0, 1, 3, 4, 6, 7]
    assert bool((m[1:] > m[:-1]).all())          # monotone: CSR order (and fma chains) preserved


def _halo_worker(rank, world, port, out_path, chunks, ghost=None, full_x=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "scalable-roubust-gnn_amd"), repo]
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    from oracle import oracle as O
    from srgnn.dist import HaloPartitionedOperator

    def local_spmm(A, X, out):
        ip, ix, vv, order = A
        full = torch.from_numpy(O.spmm(ip.numpy(), ix.numpy(), vv.numpy(), X.numpy()))
        o = order.long()
        out[o] = full[o]

    ip, ix, vals, x, n = _graph()
    op = HaloPartitionedOperator(ip, ix, vals, n, chunks=chunks, hub_threshold=60, local_spmm=local_spmm,
                                 device="cpu", ghost_max_degree=ghost)
    assert op.views[-1][1] > 0 or world > 2          # some hub rows exist at this threshold
    assert ghost is None or (op.n_ghost > 0) == (ghost > 0)
    panels = op.propagate(x[op.r0:op.r1], 3, x_full=x if full_x else None)
    rows = torch.tensor([op.rows])
    all_rows = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(all_rows, rows)
    mx = int(max(r.item() for r in all_rows))
    buf = torch.zeros((mx, x.shape[1]))
    buf[: op.rows] = panels[3][: op.rows]
    full = [torch.zeros((mx, x.shape[1])) for _ in range(world)]
    dist.all_gather(full, buf)
    if rank == 0:
        res = torch.cat([full[q][: int(all_rows[q].item())] for q in range(world)])
        np.save(out_path, res.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks,ghost,full_x", [(2, 3, None, False), (3, 2, None, False), (2, 2, 0, False),
                                                      (3, 3, 16, False), (2, 2, None, True), (3, 2, 8, True)])
def test_halo_exchange_bitwise_equals_single(tmp_path, oracle_mod, world, chunks, ghost, full_x):
    """Halo exchange (only referenced remote rows, grouped all_to_all_single; ghost rows computed
    locally, exchanged once with X -- or, with the whole X on every rank, gathered from it) over
    gloo ranks."""
    out = str(tmp_path / "halo.npy")
    mp.spawn(_halo_worker, args=(world, _free_port(), out, chunks, ghost, full_x), nprocs=world, join=True)
    ip, ix, vals, x, n = _graph()
    want = oracle_mod.propagate(ip.numpy(), ix.numpy(), vals.numpy(), x.numpy(), 3)[3]
    np.testing.assert_array_equal(np.load(out), want)


def test_halo_layout_virtual_ranks(oracle_mod):
    """Halo sizes never exceed the all-gather volume, and the layout reproduces the product."""
    from srgnn.dist import HaloPartitionedOperator
    ip, ix, vals, x, n = _graph()

    def local_spmm(A, X, out):
        lip, lix, lvv, order = A
        full = torch.from_numpy(oracle_mod.spmm(lip.numpy(), lix.numpy(), lvv.numpy(), X.numpy()))
        o = order.long()
        out[o] = full[o]

    for world in (1, 4):
        shares = [HaloPartitionedOperator(ip, ix, vals, n, chunks=2, device="cpu", rank=q, world=world,
                                          local_spmm=local_spmm) for q in range(world)]
        for s in shares:
            assert s.halo <= n - s.rows
            assert sum(map(sum, s.recv_counts)) == s.n_recv
            assert sum(s.ghost_recv_counts) == s.n_ghost and s.n_recv + s.n_ghost == s.halo
        # every send list matches the receiver's count
        for g in range(shares[0].n_groups):
            for q, sq in enumerate(shares):
                for src, ss in enumerate(shares):
                    if src != q:
                        assert ss.send_counts[g][q] == sq.recv_counts[g][src]
        for q, sq in enumerate(shares):
            for src, ss in enumerate(shares):
                if src != q:
                    assert ss.ghost_send_counts[q] == sq.ghost_recv_counts[src]


@pytest.mark.parametrize("world,cap", [(2, 0), (2, 8), (3, 64), (4, 3)])
def test_halo_ghost_rows_virtual_ranks_bitwise(oracle_mod, world, cap):
    """Ghost rows (low-degree halo rows computed locally instead of received) with the oracle as
    the local product: K hops over P virtual ranks are bitwise the single-rank propagation, and
    the ghosts really replace received rows."""
    from srgnn.dist import HaloPartitionedOperator, simulate_halo_propagate
    ip, ix, vals, x, n = _graph()

    def local_spmm(A, X, out):
        lip, lix, lvv, order = A
        full = torch.from_numpy(oracle_mod.spmm(lip.numpy(), lix.numpy(), lvv.numpy(), X.numpy()))
        o = order.long()
        out[o] = full[o]

    shares = [HaloPartitionedOperator(ip, ix, vals, n, chunks=2, hub_threshold=60, device="cpu", rank=q,
                                      world=world, local_spmm=local_spmm, ghost_max_degree=cap)
              for q in range(world)]
    full_halo = [HaloPartitionedOperator(ip, ix, vals, n, chunks=2, device="cpu", rank=q, world=world,
                                         local_spmm=local_spmm, ghost_max_degree=0).halo for q in range(world)]
    for s, h in zip(shares, full_halo):
        assert s.halo == h and s.ghost_max_degree == cap
        assert (s.n_ghost > 0) == (cap > 0)
    got = simulate_halo_propagate(ip, ix, vals, n, x, 4, world, shares=shares)
    want = oracle_mod.propagate(ip.numpy(), ix.numpy(), vals.numpy(), x.numpy(), 4)
    for k in range(5):
        np.testing.assert_array_equal(got[k].numpy(), want[k])


def test_ghost_plan_cost_model():
    """The automatic cap: no ghosts when the links are (modelled as) free, ghosts when they are
    slow; every cap is one of the candidates, and all ranks agree."""
    import srgnn.dist as D
    ip, ix, vals, x, n = _graph()
    saved = D.GHOST_LINK_BPS
    try:
        D.GHOST_LINK_BPS = 1e30
        caps = {D.HaloPartitionedOperator(ip, ix, vals, n, chunks=2, device="cpu", rank=q, world=2,
                                          local_spmm=lambda *a: None).ghost_max_degree for q in range(2)}
        assert caps == {0}
        D.GHOST_LINK_BPS = 1e3
        caps = {D.HaloPartitionedOperator(ip, ix, vals, n, chunks=2, device="cpu", rank=q, world=2,
                                          local_spmm=lambda *a: None).ghost_max_degree for q in range(2)}
        assert len(caps) == 1 and caps.pop() in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64)
    finally:
        D.GHOST_LINK_BPS = saved


def _cpu_epilogue(Tn, Tc, To, mode, a1, a2, coef_prev, coef, R):
    """srg_cheby_epilogue_f32's arithmetic in torch fp32 (CPU ranks), every mode: INIT (0), STEP
    (1), INIT_T (2), STEP_FIRST (3), with the NO_T flag (0x10)."""
    a1, a2 = torch.tensor(a1, dtype=torch.float32), torch.tensor(a2, dtype=torch.float32)
    f32 = lambda v: torch.tensor(v, dtype=torch.float32)  # noqa: E731
    m, ns = mode & 0xF, R.shape[0]
    if m in (0, 2):
        t = (Tn - a2 * Tc) / a1
        if m == 0:
            for s in range(ns):
                R[s] = (0.5 * f32(coef_prev[s])) * Tc + f32(coef[s]) * t
    elif m == 3:
        t = Tn - To
        for s in range(ns):
            R[s] = ((0.5 * f32(coef_prev[s])) * To + f32(coef_prev[ns + s]) * Tc) + f32(coef[s]) * t
    else:
        t = Tn - To
        for s in range(ns):
            R[s] = R[s] + f32(coef[s]) * t
    if not mode & 0x10:
        Tn.copy_(t)


def _wavelet_graph():
    from srgnn import synth
    from srgnn.normalize import sym_norm_edges_blocked
    n = 1200
    u, v = synth.rmat_undirected_t(n, 7000, seed=21)
    ip, ix, lv = sym_norm_edges_blocked(u.to(torch.int32), v.to(torch.int32), n, kind="laplacian")
    S = synth.uniform_features_t(n, 20, seed=4)
    return ip, ix, lv, S, n


def _wavelet_worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "scalable-roubust-gnn_amd"), repo]
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    from oracle import oracle as O
    from srgnn.dist import HaloWaveletFilter

    def local_spmm(A, X, out):
        lip, lix, lvv, order = A
        full = torch.from_numpy(O.spmm(lip.numpy(), lix.numpy(), lvv.numpy(), X.numpy()))
        o = order.long()
        out[o] = full[o]

    ip, ix, lv, S, n = _wavelet_graph()
    f = HaloWaveletFilter(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=40.0, chunks=2, hub_threshold=30,
                          device="cpu", local_spmm=local_spmm, epilogue=_cpu_epilogue)
    R = f.apply(S[f.r0:f.r1])
    parts = [None] * world
    dist.all_gather_object(parts, (f.r0, f.r1, R.numpy()))
    if rank == 0:
        full = np.concatenate([p[2] for p in sorted(parts, key=lambda t: t[0])], axis=1)
        np.save(out_path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_halo_wavelet_bitwise_equals_single_rank(tmp_path, oracle_mod, world):
    """The distributed Chebyshev filter bank (one halo exchange per order) over gloo ranks equals
    the same computation on one rank, bit for bit."""
    from srgnn.dist import HaloWaveletFilter
    out = str(tmp_path / "wav.npy")
    mp.spawn(_wavelet_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    ip, ix, lv, S, n = _wavelet_graph()

    def local_spmm(A, X, o_):
        lip, lix, lvv, order = A
        full = torch.from_numpy(oracle_mod.spmm(lip.numpy(), lix.numpy(), lvv.numpy(), X.numpy()))
        o = order.long()
        o_[o] = full[o]

    single = HaloWaveletFilter(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=40.0, chunks=2, hub_threshold=30,
                               device="cpu", rank=0, world=1, local_spmm=local_spmm, epilogue=_cpu_epilogue)
    R = single.apply(S)
    np.testing.assert_array_equal(np.load(out), R.numpy())


def _sampled_parity_worker(rank, world, port, out_path, corrupt):
    import importlib.util
    import json
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "scalable-roubust-gnn_amd"), repo]
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    from oracle import oracle as O
    from srgnn.dist import HaloPartitionedOperator
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def local_spmm(A, X, out):
        ip, ix, vv, order = A
        full = torch.from_numpy(O.spmm(ip.numpy(), ix.numpy(), vv.numpy(), X.numpy()))
        o = order.long()
        out[o] = full[o]

    ip, ix, vals, x, n = _graph()
    K = 3
    op = HaloPartitionedOperator(ip, ix, vals, n, chunks=2, hub_threshold=60, local_spmm=local_spmm,
                                 device="cpu", ghost_max_degree=4)
    panels = op.propagate(x[op.r0:op.r1], K, x_full=x)
    if corrupt == "own" and rank == world - 1:         # one bit of one own row of hop K
        panels[K][0, 1] = torch.nextafter(panels[K][0, 1], torch.tensor(float("inf")))
    if corrupt == "halo" and rank == 0:                # one bit of every halo row of panel K-1
        panels[K - 1][op.rows:op.rows + op.halo, 0] = torch.nextafter(
            panels[K - 1][op.rows:op.rows + op.halo, 0], torch.tensor(float("inf")))
    res = bench.dist_sampled_parity(op, panels, K, n_random=op.rows, n_top=5, n_halo=op.halo)
    dev = bench.rank_devices(torch.device("cpu"), "gloo", world)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"parity": res, "devices": dev}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", ["none", "own", "halo"])
def test_bench_sampled_dist_parity_on_gloo_ranks(tmp_path, oracle_mod, corrupt):
    """bench.py's N-GPU check for the configurations whose whole-graph reference does not fit a
    rank (papers100M, RMAT-26): sampled own rows of hop 1 and hop K against the oracle fed with the
    rank's previous panel, and sampled halo rows against their owners -- green on a correct run,
    and a flipped bit in an own row or in the halo is caught; the device record lists every rank."""
    import json
    out = str(tmp_path / "par.json")
    world = 2
    mp.spawn(_sampled_parity_worker, args=(world, _free_port(), out, corrupt), nprocs=world, join=True)
    with open(out) as f:
        rec = json.load(f)
    par = rec["parity"]
    assert par["hops_checked"] == [1, 3] and par["rows_checked_rank0"] > 0
    # (a corrupted halo row also feeds the oracle a value the hop did not read: both checks see it)
    assert par["bit_exact"] == (corrupt == "none")
    assert par["halo_equal_to_owners"] == (corrupt != "halo")
    assert rec["devices"]["world_size"] == 2 and rec["devices"]["backend"] == "gloo"
    assert [r["rank"] for r in rec["devices"]["ranks"]] == [0, 1]


@pytest.mark.parametrize("world,chunks,hub", [(2, 2, 30), (3, 4, None), (4, 3, 0), (3, 2, -1)])
def test_halo_wavelet_f64_group_schedules(world, chunks, hub):
    """The fp64 halo filter's launch schedules (host logic, no device): one launch per exchange group of the
    halo plan, the hub group first, every own row in exactly one launch, each launch's rows by decreasing
    length with its hub rows first (the hub group's rows above min(rule, HUB_GROUP64_MIN), the chunks' above
    the rule; none with hub_threshold < 0); the one-launch schedule is every own row once, longest first."""
    from srgnn.dist import HUB_GROUP64_MIN, HaloWaveletFilter
    from srgnn.wavelet import HeatWaveletFilter
    ip, ix, lv, _, n = _wavelet_graph()
    for q in range(world):
        f = HaloWaveletFilter(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=40.0, chunks=chunks, hub_threshold=hub,
                              device="cpu", rank=q, world=world, dtype=torch.float64)
        deg = (f.opL._lip[1:f.rows + 1] - f.opL._lip[:f.rows]).to(torch.int64)
        t = HeatWaveletFilter.hub64_rule(int(deg.sum())) if hub is None else hub
        groups = f._sched64_groups
        assert [g for g, _ in groups] == [f.opL.C] + list(range(f.opL.C))
        rows = torch.cat([o.to(torch.int64) for _, (o, _) in groups])
        assert torch.equal(torch.sort(rows).values, torch.arange(f.rows))
        for g, (o, nh) in groups:
            dg = deg[o.to(torch.int64)]
            assert bool((dg[:-1] >= dg[1:]).all())
            tg = min(t, HUB_GROUP64_MIN) if g == f.opL.C else t
            assert nh == (int((dg > tg).sum()) if t >= 0 else 0)
        assert torch.equal(torch.sort(f._sched64.to(torch.int64)).values, torch.arange(f.rows))
        assert f._n_hub64 == (int((deg > t).sum()) if t >= 0 else 0)
        assert f.new_panel(8).dtype == torch.float64 and f.new_panel(8).shape == (f.rows + f.opL.halo, 8)
