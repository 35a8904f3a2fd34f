"""Wavelet basis on the GPU (fused Chebyshev launches) vs the CPU oracle.

fp64: the kernel follows the oracle's operation order (sequential CSR chains of separate multiply
and add, uncontracted epilogue), so results are compared BIT FOR BIT.  fp32: normwise relative
error <= 1e-5 against the fp64 oracle.  (Parity with pygsp itself is unpinned; see
tests/test_wavelet_cpu.py for the oracle's validation against a dense eigendecomposition.)"""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import torch

pytestmark = pytest.mark.gpu


def graphs():
    from srgnn import synth
    rng = np.random.default_rng(0)
    m = np.triu(rng.random((60, 60)) < 0.1, 1)
    a = sp.csr_matrix((m + m.T).astype(float))
    n = 3000
    u, v = synth.rmat_undirected_t(n, 15000, seed=8)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    b = sp.csr_matrix((np.ones(ix.numel()), ix.numpy(), ip.numpy()), shape=(n, n))
    return {"small": a, "rmat3000": b}


@pytest.mark.parametrize("gname", ["small", "rmat3000"])
@pytest.mark.parametrize("d", [5, 64, 128])
def test_heat_filter_f64_bit_exact(oracle_mod, gname, d):
    from srgnn import wavelet as W
    a = graphs()[gname]
    L = W.laplacian_from_adj(a)
    n = a.shape[0]
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, device="cuda")
    S = np.random.default_rng(d).standard_normal((n, d))
    R = f.apply(torch.from_numpy(S).cuda()).cpu().numpy()
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S, f.lmax)
    np.testing.assert_array_equal(R, want)


def _hub_graph():
    """rmat3000 plus three hub nodes: node 7 joined to every node (a ~3,000-entry row: six 512-entry
    windows, the last partial), node 11 to 1,100 nodes, node 13 to 520."""
    a = graphs()["rmat3000"].tolil()
    n = a.shape[0]
    rng = np.random.default_rng(4)
    for hub, k in ((7, n), (11, 1100), (13, 520)):
        for j in (np.arange(n) if k >= n else rng.choice(n, k, replace=False)):
            if j != hub:
                a[hub, j] = a[j, hub] = 1.0
    return sp.csr_matrix(a)


@pytest.mark.parametrize("hub", [500, 0, 6])
@pytest.mark.parametrize("d", [5, 16, 64, 100, 128, 130])
def test_heat_filter_f64_hub_rows_bit_exact(oracle_mod, hub, d):
    """srg_cheby_step_hub_f64: the schedule's hub rows (> hub entries) as hub workgroups on the side
    stream, the other rows as row waves -- bit for bit the oracle's cheby_op and the all-row-wave
    step.  hub = 0: every non-empty row a hub row (one short window each); d = 5: odd, every row a row
    wave; d = 100 / 130: a partial last slice."""
    from srgnn import wavelet as W
    a = _hub_graph()
    L = W.laplacian_from_adj(a)
    n = a.shape[0]
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, device="cuda", hub_threshold=hub)
    g = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=f.lmax, device="cuda", hub_threshold=-1)
    assert f.n_hub == (int((np.diff(L.indptr) > hub).sum())) and f.n_hub >= 3 and g.n_hub == 0
    S = np.random.default_rng(d).standard_normal((n, d))
    St = torch.from_numpy(S).cuda()
    R = f.apply(St).cpu().numpy()
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S, f.lmax)
    np.testing.assert_array_equal(R.view(np.uint64), want.view(np.uint64))
    np.testing.assert_array_equal(g.apply(St).cpu().numpy().view(np.uint64), R.view(np.uint64))


def test_fp64_hub_step_nojoin_then_rows_beside():
    """srg_cheby_step_hub_f64 with SRG_CHEBY_HUB_NOJOIN: the hub rows' launch left running on the hub side
    stream, the other rows as separate launches on the stream beside it, then srg_hub_join -- bit for bit the
    one joined launch over every row (the halo ranks' overlapped orders)."""
    import ctypes
    from srgnn import _lib, wavelet as W
    a = _hub_graph()
    L = W.laplacian_from_adj(a)
    n = a.shape[0]
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, device="cuda", hub_threshold=200)
    assert f.n_hub >= 3
    rng = np.random.default_rng(3)
    Tc, To = (torch.from_numpy(rng.standard_normal((n, 64))).cuda() for _ in range(2))
    cc = (ctypes.c_double * 2)(*f.coeffs[:, 2])
    dev, st = Tc.device, _lib.stream(Tc.device)

    def step(rows, n_hub, mode, Tn, R):
        _lib.call(dev, "srg_cheby_step_hub_f64", f.indptr.data_ptr(), f.indices.data_ptr(), f.fvals.data_ptr(),
                  rows.numel(), rows.data_ptr(), n_hub, Tc.data_ptr(), To.data_ptr(), Tn.data_ptr(), 64, 64, mode,
                  f.a1, f.a2, None, cc, 2, R.data_ptr(), n * 64, st)
    want_T, want_R = torch.empty_like(Tc), torch.zeros((2, n, 64), dtype=torch.float64, device="cuda")
    step(f.order, f.n_hub, _lib.SRG_CHEBY_STEP, want_T, want_R)
    got_T, got_R = torch.empty_like(Tc), torch.zeros_like(want_R)
    hubs, rest = f.order[: f.n_hub].contiguous(), f.order[f.n_hub:]
    step(hubs, f.n_hub, _lib.SRG_CHEBY_STEP | _lib.SRG_CHEBY_HUB_NOJOIN, got_T, got_R)
    for part in torch.chunk(rest, 3):
        step(part.contiguous(), 0, _lib.SRG_CHEBY_STEP, got_T, got_R)
    _lib.call(dev, "srg_hub_join", st)
    torch.cuda.synchronize()
    assert torch.equal(got_T, want_T) and torch.equal(got_R, want_R)


@pytest.mark.parametrize("B,hub,wm", [(2, None, None), (4, None, None), (7, 500, None), (4, 0, None), (16, 40, None),
                                      (4, None, 100), (6, 500, 12)])
@pytest.mark.parametrize("d", [5, 64, 100, 128])
def test_heat_filter_f64_column_blocked_bit_exact(oracle_mod, B, hub, wm, d):
    """srg_plan_cheby_step_f64: the fp64 orders through a column-blocked plan (spans of the filter's arrays,
    block 0's cut rows and whole rows, blocks 1.. continuing every chain from the fp64 partial sum in Tn,
    the epilogue where the chain ends, whole hub rows as hub workgroups on the side stream) == the oracle's
    cheby_op == the one-launch steps, bit for bit.  hub None: the fp64 rule (node 7's ~3,000 entries >
    2,048: one whole hub row); 500: explicit (SRG_PLAN_WHOLE_HUBS, three rows); 0 / 40: every row of more
    than 48 entries a whole hub row (no cut rows at all); wm: block 0's whole-row limit (SRG_PLAN_WHOLE_MAX);
    d = 5: 1-wide lanes and the hub rows as row waves."""
    from srgnn import wavelet as W
    a = _hub_graph()
    L = W.laplacian_from_adj(a)
    n = a.shape[0]
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, device="cuda")
    f.col_blocks64, f.hub64_threshold, f.whole64_max = B, hub, wm
    S = np.random.default_rng(d + B).standard_normal((n, d))
    St = torch.from_numpy(S).cuda()
    R = f.apply(St).cpu().numpy()
    P = f._plan64(d)
    assert P is not None and P.col_blocks == B and P.fp64
    deg = np.diff(L.indptr)
    t = W.HeatWaveletFilter.hub64_rule(L.nnz) if hub is None else hub
    whole = int((deg > max(t, wm or 48)).sum())            # block 0's whole rows (<= 48 entries) run whole anyway
    assert P.hub_rows_whole == whole and whole >= 1
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S, f.lmax)
    np.testing.assert_array_equal(R.view(np.uint64), want.view(np.uint64))
    g = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=f.lmax, device="cuda")
    assert g._plan64(d) is None                    # a small panel: one launch per order
    np.testing.assert_array_equal(g.apply(St).cpu().numpy().view(np.uint64), R.view(np.uint64))
    f.drop_layouts()


@pytest.mark.parametrize("order", [1, 2, 3, 5])
@pytest.mark.parametrize("B", [None, 5])
def test_fp64_lean_sequence_bit_identical(oracle_mod, order, B):
    """The fused fp64 steps' lean epilogue sequence (INIT_T, STEP_FIRST, ..., STEP | NO_T) == INIT + STEP ...
    == the oracle, bit for bit, one launch per order (with its hub rows) or over a 5-block plan."""
    from srgnn import wavelet as W
    a = _hub_graph()
    L = W.laplacian_from_adj(a)
    n = a.shape[0]
    f = W.HeatWaveletFilter(L, [-1.0, 0.3, 2.0], order=order, lmax=None, device="cuda", hub_threshold=500)
    f.col_blocks64, f.hub64_threshold = B, (500 if B else None)
    S = np.random.default_rng(order).standard_normal((n, 64))
    St = torch.from_numpy(S).cuda()
    lean = f.apply(St).cpu().numpy()
    f.lean_epilogue = False
    full = f.apply(St).cpu().numpy()
    assert (f._plan64(64) is not None) == bool(B)
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S, f.lmax)
    np.testing.assert_array_equal(lean.view(np.uint64), want.view(np.uint64))
    np.testing.assert_array_equal(full.view(np.uint64), want.view(np.uint64))
    f.drop_layouts()


@pytest.mark.parametrize("case", ["no_edges", "d1", "d2", "one_hub_only"])
def test_fp64_blocked_edge_cases(oracle_mod, case):
    """Blocked fp64 steps on degenerate layouts: a Laplacian without edges (every row a 1-entry whole row,
    the cut launches empty), 1- and 2-column panels, and a star whose centre is the only cut row (a whole
    hub row; every other row whole) -- the oracle's bits."""
    from srgnn import wavelet as W
    if case == "no_edges":
        a = sp.csr_matrix((500, 500))
    elif case == "one_hub_only":
        n0 = 3000
        a = sp.csr_matrix((np.ones(n0 - 1), (np.zeros(n0 - 1, dtype=np.int64), np.arange(1, n0))), shape=(n0, n0))
        a = a + a.T
    else:
        a = _hub_graph()
    d = {"d1": 1, "d2": 2}.get(case, 8)
    L = W.laplacian_from_adj(a)
    n = a.shape[0]
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None if case != "no_edges" else 2.0, device="cuda")
    f.col_blocks64 = 3
    S = np.random.default_rng(3).standard_normal((n, d))
    R = f.apply(torch.from_numpy(S).cuda()).cpu().numpy()
    P = f._plan64(d)
    assert P is not None and P.col_blocks == 3
    if case == "one_hub_only":
        assert P.hub_rows_whole == 1
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S, f.lmax)
    np.testing.assert_array_equal(R.view(np.uint64), want.view(np.uint64))
    f.drop_layouts()


def test_plan_cheby_step_argument_checks():
    """srg_plan_cheby_step_f64 refuses a compact plan (its ids are copies, the fp64 values are not), a
    blocked plan with block 0 as one launch, null values and unknown modes; nothing runs."""
    import ctypes as C
    from srgnn import _lib
    from srgnn.plan import NativePlan
    from srgnn.csr import DeviceCSR
    a = _hub_graph()
    n = a.shape[0]
    A = DeviceCSR.from_scipy(sp.csr_matrix(a, dtype=np.float32), device="cuda")
    T = torch.zeros((n, 64), dtype=torch.float64, device="cuda")
    R = torch.zeros((2, n, 64), dtype=torch.float64, device="cuda")
    v = torch.ones(A.nnz, dtype=torch.float64, device="cuda")
    coef = (C.c_double * 2)(1.0, 1.0)

    def step(P, vals=v, mode=_lib.SRG_CHEBY_STEP):
        _lib.call(P.device, "srg_plan_cheby_step_f64", P._p, vals.data_ptr() if vals is not None else None,
                  T.data_ptr(), T.data_ptr(), T.data_ptr(), 64, 64, mode, 1.0, 1.0, None, coef, 2, R.data_ptr(), n * 64,
                  _lib.stream(P.device))
    P = NativePlan(A, 64, 20, col_blocks=3, compact=True, split_block0=True)
    with pytest.raises(_lib.SrgError, match="SRG_PLAN_SPANS"):
        step(P)
    P.close()
    P = NativePlan(A, 64, 20, col_blocks=3, compact=False, split_block0=False)
    with pytest.raises(_lib.SrgError, match="SPLIT_BLOCK0"):
        step(P)
    P.close()
    P = NativePlan(A, 64, 20, col_blocks=3, fp64=True)
    with pytest.raises(_lib.SrgError, match="null values"):
        step(P, vals=None)
    with pytest.raises(_lib.SrgError, match="cheby mode"):
        step(P, mode=9)
    P.close()


def test_fp64_plan_refuses_fp32_hops():
    """A plan built without fp32 values (the fp64 steps' layout) is refused by the fp32 entry points."""
    from srgnn import _lib
    from srgnn import wavelet as W
    a = _hub_graph()
    f = W.HeatWaveletFilter(W.laplacian_from_adj(a), [-0.5, 0.5], order=3, lmax=None, device="cuda")
    f.col_blocks64 = 3
    P = f._plan64(64)
    X = torch.zeros((a.shape[0], 64), device="cuda")
    with pytest.raises(_lib.SrgError, match="without fp32 values"):
        P.propagate([X, torch.empty_like(X)], 64, 64, 1)
    with pytest.raises(_lib.SrgError, match="without fp32 values"):
        P.hop(X, torch.empty_like(X), 64)
    f.drop_layouts()


@pytest.mark.parametrize("order", [1, 2, 5])
def test_heat_filter_orders(oracle_mod, order):
    from srgnn import wavelet as W
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-1.0, 0.3, 2.0], order=order, lmax=7.5, device="cuda")
    S = np.random.default_rng(1).standard_normal((a.shape[0], 16))
    R = f.apply(torch.from_numpy(S).cuda()).cpu().numpy()
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S, 7.5)
    np.testing.assert_array_equal(R, want)


def test_heat_filter_f32_within_tolerance(oracle_mod):
    from srgnn import wavelet as W
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, dtype=torch.float32, device="cuda")
    S = np.random.default_rng(3).standard_normal((a.shape[0], 256)).astype(np.float32)
    R = f.apply(torch.from_numpy(S).cuda()).cpu().numpy().astype(np.float64)
    want = oracle_mod.cheby_op((L.indptr, L.indices, L.data), f.coeffs, S.astype(np.float64), f.lmax)
    rel = np.linalg.norm(R - want) / np.linalg.norm(want)
    assert rel <= 1e-5, rel


def test_wavelet_basis_matches_oracle_restatement(oracle_mod):
    """phi / phi^-1 as SpectralModel.calculate_wavelet + normalize_matrices build them."""
    from srgnn import wavelet as W
    a = graphs()["small"]
    n = a.shape[0]
    phi, phi_inv, lmax = W.wavelet_basis(a, scale=0.5, order=3, tolerance=1e-4, batch=25, device="cuda")
    L = W.laplacian_from_adj(a)
    coeffs = np.stack([oracle_mod.cheby_coeffs(t, lmax, 3) for t in (-0.5, 0.5)])
    R = oracle_mod.cheby_op((L.indptr, L.indices, L.data), coeffs, np.eye(n), lmax)
    from sklearn.preprocessing import normalize   # what the reference calls (base_model.py:290)
    for s, got in enumerate((phi, phi_inv)):
        m = R[s].copy()
        m[m < 1e-4] = 0
        want = normalize(sp.csr_matrix(m.astype(np.float32)), norm="l1", axis=1)
        assert got.dtype == np.float32
        np.testing.assert_array_equal(got.indptr, want.indptr)
        np.testing.assert_array_equal(got.indices, want.indices)
        np.testing.assert_array_equal(got.data, want.data)      # bit-exact (sklearn's arithmetic)


def test_spectral_features_vs_dense_fp64(oracle_mod):
    """SpectralModel.preprocess's processed_feature [X | relu(phi phi^-1 X)] vs a dense fp64
    evaluation on the same phi / phi^-1 (the product association differs: tolerance 1e-5)."""
    from srgnn import wavelet as W
    a = graphs()["rmat3000"]
    n = a.shape[0]
    X = np.random.default_rng(5).random((n, 24)).astype(np.float32)
    out, phi, phi_inv, lmax = W.spectral_features(a, X, scale=0.5, order=3, tolerance=1e-4, batch=700, device="cuda")
    assert out.shape == (n, 48) and out.dtype == torch.float32
    np.testing.assert_array_equal(out[:, :24].numpy(), X)
    want = np.maximum((phi.toarray().astype(np.float64) @ phi_inv.toarray().astype(np.float64)) @ X.astype(np.float64), 0)
    got = out[:, 24:].numpy().astype(np.float64)
    assert np.linalg.norm(got - want) / np.linalg.norm(want) <= 1e-5


@pytest.mark.parametrize("thr", [(None, None), (0, -1), (-1, -1), (4, 40)])
@pytest.mark.parametrize("d,cb", [(128, None), (100, 32), (256, 64), (36, 8), (130, None), (96, None), (64, 16)])
def test_split_path_bit_identical_to_fused(d, cb, thr):
    """fp32 split path (load-balanced SpMM with the Chebyshev epilogue fused into its store,
    srg_spmm_cheby_f32, T_{k+1} written over T_{k-1}; and the two-launch form, SpMM +
    srg_cheby_epilogue_f32; column blocks writing into strided views of R) == the fused
    srg_cheby_step_f32 kernel, bit for bit.  The shapes reach every store site: packed light rows
    (d = 64 / 128 / 256 blocks), narrow rows (blocks of 4 / 8 / 16 / 32), row waves with 2- and
    1-wide lanes (130, 96), slice waves and hub workgroups (thresholds)."""
    from srgnn import wavelet as W
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5, 1.5], order=4, lmax=None, dtype=torch.float32, device="cuda",
                            heavy_threshold=thr[0], hub_threshold=thr[1])
    S = torch.from_numpy(np.random.default_rng(d).standard_normal((a.shape[0], d)).astype(np.float32)).cuda()
    fused = f.apply(S, split=False)
    split = f.apply(S, split=True, col_block=cb)
    assert torch.equal(fused, split)
    one_launch = f.apply(S, split=True, col_block=cb, fused_epilogue=True)
    assert torch.equal(fused, one_launch)
    # into a caller-provided stack, and from a strided column window of a wider panel
    wide = torch.zeros((a.shape[0], d + 12), device="cuda")
    wide[:, 4:4 + d] = S
    for fe in (True, False):
        out = torch.full((3, a.shape[0], d), float("nan"), device="cuda")
        f.apply(wide[:, 4:4 + d], split=True, col_block=cb, out=out, fused_epilogue=fe)
        assert torch.equal(fused, out)


@pytest.mark.parametrize("order", [1, 2, 3, 5])
@pytest.mark.parametrize("cb", [None, 32])
def test_lean_epilogue_bit_identical(order, cb):
    """Split path with the lean epilogue sequence (order 1 stores T1 only, order 2 forms R from
    T0, T1, T2, the last order stores no T) == the INIT + STEP epilogues == the fused kernel."""
    from srgnn import wavelet as W
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5, 1.5], order=order, lmax=None, dtype=torch.float32, device="cuda",
                            heavy_threshold=40, hub_threshold=400)
    S = torch.from_numpy(np.random.default_rng(order).standard_normal((a.shape[0], 96)).astype(np.float32)).cuda()
    fused = f.apply(S, split=False)
    f.lean_epilogue = True
    lean = f.apply(S, split=True, col_block=cb)
    f.lean_epilogue = False
    plain = f.apply(S, split=True, col_block=cb)
    assert torch.equal(fused, lean) and torch.equal(fused, plain)


@pytest.mark.parametrize("B", [2, 3])
def test_split_path_column_blocked_bit_identical(monkeypatch, B):
    """The split path's SpMMs as column-blocked hops (spmm.hop, forced here; automatic for panels of
    512 MiB .. 16 GiB) == the fused kernel, bit for bit."""
    from srgnn import spmm as S_, wavelet as W
    monkeypatch.setattr(S_, "FORCE_COL_BLOCKS", B)
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, dtype=torch.float32, device="cuda",
                            heavy_threshold=40, hub_threshold=400)
    from srgnn.plan import cached
    S = torch.from_numpy(np.random.default_rng(9).standard_normal((a.shape[0], 128)).astype(np.float32)).cuda()
    assert torch.equal(f.apply(S, split=False), f.apply(S, split=True, col_block=64))
    assert cached(f._csr(f.fvals), 64).col_blocks == B


def test_split_path_runs_the_native_plan(monkeypatch):
    """Automatic thresholds: prepare_column_blocks lays L and F out with the native plan (srgnn.plan)
    and the split path's hops -- over column slices of the panel, a leading dimension other than the
    work panels' -- run through srg_plan_hop_f32: bit for bit the fused kernel."""
    from srgnn import spmm as S_, wavelet as W
    from srgnn.plan import cached
    monkeypatch.setattr(S_, "FORCE_COL_BLOCKS", 3)
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=4, lmax=None, dtype=torch.float32, device="cuda")
    assert f.prepare_column_blocks(64, hops=8) == 3
    assert cached(f._csr(f.fvals), 64) is not None and cached(f._csr(f.lvals), 64) is not None
    S = torch.from_numpy(np.random.default_rng(5).standard_normal((a.shape[0], 128)).astype(np.float32)).cuda()
    assert torch.equal(f.apply(S, split=False), f.apply(S, split=True, col_block=64))


def test_split_path_plans_in_torch_memory(monkeypatch):
    """The filter's plans hold their memory as torch allocations (srg_plan_build_in: what the RMAT-26
    filter bank needs, whose graph build leaves torch's cache full of reusable blocks); bit for bit the
    fused kernel; drop_layouts frees every cached plan and returns the memory to torch."""
    from srgnn import spmm as S_, wavelet as W
    from srgnn.plan import cached
    monkeypatch.setattr(S_, "FORCE_COL_BLOCKS", 3)
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=4, lmax=None, dtype=torch.float32, device="cuda")
    before = torch.cuda.memory_allocated()
    assert f.prepare_column_blocks(64, hops=8) == 3
    Fm = f._csr(f.fvals)
    P = cached(Fm, 64)
    assert P is not None and P._keep is not None and P._keep.numel() >= P.device_bytes
    assert torch.cuda.memory_allocated() - before >= P.device_bytes
    S = torch.from_numpy(np.random.default_rng(6).standard_normal((a.shape[0], 128)).astype(np.float32)).cuda()
    assert torch.equal(f.apply(S, split=False), f.apply(S, split=True, col_block=64))
    f.drop_layouts()
    assert not Fm._blocks and P._p is None and P._keep is None


def test_spmm_cheby_in_place_and_argument_checks():
    """srg_spmm_cheby_f32 directly: a step written over T_{k-1} equals the step into a fresh panel
    and the two-launch form; aliasing and flag misuse are rejected before any launch."""
    from srgnn import _lib, wavelet as W
    from srgnn.spmm import spmm, spmm_cheby
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    f = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=None, dtype=torch.float32, device="cuda")
    n = a.shape[0]
    rng = np.random.default_rng(11)
    Tc, To = (torch.from_numpy(rng.standard_normal((n, 128)).astype(np.float32)).cuda() for _ in range(2))
    Fm = f._csr(f.fvals)
    R0 = torch.from_numpy(rng.standard_normal((2, n, 128)).astype(np.float32)).cuda()
    fresh, Rf = torch.empty_like(To), R0.clone()
    spmm_cheby(Fm, Tc, fresh, _lib.SRG_CHEBY_STEP, f.a1, f.a2, To, None, f.coeffs[:, 2], Rf)
    inplace, Ri = To.clone(), R0.clone()
    spmm_cheby(Fm, Tc, inplace, _lib.SRG_CHEBY_STEP, f.a1, f.a2, inplace, None, f.coeffs[:, 2], Ri)
    y, Rs = spmm(Fm, Tc), R0.clone()
    cp = (ctypes.c_float * 2)(*f.coeffs[:, 2])
    _lib.call(y.device, "srg_cheby_epilogue_f32", y.data_ptr(), 128, None, 128, To.data_ptr(), 128, n, 128,
              _lib.SRG_CHEBY_STEP, f.a1, f.a2, None, cp, 2, Rs.data_ptr(), 128, n * 128, _lib.stream(y.device))
    assert torch.equal(fresh, inplace) and torch.equal(fresh, y)
    assert torch.equal(Rf, Ri) and torch.equal(Rf, Rs)
    with pytest.raises(_lib.SrgError, match="alias Tc"):
        spmm_cheby(Fm, Tc, Tc, _lib.SRG_CHEBY_STEP, f.a1, f.a2, To, None, f.coeffs[:, 2], Rf)
    with pytest.raises(_lib.SrgError, match="must not alias a T panel"):
        spmm_cheby(Fm, Tc, fresh, _lib.SRG_CHEBY_STEP, f.a1, f.a2, To, None, f.coeffs[:1, 2], fresh.view(1, n, 128))
    with pytest.raises(_lib.SrgError, match="needs To"):
        spmm_cheby(Fm, Tc, fresh, _lib.SRG_CHEBY_STEP, f.a1, f.a2, None, None, f.coeffs[:, 2], Rf)


def test_device_built_filter_equals_host_built():
    """HeatWaveletFilter.from_device (device Laplacian from the edge list) == the host-built filter."""
    from srgnn import normalize, synth, wavelet as W
    n = 3000
    u, v = synth.rmat_undirected_t(n, 15000, seed=8)
    ip, ix, lv = normalize.sym_norm_edges_blocked(u.cuda().to(torch.int32), v.cuda().to(torch.int32), n,
                                                  kind="laplacian")
    a = graphs()["rmat3000"]
    L = W.laplacian_from_adj(a)
    host = W.HeatWaveletFilter(L, [-0.5, 0.5], order=3, lmax=9.0, dtype=torch.float32, device="cuda")
    dev = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=9.0, dtype=torch.float32)
    assert torch.equal(host.fvals, dev.fvals) and torch.equal(host.lvals, dev.lvals)
    S = torch.from_numpy(np.random.default_rng(2).standard_normal((n, 64)).astype(np.float32)).cuda()
    assert torch.equal(host.apply(S), dev.apply(S, col_block=16))


@pytest.mark.parametrize("world,chunks", [(2, 3), (8, 4)])
def test_halo_wavelet_virtual_ranks_bitwise(world, chunks):
    """The wavelet filter bank over the halo partition (P virtual ranks on one GPU, one exchange per
    Chebyshev order) == HeatWaveletFilter's split path on one GPU, bit for bit."""
    from srgnn import normalize, synth, wavelet as W
    from srgnn.dist import simulate_halo_wavelet
    n = 4000
    u, v = synth.rmat_undirected_t(n, 40000, seed=17, device="cuda")
    ip, ix, lv = normalize.sym_norm_edges_blocked(u.to(torch.int32), v.to(torch.int32), n, kind="laplacian")
    S = synth.uniform_features_t(n, 64, seed=5, device="cuda")
    lmax = 2.0 * float((ip[1:] - ip[:-1]).max())
    one = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float32)
    want = one.apply(S, split=True)
    got = simulate_halo_wavelet(ip, ix, lv, n, S, [-0.5, 0.5], 3, lmax, world, chunks=chunks, device="cuda")
    assert torch.equal(got, want)


@pytest.mark.parametrize("world,hub,blocks", [(2, None, 1), (3, 100, 1), (8, None, 1), (4, 0, 1),
                                               (2, None, 4), (3, 100, 3), (4, None, 7), (2, None, None)])
def test_halo_wavelet_f64_virtual_ranks_bitwise(oracle_mod, world, hub, blocks):
    """The fp64 filter bank (pygsp cheby_op's precision) over the halo partition: P virtual ranks on one GPU,
    each order one fused srg_cheby_step_hub_f64 launch over the rank's rows (hub rows: the fp64 rule, or
    rows > 100 entries, or every row) -- or, forced, the rank's column-blocked fp64 plan over its [rows + halo]
    panel -- and one exchange of fp64 halo rows == the one-GPU fp64 filter == the oracle's cheby_op, bit for
    bit."""
    from srgnn import normalize, synth, wavelet as W
    from srgnn.dist import simulate_halo_wavelet
    n = 4000
    u, v = synth.rmat_undirected_t(n, 40000, seed=17, device="cuda")
    ip, ix, lv = normalize.sym_norm_edges_blocked(u.to(torch.int32), v.to(torch.int32), n, kind="laplacian")
    S = synth.uniform_features_t(n, 64, seed=5, device="cuda").to(torch.float64)
    lmax = 2.0 * float((ip[1:] - ip[:-1]).max())
    one = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float64)
    want = one.apply(S)
    got = simulate_halo_wavelet(ip, ix, lv, n, S, [-0.5, 0.5], 3, lmax, world, chunks=3, device="cuda",
                                hub_threshold=hub, dtype=torch.float64, col_blocks64=blocks)
    assert got.dtype == torch.float64 and torch.equal(got, want)
    ref = oracle_mod.cheby_op((ip.cpu().numpy(), ix.cpu().numpy(), lv.to(torch.float64).cpu().numpy()), one.coeffs,
                              S.cpu().numpy(), lmax)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("world,d,order", [(8, 1, 1), (5, 3, 2), (8, 64, 5), (3, 7, 3), (7, 2, 4)])
def test_halo_wavelet_f64_ragged_edge_cases(oracle_mod, world, d, order):
    """The fp64 halo filter bank on a ragged operator: a third of the rows empty (no diagonal either), a few
    ranks holding only a handful of rows, odd and one-column panels (the hub workgroups need an even d, so
    those run as row waves only), orders 1 (no lean sequence) to 5 == the one-GPU fp64 filter == the
    oracle's cheby_op, bit for bit."""
    from srgnn import wavelet as W
    from srgnn.dist import simulate_halo_wavelet
    rng = np.random.default_rng(world * 100 + d)
    n = 60
    deg = rng.integers(0, 12, n)
    deg[40:] = 0
    deg[3] = 45
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) for k in deg] + [np.zeros(0, np.int64)])
    lv = rng.standard_normal(ix.size).astype(np.float32)
    ip_t, ix_t, lv_t = (torch.from_numpy(a).cuda() for a in (ip, ix.astype(np.int32), lv))
    S = torch.from_numpy(rng.standard_normal((n, d))).cuda()
    lmax = 9.0
    one = W.HeatWaveletFilter.from_device(ip_t, ix_t, lv_t, n, [-0.5, 0.5], order=order, lmax=lmax,
                                          dtype=torch.float64)
    want = one.apply(S)
    got = simulate_halo_wavelet(ip_t, ix_t, lv_t, n, S, [-0.5, 0.5], order, lmax, world, chunks=2, device="cuda",
                                hub_threshold=8, dtype=torch.float64)
    assert got.shape == (2, n, d) and torch.equal(got, want)
    ref = oracle_mod.cheby_op((ip, ix.astype(np.int32), lv.astype(np.float64)), one.coeffs, S.cpu().numpy(), lmax)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("name", ["wav_rand", "wav_cora"])
def test_wavelet_basis_equals_reference_spectral_model(name):
    """The GPU wavelet basis against the REFERENCE's own SpectralModel.preprocess (golden wav_*,
    pygsp restated in the fixture generator): phi and phi^-1 bit for bit (fp64 recurrence, threshold,
    fp32 blocks, L1 normalisation), processed_feature = [X | relu(phi phi^-1 X)] within 1e-5 of its
    scale (the reference forms phi phi^-1 with a sparse-sparse product first; here phi (phi^-1 X))."""
    import golden_cases as G
    from srgnn.wavelet import spectral_features
    z = np.load(f"{G.GOLDEN}/{name}.npz", allow_pickle=False)
    n = z["adj_indptr"].size - 1
    adj = sp.csr_matrix((z["adj_data"], z["adj_indices"], z["adj_indptr"]), shape=(n, n))
    feat, phi, phi_inv, lmax = spectral_features(adj, z["x"], float(z["scale"]), int(z["order"]),
                                                 float(z["tolerance"]), lmax=float(z["lmax"]), device="cuda")
    for s, m in enumerate((phi, phi_inv)):
        m = sp.csr_matrix(m)
        np.testing.assert_array_equal(m.indptr, z[f"phi{s}_indptr"])
        np.testing.assert_array_equal(m.indices, z[f"phi{s}_indices"])
        assert np.array_equal(m.data, z[f"phi{s}_data"]), f"phi{s} values differ"
    want = z["processed_feature"]
    assert feat.shape == want.shape and feat.dtype == torch.float32
    np.testing.assert_allclose(feat.numpy(), want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
