"""Wavelet basis restatement (parity UNPINNED: pygsp is absent from the reference tree and this
image).  The oracle's Chebyshev recurrence is validated against a dense eigendecomposition, and the
product's host-side helpers (Laplacian, coefficients) against the oracle's independent versions."""
import numpy as np
import pytest
import scipy.sparse as sp

from srgnn import wavelet as W


def small_graph(n=40, seed=0, weighted=False):
    rng = np.random.default_rng(seed)
    m = rng.random((n, n)) < 0.12
    m = np.triu(m, 1)
    w = rng.integers(1, 5, size=(n, n)).astype(float) if weighted else np.ones((n, n))
    a = np.where(m, w, 0.0)
    a = a + a.T
    a[3, :] = a[:, 3] = 0.0                        # an isolated node
    return sp.csr_matrix(a)


def dense_cheby(Ld, coeffs, S, lmax):
    lam, U = np.linalg.eigh(Ld)
    a1 = a2 = lmax / 2
    x = (lam - a2) / a1
    T = [np.ones_like(x), x]
    for _ in range(2, coeffs.shape[1]):
        T.append(2 * x * T[-1] - T[-2])
    out = []
    for c in coeffs:
        p = 0.5 * c[0] * T[0] + sum(c[k] * T[k] for k in range(1, len(c)))
        out.append(U @ (p[:, None] * (U.T @ S)))
    return np.stack(out), lam, U


@pytest.mark.parametrize("weighted", [False, True])
def test_oracle_cheby_equals_dense_polynomial(oracle_mod, weighted):
    a = small_graph(weighted=weighted)
    n = a.shape[0]
    L = oracle_mod.laplacian(a.indptr, a.indices, a.data, n)
    Ld = sp.csr_matrix((L[2], L[1], L[0]), shape=(n, n)).toarray()
    lmax = float(np.linalg.eigvalsh(Ld).max()) * 1.01
    coeffs = np.stack([oracle_mod.cheby_coeffs(t, lmax, 3) for t in (-0.5, 0.5)])
    S = np.random.default_rng(1).standard_normal((n, 5))
    R = oracle_mod.cheby_op(L, coeffs, S, lmax)
    want, lam, U = dense_cheby(Ld, coeffs, S, lmax)
    np.testing.assert_allclose(R, want, rtol=1e-10, atol=1e-10)
    # and order 3 already approximates the heat kernel itself (loose: approximation error)
    heat = U @ (np.exp(-0.5 * lam / lmax)[:, None] * (U.T @ S))
    assert np.abs(R[1] - heat).max() < 5e-2 * np.abs(heat).max()


def test_laplacian_and_coefficients_match_oracle(oracle_mod):
    a = small_graph(weighted=True)
    # store a conflicting upper/lower pair: nx.Graph keeps the last stored (lower-triangle) weight
    a = a.tolil()
    a[5, 9], a[9, 5] = 2.0, 7.0
    a = a.tocsr()
    n = a.shape[0]
    L_prod = W._explicit_diagonal(W.laplacian_from_adj(a))
    ip, ix, v = oracle_mod.laplacian(a.indptr, a.indices, a.data, n)
    np.testing.assert_array_equal(L_prod.indptr, ip)
    np.testing.assert_array_equal(L_prod.indices, ix)
    np.testing.assert_array_equal(L_prod.data, v)
    assert L_prod[5, 9] == -7.0 and L_prod[9, 5] == -7.0
    for tau in (-0.5, 0.5, 2.0):
        np.testing.assert_array_equal(W.heat_cheby_coeffs(tau, 3.7, 3), oracle_mod.cheby_coeffs(tau, 3.7, 3))


def test_estimate_lmax_upper_bounds_spectrum():
    a = small_graph()
    L = W.laplacian_from_adj(a)
    lmax = W.estimate_lmax(L)
    true = np.linalg.eigvalsh(L.toarray()).max()
    assert true <= lmax <= true * 1.03


def test_device_laplacian_builder_matches_host_laplacian():
    """normalize.sym_norm_edges_blocked(kind="laplacian") == wavelet.laplacian_from_adj on the
    same binary symmetric graph (structure with the explicit diagonal, and values)."""
    import scipy.sparse as sp
    import torch
    from srgnn import normalize, synth, wavelet
    n, m = 3000, 15000
    u, v = synth.rmat_undirected_t(n, m, seed=9)
    ip, ix, lv = normalize.sym_norm_edges_blocked(u.to(torch.int32), v.to(torch.int32), n, kind="laplacian",
                                                  block_nnz=1 << 12)
    adj = sp.csr_matrix((np.ones(2 * m), (np.r_[u.numpy(), v.numpy()], np.r_[v.numpy(), u.numpy()])), shape=(n, n))
    L = wavelet.laplacian_from_adj(adj)
    np.testing.assert_array_equal(ip.numpy(), L.indptr)
    np.testing.assert_array_equal(ix.numpy(), L.indices)
    np.testing.assert_array_equal(lv.numpy(), L.data.astype(np.float32))


def test_l1_normalization_restatement_matches_sklearn():
    """The arithmetic srgnn.wavelet.l1_normalize_rows runs on the GPU (sequential fp64 sum of |x|,
    fp64 divide, round to fp32; empty rows kept), restated in numpy, equals sklearn's normalize."""
    import scipy.sparse as sp
    from sklearn.preprocessing import normalize
    rng = np.random.default_rng(3)
    M = sp.random(400, 300, density=0.2, format="csr", dtype=np.float32, random_state=4)
    M.data = (rng.random(M.nnz).astype(np.float32) * 3 - 1).astype(np.float32)
    M = sp.csr_matrix(M)
    got = M.copy()
    for i in range(M.shape[0]):
        lo, hi = M.indptr[i], M.indptr[i + 1]
        acc = 0.0
        for x in M.data[lo:hi].tolist():
            acc += abs(x)
        if acc != 0.0:
            got.data[lo:hi] = (M.data[lo:hi].astype(np.float64) / acc).astype(np.float32)
    want = normalize(M, norm="l1", axis=1)
    np.testing.assert_array_equal(got.data, want.data)


def _wavelet_golden(name):
    import golden_cases as G
    z = np.load(f"{G.GOLDEN}/{name}.npz", allow_pickle=False)
    n = z["adj_indptr"].size - 1
    adj = sp.csr_matrix((z["adj_data"], z["adj_indices"], z["adj_indptr"]), shape=(n, n))
    return z, adj, n


@pytest.mark.parametrize("name", ["wav_rand", "wav_cora"])
def test_oracle_wavelet_basis_equals_reference_spectral_model(oracle_mod, name):
    """phi and phi^-1 of the REFERENCE's own SpectralModel.preprocess (tests/golden/make_golden_wavelet.py:
    real networkx, its impulse batches, threshold, float32 blocks and sklearn normalisation; pygsp
    restated) equal the oracle's restatement bit for bit, with the fixture's lmax."""
    from sklearn.preprocessing import normalize
    z, adj, n = _wavelet_golden(name)
    lmax, scale, order, tol = float(z["lmax"]), float(z["scale"]), int(z["order"]), float(z["tolerance"])
    L = oracle_mod.laplacian(adj.indptr, adj.indices, adj.data, n)
    Lh = W.laplacian_from_adj(adj)
    assert np.array_equal(Lh.indptr, L[0]) and np.array_equal(Lh.indices, L[1]) and np.array_equal(Lh.data, L[2])
    coeffs = np.stack([oracle_mod.cheby_coeffs(t, lmax, order) for t in (-scale, scale)])
    blocks = [[], []]
    for c0 in range(0, n, 1000):
        w = min(1000, n - c0)
        S = np.zeros((n, w))
        S[np.arange(c0, c0 + w), np.arange(w)] = 1
        R = oracle_mod.cheby_op(L, coeffs, S, lmax)
        for s in range(2):
            sub = R[s].copy()
            sub[sub < tol] = 0
            blocks[s].append(sp.csr_matrix(sub.astype(np.float32)))
    for s in range(2):
        phi = normalize(sp.hstack(blocks[s]).tocsr(), norm="l1", axis=1)
        np.testing.assert_array_equal(phi.indptr, z[f"phi{s}_indptr"])
        np.testing.assert_array_equal(phi.indices, z[f"phi{s}_indices"])
        assert np.array_equal(phi.data, z[f"phi{s}_data"])
