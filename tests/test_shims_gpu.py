"""The wavelet model's third-party calls on the GPU through the package's pygsp / torch_sparse
(SSRG/models/base_scalable/base_model.py:180-265): the shim cheby_op against the oracle's
recurrence, spspmm / spmm against scipy's products of the same fp32 operands (the arithmetic of
torch_sparse's CPU kernels; torch_sparse itself is absent, so that part is parity-unpinned), and
SpectralModel.preprocess's call sequence end to end against the fixtures of the reference's own
preprocess (tests/golden/wav_*.npz)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wav(name):
    return np.load(os.path.join(REPO, "tests", "golden", name + ".npz"), allow_pickle=False)


def _adj(z):
    n = z["adj_indptr"].size - 1
    return sp.csr_matrix((z["adj_data"], z["adj_indices"], z["adj_indptr"]), shape=(n, n))


@pytest.mark.parametrize("name", ["wav_cora", "wav_rand"])
def test_cheby_op_bit_exact_vs_oracle(oracle_mod, name):
    """pygsp.filters.approximations.cheby_op on impulse batches (one scale, and two scales at once;
    the ragged last batch; a 1-D signal) == the oracle's fp64 recurrence, bit for bit."""
    import networkx as nx
    from pygsp import filters, graphs
    z = _wav(name)
    G = graphs.Graph(nx.adjacency_matrix(nx.Graph(_adj(z))))
    G.lmax = float(z["lmax"])
    m = int(z["order"])
    L = oracle_mod.laplacian(z["adj_indptr"], z["adj_indices"], z["adj_data"], G.N)
    cs = [filters.approximations.compute_cheby_coeff(filters.Heat(G, tau=[t]), m=m)
          for t in (-float(z["scale"]), float(z["scale"]))]
    n = G.N
    for c0, w in ((0, min(100, n)), (max(0, n - 37), min(37, n))):
        S = np.zeros((n, w))
        S[c0:c0 + w, :] = np.eye(w, dtype=int)
        for c in (cs[0], np.stack(cs)):
            got = filters.approximations.cheby_op(G, c, S)
            want = oracle_mod.cheby_op(L, c, S, G.lmax).reshape(-1, w)
            assert got.shape == want.shape
            np.testing.assert_array_equal(got, want)
    v = np.random.default_rng(3).standard_normal(n)
    got = filters.approximations.cheby_op(G, cs[1], v)
    assert got.shape == (n,)
    np.testing.assert_array_equal(got, oracle_mod.cheby_op(L, cs[1], v[:, None], G.lmax).reshape(-1))


def _spectral_preprocess(adj, feature, scale, order, tolerance, lmax):
    """SpectralModel.preprocess's calls (base_model.py:180-219, 236-265, 287-290) through the
    package's pygsp / torch_sparse, in the same order with the same arguments: nx graph ->
    pygsp Graph -> per scale Heat + compute_cheby_coeff + cheby_op on 1000-column impulse batches
    (ragged last batch), entries < tolerance zeroed, fp32 csr blocks, hstack -> sklearn L1 row
    normalisation -> COO index / value tensors via .nonzero() -> spspmm -> spmm -> relu -> concat.
    lmax is the fixture's (pygsp's ARPACK start vector is random)."""
    import networkx as nx
    import pygsp
    from sklearn.preprocessing import normalize
    from torch_sparse import spmm, spspmm
    Gx = nx.Graph(adj)
    G = pygsp.graphs.Graph(nx.adjacency_matrix(Gx))
    G.lmax = lmax
    n = Gx.number_of_nodes()
    phis = []
    for tau in (-scale, scale):
        c = pygsp.filters.approximations.compute_cheby_coeff(pygsp.filters.Heat(G, tau=[tau]), m=order)
        blocks = []
        for c0 in range(0, n, 1000):
            w = min(1000, n - c0)
            imp = np.zeros((n, w))
            imp[c0:c0 + w, :] = np.eye(w, dtype=int)
            co = pygsp.filters.approximations.cheby_op(G, c, imp)
            co[co < tolerance] = 0
            r, cc = co.nonzero()
            blocks.append(sp.csr_matrix((co[r, cc], (r, cc)), shape=(n, w), dtype=np.float32))
        phis.append(normalize(sp.hstack(blocks), norm="l1", axis=1))
    feat = torch.FloatTensor(feature)
    idx0 = torch.LongTensor(np.vstack(phis[0].nonzero()))
    val0 = torch.FloatTensor(np.asarray(phis[0][phis[0].nonzero()])).view(-1)
    idx1 = torch.LongTensor(np.vstack(phis[1].nonzero()))
    val1 = torch.FloatTensor(np.asarray(phis[1][phis[1].nonzero()])).view(-1)
    pi, pv = spspmm(idx0, val0, idx1, val1, n, n, n)
    loc = torch.nn.functional.relu(spmm(pi, pv, n, n, feat))
    return phis, torch.concat((feat, loc), dim=1), (pi, pv)


@pytest.mark.parametrize("name", ["wav_cora", "wav_rand"])
def test_spectral_preprocess_through_the_shims_matches_the_reference(name):
    """The reference's preprocess sequence on the package's pygsp / torch_sparse: phi, phi^-1 and
    processed_feature equal the reference's own outputs (fixtures), bit for bit."""
    z = _wav(name)
    phis, processed, (pi, pv) = _spectral_preprocess(_adj(z), z["x"], float(z["scale"]), int(z["order"]),
                                                     float(z["tolerance"]), float(z["lmax"]))
    for k in range(2):
        phi = sp.csr_matrix(phis[k])
        np.testing.assert_array_equal(phi.indptr, z[f"phi{k}_indptr"])
        np.testing.assert_array_equal(phi.indices, z[f"phi{k}_indices"])
        np.testing.assert_array_equal(phi.data.view(np.uint32), z[f"phi{k}_data"].view(np.uint32))
    assert pi.device.type == "cpu" and pv.dtype == torch.float32 and processed.device.type == "cpu"
    np.testing.assert_array_equal(processed.numpy().view(np.uint32), z["processed_feature"].view(np.uint32))


def _rand_csr(rng, m, n, density, dup_rows=False):
    A = sp.random(m, n, density=density, format="csr", random_state=rng, dtype=np.float32)
    A.data = (rng.standard_normal(A.nnz) * 2).astype(np.float32)
    A.data[rng.random(A.nnz) < 0.05] = 0.0                      # explicit zeros
    return A


def _coo(A):
    C = A.tocoo()
    return torch.from_numpy(np.vstack([C.row, C.col]).astype(np.int64)), torch.from_numpy(C.data.astype(np.float32))


@pytest.mark.parametrize("m,k,n,da,db", [(300, 250, 280, 0.05, 0.08), (2000, 1500, 40000, 0.003, 0.002),
                                         (1, 1, 1, 1.0, 1.0), (64, 30, 20000, 0.3, 0.01), (500, 400, 16384, 0.02, 0.02)])
def test_spspmm_equals_scipy_product(m, k, n, da, db):
    """torch_sparse.spspmm == scipy's fp32 A @ B (csr_matmat: products rounded, added in A's
    order, zero sums dropped) after sorting scipy's columns -- bit for bit, for the LDS accumulator
    (<= 16384 columns) and the scratch accumulator (more columns)."""
    import torch_sparse
    rng = np.random.default_rng(m + n)
    A, B = _rand_csr(rng, m, k, da), _rand_csr(rng, k, n, db)
    ia, va = _coo(A)
    ib, vb = _coo(B)
    idx, val = torch_sparse.spspmm(ia, va, ib, vb, m, k, n)
    C = (A @ B).tocsr()
    C.sort_indices()
    C = C.tocoo()
    keep = C.data != 0
    np.testing.assert_array_equal(idx[0].numpy(), C.row[keep])
    np.testing.assert_array_equal(idx[1].numpy(), C.col[keep])
    np.testing.assert_array_equal(val.numpy().view(np.uint32), C.data[keep].view(np.uint32))


def test_spspmm_unsorted_duplicates_and_coalesced():
    """B rows with repeated column ids (each B row walked in order by one lane) and coalesced=True
    with shuffled COO input (sorted by (row, col) first, duplicates kept)."""
    import torch_sparse
    rng = np.random.default_rng(7)
    m, k, n = 50, 40, 30
    rows = rng.integers(0, k, 600)
    cols = rng.integers(0, n, 600)
    order = np.lexsort((np.arange(600), rows))
    rows, cols = rows[order], cols[order]
    vb = rng.standard_normal(600).astype(np.float32)
    A = _rand_csr(rng, m, k, 0.2)
    ia, va = _coo(A)
    ib = torch.from_numpy(np.vstack([rows, cols]).astype(np.int64))
    idx, val = torch_sparse.spspmm(ia, va, ib, torch.from_numpy(vb), m, k, n)
    # host restatement: sums per (i, j) in A's order then B's stored order
    want = {}
    Ad = A.tocsr()
    for i in range(m):
        for e in range(Ad.indptr[i], Ad.indptr[i + 1]):
            kk, a = Ad.indices[e], Ad.data[e]
            for q in np.flatnonzero(rows == kk):
                key = (i, int(cols[q]))
                want[key] = np.float32(want.get(key, np.float32(0)) + np.float32(a * vb[q]))
    keys = sorted(kk for kk, v in want.items() if v != 0)
    np.testing.assert_array_equal(idx.numpy().T, np.array(keys).reshape(-1, 2))
    np.testing.assert_array_equal(val.numpy(), np.array([want[kk] for kk in keys], np.float32))
    # coalesced=True sorts both inputs by (row, col) and keeps duplicates (torch_sparse 0.6.x builds
    # SparseTensor(..., is_sorted=False), which sorts without summing): every duplicate's product is
    # rounded and added on its own, in the stably sorted order
    perm = rng.permutation(ia.shape[1])
    bperm = rng.permutation(rows.size)
    ib2 = ib[:, bperm]
    vb2 = vb[bperm]
    idx2, val2 = torch_sparse.spspmm(ia[:, perm], va[perm], ib2, torch.from_numpy(vb2), m, k, n, coalesced=True)
    r2, c2 = ib2[0].numpy(), ib2[1].numpy()
    bord = np.lexsort((np.arange(rows.size), c2, r2))   # stable by (row, col)
    brow = {}
    for q in bord:
        brow.setdefault(int(r2[q]), []).append((int(c2[q]), vb2[q]))
    want2 = {}
    As = Ad.sorted_indices()                    # A's entries by (row, col)
    for i in range(m):
        for e in range(As.indptr[i], As.indptr[i + 1]):
            kk, a = As.indices[e], As.data[e]
            for cc, v in brow.get(int(kk), []):
                key = (i, cc)
                want2[key] = np.float32(want2.get(key, np.float32(0)) + np.float32(a * v))
    keys2 = sorted(kk for kk, v in want2.items() if v != 0)
    assert len({(int(r), int(c)) for r, c in zip(rows, cols)}) < rows.size   # the fixture has duplicates
    np.testing.assert_array_equal(idx2.numpy().T, np.array(keys2).reshape(-1, 2))
    np.testing.assert_array_equal(val2.numpy(), np.array([want2[kk] for kk in keys2], np.float32))


@pytest.mark.parametrize("d", [1, 16, 64, 130])
def test_spmm_equals_scipy_and_scatter_add(d):
    """torch_sparse.spmm == scipy's csr @ dense (fp32, products added in index order from 0) and the
    index_select / mul / scatter_add composition on the CPU, bit for bit; the gradients of matrix
    and value match the same composition's autograd."""
    import torch_sparse
    rng = np.random.default_rng(d)
    m, n = 700, 500
    A = _rand_csr(rng, m, n, 0.02)
    idx, val = _coo(A)
    X = torch.from_numpy(rng.standard_normal((n, d)).astype(np.float32))
    got = torch_sparse.spmm(idx, val, m, n, X)
    want = np.asarray(A @ X.numpy(), dtype=np.float32)
    np.testing.assert_array_equal(got.numpy().view(np.uint32), want.view(np.uint32))
    ref = torch.zeros(m, d).index_add_(0, idx[0], X.index_select(0, idx[1]) * val.unsqueeze(-1))
    np.testing.assert_array_equal(got.numpy().view(np.uint32), ref.numpy().view(np.uint32))
    # gradients
    Xg, vg = X.clone().requires_grad_(True), val.clone().requires_grad_(True)
    g = torch.from_numpy(rng.standard_normal((m, d)).astype(np.float32))
    torch_sparse.spmm(idx, vg, m, n, Xg).backward(g)
    Xr, vr = X.clone().requires_grad_(True), val.clone().requires_grad_(True)
    torch.zeros(m, d).index_add(0, idx[0], Xr.index_select(0, idx[1]) * vr.unsqueeze(-1)).backward(g)
    np.testing.assert_array_equal(Xg.grad.numpy(), Xr.grad.numpy())
    # d-term dot products: the reduction order of the sum over columns is the device's
    torch.testing.assert_close(vg.grad, vr.grad, rtol=1e-5, atol=1e-5 * float(vr.grad.abs().max()))
    with pytest.raises(IndexError):            # torch_sparse asserts n == matrix.size(-2) first
        torch_sparse.spmm(idx, val, m, n, X[:, 0])


def test_coalesce_sorts_and_sums_in_order():
    import torch_sparse
    idx = torch.tensor([[2, 0, 2, 1, 0], [1, 3, 1, 0, 3]])
    val = torch.tensor([1.0, 2.0, 3.0, 4.0, 5.0])
    i, v = torch_sparse.coalesce(idx, val, 3, 4)
    assert i.tolist() == [[0, 1, 2], [3, 0, 1]] and v.tolist() == [7.0, 4.0, 4.0]
    i2, v2 = torch_sparse.coalesce(idx, torch.stack([val, -val], 1), 3, 4)
    assert torch.equal(i2, i) and v2[:, 1].tolist() == [-7.0, -4.0, -4.0]


def test_sparse_products_edge_cases():
    """Empty operands, rows without entries, products that cancel to zero (dropped, as scipy and
    torch_sparse drop them), a single entry, and an empty sparse operand in spmm."""
    import torch_sparse
    e = torch.zeros((2, 0), dtype=torch.int64)
    ev = torch.zeros(0)
    idx, val = torch_sparse.spspmm(e, ev, e, ev, 5, 4, 3)
    assert idx.shape == (2, 0) and val.numel() == 0
    # a @ b where two products cancel exactly: (1 * 2) + (-1 * 2) = 0 -> dropped
    ia = torch.tensor([[0, 0, 2], [0, 1, 1]])
    va = torch.tensor([1.0, -1.0, 3.0])
    ib = torch.tensor([[0, 1, 1], [2, 2, 0]])
    vb = torch.tensor([2.0, 2.0, 5.0])
    idx, val = torch_sparse.spspmm(ia, va, ib, vb, 3, 2, 3)
    assert idx.tolist() == [[0, 2, 2], [0, 0, 2]] and val.tolist() == [-5.0, 15.0, 6.0]
    one_i, one_v = torch_sparse.spspmm(torch.tensor([[0], [0]]), torch.tensor([3.0]), torch.tensor([[0], [0]]),
                                       torch.tensor([0.5]), 1, 1, 1)
    assert one_i.tolist() == [[0], [0]] and one_v.tolist() == [1.5]
    y = torch_sparse.spmm(e, ev, 4, 3, torch.ones(3, 2))
    assert y.shape == (4, 2) and bool((y == 0).all())


def test_sparse_products_reject_bad_csr_and_out():
    """srgnn.sparse validates what its kernels trust: row pointers from 0 to nnz without decreasing,
    ids and values of one length, and an `out` of the product's shape (ValueError, nothing launched)."""
    from srgnn import sparse as S
    ip = torch.tensor([0, 2, 3], dtype=torch.int64, device="cuda")
    ix = torch.tensor([0, 1, 1], dtype=torch.int32, device="cuda")
    v = torch.tensor([1.0, 2.0, 3.0], device="cuda")
    X = torch.ones((2, 4), device="cuda")
    assert torch.equal(S.spmm_scatter(ip, ix, v, X), torch.tensor([[3.0] * 4, [3.0] * 4], device="cuda"))
    for bad in (torch.tensor([0, 2, 4], dtype=torch.int64, device="cuda"),     # ends past nnz
                torch.tensor([0, 3, 2], dtype=torch.int64, device="cuda"),     # decreasing
                torch.tensor([1, 2, 3], dtype=torch.int64, device="cuda")):    # does not start at 0
        with pytest.raises(ValueError):
            S.spmm_scatter(bad, ix, v, X)
        with pytest.raises(ValueError):
            S.spgemm(bad, ix, v, ip, ix, v, 2)
    with pytest.raises(ValueError):
        S.spmm_scatter(ip, ix, v[:2], X)
    for out in (torch.empty((1, 4), device="cuda"), torch.empty((2, 3), device="cuda"),
                torch.empty((4, 2), device="cuda").t(), torch.empty((2, 4), dtype=torch.float64, device="cuda")):
        with pytest.raises(ValueError):
            S.spmm_scatter(ip, ix, v, X, out=out)
