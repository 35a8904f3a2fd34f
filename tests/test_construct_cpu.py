"""Host logic of the device construct_adj (srgnn.construct), run here with torch CPU tensors and a
numpy sequential segment sum in place of srg_segment_sum_f64: equal to the oracle's restatement
and to the reference's Â stored in the golden fixtures, bit for bit."""
import numpy as np
import pytest
import torch

import golden_cases as G
from srgnn import construct as C


def segsum_np(ptr, vals):
    p, v = ptr.numpy(), vals.numpy()
    out = np.zeros(p.size - 1)
    for s in range(p.size - 1):
        acc = 0.0
        for j in range(p[s], p[s + 1]):
            acc += v[j]
        out[s] = acc
    return torch.from_numpy(out)


def mirror_np(indptr, indices32, rows):
    """srg_csr_mirror restated: position of (c, r) in row c for each entry (r, c), or -1."""
    ip, ix, rw = indptr.numpy(), indices32.numpy(), rows.numpy()
    out = np.full(ix.size, -1, dtype=np.int64)
    for e in range(ix.size):
        c = ix[e]
        k = ip[c] + np.searchsorted(ix[ip[c]:ip[c + 1]], rw[e])
        if k < ip[c + 1] and ix[k] == rw[e]:
            out[e] = k
    return torch.from_numpy(out)


@pytest.mark.parametrize("fast", [False, True])
@pytest.mark.parametrize("name", [n for n in G.names("norm") if G.manifest()[n]["n"] <= 5000])
def test_sym_and_ppr_equal_reference(oracle_mod, name, fast):
    """The general path (sorts) and the fast path (diagonal merged in place for canonical input;
    the transpose from mirror positions for a symmetric structure) both give the reference's Â."""
    c = G.Case(name)
    a = c.adj()
    r = c.meta["r"]
    kw = dict(device="cpu", segsum=segsum_np, mirror=mirror_np, fast=fast)
    if c.meta["op"] == "ppr":
        ip, ix, v = C.ppr_norm(a.indptr, a.indices, a.data, c.n, r, c.meta["alpha"], **kw)
    else:
        ip, ix, v = C.sym_norm(a.indptr, a.indices, a.data, c.n, r, **kw)
    np.testing.assert_array_equal(ip.numpy(), c["ahat_indptr"])
    np.testing.assert_array_equal(ix.numpy(), c["ahat_indices"])
    np.testing.assert_array_equal(v.numpy(), c["ahat_data64"])


def test_fast_paths_taken_and_refused():
    """Which inputs take the in-place A+I merge: canonical ones (with or without stored diagonal
    entries); not unsorted rows, duplicates, explicit zeros, or a diagonal entry of -1 (A+I drops
    it to zero)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(3)
    n = 60
    d = sp.random(n, n, density=0.1, random_state=4, format="csr")
    d.data[:] = rng.random(d.nnz) + 0.5
    d = d + d.T
    d.setdiag(0.0)
    d.eliminate_zeros()
    d.sort_indices()

    def api(a):
        ip = torch.from_numpy(a.indptr.astype(np.int64))
        ix = torch.from_numpy(a.indices.astype(np.int64))
        rows = torch.repeat_interleave(torch.arange(n), ip[1:] - ip[:-1])
        return C._canonical_plus_identity(ip, ix, torch.from_numpy(a.data.astype(np.float64)), rows, n)

    for a in (d, d + sp.identity(n, format="csr") * 0.25):
        a = sp.csr_matrix(a)
        a.sort_indices()
        got = api(a)
        assert got is not None
        want = sp.csr_matrix(a + sp.identity(n, format="csr"))
        np.testing.assert_array_equal(got[0].numpy(), want.indptr)
        np.testing.assert_array_equal(got[1].numpy(), want.indices)
        np.testing.assert_array_equal(got[2].numpy(), want.data)
    neg = sp.csr_matrix(d + sp.identity(n, format="csr") * -1.0)
    neg.sort_indices()
    assert api(neg) is None
    zero = d.copy()
    zero.data[3] = 0.0
    assert api(zero) is None
    unsorted = d.copy()
    unsorted.indices[unsorted.indptr[5]:unsorted.indptr[6]] = unsorted.indices[unsorted.indptr[5]:unsorted.indptr[6]][::-1]
    assert d.indptr[6] - d.indptr[5] < 2 or api(unsorted) is None


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_weighted_noncanonical_equal_oracle(oracle_mod, seed):
    """Unsorted rows with duplicates and non-integer weights: the restatement's order."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    n, m = 200, 1500
    r, c = rng.integers(0, n, m), rng.integers(0, n, m)
    v = rng.random(m) * 3 - 1
    order = np.lexsort((rng.random(m), r))
    r, c, v = r[order], c[order], v[order]
    ptr = np.r_[0, np.cumsum(np.bincount(r, minlength=n))]
    for rr in (0.5, 0.3, 1.0):
        ip, ix, vals = C.sym_norm(ptr, c.astype(np.int32), v, n, rr, device="cpu", segsum=segsum_np)
        want = oracle_mod.sym_norm(ptr, c, v, n, rr)
        np.testing.assert_array_equal(ip.numpy(), want[0])
        np.testing.assert_array_equal(ix.numpy(), want[1])
        np.testing.assert_array_equal(vals.numpy(), want[2])
        want = oracle_mod.ppr_norm(ptr, c, v, n, rr, 0.15)
        ip, ix, vals = C.ppr_norm(ptr, c.astype(np.int32), v, n, rr, 0.15, device="cpu", segsum=segsum_np)
        np.testing.assert_array_equal(vals.numpy(), want[2])
        np.testing.assert_array_equal(ix.numpy(), want[1])


def test_edge_index_ingestion_equals_scipy():
    """edge_index.pt (Cora, int64 [2, E] upper triangle) -> csr_matrix((ones, (row, col))), as
    stored and symmetrised."""
    import os
    import scipy.sparse as sp
    c = G.Case("cora_asstored_k3")
    a = c.adj()
    coo = a.tocoo()
    e = np.stack([coo.row, coo.col]).astype(np.int64)
    for sym in (False, True):
        ip, ix, v = C.edge_index_to_adj(e, c.n, symmetric=sym, device="cpu", segsum=segsum_np)
        row, col = (np.r_[e[0], e[1]], np.r_[e[1], e[0]]) if sym else (e[0], e[1])
        want = sp.csr_matrix((np.ones(row.size), (row, col)), shape=(c.n, c.n))
        np.testing.assert_array_equal(ip.numpy(), want.indptr)
        np.testing.assert_array_equal(ix.numpy(), want.indices)
        np.testing.assert_array_equal(v.numpy(), want.data)
    with pytest.raises(ValueError):
        C.edge_index_to_adj(np.array([[0, 1], [2, c.n]]), c.n, device="cpu", segsum=segsum_np)
