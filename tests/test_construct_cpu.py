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


@pytest.mark.parametrize("name", [n for n in G.names("norm") if G.manifest()[n]["n"] <= 5000])
def test_sym_and_ppr_equal_reference(oracle_mod, name):
    c = G.Case(name)
    a = c.adj()
    r = c.meta["r"]
    if c.meta["op"] == "ppr":
        ip, ix, v = C.ppr_norm(a.indptr, a.indices, a.data, c.n, r, c.meta["alpha"], device="cpu", segsum=segsum_np)
    else:
        ip, ix, v = C.sym_norm(a.indptr, a.indices, a.data, c.n, r, device="cpu", segsum=segsum_np)
    np.testing.assert_array_equal(ip.numpy(), c["ahat_indptr"])
    np.testing.assert_array_equal(ix.numpy(), c["ahat_indices"])
    np.testing.assert_array_equal(v.numpy(), c["ahat_data64"])


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
