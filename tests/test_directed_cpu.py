"""Host logic of the directed families' construct_adj (srgnn.directed), run here on torch CPU tensors
with the oracle's sequential segment sum and fp64 scipy-order product standing in for
srg_segment_sum_f64/_f32 and srg_spmm_csr_f64, against the REFERENCE's own operators
(tests/golden/dir_*.npz, made by tests/golden/make_golden_directed.py).

Bit-identical: the magnetic Laplacian (two parameter sets), the complex PPR operator, the PyG-SD
magnetic variant (one documented diagonal entry aside) and the undirected part of the in/out
operator.  Tolerance (the reference's values come from CPU BLAS / LAPACK reductions): the in/out
second-order operators, the fast PPR operator and the second-order two-order operator to 2e-6
relative (a few fp32 ulps; the same sparsity exactly); the first-order two-order operator to 1e-3
relative against the reference (its stationary vector is an fp32 sgeev eigenvector) and to 1e-6
against the fp64 stationary vector of a dense eigendecomposition."""
import numpy as np
import pytest
import torch

import golden_cases as G
from srgnn import directed as D

EXACT_TOL = {"mag_lap": 0, "mag_lap_q01_r03": 0, "mag_comppr": 0, "pygsd_mag": 0}
ULP_RTOL = 2e-6


@pytest.fixture(scope="module")
def standins(oracle_mod):
    def segsum(ptr, v):
        return torch.from_numpy(oracle_mod.segment_sum(ptr.numpy(), v.numpy()))

    def spmv(ip, ix, v, x):
        return torch.from_numpy(oracle_mod.spmm64(ip.numpy(), ix.numpy(), v.numpy(), x.numpy()))
    return segsum, spmv


def directed_cases():
    return [k for k in G.names() if k.startswith("dir_")]


def build(name, segsum, spmv):
    c = G.Case(name)
    kw, n, op = c.meta["kwargs"], c.n, c.meta["operator"]
    a = c.adj().tocoo()
    if op in ("mag_lap", "mag_lap_q01_r03"):
        mats = D.magnetic_norm(a.row, a.col, a.data, n, kw["r"], kw["q"], device="cpu", segsum=segsum)
    elif op == "mag_comppr":
        mats = D.magnetic_com_ppr(a.row, a.col, a.data, n, kw["r"], kw["q"], kw["ppr_alpha"], device="cpu",
                                  segsum=segsum)
    elif op == "pygsd_mag":
        mats = D.pygsd_magnetic_norm(a.row, a.col, a.data, n, kw["r"], kw["q"], device="cpu", segsum=segsum)
    elif op == "two_dir":
        mats = D.in_out_norm(a.row, a.col, n, kw["r"], device="cpu", segsum=segsum)
    elif op == "fast_ppr":
        mats = (D.fast_ppr_norm(a.row, a.col, n, kw["r"], kw["ppr_alpha"], device="cpu", segsum=segsum, spmv=spmv),)
    else:
        mats = D.two_order_norm(a.row, a.col, n, kw["r"], kw["ppr_alpha"], device="cpu", segsum=segsum, spmv=spmv)
    return c, dict(zip(c.meta["matrices"], mats))


def pygsd_known_entries(c, ip):
    """Diagonal entries scipy sums from three duplicates (a stored self-loop, +1, -1) in a row of
    more than 16 stored entries: their order is that of libstdc++'s introsort, not input order."""
    adj = c.adj()
    rows = [i for i in range(c.n) if adj[i, i] != 0 and ip[i + 1] - ip[i] > 16]
    return rows


@pytest.mark.parametrize("name", directed_cases())
def test_directed_norm_matches_reference(standins, name):
    c, got = build(name, *standins)
    op = c.meta["operator"]
    for m, (ip, ix, v) in got.items():
        np.testing.assert_array_equal(ip.numpy(), c[f"m_{m}_indptr"], err_msg=f"{name} {m} indptr")
        np.testing.assert_array_equal(ix.numpy(), c[f"m_{m}_indices"], err_msg=f"{name} {m} indices")
        want = c[f"m_{m}_data"]
        v = v.numpy()
        assert v.dtype == want.dtype, (name, m, v.dtype, want.dtype)
        if op in EXACT_TOL or (op == "two_dir" and m == "un"):
            if op == "pygsd_mag" and m == "real":
                ipn = ip.numpy()
                skip = np.zeros(v.size, dtype=bool)
                for r in pygsd_known_entries(c, ipn):
                    row = slice(ipn[r], ipn[r + 1])
                    skip[row] = ix.numpy()[row] == r
                np.testing.assert_allclose(v[skip], want[skip], rtol=0, atol=4.5e-16)   # (x + 1) - 1 vs (x - 1) + 1: ulp(1)
                v, want = v[~skip], want[~skip]
            assert np.array_equal(v.view(np.uint8), want.view(np.uint8)), f"{name} {m}: not bit-identical"
        elif op == "two_order" and m == "one":
            np.testing.assert_allclose(v, want, rtol=1e-3, err_msg=f"{name} {m}")
        else:
            np.testing.assert_allclose(v, want, rtol=ULP_RTOL, err_msg=f"{name} {m}")


def test_two_order_stationary_vector_equals_dense_eigenvector(standins):
    """The fp64 power iteration's fixed point equals the left Perron vector of the reference's
    (N+1) x (N+1) chain (utils.py:338-356), computed here by a dense fp64 eigendecomposition."""
    import scipy.linalg
    segsum, spmv = standins
    c = G.Case("dir_rand_two_order")
    n, alpha = c.n, c.meta["kwargs"]["ppr_alpha"]
    a = c.adj().tocoo()
    R, C, ew = D._loops_appended(torch.from_numpy(a.row.astype(np.int64)), torch.from_numpy(a.col.astype(np.int64)),
                                 n, torch.device("cpu"))
    deg = D._row_scatter(R, ew, n, segsum)
    inv = D._host_pow(deg, -1)
    pip, pix, pv = D._csr_from_coo(R, C, inv[R] * ew, n, segsum)
    P = np.zeros((n, n))
    rows = np.repeat(np.arange(n), np.diff(pip.numpy()))
    P[rows, pix.numpy()] = pv.numpy()
    Pv = np.zeros((n + 1, n + 1))
    Pv[:n, :n] = (1 - alpha) * P
    Pv[n, :n] = 1.0 / n
    Pv[:n, n] = alpha
    w, vl = scipy.linalg.eig(Pv, left=True, right=False)
    want = vl[:, np.argmax(w.real)].real[:n]
    want = want / want.sum()
    prow = torch.from_numpy(rows)
    key, perm = torch.sort(pix.to(torch.int64) * n + prow, stable=True)
    got = D._stationary(D._indptr(key // n, n), (key % n).to(torch.int32), pv[perm].to(torch.float64), n, alpha, spmv)
    np.testing.assert_allclose(got.numpy(), want, rtol=1e-9)


def test_oracle_segment_sum_is_sequential(oracle_mod):
    v = np.array([1e16, 1.0, -1e16, 1.0, 3.0], dtype=np.float64)
    out = oracle_mod.segment_sum(np.array([0, 3, 5]), v)
    assert out[0] == ((0.0 + 1e16) + 1.0) + -1e16 and out[1] == 4.0
    v32 = np.array([1e8, 1.0, -1e8], dtype=np.float32)
    assert oracle_mod.segment_sum(np.array([0, 3]), v32).dtype == np.float32


def test_dense_steps_refuse_huge_graphs():
    row = torch.zeros(1, dtype=torch.int64)
    with pytest.raises(ValueError, match="dense"):
        D.in_out_norm(row, row, D._DENSE_LIMIT + 1, 0.5, device="cpu",
                      segsum=lambda p, v: torch.zeros(p.numel() - 1, dtype=v.dtype))
