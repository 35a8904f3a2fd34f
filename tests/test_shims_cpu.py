"""The pygsp / torch_sparse API surface the reference's wavelet model imports (package directory on
sys.path): host-side pieces on the CPU, and that the product entry points refuse to run without a
HIP device (no CPU fallback).  The GPU results are tests/test_shims_gpu.py."""
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "scalable-roubust-gnn_amd")
REF = "/root/reference/Scalable Spectral Robust GNN"


def _wav(name):
    return np.load(os.path.join(REPO, "tests", "golden", name + ".npz"), allow_pickle=False)


def test_shim_modules_resolve_to_the_package():
    import pygsp
    import torch_sparse
    assert os.path.realpath(pygsp.__file__).startswith(os.path.realpath(PKG))
    assert os.path.realpath(torch_sparse.__file__).startswith(os.path.realpath(PKG))
    from pygsp.filters import approximations
    assert callable(approximations.cheby_op) and callable(approximations.compute_cheby_coeff)
    assert callable(torch_sparse.spspmm) and callable(torch_sparse.spmm) and callable(torch_sparse.coalesce)


@pytest.mark.parametrize("name", ["wav_cora", "wav_rand"])
def test_graph_laplacian_lmax_and_coefficients(oracle_mod, name):
    """Graph(W) of nx.adjacency_matrix(nx.Graph(adj)) (what SpectralModel passes): L = D - W;
    estimate_lmax reproduces the fixture's lmax (same estimator and start vector); the Heat
    filter's Chebyshev coefficients equal the oracle's restatement bit for bit."""
    import networkx as nx
    from pygsp import filters, graphs
    z = _wav(name)
    n = z["adj_indptr"].size - 1
    adj = sp.csr_matrix((z["adj_data"], z["adj_indices"], z["adj_indptr"]), shape=(n, n))
    W = nx.adjacency_matrix(nx.Graph(adj))
    G = graphs.Graph(W)
    assert G.N == n
    Wd = sp.csr_matrix(W).toarray().astype(np.float64)
    np.testing.assert_array_equal(G.L.toarray(), np.diag(Wd.sum(0)) - Wd)
    # the oracle's Laplacian (nx semantics from the raw adjacency) has the same entries
    ip, ix, lv = oracle_mod.laplacian(z["adj_indptr"], z["adj_indices"], z["adj_data"], n)
    np.testing.assert_array_equal(sp.csr_matrix((lv, ix, ip), shape=(n, n)).toarray(), G.L.toarray())
    assert G.estimate_lmax() == float(z["lmax"])
    for tau in (-float(z["scale"]), float(z["scale"])):
        f = filters.Heat(G, tau=[tau])
        c = filters.approximations.compute_cheby_coeff(f, m=int(z["order"]))
        np.testing.assert_array_equal(c, oracle_mod.cheby_coeffs(tau, float(z["lmax"]), int(z["order"])))
        x = np.linspace(0, G.lmax, 7)
        np.testing.assert_array_equal(f.evaluate(x)[0], np.exp(-tau * x / G.lmax))


def test_product_entries_fail_loudly_without_a_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    import torch_sparse
    from pygsp import graphs
    from pygsp.filters import approximations
    G = graphs.Graph(sp.csr_matrix(np.array([[0, 1.0], [1.0, 0]])))
    G.lmax = 2.0
    with pytest.raises(RuntimeError):
        approximations.cheby_op(G, [1.0, 0.5, 0.25], np.eye(2))
    idx = torch.tensor([[0, 1], [1, 0]])
    val = torch.ones(2)
    with pytest.raises(RuntimeError):
        torch_sparse.spspmm(idx, val, idx, val, 2, 2, 2)
    with pytest.raises(RuntimeError):
        torch_sparse.spmm(idx, val, 2, 2, torch.ones(2, 3))
    with pytest.raises(TypeError):
        approximations.cheby_op(G, [1.0], np.eye(2))        # pygsp: fewer than 2 coefficients


_IMPORT_REFERENCE_MODEL = r"""
import os, sys, tempfile
sys.pycache_prefix = tempfile.mkdtemp()          # nothing read from or written next to the reference
sys.path[:0] = [sys.argv[1], sys.argv[2]]        # this package first, then the reference's root
import models.base_scalable.base_model as bm
import pygsp, torch_sparse
assert bm.pygsp is pygsp and pygsp.__file__.startswith(sys.argv[1]), pygsp.__file__
assert bm.spspmm is torch_sparse.spspmm and bm.spmm is torch_sparse.spmm
import models.base_scalable.simple_models as smod
assert smod.spspmm is torch_sparse.spspmm
print("ok", bm.SpectralModel.__name__)
"""


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is only in the development container")
def test_reference_wavelet_model_imports_with_the_shims():
    """The unchanged reference model modules (base_model.py:9,13; simple_models.py:3) import with
    this package on sys.path, and their pygsp / spspmm / spmm names are the HIP-backed ones."""
    r = subprocess.run([sys.executable, "-c", _IMPORT_REFERENCE_MODEL, PKG, REF], capture_output=True,
                       timeout=300, env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert r.stdout.decode().strip().endswith("ok SpectralModel")
