"""Golden fixtures for the wavelet basis: the REFERENCE's own SpectralModel.preprocess
(SSRG/models/base_scalable/base_model.py:171-219, 236-265, 287-290), run in the development container.

    python tests/golden/make_golden_wavelet.py

What runs unmodified: SpectralModel.preprocess, calculate_wavelet (1000-column impulse batches, the
`< tolerance` threshold, float32 csr blocks, hstack), normalize_matrices (sklearn), the feature
handling and the phi phi^-1 X product, with the real networkx (nx.Graph(adj), nx.adjacency_matrix).

Stubs (test infrastructure; the libraries are absent from the image and the reference pins no versions):
  * pygsp 0.5.x, restated from its published source:
      graphs.Graph(W): combinatorial L = diag(W.sum(0)) - W, stored CSC;
      Graph.estimate_lmax(): pygsp takes the largest eigenvalue from ARPACK (eigsh, tol 5e-3, random
        start) times 1.01 -- not reproducible; the stub uses a fixed start vector and stores the
        value, which the tests pass to the build as its explicit lmax input;
      filters.Heat(G, tau=[t]): kernel exp(-t x / lmax);
      filters.approximations.compute_cheby_coeff(f, m): N = m + 1 Chebyshev nodes on [0, lmax];
      filters.approximations.cheby_op(G, c, S): T0 = S, T1 = (L S - a2 S) / a1,
        T_{k+1} = (2/a1)(L - a2 I) T_k - T_{k-1}, r = c0/2 T0 + sum c_k T_k, a1 = a2 = lmax / 2;
  * torch_sparse spspmm / spmm: the sparse product phi @ phi^-1 and its product with X, through scipy
    (fp32); the build evaluates phi (phi^-1 X) instead, so that output is compared within tolerance;
  * tqdm (unused here) and the operators stubs of make_golden.py.
Only data is written: the inputs, lmax, phi and phi^-1 (csr arrays) and processed_feature.
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import scipy.sparse as sparse
import scipy.sparse.linalg as sla
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402


def _pygsp_stub():
    pygsp = types.ModuleType("pygsp")
    graphs = types.ModuleType("pygsp.graphs")
    filters = types.ModuleType("pygsp.filters")
    approximations = types.ModuleType("pygsp.filters.approximations")

    class Graph:
        def __init__(self, W, lap_type="combinatorial"):
            self.W = sparse.lil_matrix(W)
            self.N = W.shape[0]
            deg = np.ravel(self.W.sum(0))
            self.L = (sparse.diags(deg, 0) - self.W).tocsc()

        def estimate_lmax(self):
            v0 = np.ones(self.N) / np.sqrt(self.N)
            lmax = sla.eigsh(self.L, k=1, tol=5e-3, ncv=min(self.N, 10), v0=v0, return_eigenvectors=False)[0]
            self.lmax = float(np.real(lmax) * 1.01)

    class Heat:
        def __init__(self, G, tau=10, normalize=False):
            taus = tau if isinstance(tau, (list, tuple, np.ndarray)) else [tau]
            self.G = G
            self._kernels = [lambda x, t=t: np.exp(-t * x / G.lmax) for t in taus]

    def compute_cheby_coeff(f, m=30, N=None, i=0):
        G = f.G
        if not N:
            N = m + 1
        a1 = (G.lmax - 0) / 2
        a2 = (G.lmax + 0) / 2
        c = np.zeros(m + 1)
        tmpN = np.arange(N)
        num = np.cos(np.pi * (tmpN + 0.5) / N)
        for o in range(m + 1):
            c[o] = 2. / N * np.dot(f._kernels[i](a1 * num + a2), np.cos(np.pi * o * (tmpN + 0.5) / N))
        return c

    def cheby_op(G, c, signal):
        c = np.atleast_2d(np.array(c))
        n_scales, M = c.shape
        if M < 2:
            raise TypeError("The coefficients have an invalid shape")
        r = np.zeros((G.N * n_scales, np.shape(signal)[1])) if np.ndim(signal) > 1 else np.zeros(G.N * n_scales)
        a1 = float(G.lmax - 0) / 2.
        a2 = float(G.lmax + 0) / 2.
        twf_old = signal
        twf_cur = (G.L.dot(signal) - a2 * signal) / a1
        rows = np.arange(G.N, dtype=int)
        for i in range(n_scales):
            r[rows + G.N * i] = 0.5 * c[i, 0] * twf_old + c[i, 1] * twf_cur
        factor = 2 / a1 * (G.L - a2 * sparse.eye(G.N))
        for k in range(2, M):
            twf_new = factor.dot(twf_cur) - twf_old
            for i in range(n_scales):
                r[rows + G.N * i] += c[i, k] * twf_new
            twf_old = twf_cur
            twf_cur = twf_new
        return r

    graphs.Graph = Graph
    filters.Heat = Heat
    approximations.compute_cheby_coeff = compute_cheby_coeff
    approximations.cheby_op = cheby_op
    filters.approximations = approximations
    pygsp.graphs, pygsp.filters = graphs, filters
    return {"pygsp": pygsp, "pygsp.graphs": graphs, "pygsp.filters": filters,
            "pygsp.filters.approximations": approximations}


def _torch_sparse_products(mod):
    def spspmm(indexA, valueA, indexB, valueB, m, k, n, coalesced=False):
        A = sparse.csr_matrix((valueA.numpy(), (indexA[0].numpy(), indexA[1].numpy())), shape=(m, k))
        B = sparse.csr_matrix((valueB.numpy(), (indexB[0].numpy(), indexB[1].numpy())), shape=(k, n))
        C = (A @ B).tocoo()
        order = np.lexsort((C.col, C.row))
        idx = torch.from_numpy(np.vstack((C.row[order], C.col[order])).astype(np.int64))
        return idx, torch.from_numpy(C.data[order].astype(np.float32))

    def spmm(index, value, m, n, matrix):
        A = sparse.csr_matrix((value.numpy(), (index[0].numpy(), index[1].numpy())), shape=(m, n))
        return torch.from_numpy(np.asarray(A @ matrix.numpy(), dtype=np.float32))
    mod.spspmm, mod.spmm = spspmm, spmm


def directed_weighted(n, density, seed):
    """A small graph with weights, reciprocal edges of different weight, self-loops and isolated nodes
    (nx.Graph keeps one weight per pair: the last one it is given)."""
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < density
    mask[[4, n - 5], :] = False
    mask[:, [4, n - 5]] = False
    np.fill_diagonal(mask, rng.random(n) < 0.1)
    w = rng.integers(1, 9, size=(n, n)) / 2.0
    return sparse.csr_matrix(np.where(mask, w, 0.0))


def main():
    MG.import_reference()
    sys.modules.update(_pygsp_stub())
    if "tqdm" not in sys.modules:
        try:
            import tqdm  # noqa: F401
        except ImportError:
            sys.modules["tqdm"] = types.ModuleType("tqdm")
    import torch_sparse
    _torch_sparse_products(torch_sparse)
    from models.base_scalable.base_model import SpectralModel
    synth = MG._load_synth()
    cases = {}
    adj, _ = MG.planetoid_adj("cora_0_0", True)
    cases["wav_cora"] = (adj, synth.uniform_features_np(adj.shape[0], 16, seed=90), 0.5, 3, 1e-4)
    adj = directed_weighted(130, 0.05, seed=91)
    cases["wav_rand"] = (adj, synth.uniform_features_np(130, 8, seed=92), 0.7, 4, 1e-3)
    for name, (adj, X, scale, order, tol) in cases.items():
        model = SpectralModel(scale, order, tol)
        model.preprocess(adj, X)
        arrs = {"adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int32),
                "adj_data": adj.data.astype(np.float64), "x": X, "lmax": np.array(model.pygsp_graph.lmax),
                "scale": np.array(scale), "order": np.array(order), "tolerance": np.array(tol),
                "processed_feature": model.processed_feature.numpy()}
        for k, phi in enumerate(model.phi_matrices):
            phi = sparse.csr_matrix(phi)
            arrs[f"phi{k}_indptr"] = phi.indptr.astype(np.int64)
            arrs[f"phi{k}_indices"] = phi.indices.astype(np.int32)
            arrs[f"phi{k}_data"] = phi.data
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print(name, "n", adj.shape[0], "lmax", model.pygsp_graph.lmax, "phi nnz", [m.nnz for m in model.phi_matrices],
              flush=True)


if __name__ == "__main__":
    tempfile.tempdir = None
    main()
