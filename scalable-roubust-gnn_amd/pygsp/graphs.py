"""pygsp.graphs.Graph (0.5.x restated): a weighted undirected graph and its combinatorial Laplacian.

Only what the reference's wavelet model reads is provided: Graph(W), N, W, L, d, Ne, lmax,
estimate_lmax().  L = diag(W.sum(0)) - W, stored CSC as pygsp stores it.  The device copy of L that
cheby_op runs on (CSR, every diagonal slot stored) is built once per graph.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sparse


class Graph:
    """pygsp.graphs.Graph(W, lap_type='combinatorial')."""

    def __init__(self, W, lap_type="combinatorial", coords=None, plotting=None, **kwargs):
        if lap_type != "combinatorial":
            raise NotImplementedError(f"lap_type={lap_type!r}: the wavelet model uses the combinatorial Laplacian")
        if W.shape[0] != W.shape[1]:
            raise ValueError("W must be a square matrix")
        self.lap_type = lap_type
        self.W = sparse.lil_matrix(W)
        self.N = W.shape[0]
        self.coords = coords
        self.plotting = plotting or {}
        deg = np.ravel(self.W.sum(0))
        self.d = deg
        self.dw = deg
        self.L = (sparse.diags(deg, 0) - self.W).tocsc()
        Wc = sparse.csr_matrix(self.W)
        self.Ne = int((Wc.nnz + int(np.count_nonzero(Wc.diagonal()))) // 2)
        self._lmax = None
        self._device_L = None

    # -- largest eigenvalue ------------------------------------------------------------------------
    @property
    def lmax(self):
        if self._lmax is None:
            self.estimate_lmax()
        return self._lmax

    @lmax.setter
    def lmax(self, value):
        self._lmax = float(value)

    def estimate_lmax(self, method="lanczos"):
        """pygsp 0.5.x: the largest eigenvalue of L from ARPACK (eigsh, k = 1, tol 5e-3,
        ncv = min(N, 10)) times 1.01.  pygsp starts ARPACK from a random vector; here the start
        vector is the constant unit vector (what the fixtures were generated with), so the estimate
        is reproducible.  Graphs of <= 2 nodes use a dense eigensolver."""
        if method != "lanczos":
            raise NotImplementedError(f"estimate_lmax(method={method!r})")
        if self.N <= 2:
            lam = float(np.linalg.eigvalsh(self.L.toarray()).max()) if self.N else 0.0
        else:
            from scipy.sparse.linalg import eigsh
            v0 = np.ones(self.N) / np.sqrt(self.N)
            lam = float(np.real(eigsh(self.L, k=1, tol=5e-3, ncv=min(self.N, 10), v0=v0,
                                      return_eigenvectors=False)[0]))
        self._lmax = lam * 1.01
        return self._lmax

    def is_directed(self):
        W = sparse.csr_matrix(self.W)
        return (W != W.T).nnz != 0

    # -- device operand (srgnn) --------------------------------------------------------------------
    def device_laplacian(self, device=None):
        """(indptr int64, indices int32, values fp64) of L on the device, every diagonal slot
        stored (so that L - a2 I keeps its structure), built once."""
        import torch
        from srgnn.wavelet import _explicit_diagonal
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self._device_L is None or self._device_L[0].device != dev:
            L = _explicit_diagonal(sparse.csr_matrix(self.L))
            self._device_L = (torch.from_numpy(L.indptr.astype(np.int64)).to(dev),
                              torch.from_numpy(L.indices.astype(np.int32)).to(dev),
                              torch.from_numpy(L.data.astype(np.float64)).to(dev))
        return self._device_L
