"""pygsp.filters (0.5.x restated): the Heat kernel filter the reference's wavelet model builds."""
from __future__ import annotations

import numpy as np

from . import approximations  # noqa: F401


class Filter:
    """pygsp.filters.Filter(G, kernels): a bank of Nf kernels g_i(lambda) on graph G."""

    def __init__(self, G, kernels):
        self.G = G
        self._kernels = list(kernels) if isinstance(kernels, (list, tuple)) else [kernels]
        self.Nf = len(self._kernels)

    def evaluate(self, x):
        """[Nf, len(x)] kernel values."""
        x = np.asarray(x, dtype=np.float64)
        return np.stack([np.asarray(k(x), dtype=np.float64) for k in self._kernels])


class Heat(Filter):
    """pygsp.filters.Heat(G, tau=10, normalize=False): g(x) = exp(-tau x / lmax) per tau."""

    def __init__(self, G, tau=10, normalize=False):
        if normalize:
            raise NotImplementedError("Heat(normalize=True) needs L's spectrum; the wavelet model uses False")
        taus = tau if isinstance(tau, (list, tuple, np.ndarray)) else [tau]
        self.tau = list(taus)
        super().__init__(G, [lambda x, t=t: np.exp(-t * x / G.lmax) for t in taus])


__all__ = ["Filter", "Heat", "approximations"]
