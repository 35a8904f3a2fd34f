"""pygsp's API surface used by the reference's wavelet model, backed by libsrgnn_hip (gfx950).

SpectralModel.preprocess (SSRG/models/base_scalable/base_model.py:180-265) calls
    pygsp.graphs.Graph(W), Graph.estimate_lmax(), pygsp.filters.Heat(G, tau=[s]),
    pygsp.filters.approximations.compute_cheby_coeff(f, m=order) and
    pygsp.filters.approximations.cheby_op(G, c, impulse)
(and WAV/utils.py the same).  pygsp is not installed in this image and the reference pins no
version; this package restates pygsp 0.5.x for those names -- the same restatement the wavelet
fixtures were generated with (tests/golden/make_golden_wavelet.py) -- and runs cheby_op's
Chebyshev recurrence on the GPU (srg_cheby_step_f64: one fused launch per order, every scale of
the coefficient array from one recurrence; fp64 in scipy's operation order, so bit for bit the
host recurrence).  With the package directory on sys.path, `import pygsp` resolves here.
"""
from . import filters, graphs  # noqa: F401

__version__ = "0.5.1-srgnn-hip"
__all__ = ["graphs", "filters"]
