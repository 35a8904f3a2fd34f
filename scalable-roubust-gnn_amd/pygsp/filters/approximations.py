"""pygsp.filters.approximations (0.5.x restated): Chebyshev coefficients and the Chebyshev operator.

cheby_op runs on the GPU: the recurrence
    T0 = S,  T1 = (L S - a2 S) / a1,  T_{k+1} = (2/a1)(L - a2 I) T_k - T_{k-1},  a1 = a2 = lmax / 2,
    r_i = (c_i0 / 2) T0 + sum_{k >= 1} c_ik T_k          for every coefficient row i
is srgnn.wavelet.HeatWaveletFilter's fp64 path (srg_cheby_step_f64): one launch per order forms
T_{k+1} and every row's r_i in the same pass, in scipy's operation order (separately rounded
multiply and add), so the result is pygsp's host recurrence bit for bit (tests/test_pygsp_shim_gpu.py
against the oracle and the wav_* fixtures of the reference's SpectralModel).
"""
from __future__ import annotations

import numpy as np

_MAX_SCALES = 8          # coefficient rows per recurrence (the kernels' limit; more run in groups)


def compute_cheby_coeff(f, m=30, N=None, *args, **kwargs):
    """The m + 1 Chebyshev coefficients of filter f's i-th kernel on [0, lmax], from N = m + 1
    (default) Chebyshev nodes."""
    G = f.G
    i = kwargs.pop("i", 0)
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


def cheby_op(G, c, signal, **kwargs):
    """Chebyshev polynomial approximation of the filter with coefficients c ([M] or [Nscales, M])
    applied to `signal` ([N] or [N, Nv]): [N * Nscales] or [N * Nscales, Nv], scale i in rows
    i*N .. (i+1)*N - 1 (pygsp's layout).  Computed on the current HIP device in fp64."""
    import torch
    from srgnn.wavelet import HeatWaveletFilter
    c = np.atleast_2d(np.array(c, dtype=np.float64))
    n_scales, M = c.shape
    if M < 2:
        raise TypeError("The coefficients have an invalid shape")
    sig = np.asarray(signal, dtype=np.float64)
    one_d = sig.ndim == 1
    S = sig.reshape(G.N, -1)
    if S.shape[0] != G.N:
        raise ValueError(f"signal has {sig.shape[0]} rows, the graph {G.N} nodes")
    ip, ix, lv = G.device_laplacian()
    dev = ip.device
    St = torch.from_numpy(np.ascontiguousarray(S)).to(dev)
    r = np.zeros((G.N * n_scales, S.shape[1]))
    for s0 in range(0, n_scales, _MAX_SCALES):
        cs = c[s0:s0 + _MAX_SCALES]
        filt = HeatWaveletFilter.from_device(ip, ix, lv, G.N, None, lmax=float(G.lmax), dtype=torch.float64,
                                             coeffs=cs)
        R = filt.apply(St)
        r[s0 * G.N:(s0 + cs.shape[0]) * G.N] = R.reshape(cs.shape[0] * G.N, -1).cpu().numpy()
    return r.reshape(-1) if one_d else r
