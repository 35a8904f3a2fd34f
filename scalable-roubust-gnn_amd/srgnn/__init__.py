"""srgnn -- MI355X (gfx950) runtime for the spectral feature-propagation hot path of
yyysyyy/Scalable-Roubust-GNN.

    _lib      ctypes binding of libsrgnn_hip.so (include/srgnn_hip.h); no fallback
    csr       DeviceCSR: device-resident normalised adjacency + its row schedule
    spmm      spmm() / propagate(): one hop / K hops on the GPU
    normalize construct_adj on the GPU (bit-exact to SSRG/operators/utils.py:81-93)
    wavelet   Chebyshev heat-kernel filter bank (SpectralModel's wavelet basis)
    dist      1-D row partition over torch.distributed (RCCL over xGMI), one process per GPU
    synth     deterministic synthetic graphs / features (counter-based hash, CPU == GPU)
    roofline  byte models of SURVEY.md §8(d)

The reference-compatible Python API lives in the sibling package `operators` (same module paths
as SSRG/operators), which is what models/ and main.py import.
"""
from ._lib import SrgError, version  # noqa: F401
