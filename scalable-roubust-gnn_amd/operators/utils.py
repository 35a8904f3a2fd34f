"""Reference-compatible helpers of the propagation path (mirror of SSRG/operators/utils.py).

Same names, argument meaning and error behaviour as the reference; the SpMM runs on the GPU through
libsrgnn_hip.so instead of libmatmul.so.  The directed-family normalisations (utils.py:95-424) are
built on the GPU by srgnn.directed and returned as scipy matrices, as the reference returns them.
"""
from __future__ import annotations

import os.path as osp
from ctypes import c_int

import numpy as np
import numpy.ctypeslib as ctl
import scipy.sparse as sp
import torch
from torch import Tensor

from srgnn import _lib as _srg

_LIB_DIR = osp.dirname(_srg.LIB_PATH)
_LIB_NAME = osp.basename(_srg.LIB_PATH)
_host_lib = None


def _host_entry():
    """libsrgnn_hip.so loaded through numpy.ctypeslib with the reference's argtypes (utils.py:21-36):
    the same ndpointer checks, hence the same ctypes.ArgumentError for float64 / int64 buffers."""
    global _host_lib
    if _host_lib is None:
        lib = ctl.load_library(_LIB_NAME, _LIB_DIR)
        i32 = ctl.ndpointer(dtype=np.int32, ndim=1, flags="CONTIGUOUS")
        f32 = ctl.ndpointer(dtype=np.float32, ndim=1, flags="CONTIGUOUS")
        lib.FloatCSRMulDenseOMP.argtypes = [f32, f32, i32, i32, f32, c_int, c_int]
        lib.FloatCSRMulDenseOMP.restype = None
        lib.FloatCSRMulDense.argtypes = [f32, c_int, f32, i32, i32, f32, c_int, c_int]
        lib.FloatCSRMulDense.restype = c_int
        lib.srg_last_error_code.restype = c_int
        lib.srg_last_error.restype = __import__("ctypes").c_char_p
        _host_lib = lib
    return _host_lib


def _raise_if_failed(lib, what):
    code = lib.srg_last_error_code()
    if code != 0:
        raise RuntimeError(f"{what}: {lib.srg_last_error().decode(errors='replace')}")


def csr_sparse_dense_matmul(adj, feature):
    """adj @ feature on the GPU with the reference's host-buffer contract (utils.py:17-47):
    the answer starts zeroed and every element is one fma chain in CSR order (bit-identical to
    FloatCSRMulDenseOMP)."""
    lib = _host_entry()
    answer = np.zeros(feature.shape, dtype=np.float32).flatten()
    data = adj.data.astype(np.float32)
    mat = feature.flatten()
    mat_row, mat_col = feature.shape
    lib.FloatCSRMulDenseOMP(answer, data, adj.indices, adj.indptr, mat, mat_row, mat_col)
    _raise_if_failed(lib, "FloatCSRMulDenseOMP")
    return answer.reshape(feature.shape)


def cuda_csr_sparse_dense_matmul(adj, feature):
    """The reference's (never called) cuSPARSE variant, utils.py:49-79: beta = 0 overwrite."""
    lib = _host_entry()
    answer = np.zeros(feature.shape, dtype=np.float32).flatten()
    data = adj.data.astype(np.float32)
    mat = feature.flatten()
    mat_row, mat_col = feature.shape
    rc = lib.FloatCSRMulDense(answer, len(data), data, adj.indices, adj.indptr, mat, mat_row, mat_col)
    if rc != 0:
        _raise_if_failed(lib, "FloatCSRMulDense")
    return answer.reshape(feature.shape)


def adj_to_symmetric_norm(adj, r):
    """D^(r-1) (A+I)^T D^(-r) with D = rowsum(A+I), as SSRG/operators/utils.py:81-93 computes it
    (fp64, degree powers through np.power, inf -> 0).  Returns a scipy sparse matrix whose csr form
    is element-for-element the reference's.

    Element (i, j) of the result is ((A+I)[j, i] * deg_i^(r-1)) * deg_j^(-r), evaluated in that
    order, exactly as the reference's column scaling, transpose and second column scaling do."""
    a_hat = sp.csr_matrix(adj + sp.eye(adj.shape[0]))
    deg = np.asarray(a_hat.sum(1)).flatten()
    with np.errstate(divide="ignore"):
        left = np.power(deg, r - 1)
        right = np.power(deg, -r)
    left[np.isinf(left)] = 0.0
    right[np.isinf(right)] = 0.0
    # (A+I) * diag(left): scales column i of (A+I) by left[i]
    scaled = a_hat @ sp.diags(left)
    # transpose, then scale column j by right[j]
    return scaled.transpose() @ sp.diags(right)


def _coo_of(adj):
    """The reference reads adj.row / adj.col / adj.data (a coo_matrix, utils.py:97-98, 197-198)."""
    if not isinstance(adj, sp.coo_matrix):
        adj = sp.coo_matrix(adj)
    return adj.row, adj.col, adj.data, adj.shape[0]


def _scipy(csr, n):
    from srgnn.construct import to_scipy
    return to_scipy(*csr, n)


def adj_to_directed_symmetric_mag_norm(adj, r, q):
    """Magnetic Laplacian normalisation, utils.py:95-138: (real, imag) csr_matrix parts of
    D_s^(r-1) (A_s + I) D_s^(-r) * exp(i 2 pi q (A - A^T)), A_s = (A + A^T) / 2 (GPU, bit-identical)."""
    from srgnn.directed import magnetic_norm
    row, col, data, n = _coo_of(adj)
    re, im = magnetic_norm(row, col, data, n, r, q)
    return _scipy(re, n), _scipy(im, n)


def PyGSD_adj_to_directed_symmetric_mag_norm(adj, r, q):
    """utils.py:140-193 (PyTorch Geometric Signed Directed's variant: no self-loops in the degrees,
    L = I - A_norm scaled by 2 / lambda_max with lambda_max = 2, a second set of -1 loops on the
    real part).  GPU; bit-identical except, in a row of more than 16 stored entries that also stores
    a self-loop, the last bit of that diagonal entry (scipy sums its three duplicates in the order
    its introsort leaves them)."""
    from srgnn.directed import pygsd_magnetic_norm
    row, col, data, n = _coo_of(adj)
    re, im = pygsd_magnetic_norm(row, col, data, n, r, q)
    return _scipy(re, n), _scipy(im, n)


def adj_to_un_in_out_dir_symmetric_norm(adj, r):
    """utils.py:195-260: (un, in, out) csr_matrix operators.  un is bit-identical; in / out come from
    the dense P^T P and P P^T (P = D^-1 (A + I)), here fp64 GEMMs on the GPU rounded to fp32, so
    they match the reference's fp32 sgemm values to a few ulps (same sparsity)."""
    from srgnn.directed import in_out_norm
    row, col, _, n = _coo_of(adj)
    un, i, o = in_out_norm(row, col, n, r)
    return _scipy(un, n), _scipy(i, n), _scipy(o, n)


def adj_to_fast_ppr_approx_symmetric_norm(adj, r, ppr_alpha, max_iter=100):
    """utils.py:262-322: the symmetric normalisation of (Pi^1/2 P Pi^-1/2 + Pi^-1/2 P^T Pi^1/2) / 2,
    Pi from the reference's power iteration (fp64 on the GPU; its dot product and norm are BLAS
    reductions in the reference, so values agree to a few fp32 ulps, same sparsity)."""
    from srgnn.directed import fast_ppr_norm
    row, col, _, n = _coo_of(adj)
    return _scipy(fast_ppr_norm(row, col, n, r, ppr_alpha, max_iter), n)


def adj_to_slow_first_second_ppr_approx_symmetric_norm(adj, r, ppr_alpha):
    """utils.py:324-424: (first-order, second-order) csr_matrix operators.  The stationary
    distribution comes from a fp64 power iteration on the GPU instead of the reference's fp32 dense
    eigendecomposition (scipy.linalg.eig of a float32 matrix), so the first-order values differ from
    the reference's by that eigenvector's fp32 error (up to ~5e-4 relative on Cora); the
    second-order operator matches to a few ulps (fp64 GEMMs vs the reference's sgemm)."""
    from srgnn.directed import two_order_norm
    row, col, _, n = _coo_of(adj)
    one, two = two_order_norm(row, col, n, r, ppr_alpha)
    return _scipy(one, n), _scipy(two, n)


def one_dim_weighted_add(feat_list, weight_list):
    """Mirror of utils.py:426-437 (hop aggregation with one weight per hop)."""
    if not isinstance(feat_list, list) or not isinstance(weight_list, Tensor):
        raise TypeError("This function is designed for list(feature) and tensor(weight)!")
    elif len(feat_list) != weight_list.shape[0]:
        raise ValueError("The feature list and the weight list have different lengths!")
    elif len(weight_list.shape) != 1:
        raise ValueError("The weight list should be a 1d tensor!")
    shape = feat_list[0].shape
    stacked = torch.vstack([f.reshape(1, -1).squeeze(0) for f in feat_list])
    return (stacked * weight_list.view(-1, 1)).sum(dim=0).view(shape)


def two_dim_weighted_add(feat_list, weight_list):
    """Mirror of utils.py:439-449 (per-node hop weights)."""
    if not isinstance(feat_list, list) or not isinstance(weight_list, Tensor):
        raise TypeError("This function is designed for list(feature) and tensor(weight)!")
    elif len(feat_list) != weight_list.shape[1]:
        raise ValueError("The feature list and the weight list have different lengths!")
    elif len(weight_list.shape) != 2:
        raise ValueError("The weight list should be a 2d tensor!")
    stacked = torch.stack(feat_list, dim=2)
    return torch.bmm(stacked, weight_list.unsqueeze(dim=2)).squeeze(dim=2)


def squeeze_first_dimension(feat_list):
    """Mirror of utils.py:452-460: drop a leading batch dimension of 3-d feature tensors
    (in place for a list, like the reference)."""
    if isinstance(feat_list, Tensor):
        return feat_list[0] if feat_list.dim() == 3 else feat_list
    if isinstance(feat_list, list) and feat_list[0].dim() == 3:
        feat_list[:] = [f.squeeze(dim=0) for f in feat_list]
    return feat_list
