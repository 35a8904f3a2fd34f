"""TEST INFRASTRUCTURE ONLY -- the parity oracle.

CPU restatement of the reference's propagation path.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product (scalable-roubust-gnn_amd/) never
does, and it must not be used as a fallback.

  sym_norm        restates adj_to_symmetric_norm      SSRG/operators/utils.py:81-93
  spmm / propagate restate FloatCSRMulDenseOMP + the   SSRG/operators/csrc/matmul.c:23-40,
                  GraphOp hop loop                     SSRG/operators/base_operator.py:19-36
  spmm64          fp64 product in scipy's csr_matvecs order (the directed families' power iterations)
  segment_sum     sequential per-segment sums (scatter_add / duplicate merges), any float dtype
  ref_spmm        the reference's own matmul.c, compiled from its source by oracle/Makefile into
                  oracle/_ref/libmatmul_ref.so (the shipped prebuilt libmatmul.so is never loaded)
  combine         restates MessageOp.combine for last / sum / mean / simple_weighted with the same
                  torch CPU operations           SSRG/operators/message_operator/*_message_op.py,
                                                 SSRG/operators/utils.py:426-437
  laplacian, cheby_coeffs, cheby_op
                  restate the wavelet basis' pygsp calls (SSRG/models/base_scalable/
                  base_model.py:180-191, 236-265); pygsp is not in the reference tree nor installed
                  here.  Pinned on the reference's own SpectralModel.preprocess run with pygsp
                  restated (tests/golden/wav_*.npz, bit-identical phi / phi^-1) and validated
                  against a dense eigendecomposition.

Pinning: sym_norm/spmm/propagate are checked against tests/golden/*.npz, produced by running the
reference's own Python operators (tests/golden/make_golden.py), and spmm against ref_spmm.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "libsrg_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libmatmul_ref.so")

_oracle = None
_ref = None


def build(quiet=True):
    """make -C oracle (our restatement always; the reference's matmul.c when its source exists)."""
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        p, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        L.srg_oracle_spmm_f32.argtypes = [p, p, p, i64, p, i64, p, i64, i32, ctypes.c_int]
        L.srg_oracle_spmm_f32.restype = None
        L.srg_oracle_spmm_f64.argtypes = [p, p, p, i64, p, i64, p, i64, i32]
        L.srg_oracle_spmm_f64.restype = None
        L.srg_oracle_cheby_f64.argtypes = [p, p, p, i64, p, i32, p, i32, i32, ctypes.c_double,
                                           p, p, p, p, p]
        L.srg_oracle_cheby_f64.restype = ctypes.c_int
        L.srg_oracle_num_threads.restype = ctypes.c_int
        _oracle = L
    return _oracle


def ref_lib():
    """oracle/_ref/libmatmul_ref.so (reference matmul.c built from source) or None if absent."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        L = ctypes.CDLL(REF_SO)
        p, ci = ctypes.c_void_p, ctypes.c_int
        for name in ("FloatCSRMulDenseOMP", "FloatCSRMulDenseRAW"):
            getattr(L, name).argtypes = [p, p, p, p, p, ci, ci]
            getattr(L, name).restype = None
        _ref = L
    return _ref


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ------------------------------------------------------------------------------------------------
# normalisation (utils.py:81-93), restated without scipy
# ------------------------------------------------------------------------------------------------
def _coo(indptr, indices, data, n):
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(np.asarray(indptr, dtype=np.int64)))
    return rows, np.asarray(indices, dtype=np.int64), np.asarray(data, dtype=np.float64)


def _sum_duplicates_sorted(rows, cols, vals, n):
    """Canonical CSR triplets: sorted by (row, col), duplicates summed, explicit zeros dropped."""
    key = rows * n + cols
    order = np.argsort(key, kind="stable")
    key, vals = key[order], vals[order]
    if key.size:
        # left-to-right sums from +0 (scipy's csr_binop / sum_duplicates order); np.add.reduceat
        # would add the tail of a run pairwise, a different rounding for 3+ duplicates
        start = np.flatnonzero(np.r_[True, key[1:] != key[:-1]])
        lens = np.diff(np.r_[start, key.size])
        out = vals[start] + 0.0
        for i in np.flatnonzero(lens > 1).tolist():
            acc = 0.0
            for x in vals[start[i]:start[i] + lens[i]].tolist():
                acc += x
            out[i] = acc
        vals = out
        key = key[start]
    keep = vals != 0
    key, vals = key[keep], vals[keep]
    return key // n, key % n, vals


def sym_norm(indptr, indices, data, n, r):
    """Â = D^(r-1) (A+I)^T D^(-r), D = rowsum(A+I) (fp64), as CSR arrays.

    Returns (indptr int64, indices int32, values fp64).  Element (i, j) is
    ((A+I)[j, i] * deg_i^(r-1)) * deg_j^(-r), products evaluated in that order (fp64), with
    np.power for the degree powers and inf -> 0, zero products dropped (scipy's sparse products
    keep only nonzero results)."""
    rows, cols, vals = _coo(indptr, indices, data, n)
    diag = np.arange(n, dtype=np.int64)
    rows, cols, vals = _sum_duplicates_sorted(np.r_[rows, diag], np.r_[cols, diag],
                                              np.r_[vals, np.ones(n)], n)
    deg = np.zeros(n, dtype=np.float64)
    for i, v in zip(rows.tolist(), vals.tolist()):   # sequential fp64 row sums, column order
        deg[i] += v
    with np.errstate(divide="ignore"):
        left = np.power(deg, r - 1)
        right = np.power(deg, -r)
    left[np.isinf(left)] = 0.0
    right[np.isinf(right)] = 0.0
    # (A+I)[j, i] lands at (i, j)
    t_rows, t_cols = cols, rows
    step1 = vals * left[t_rows]          # (A+I)[j,i] * left[i]
    step2 = step1 * right[t_cols]        # ... * right[j]
    keep1 = step1 != 0
    t_rows, t_cols, step2 = t_rows[keep1], t_cols[keep1], step2[keep1]
    keep2 = step2 != 0
    t_rows, t_cols, step2 = t_rows[keep2], t_cols[keep2], step2[keep2]
    order = np.lexsort((t_cols, t_rows))
    t_rows, t_cols, step2 = t_rows[order], t_cols[order], step2[order]
    out_ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(out_ptr, t_rows + 1, 1)
    return np.cumsum(out_ptr), t_cols.astype(np.int32), step2


def ppr_norm(indptr, indices, data, n, r, alpha):
    """(1 - alpha) Â + alpha I (symmetrical_simgraph_ppr_operator.py:19-20), fp64."""
    ip, ix, v = sym_norm(indptr, indices, data, n, r)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip))
    diag = np.arange(n, dtype=np.int64)
    r2, c2, v2 = _sum_duplicates_sorted(np.r_[rows, diag], np.r_[ix.astype(np.int64), diag],
                                        np.r_[(1 - alpha) * v, np.full(n, alpha)], n)
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ptr, r2 + 1, 1)
    return np.cumsum(ptr), c2.astype(np.int32), v2


# ------------------------------------------------------------------------------------------------
# SpMM / K-hop propagation (matmul.c:23-40, base_operator.py:19-36)
# ------------------------------------------------------------------------------------------------
def spmm(indptr, indices, values, X, out=None, accumulate=False):
    """Y = A @ X with one sequential fp32 fma chain per element, CSR order (C oracle)."""
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    values = np.ascontiguousarray(values, dtype=np.float32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    n_rows = indptr.size - 1
    d = X.shape[1]
    if out is None:
        out = np.zeros((n_rows, d), dtype=np.float32)
    lib().srg_oracle_spmm_f32(_ptr(indptr), _ptr(indices), _ptr(values), n_rows, _ptr(X), d,
                              _ptr(out), out.shape[1], d, 1 if accumulate else 0)
    return out


def propagate(indptr, indices, values, X, K):
    out = [np.asarray(X, dtype=np.float32)]
    for _ in range(K):
        out.append(spmm(indptr, indices, values, out[-1]))
    return out


def spmm64(indptr, indices, values, X):
    """fp64 Y = A @ X in scipy's csr_matvecs order: each element from 0, adding the separately
    rounded products in storage order (C oracle)."""
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    values = np.ascontiguousarray(values, dtype=np.float64)
    X2 = np.ascontiguousarray(np.asarray(X, dtype=np.float64).reshape(np.shape(X)[0], -1))
    n_rows, d = indptr.size - 1, X2.shape[1]
    out = np.zeros((n_rows, d), dtype=np.float64)
    lib().srg_oracle_spmm_f64(_ptr(indptr), _ptr(indices), _ptr(values), n_rows, _ptr(X2), d, _ptr(out), d, d)
    return out.reshape((n_rows,) + tuple(np.shape(X)[1:]))


def segment_sum(ptr, vals):
    """out[s] = ((0 + v[p[s]]) + v[p[s]+1]) + ..., left to right in vals' dtype (torch_scatter's
    scatter_add / scipy's duplicate merge order); vectorised across segments."""
    ptr = np.asarray(ptr, dtype=np.int64)
    vals = np.asarray(vals)
    lens = np.diff(ptr)
    out = np.zeros(lens.size, dtype=vals.dtype)
    for k in range(int(lens.max()) if lens.size else 0):
        live = lens > k
        out[live] = out[live] + vals[ptr[:-1][live] + k]
    return out


def ref_spmm(indptr, indices, values, X):
    """The reference's own FloatCSRMulDenseOMP (from matmul.c source) on a zeroed answer."""
    L = ref_lib()
    if L is None:
        raise FileNotFoundError(REF_SO)
    indptr = np.ascontiguousarray(indptr, dtype=np.int32)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    values = np.ascontiguousarray(values, dtype=np.float32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    ans = np.zeros(X.shape, dtype=np.float32)
    L.FloatCSRMulDenseOMP(_ptr(ans), _ptr(values), _ptr(indices), _ptr(indptr), _ptr(X),
                          X.shape[0], X.shape[1])
    return ans


# ------------------------------------------------------------------------------------------------
# wavelet basis (restates pygsp 0.5.x; pinned by tests/golden/wav_*.npz from the reference's SpectralModel)
# ------------------------------------------------------------------------------------------------
def laplacian(indptr, indices, data, n):
    """Combinatorial Laplacian L = D - W of nx.Graph(adj) (base_model.py:181-183): W is the
    symmetrised adjacency (an undirected graph keeps one weight per pair: the last stored one in
    row-major order, i.e. the lower-triangle entry when both exist).  Every diagonal entry is
    stored (zero-degree rows included) so that L - a2*I keeps the CSR structure.
    Returns (indptr int64, indices int32, values fp64)."""
    rows, cols, vals = _coo(indptr, indices, data, n)
    w = {}
    for u, v, x in zip(rows.tolist(), cols.tolist(), vals.tolist()):
        w[(min(u, v), max(u, v))] = x
    pr, pc, pv = [], [], []
    for (u, v), x in w.items():
        pr.append(u); pc.append(v); pv.append(x)
        if u != v:
            pr.append(v); pc.append(u); pv.append(x)
    pr, pc, pv = np.array(pr, dtype=np.int64), np.array(pc, dtype=np.int64), np.array(pv, dtype=np.float64)
    deg = np.zeros(n)
    np.add.at(deg, pr, pv)
    diag = np.arange(n, dtype=np.int64)
    key_rows = np.r_[pr, diag]
    key_cols = np.r_[pc, diag]
    key_vals = np.r_[-pv, deg]
    key = key_rows * n + key_cols
    order = np.argsort(key, kind="stable")
    key, key_vals = key[order], key_vals[order]
    start = np.flatnonzero(np.r_[True, key[1:] != key[:-1]]) if key.size else np.zeros(0, np.int64)
    vals_s = np.add.reduceat(key_vals, start) if key.size else key_vals
    key = key[start] if key.size else key
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ptr, key // n + 1, 1)
    return np.cumsum(ptr), (key % n).astype(np.int32), vals_s


def heat_kernel(x, tau, lmax):
    """pygsp filters.Heat kernel (normalize=False): exp(-tau * x / lmax)."""
    return np.exp(-tau * x / lmax)


def cheby_coeffs(tau, lmax, m):
    """pygsp compute_cheby_coeff(Heat(tau), m): m+1 coefficients, N = m+1 Chebyshev nodes."""
    N = m + 1
    a1 = a2 = lmax / 2.0
    k = np.arange(N)
    nodes = np.cos(np.pi * (k + 0.5) / N)
    c = np.zeros(m + 1)
    for o in range(m + 1):
        c[o] = 2.0 / N * np.dot(heat_kernel(a1 * nodes + a2, tau, lmax), np.cos(np.pi * o * (k + 0.5) / N))
    return c


def cheby_op(L, coeffs, S, lmax):
    """pygsp cheby_op(G, c, S): R[s] = sum_k c[s,k] T_k(L~) S for every scale s (C oracle)."""
    ip, ix, lv = (np.ascontiguousarray(L[0], dtype=np.int64), np.ascontiguousarray(L[1], dtype=np.int32),
                  np.ascontiguousarray(L[2], dtype=np.float64))
    coeffs = np.ascontiguousarray(np.atleast_2d(coeffs), dtype=np.float64)
    S = np.ascontiguousarray(S, dtype=np.float64)
    n, d = S.shape
    ns, nc = coeffs.shape
    R = np.zeros((ns, n, d))
    w = [np.zeros((n, d)) for _ in range(3)]
    fv = np.zeros(lv.size)
    rc = lib().srg_oracle_cheby_f64(_ptr(ip), _ptr(ix), _ptr(lv), n, _ptr(S), d, _ptr(coeffs), ns, nc,
                                    float(lmax), _ptr(R), _ptr(w[0]), _ptr(w[1]), _ptr(w[2]), _ptr(fv))
    if rc != 0:
        raise ValueError("cheby_op needs at least 2 coefficients")
    return R


def combine(aggr, feat_list, start=None, end=None, alpha=None, weight_list=None):
    """MessageOp.combine on a list of torch CPU fp32 panels, with the reference's own torch ops:
    last_message_op.py:9-10, sum_message_op.py:9-10, mean_message_op.py:9-10 and
    simple_weighted_message_op.py:36-53 -> utils.py:426-437 (vstack of flattened panels, product
    with the fp32 weight column, dim-0 sum)."""
    import torch
    if aggr == "last":
        return feat_list[-1]
    if aggr == "sum":
        return sum(feat_list[start:end])
    if aggr == "mean":
        return sum(feat_list[start:end]) / (end - start)
    if aggr == "simple_weighted":
        if alpha is not None:
            w = [alpha]
            for _ in range(len(feat_list) - 1):
                w.append((1 - alpha) * w[-1])
            w = torch.FloatTensor(w[start:end])
        else:
            w = torch.FloatTensor(weight_list)
        sel = feat_list[start:end]
        assert len(sel) == w.shape[0]
        shape = sel[0].shape
        stack = torch.vstack([f.view(1, -1).squeeze(0) for f in sel])
        return (stack * w.view(-1, 1)).sum(dim=0).view(shape)
    raise ValueError(aggr)
