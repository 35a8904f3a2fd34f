"""Sparse x sparse and scatter-order sparse x dense products on the device (the wavelet model's
phi * phi^-1 and its product with the features, SSRG/models/base_scalable/base_model.py:208-219).

The reference calls torch_sparse 0.6.x (absent here; the reference pins no version).  Its CPU
kernels have scipy csr_matmat's arithmetic, which is what libsrgnn_hip restates on the GPU:
  * spgemm: C[i, j] = ((0 + A[i,k1] B[k1,j]) + A[i,k2] B[k2,j]) + ... over row i of A in stored
    order, every product rounded before it is added; zero sums dropped; columns ascending
    (srg_spgemm_f32: count pass, prefix sum, fill pass);
  * spmm_scatter: Y[r] = ((0 + v1 X[c1]) + v2 X[c2]) + ... in the entries' order (index_select,
    mul, scatter_add; srg_spmm_muladd_f32).
Parity: pinned against scipy's products of the same fp32 operands (bit for bit: scipy's
csr_matmat and csr_matvecs use the same separately rounded multiply-add in the same order) and
against the wavelet fixtures' processed_feature (tests/golden/wav_*.npz, whose torch_sparse
products the generator took from scipy).  torch_sparse itself: parity unpinned.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _dev(t: torch.Tensor):
    if not t.is_cuda:
        raise RuntimeError("srgnn.sparse runs on a HIP device")
    return t.device


def csr_from_coo(row: torch.Tensor, col: torch.Tensor, value: torch.Tensor, m: int, sort_cols: bool = False):
    """(indptr int64 [m+1], indices int32, values) with every row's entries in their COO order (a
    stable sort by row; with sort_cols by (row, col)), on the tensors' device."""
    row = row.to(torch.int64)
    col = col.to(torch.int64)
    if row.numel():
        if int(row.min()) < 0 or int(row.max()) >= m:
            raise ValueError(f"row index out of range [0, {m})")
    key = row * (int(col.max()) + 1 if col.numel() else 1) + col if sort_cols else row
    perm = torch.sort(key, stable=True).indices
    counts = torch.bincount(row, minlength=m) if row.numel() else torch.zeros(m, dtype=torch.int64, device=row.device)
    ip = torch.zeros(m + 1, dtype=torch.int64, device=row.device)
    torch.cumsum(counts, 0, out=ip[1:])
    return ip, col[perm].to(torch.int32).contiguous(), value[perm].contiguous()


def _rows_have_unique_cols(ip: torch.Tensor, ix: torch.Tensor, n_rows: int) -> bool:
    if ix.numel() < 2:
        return True
    rows = torch.repeat_interleave(torch.arange(n_rows, device=ix.device), ip[1:] - ip[:-1])
    key = rows * (int(ix.max()) + 1) + ix.to(torch.int64)
    ks = torch.sort(key).values
    return not bool((ks[1:] == ks[:-1]).any())


def _check_csr(ip: torch.Tensor, ix: torch.Tensor, v: torch.Tensor) -> None:
    """The kernels trust the row pointers: int64, from 0 to nnz, non-decreasing."""
    if ip.dtype != torch.int64 or ip.dim() != 1 or ip.numel() < 1:
        raise ValueError("indptr must be a 1-D int64 tensor of n_rows + 1 entries")
    if ix.numel() != v.numel():
        raise ValueError(f"indices ({ix.numel()}) and values ({v.numel()}) differ in length")
    if int(ip[0]) != 0 or int(ip[-1]) != ix.numel() or (ip.numel() > 1 and bool((ip[1:] < ip[:-1]).any())):
        raise ValueError("indptr must run from 0 to nnz without decreasing")


def spgemm(a_ip, a_ix, a_v, b_ip, b_ix, b_v, n_cols: int, scratch_limit: int | None = None):
    """C = A @ B for device CSRs (A: m x k with column ids < k = rows of B; B: k x n_cols), fp32,
    in torch_sparse / scipy's arithmetic (module docstring).  Returns (indptr, indices, values)."""
    dev = _dev(a_ip)
    m, k = a_ip.numel() - 1, b_ip.numel() - 1
    for t in (a_ix, b_ix):
        if t.dtype != torch.int32:
            raise TypeError("column ids must be int32")
    for t in (a_v, b_v):
        if t.dtype != torch.float32:
            raise TypeError(f"spgemm computes in fp32, got {t.dtype}")
    _check_csr(a_ip, a_ix, a_v)
    _check_csr(b_ip, b_ix, b_v)
    if a_ix.numel() and (int(a_ix.min()) < 0 or int(a_ix.max()) >= k):
        raise ValueError("A's column ids must index B's rows")
    if b_ix.numel() and (int(b_ix.min()) < 0 or int(b_ix.max()) >= n_cols):
        raise ValueError(f"B's column ids must be < {n_cols}")
    a_ip, a_ix, a_v = a_ip.contiguous(), a_ix.contiguous(), a_v.contiguous()
    b_ip, b_ix, b_v = b_ip.contiguous(), b_ix.contiguous(), b_v.contiguous()
    flags = 0 if _rows_have_unique_cols(b_ip, b_ix, k) else _lib.SRG_SPGEMM_SERIAL_B
    need = ctypes.c_int64(0)
    _lib.check(_lib.query("srg_spgemm_scratch_bytes", m, int(n_cols), ctypes.byref(need)), "srg_spgemm_scratch_bytes")
    scratch = None
    if need.value:
        free, _ = torch.cuda.mem_get_info(dev)
        budget = min(need.value, scratch_limit if scratch_limit is not None else free // 4)
        per = 4 * n_cols + 4 * ((n_cols + 31) // 32)
        budget = max(per, budget // per * per)
        scratch = torch.empty(budget, dtype=torch.uint8, device=dev)
    sp = (scratch.data_ptr() if scratch is not None else None, scratch.numel() if scratch is not None else 0)
    cnt = torch.empty(m, dtype=torch.int64, device=dev)
    st = _lib.stream(dev)

    def run(phase, c_ptr, c_ix, c_v):
        _lib.call(dev, "srg_spgemm_f32", phase, a_ip.data_ptr(), a_ix.data_ptr() if a_ix.numel() else None,
                  a_v.data_ptr() if a_v.numel() else None, m, b_ip.data_ptr(),
                  b_ix.data_ptr() if b_ix.numel() else None, b_v.data_ptr() if b_v.numel() else None,
                  int(n_cols), cnt.data_ptr() if m else None, c_ptr, c_ix, c_v, sp[0], sp[1], flags, st)
    run(0, None, None, None)
    c_ip = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    if m:
        torch.cumsum(cnt, 0, out=c_ip[1:])
    nnz = int(c_ip[-1])
    c_ix = torch.empty(nnz, dtype=torch.int32, device=dev)
    c_v = torch.empty(nnz, dtype=torch.float32, device=dev)
    if nnz:
        run(1, c_ip.data_ptr(), c_ix.data_ptr(), c_v.data_ptr())
    return c_ip, c_ix, c_v


def spmm_scatter(ip, ix, v, X: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Y = A @ X with torch_sparse.spmm's arithmetic (srg_spmm_muladd_f32): per row, the entries'
    products rounded and added in stored order from +0.  A: device CSR, X: [rows of A's columns, d]
    fp32 with unit column stride."""
    dev = _dev(X)
    if X.dtype != torch.float32 or v.dtype != torch.float32:
        raise TypeError("spmm_scatter computes in fp32")
    if X.dim() != 2 or X.stride(1) != 1:
        X = X.reshape(X.shape[0], -1).contiguous()
    n_rows, d = ip.numel() - 1, X.shape[1]
    _check_csr(ip, ix, v)
    if ix.numel() and (int(ix.min()) < 0 or int(ix.max()) >= X.shape[0]):
        raise ValueError("column ids must index X's rows")
    if out is None:
        out = torch.empty((n_rows, d), dtype=torch.float32, device=dev)
    elif (out.dtype != torch.float32 or out.device != dev or out.dim() != 2 or tuple(out.shape) != (n_rows, d)
          or (d > 1 and out.stride(1) != 1)):
        raise ValueError(f"out must be a float32 [{n_rows}, {d}] tensor with unit column stride on {dev}")
    _lib.call(dev, "srg_spmm_muladd_f32", ip.data_ptr(), ix.data_ptr() if ix.numel() else None,
              v.data_ptr() if v.numel() else None, n_rows, X.data_ptr(), X.stride(0) if X.shape[0] > 1 else d,
              out.data_ptr(), out.stride(0) if n_rows > 1 else d, d, _lib.stream(dev))
    return out
