"""torch_sparse's functional API, backed by libsrgnn_hip (gfx950).

The wavelet model of the reference imports `from torch_sparse import spspmm, spmm`
(SSRG/models/base_scalable/base_model.py:13, simple_models.py:3) and its operators import
`coalesce` (SSRG/operators/utils.py:10).  torch_sparse is not installed in this image and the
reference pins no version; these are the published torch_sparse 0.6.x semantics, run on the GPU
(the package directory on sys.path makes `import torch_sparse` resolve here):

  spspmm(indexA, valueA, indexB, valueB, m, k, n, coalesced=False) -> (index [2, nnz], value)
      SparseTensor(A) @ SparseTensor(B) (spspmm_sum): per output row, the products of A's entries
      in stored order with B's rows, each rounded then added from 0; zero sums dropped; entries
      sorted by (row, col).  With coalesced=False the inputs are taken as sorted by row (torch_sparse
      builds its row pointers from them as given); coalesced=True sorts both inputs by (row, col)
      first and KEEPS duplicate entries (0.6.x builds SparseTensor(..., is_sorted=not coalesced),
      which sorts without summing, whatever its docstring says: a1*b and a2*b are rounded and added
      separately).  Parity unpinned: torch_sparse is absent and the reference never passes it.
      -> srgnn.sparse.spgemm (srg_spgemm_f32).
  spmm(index, value, m, n, matrix) -> [m, ...] dense
      index_select, mul, scatter_add: each output row is the sum of its entries' rounded products in
      index order from 0 -> srgnn.sparse.spmm_scatter (srg_spmm_muladd_f32); differentiable in
      `matrix` and `value` (the adjoint scatter runs through the same kernel).
  coalesce(index, value, m, n, op="add") -> (index, value)
      sorted by row * n + col, each run of equal keys summed in order (srgnn.directed).

Inputs may live on the host (as in the reference): they are moved to the current HIP device, and
the results come back to the inputs' device.  No CPU fallback: without a HIP device these raise.
Computation is fp32 (the reference passes torch.FloatTensor values).
"""
from __future__ import annotations

import torch

__version__ = "0.6.x-srgnn-hip"

__all__ = ["spspmm", "spmm", "coalesce", "transpose"]


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("torch_sparse (srgnn HIP build) needs a HIP device")
    return torch.device("cuda", torch.cuda.current_device())


def _on(t: torch.Tensor, dev):
    return t.to(dev) if t.device != dev else t


def spspmm(indexA, valueA, indexB, valueB, m, k, n, coalesced=False):
    """Matrix product of two sparse tensors in COO form (torch_sparse 0.6.x `spspmm`)."""
    from srgnn.sparse import csr_from_coo, spgemm
    if torch.is_grad_enabled() and (getattr(valueA, "requires_grad", False) or getattr(valueB, "requires_grad", False)):
        raise NotImplementedError("spspmm: gradients through the sparse product are outside the "
                                  "preprocessing path this build covers (SpectralModel.preprocess)")
    home = valueA.device
    dev = _device()
    iA, vA, iB, vB = (_on(t, dev) for t in (indexA, valueA, indexB, valueB))
    for v in (vA, vB):
        if v.dtype != torch.float32:
            raise TypeError(f"spspmm computes in float32, got {v.dtype}")
    # coalesced=True: both inputs sorted by (row, col), duplicates kept in their stored order
    # (torch_sparse 0.6.x: SparseTensor(row, col, value, is_sorted=not coalesced) sorts, never sums)
    a = csr_from_coo(iA[0], iA[1], vA, int(m), sort_cols=bool(coalesced))
    b = csr_from_coo(iB[0], iB[1], vB, int(k), sort_cols=bool(coalesced))
    if a[1].numel() and int(a[1].max()) >= int(k):
        raise ValueError(f"indexA has a column >= k = {k}")
    c_ip, c_ix, c_v = spgemm(*a, *b, int(n))
    rows = torch.repeat_interleave(torch.arange(int(m), device=dev), c_ip[1:] - c_ip[:-1])
    index = torch.stack([rows, c_ix.to(torch.int64)], dim=0)
    return index.to(home), c_v.to(home)


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, row, col, value, m, matrix):
        from srgnn.sparse import csr_from_coo, spmm_scatter
        ip, ix, v = csr_from_coo(row, col, value.detach(), m)
        ctx.save_for_backward(row, col, value, matrix)
        ctx.m = m
        return spmm_scatter(ip, ix, v, matrix.detach())

    @staticmethod
    def backward(ctx, grad):
        from srgnn.sparse import csr_from_coo, spmm_scatter
        row, col, value, matrix = ctx.saved_tensors
        g_val = g_mat = None
        if ctx.needs_input_grad[4]:
            # adjoint of the scatter: grad_matrix[c] = sum over entries with column c of v * grad[r]
            ip, ix, v = csr_from_coo(col, row, value.detach(), matrix.shape[0])
            g_mat = spmm_scatter(ip, ix, v, grad.contiguous())
        if ctx.needs_input_grad[2]:
            g_val = (grad[row] * matrix[col]).sum(dim=-1)
        return None, None, g_val, None, g_mat


def spmm(index, value, m, n, matrix):
    """Matrix product of a sparse matrix (COO `index`, `value`, shape m x n) with a dense matrix
    (torch_sparse 0.6.x `spmm`)."""
    if matrix.size(-2) != n:         # torch_sparse's first check (a 1-D matrix raises IndexError here)
        raise AssertionError(f"matrix has {matrix.size(-2)} rows, the sparse matrix {n} columns")
    home = matrix.device
    dev = _device()
    mat = _on(matrix, dev)
    if mat.dim() != 2:
        raise NotImplementedError("spmm: batched dense operands are not supported by this build")
    if mat.dtype != torch.float32 or value.dtype != torch.float32:
        raise TypeError("spmm computes in float32")
    idx, val = _on(index, dev), _on(value, dev)
    return _SpMM.apply(idx[0], idx[-1], val, int(m), mat.contiguous()).to(home)


def coalesce(index, value, m, n, op="add"):
    """Row-major sorted COO with duplicate entries summed in order (torch_sparse 0.6.x `coalesce`)."""
    from srgnn.directed import _coalesce, segment_sum
    if op not in ("add", "sum"):
        raise NotImplementedError(f"coalesce op={op!r}: only 'add' is supported")
    home = index.device
    dev = _device()
    idx = _on(index, dev).to(torch.int64)
    if value is None:
        r, c, _ = _coalesce(idx[0], idx[1], [], int(n), segment_sum)
        return torch.stack([r, c]).to(home), None
    val = _on(value, dev)
    cols = [val] if val.dim() == 1 else [val[:, j].contiguous() for j in range(val.shape[1])]
    r, c, out = _coalesce(idx[0], idx[1], cols, int(n), segment_sum)
    v = out[0] if val.dim() == 1 else torch.stack(out, dim=1)
    return torch.stack([r, c]).to(home), v.to(home)


def transpose(index, value, m, n, coalesced=True):
    """The transposed COO matrix (torch_sparse 0.6.x `transpose`)."""
    row, col = index[0], index[1]
    index = torch.stack([col, row], dim=0)
    if coalesced:
        return coalesce(index, value, n, m)
    return index, value
