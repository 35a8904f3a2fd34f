"""construct_adj on the device: Â of SymLaplacianGraphOp / PprGraphOp
from any scipy-style adjacency, bit-identical to the reference's scipy arithmetic.

Reference (SSRG/operators/utils.py:81-93, symmetrical_simgraph_ppr_operator.py:13-21):
    adj = adj + I                                   duplicates merged left to right, zeros dropped
    deg = adj.sum(1)                                fp64 row sums in column order
    left = deg^(r-1), right = deg^(-r)              np.power, inf -> 0
    Â = (adj . diag(left))^T . diag(right)          Â[i, j] = ((A+I)[j, i] * left[i]) * right[j]
    PPR: (1 - alpha) * Â + alpha * I
Every step is an elementwise fp64 product, a sort, or a sequential segment sum
(srg_segment_sum_f64), so the device result equals scipy's bit for bit; np.power stays on the
host (N values through the same libm call as the reference).  Canonical inputs are pinned by the
golden fixtures; for non-canonical weighted inputs scipy sums a row in its own merge order, so
the last fp64 bit may differ there (integer weights are exact in any order).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from .normalize import degree_powers


def segment_sum_device(seg_ptr: torch.Tensor, vals: torch.Tensor) -> torch.Tensor:
    n_seg = seg_ptr.numel() - 1
    out = torch.empty(n_seg, dtype=torch.float64, device=vals.device)
    _lib.call(vals.device, "srg_segment_sum_f64", seg_ptr.data_ptr(), vals.data_ptr() if vals.numel() else None,
              n_seg, out.data_ptr(), _lib.stream(vals.device))
    return out


def mirror_device(indptr: torch.Tensor, indices32: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """srg_csr_mirror: position of entry (c, r) in row c for every entry (r, c), or -1."""
    out = torch.empty(indices32.numel(), dtype=torch.int64, device=indices32.device)
    _lib.call(indices32.device, "srg_csr_mirror", indptr.data_ptr(), indices32.data_ptr(), rows.data_ptr(),
              indptr.numel() - 1, indices32.numel(), out.data_ptr(), _lib.stream(indices32.device))
    return out


def _canonical_plus_identity(ip, ix, v, rows, n):
    """adj + I without a sort when adj is canonical (strictly increasing column ids within rows,
    no explicit zeros) and no diagonal entry becomes 0: each row gets its diagonal entry merged at
    its sorted position (an existing one becomes A[i,i] + 1.0, scipy's csr_plus_csr sum).  Returns
    (indptr, indices, values, rows) or None when the input needs the general path."""
    nnz = ix.numel()
    key = rows * n + ix
    if nnz and not (bool((key[1:] > key[:-1]).all()) and bool((v != 0).all())):
        return None
    dev = ix.device
    ar = torch.arange(n, device=dev)
    pos = torch.searchsorted(key, ar * (n + 1))            # first entry >= (r, r) in row r
    has = (pos < ip[1:]) & (ix[pos.clamp(max=max(nnz - 1, 0))] == ar) if nnz else torch.zeros(n, dtype=torch.bool, device=dev)
    vv = v.clone()
    if bool(has.any()):
        dpos = pos[has]
        vv[dpos] = v[dpos] + 1.0
        if not bool((vv[dpos] != 0).all()):
            return None
    ins = (~has).to(torch.int64)
    before = torch.cumsum(ins, 0) - ins                  # inserted diagonals in earlier rows
    n_new = nnz + int(ins.sum().item())
    new_ip = torch.empty(n + 1, dtype=torch.int64, device=dev)
    new_ip[:-1] = ip[:-1] + before
    new_ip[-1] = n_new
    new_pos = torch.arange(nnz, device=dev) + before[rows] + (ins[rows] * (ix > rows))
    new_ix = torch.empty(n_new, dtype=torch.int64, device=dev)
    new_v = torch.empty(n_new, dtype=torch.float64, device=dev)
    new_ix[new_pos] = ix
    new_v[new_pos] = vv
    r_ins = torch.nonzero(ins).squeeze(1)
    at = new_ip[r_ins] + (pos[r_ins] - ip[r_ins])
    new_ix[at] = r_ins
    new_v[at] = 1.0
    new_rows = torch.repeat_interleave(ar, new_ip[1:] - new_ip[:-1], output_size=n_new)
    return new_ip, new_ix, new_v, new_rows


def _runs(keys: torch.Tensor):
    """Start offsets (+ end) of the runs of equal values in a sorted 1-D tensor."""
    if keys.numel() == 0:
        return torch.zeros(1, dtype=torch.int64, device=keys.device)
    new = torch.ones(keys.numel(), dtype=torch.bool, device=keys.device)
    new[1:] = keys[1:] != keys[:-1]
    starts = torch.nonzero(new).squeeze(1)
    return torch.cat([starts, torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)])


def _kept(keep: torch.Tensor, *ts):
    """ts[i][keep] for each tensor -- or ts themselves when every entry is kept (the usual case:
    a boolean selection of 1e8 entries costs milliseconds, the check one reduction)."""
    if bool(keep.all()):
        return ts
    return tuple(t[keep] for t in ts)


def canonical_sum(rows, cols, vals, n_cols, segsum):
    """Sorted (row, col) triplets with duplicates summed in input order and zeros dropped."""
    key = rows * n_cols + cols
    key, perm = torch.sort(key, stable=True)
    ptr = _runs(key)
    summed = segsum(ptr, vals[perm])
    key = key[ptr[:-1]]
    key, summed = _kept(summed != 0, key, summed)
    return key // n_cols, key % n_cols, summed


def _indptr(rows, n):
    """Row pointers of SORTED row ids (every caller's rows come out of a sort): ptr[i] = the
    number of entries in rows < i, one binary search per row (a bincount of 1e8 ids took 20 ms)."""
    return torch.searchsorted(rows, torch.arange(n + 1, dtype=rows.dtype, device=rows.device))


def sym_norm(indptr, indices, data, n: int, r: float, device=None, segsum=None, mirror=None, fast=True):
    """Â = D^(r-1) (A+I)^T D^(-r) of the CSR (indptr, indices, data) (host arrays or tensors).
    Returns device tensors (indptr int64, indices int32, values fp64), canonical CSR.

    fast: a canonical adj (the reference's datasets: csr_matrix((ones, (row, col))) is canonical)
    gets A+I by merging the diagonals in place instead of a sort, and a structurally symmetric one
    (undirected graphs) its transpose from one binary search per entry (srg_csr_mirror) instead of
    a second sort -- the same values from the same fp64 operations, so the same bits; anything else
    takes the general path."""
    segsum = segsum or segment_sum_device
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    # copy in the stored dtypes and widen on the device (a host-side int32 -> int64 conversion of
    # the column ids cost 0.24 s at products size)
    ip = torch.as_tensor(np.asarray(indptr) if not torch.is_tensor(indptr) else indptr).to(dev).to(torch.int64)
    ix = torch.as_tensor(np.asarray(indices) if not torch.is_tensor(indices) else indices).to(dev).to(torch.int64)
    v = torch.as_tensor(np.asarray(data) if not torch.is_tensor(data) else data).to(dev).to(torch.float64)
    rows = torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1], output_size=ix.numel())
    api = _canonical_plus_identity(ip, ix, v, rows, n) if fast else None
    if api is not None:
        aip, cols, vals, rows = api
    else:
        diag = torch.arange(n, device=dev)
        # adj + I: the identity's entry is added after the row's own (duplicate) entries
        rows, cols, vals = canonical_sum(torch.cat([rows, diag]), torch.cat([ix, diag]),
                                         torch.cat([v, torch.ones(n, dtype=torch.float64, device=dev)]), n, segsum)
        aip = _indptr(rows, n)
    del ip, ix, v
    deg = segsum(aip, vals)
    left, right = degree_powers(deg.cpu().numpy(), r)
    left_t = torch.from_numpy(left).to(dev)
    right_t = torch.from_numpy(right).to(dev)
    if mirror is None and dev.type == "cuda":
        mirror = mirror_device
    if fast and mirror is not None and vals.numel():
        cols32 = cols.to(torch.int32)
        m = mirror(aip, cols32, rows)
        if bool((m >= 0).all()):
            # symmetric structure: Â[i, j] = ((A+I)[j, i] * left[i]) * right[j] at A+I's own positions
            vhat = (vals[m] * left_t[rows]) * right_t[cols]
            if bool((vhat != 0).all()):
                return aip, cols32, vhat
        del m, cols32
    # stored (rows, cols) of A+I lands at (cols, rows) of Â
    step1 = vals * left_t[cols]
    rows, cols, step1 = _kept(step1 != 0, rows, cols, step1)
    step2 = step1 * right_t[rows]
    t_cols, t_rows, step2 = _kept(step2 != 0, rows, cols, step2)
    key, perm = torch.sort(t_rows * n + t_cols)
    return _indptr(key // n, n), (key % n).to(torch.int32), step2[perm]


def ppr_norm(indptr, indices, data, n: int, r: float, alpha: float, device=None, segsum=None, mirror=None,
             fast=True):
    """(1 - alpha) Â + alpha I (symmetrical_simgraph_ppr_operator.py:19-21) on the device."""
    segsum = segsum or segment_sum_device
    ip, ix, v = sym_norm(indptr, indices, data, n, r, device, segsum, mirror, fast)
    dev = ip.device
    rows = torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1])
    v = (1 - alpha) * v
    diag = torch.arange(n, device=dev)
    rows, cols, vals = canonical_sum(torch.cat([rows, diag]), torch.cat([ix.to(torch.int64), diag]),
                                     torch.cat([v, torch.full((n,), alpha, dtype=torch.float64, device=dev)]),
                                     n, segsum)
    return _indptr(rows, n), cols.to(torch.int32), vals


def to_scipy(indptr, indices, values, n: int) -> sp.csr_matrix:
    """Host scipy copy (the reference keeps Â as GraphOp.adj)."""
    return sp.csr_matrix((values.cpu().numpy(), indices.cpu().numpy(), indptr.cpu().numpy()), shape=(n, n))


def edge_index_to_adj(edge_index, n: int, symmetric: bool = False, device=None, segsum=None):
    """csr_matrix((ones, (row, col)), shape=(n, n)) of an int64 [2, E] edge list on the device
    (duplicates summed), optionally symmetrised first by appending the reversed edges -- the
    dataset adjacency the reference's loaders build from edge_index.pt.
    Returns device tensors (indptr int64, indices int32, values fp64)."""
    segsum = segsum or segment_sum_device
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    e = torch.as_tensor(edge_index).to(dev, torch.int64)
    if e.dim() != 2 or e.shape[0] != 2:
        raise ValueError("edge_index must be [2, E]")
    row, col = e[0], e[1]
    if e.numel() and (int(e.min()) < 0 or int(e.max()) >= n):
        raise ValueError("edge_index holds node ids outside [0, n)")
    if symmetric:
        row, col = torch.cat([row, col]), torch.cat([col, row])
    rows, cols, vals = canonical_sum(row, col, torch.ones(row.numel(), dtype=torch.float64, device=dev), n, segsum)
    return _indptr(rows, n), cols.to(torch.int32), vals
