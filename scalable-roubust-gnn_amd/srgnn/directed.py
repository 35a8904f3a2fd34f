"""construct_adj of the directed operator families on the device (SSRG/operators/utils.py:95-424).

The reference builds these normalisations on the host with torch_sparse / torch_scatter / PyG,
scipy and dense torch CPU algebra; here the sparse steps run as device sorts, sequential segment
sums (srg_segment_sum_f64/_f32) and element-wise IEEE operations in the reference's order, and the
dense steps (the in/out products of adj_to_un_in_out_dir_symmetric_norm and the two-order
operator) as device GEMMs.  The third-party semantics followed (the reference pins no versions):
  * torch_sparse.coalesce(index, value, m, n, "add"): entries sorted by row * n + col, each run of
    equal keys summed in order by segment_csr; returned unchanged when no key repeats;
  * torch_scatter.scatter_add(src, index, dim_size): torch's scatter_add_ into zeros, i.e. a
    sequential sum in element order;
  * torch_geometric.utils.add_self_loops: arange(N) loops appended after the edges, fill_value
    after the attributes.

Exactness (tests/test_directed_*.py against the reference run in tests/golden/make_golden_directed.py):
  * magnetic Laplacian / complex PPR / PyG-SD magnetic: bit-identical.  The per-node degree powers
    and the complex phases exp(i 2 pi q theta) are evaluated by torch on the host (N values, and
    the distinct theta values), the reference's own CPU routines; everything else is sorts, sums in
    the reference's order and separately rounded products on the device;
  * the undirected part of the in/out operator: bit-identical;
  * in/out second-order products, fast PPR, two-order PPR: the reference's values come from CPU
    BLAS (sgemm; a dot product and norm in the power iteration) and LAPACK (sgeev), whose
    summation orders are the library's.  Here: fp64 GEMMs and fp64 power iterations, rounded to
    the reference's fp32 where it rounds.  Same sparsity structure, values within the tolerance
    the tests state.

Every function returns CSR device tensors (indptr int64, indices int32, values) per matrix, with the
reference's value dtype (fp64 for the magnetic family given fp64 weights, fp32 for the others).
`segsum` / `spmv` can be replaced (the CPU tests pass numpy stand-ins and torch CPU tensors).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .construct import _indptr, _runs

_DENSE_LIMIT = 1 << 16          # nodes: the dense in/out and two-order steps hold N x N fp64 panels


# ----------------------------------------------------------------------------------------------
# kernels (device) and their host-side helpers
# ----------------------------------------------------------------------------------------------
def segment_sum(seg_ptr: torch.Tensor, vals: torch.Tensor) -> torch.Tensor:
    """out[s] = ((0 + v[p[s]]) + v[p[s]+1]) + ... in the values' dtype (fp64 / fp32), on the device."""
    n_seg = seg_ptr.numel() - 1
    out = torch.empty(n_seg, dtype=vals.dtype, device=vals.device)
    name = {torch.float64: "srg_segment_sum_f64", torch.float32: "srg_segment_sum_f32"}[vals.dtype]
    _lib.call(vals.device, name, seg_ptr.data_ptr(), vals.data_ptr() if vals.numel() else None, n_seg,
              out.data_ptr(), _lib.stream(vals.device))
    return out


def spmv64(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """fp64 y = A x in scipy's csr_matvecs order (srg_spmm_csr_f64), x [n_cols] or [n_cols, d]."""
    x2 = x.reshape(x.shape[0], -1).contiguous()
    n_rows, d = indptr.numel() - 1, x2.shape[1]
    y = torch.empty((n_rows, d), dtype=torch.float64, device=x.device)
    _lib.call(x.device, "srg_spmm_csr_f64", indptr.data_ptr(), indices.data_ptr() if indices.numel() else None,
              values.data_ptr() if values.numel() else None, n_rows, x2.data_ptr(), d, y.data_ptr(), d, d,
              _lib.stream(x.device))
    return y.reshape((n_rows,) + tuple(x.shape[1:]))


def _host_pow(deg: torch.Tensor, e: float) -> torch.Tensor:
    """torch.pow(deg, e) with inf -> 0, evaluated by torch on the host (the reference's CPU kernel:
    exponent -0.5 is an rsqrt there, -1 a reciprocal) and sent back."""
    h = deg.cpu()
    p = torch.pow(h, e)
    p.masked_fill_(p == float("inf"), 0)
    return p.to(deg.device)


def _host_phase(theta: torch.Tensor, q: float, whole_limit: int = 32768):
    """(cos, sin) of torch.exp(1j * 2 * np.pi * q * theta) as the reference's CPU exp gives them.

    Up to torch's parallel grain (32768 elements) the reference evaluates the tensor in one chunk:
    vectorised routines for all but the last few elements, a scalar routine for that tail.  The
    same tensor is evaluated here the same way, on the host.  Above it the chunk boundaries (and
    their scalar tails) follow the reference's thread count, so its own bits vary with it; here
    every value is then taken from the vectorised routine: the distinct theta values are padded to
    a multiple of 16 (each in a vector lane), evaluated once and looked up on the device."""
    if theta.numel() <= whole_limit:
        z = torch.exp(1j * 2 * np.pi * q * theta.cpu())
        return z.real.to(theta.device), z.imag.to(theta.device)
    uniq, inv = torch.unique(theta, return_inverse=True)
    u = uniq.cpu()
    pad = (-u.numel()) % 16
    if pad:
        u = torch.cat([u, u[-1:].expand(pad)])
    z = torch.exp(1j * 2 * np.pi * q * u)[: uniq.numel()]
    return z.real.to(theta.device)[inv], z.imag.to(theta.device)[inv]


def _csr_from_coo(rows, cols, vals, n, segsum, drop_zeros=False):
    """csr_matrix((vals, (rows, cols)), shape=(n, n)) as scipy builds it: rows bucketed in input
    order, indices sorted, duplicates summed (the first value, then the others in order; runs here
    hold at most two entries, an edge and a loop, so their order does not matter), explicit zeros
    kept.  drop_zeros: scipy's canonical csr + csr binop instead, which drops zero results."""
    key, perm = torch.sort(rows * n + cols, stable=True)
    v = vals[perm]
    ptr = _runs(key)
    lens = ptr[1:] - ptr[:-1]
    first = ptr[:-1]
    out = v[first]
    if bool((lens > 1).any()):
        summed = segsum(ptr, v)
        out = torch.where(lens > 1, summed, out)
    key = key[first]
    if drop_zeros:
        keep = out != 0
        key, out = key[keep], out[keep]
    r = key // n
    return _indptr(r, n), (key % n).to(torch.int32), out


def _coalesce(rows, cols, attrs, n, segsum):
    """torch_sparse.coalesce(index, attrs, n, n, "add"): sorted by row * n + col, runs summed."""
    key, perm = torch.sort(rows * n + cols, stable=True)
    ptr = _runs(key)
    first = ptr[:-1]
    if first.numel() == key.numel():                 # no key repeats: returned as sorted
        out = [a[perm] for a in attrs]
    else:
        out = [segsum(ptr, a[perm]) for a in attrs]
    key = key[first]
    return key // n, key % n, out


def _coo_input(row, col, data, device):
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    r = torch.as_tensor(np.asarray(row) if not torch.is_tensor(row) else row).to(dev, torch.int64)
    c = torch.as_tensor(np.asarray(col) if not torch.is_tensor(col) else col).to(dev, torch.int64)
    v = None
    if data is not None:
        v = torch.as_tensor(np.asarray(data) if not torch.is_tensor(data) else data).to(dev)
        if v.dtype not in (torch.float64, torch.float32):
            v = v.to(torch.float64)
    return r, c, v, dev


def _segsum_default(dev, segsum):
    return segsum if segsum is not None else segment_sum


# ----------------------------------------------------------------------------------------------
# magnetic Laplacian (utils.py:95-138), complex PPR (symmetrical_directed_magnetic_comppr_operator.py:
# 32-37) and the PyG-SD variant (utils.py:140-193)
# ----------------------------------------------------------------------------------------------
def _magnetic_parts(row, col, w, n, q, segsum):
    """The symmetrised weights A_s = (A + A^T) / 2 and phases theta = A - A^T of the coalesced
    edge list (utils.py:100-108 / 145-154)."""
    rows = torch.cat([row, col])
    cols = torch.cat([col, row])
    rr, cc, (sym, theta) = _coalesce(rows, cols, (torch.cat([w, w]), torch.cat([w, -w])), n, segsum)
    return rr, cc, sym / 2, theta


def _phase_product(w, cq, sq):
    """(w + 0i) * (cos + i sin), torch's complex multiply of a promoted real tensor:
    real = w*cos - 0*sin, imag = w*sin - 0*(-cos) (separately rounded; signed zeros as torch's)."""
    z = torch.zeros_like(w)
    return w * cq - z * sq, w * sq - z * (-cq)


def magnetic_norm(row, col, data, n: int, r: float, q: float, device=None, segsum=None):
    """adj_to_directed_symmetric_mag_norm (utils.py:95-138) of the COO (row, col, data): the real
    and imaginary parts of D_s^(r-1) (A_s + I) D_s^(-r) * exp(i 2 pi q (A - A^T)), each as CSR
    device tensors (indptr int64, indices int32, values in data's dtype)."""
    row, col, w, dev = _coo_input(row, col, data, device)
    segsum = _segsum_default(dev, segsum)
    rr, cc, ws, theta = _magnetic_parts(row, col, w, n, q, segsum)
    loops = torch.arange(n, device=dev)
    # degree: the row's coalesced weights in column order, then its self-loop's 1 (:109-121)
    deg = segsum(_indptr(rr, n), ws) + 1
    left, right = _host_pow(deg, r - 1), _host_pow(deg, -r)
    R = torch.cat([rr, loops])
    C = torch.cat([cc, loops])
    ws2 = torch.cat([ws, torch.ones(n, dtype=ws.dtype, device=dev)])
    th2 = torch.cat([theta, torch.zeros(n, dtype=theta.dtype, device=dev)])
    cq, sq = _host_phase(th2, q)
    re, im = _phase_product(left[R] * ws2 * right[C], cq, sq)
    return _csr_from_coo(R, C, re, n, segsum), _csr_from_coo(R, C, im, n, segsum)


def magnetic_com_ppr(row, col, data, n: int, r: float, q: float, alpha: float, device=None, segsum=None):
    """SymDirMagComPprGraphOp.construct_adj (symmetrical_directed_magnetic_comppr_operator.py:32-37):
    real' = (1 - alpha) real + alpha I (scipy's canonical add: zero results dropped),
    imag' = (1 - alpha) imag (structure kept)."""
    (rip, rix, rv), (iip, iix, iv) = magnetic_norm(row, col, data, n, r, q, device, segsum)
    dev = rv.device
    segsum = _segsum_default(dev, segsum)
    loops = torch.arange(n, device=dev)
    rrow = torch.repeat_interleave(torch.arange(n, device=dev), rip[1:] - rip[:-1])
    real = _csr_from_coo(torch.cat([rrow, loops]), torch.cat([rix.to(torch.int64), loops]),
                         torch.cat([(1 - alpha) * rv, torch.full((n,), alpha, dtype=rv.dtype, device=dev)]),
                         n, segsum, drop_zeros=True)
    return real, (iip, iix, (1 - alpha) * iv)


def pygsd_magnetic_norm(row, col, data, n: int, r: float, q: float, device=None, segsum=None):
    """PyGSD_adj_to_directed_symmetric_mag_norm (utils.py:140-193): no self-loops in the degrees;
    L = I - A_norm scaled by 2 / lambda_max (lambda_max = 2); real part with a second set of -1
    loops.  Duplicate runs of three (a stored self-loop, the +1 and the -1 loop) are summed in input
    order, which is scipy's for rows of at most 16 stored entries."""
    row, col, w, dev = _coo_input(row, col, data, device)
    segsum = _segsum_default(dev, segsum)
    rr, cc, ws, theta = _magnetic_parts(row, col, w, n, q, segsum)
    deg = segsum(_indptr(rr, n), ws)
    left, right = _host_pow(deg, r - 1), _host_pow(deg, -r)
    cq, sq = _host_phase(theta, q)
    re, im = _phase_product(left[rr] * ws * right[cc], cq, sq)
    loops = torch.arange(n, device=dev)
    one = torch.ones(n, dtype=re.dtype, device=dev)
    # add_self_loops(edge_index, -w, fill 1+0j), then (2 * x) / 2 with inf -> 0.  torch negates a
    # complex tensor as 0 - x in its vectorised loop (so -(+0) = +0; its scalar tail flips the sign
    # instead: signed zeros of the last few entries may differ, values never do)
    z = torch.zeros_like(re)
    re1 = torch.cat([z - re, one]) * 2.0 / 2
    im1 = torch.cat([z - im, torch.zeros(n, dtype=im.dtype, device=dev)]) * 2.0 / 2
    re1.masked_fill_(re1 == float("inf"), 0)
    im1.masked_fill_(im1 == float("inf"), 0)
    R1, C1 = torch.cat([rr, loops]), torch.cat([cc, loops])
    R2, C2 = torch.cat([R1, loops]), torch.cat([C1, loops])
    re2 = torch.cat([re1, -one])
    return _csr_from_coo(R2, C2, re2, n, segsum), _csr_from_coo(R1, C1, im1, n, segsum)


# ----------------------------------------------------------------------------------------------
# in / out directed Laplacian (utils.py:195-260)
# ----------------------------------------------------------------------------------------------
def _loops_appended(row, col, n, dev):
    """add_self_loops(edge_index, ones, 1, N): (rows, cols, fp32 ones) with the loops last."""
    loops = torch.arange(n, device=dev)
    R, C = torch.cat([row, loops]), torch.cat([col, loops])
    return R, C, torch.ones(R.numel(), dtype=torch.float32, device=dev)


def _row_scatter(R, vals, n, segsum):
    """scatter_add(vals, R, dim_size=n): per row, a sequential sum in element order."""
    key, perm = torch.sort(R, stable=True)
    return segsum(_indptr(key, n), vals[perm])


def _sym_rownorm(rows, cols, vals, n, r, segsum):
    """The normalisation the reference repeats on each dense-derived operator (utils.py:230-237,
    248-255, 314-320, 383-390, 413-420): degrees by scatter_add in entry order, then
    deg^(r-1)[row] * v * deg^(-r)[col] (fp32)."""
    deg = _row_scatter(rows, vals, n, segsum)
    left, right = _host_pow(deg, r - 1), _host_pow(deg, -r)
    return left[rows] * vals * right[cols]


def _dense_guard(n, mats, dev):
    if n > _DENSE_LIMIT:
        raise ValueError(f"this operator forms dense N x N products as the reference does (utils.py:216-218, "
                         f"338-345); N = {n} exceeds the supported {_DENSE_LIMIT}")
    if dev.type == "cuda":
        free, _ = torch.cuda.mem_get_info(dev)
        need = mats * n * n * 8
        if need > 0.9 * free:
            raise MemoryError(f"dense N x N steps need {need / 2**30:.1f} GiB, {free / 2**30:.1f} GiB free")


def _dense_nonzero_csr(M32, n):
    """torch.nonzero(M) (row-major) of a dense fp32 matrix: (rows, cols, values)."""
    nz = torch.nonzero(M32, as_tuple=False)
    rows, cols = nz[:, 0], nz[:, 1]
    return rows, cols, M32[rows, cols]


def in_out_norm(row, col, n: int, r: float, device=None, segsum=None, gemm=None):
    """adj_to_un_in_out_dir_symmetric_norm (utils.py:195-260): (un, in, out) CSR device tensors, fp32.
    un = D^(r-1) (A + I) D^(-r) over the stored edges plus loops (bit-identical); in / out are the
    symmetric normalisations of P^T P and P P^T, P = D^-1 (A + I) (fp64 GEMMs rounded to fp32)."""
    row, col, _, dev = _coo_input(row, col, None, device)
    segsum = _segsum_default(dev, segsum)
    R, C, ew = _loops_appended(row, col, n, dev)
    deg = _row_scatter(R, ew, n, segsum)
    left, right = _host_pow(deg, r - 1), _host_pow(deg, -r)
    un = _csr_from_coo(R, C, left[R] * ew * right[C], n, segsum)
    _dense_guard(n, 3, dev)
    P = _dense_p(R, C, ew, deg, n, dev)
    gemm = gemm or (lambda a, b: a @ b)
    in_L = gemm(P.t(), P).to(torch.float32)
    out_L = gemm(P, P.t()).to(torch.float32)
    del P
    out_L[torch.isnan(in_L)] = 0
    in_L[torch.isnan(in_L)] = 0
    mats = []
    for M in (in_L, out_L):
        rows, cols, vals = _dense_nonzero_csr(M, n)
        w = _sym_rownorm(rows, cols, vals, n, r, segsum)
        mats.append((_indptr(rows, n), cols.to(torch.int32), w))
    return un, mats[0], mats[1]


def _dense_p(R, C, ew, deg, n, dev):
    """P = D^-1 (A + I) as a dense fp64 matrix of its fp32 entries (duplicate entries added, as
    torch.sparse to_dense does)."""
    inv = _host_pow(deg, -1)                       # deg.pow(-1), inf -> 0
    p = (inv[R] * ew).to(torch.float64)
    P = torch.zeros((n, n), dtype=torch.float64, device=dev)
    P.index_put_((R, C), p, accumulate=True)
    return P.to(torch.float32).to(torch.float64)   # the reference's entries are fp32 sums


# ----------------------------------------------------------------------------------------------
# fast PPR approximation (utils.py:262-322)
# ----------------------------------------------------------------------------------------------
def fast_ppr_norm(row, col, n: int, r: float, alpha: float, max_iter: int = 100, device=None,
                  segsum=None, spmv=None):
    """adj_to_fast_ppr_approx_symmetric_norm (utils.py:262-322): the PPR vector of A + I by the
    reference's power iteration (x <- W x + s (z^T x), until ||x - x_old|| <= 1e-6 or max_iter),
    L = (Pi^1/2 P Pi^-1/2 + Pi^-1/2 P^T Pi^1/2) / 2, then the symmetric normalisation in fp32."""
    row, col, _, dev = _coo_input(row, col, None, device)
    segsum = _segsum_default(dev, segsum)
    spmv = spmv or spmv64
    R, C, ew = _loops_appended(row, col, n, dev)
    ip, ix, a = _csr_from_coo(R, C, ew, n, segsum)            # sparse_adj (fp32, duplicates summed)
    arow = torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1])
    acol = ix.to(torch.int64)
    rsum = segsum(ip, a)                                       # sparse_adj.sum(axis=1), fp32
    d1 = torch.where(rsum != 0, 1 / rsum, torch.zeros_like(rsum))
    # W = ((1 - alpha) * A^T) @ D_1: W[i, j] = fl32(fl32(c * A[j, i]) * d1[j]), c = fl32(1 - alpha)
    c = torch.tensor(1 - alpha, dtype=torch.float32)
    wv = (a * c.to(dev)) * d1[arow]
    key, perm = torch.sort(acol * n + arow, stable=True)
    w_ip = _indptr(key // n, n)
    w_ix = (key % n).to(torch.int32)
    w_v = wv[perm].to(torch.float64)
    s = 1 / (1 + alpha) / n
    z = torch.where(rsum != 0, torch.tensor(alpha * (1 + alpha), dtype=torch.float64, device=dev),
                    torch.tensor((1 - alpha) / (1 + alpha) + alpha * (1 + alpha), dtype=torch.float64, device=dev))
    x = torch.full((n,), s, dtype=torch.float64, device=dev)
    old = torch.zeros_like(x)
    it = 0
    while float(torch.linalg.norm(x - old)) > 1e-6:
        old = x
        x = spmv(w_ip, w_ix, w_v, x) + s * torch.dot(z, x)
        it += 1
        if it >= max_iter:
            break
    x = x / x.sum()
    xs, xi = torch.pow(x, 0.5), torch.pow(x, -0.5)
    # p = D_1 * sparse_adj (fp32); L over the union of P's and P^T's structure, (a + b) / 2 (fp64)
    p = (d1[arow] * a).to(torch.float64)
    t1 = (xs[arow] * p) * xi[acol]
    t2 = (xi[acol] * p) * xs[arow]                  # the (acol, arow) entry of Pi^-1/2 P^T Pi^1/2
    lip, lix, lv = _csr_from_coo(torch.cat([arow, acol]), torch.cat([acol, arow]), torch.cat([t1, t2]), n,
                                 segsum, drop_zeros=True)
    lv = lv / 2.0
    lv = torch.nan_to_num(lv, nan=0.0).to(torch.float32)
    lrow = torch.repeat_interleave(torch.arange(n, device=dev), lip[1:] - lip[:-1])
    w = _sym_rownorm(lrow, lix.to(torch.int64), lv, n, r, segsum)
    return lip, lix, w


# ----------------------------------------------------------------------------------------------
# two-order PPR approximation (utils.py:324-424)
# ----------------------------------------------------------------------------------------------
def _stationary(Pt_ip, Pt_ix, Pt_v, n, alpha, spmv, tol=1e-15, max_iter=20000, check_every=32):
    """Left Perron vector of the (N+1) x (N+1) chain of utils.py:340-344 (row-stochastic:
    (1 - alpha) P and alpha to the extra node, which returns uniformly), normalised to sum 1 over
    the first N entries.  Lazy power iteration pi <- (pi + pi P_v) / 2 in fp64 (the same fixed point
    as the reference's sgeev eigenvector for eigenvalue 1, without its fp32 error)."""
    dev = Pt_v.device
    pi = torch.full((n,), 1.0 / (n + 1), dtype=torch.float64, device=dev)
    pv = torch.tensor(1.0 / (n + 1), dtype=torch.float64, device=dev)
    for it in range(max_iter):
        nxt = 0.5 * (pi + ((1 - alpha) * spmv(Pt_ip, Pt_ix, Pt_v, pi) + pv / n))
        nv = 0.5 * (pv + alpha * pi.sum())
        if it % check_every == check_every - 1:
            if float((nxt - pi).abs().sum() + (nv - pv).abs()) <= tol:
                pi, pv = nxt, nv
                break
        pi, pv = nxt, nv
    return pi / pi.sum()


def two_order_norm(row, col, n: int, r: float, alpha: float, device=None, segsum=None, spmv=None, gemm=None):
    """adj_to_slow_first_second_ppr_approx_symmetric_norm (utils.py:324-424): (one, two) CSR device
    tensors, fp32.  one: the symmetric normalisation of (Pi^1/2 P Pi^-1/2 + Pi^-1/2 P^T Pi^1/2) / 2
    with Pi the stationary distribution of the teleporting chain; two: of (P^T P + P P^T) / 2
    restricted to the entries where both are nonzero."""
    row, col, _, dev = _coo_input(row, col, None, device)
    segsum = _segsum_default(dev, segsum)
    spmv = spmv or spmv64
    R, C, ew = _loops_appended(row, col, n, dev)
    deg = _row_scatter(R, ew, n, segsum)
    inv = _host_pow(deg, -1)
    # P (fp32, duplicates added) as a sparse canonical matrix, and P^T for the chain
    pip, pix, pv = _csr_from_coo(R, C, inv[R] * ew, n, segsum)
    prow = torch.repeat_interleave(torch.arange(n, device=dev), pip[1:] - pip[:-1])
    pcol = pix.to(torch.int64)
    key, perm = torch.sort(pcol * n + prow, stable=True)
    pi = _stationary(_indptr(key // n, n), (key % n).to(torch.int32), pv[perm].to(torch.float64), n, alpha, spmv)
    pi32 = pi.to(torch.float32)
    pis, pii = torch.pow(pi32, 0.5), torch.pow(pi32, -0.5)
    pis.masked_fill_(pis == float("inf"), 0)
    pii.masked_fill_(pii == float("inf"), 0)
    # (Pi^1/2 P Pi^-1/2)[i, j] = fl(fl(pis_i P_ij) pii_j); (Pi^-1/2 P^T Pi^1/2)[j, i] = fl(fl(pii_j P_ij) pis_i)
    t1 = (pis[prow] * pv) * pii[pcol]
    t2 = (pii[pcol] * pv) * pis[prow]
    oip, oix, ov = _csr_from_coo(torch.cat([prow, pcol]), torch.cat([pcol, prow]), torch.cat([t1, t2]), n,
                                 segsum, drop_zeros=True)
    ov = torch.nan_to_num(ov / 2.0, nan=0.0)
    orow = torch.repeat_interleave(torch.arange(n, device=dev), oip[1:] - oip[:-1])
    one = (oip, oix, _sym_rownorm(orow, oix.to(torch.int64), ov, n, r, segsum))
    _dense_guard(n, 3, dev)
    P = torch.zeros((n, n), dtype=torch.float64, device=dev)
    P[prow, pcol] = pv.to(torch.float64)
    gemm = gemm or (lambda a, b: a @ b)
    L_in = gemm(P.t(), P).to(torch.float32)
    L_out = gemm(P, P.t()).to(torch.float32)
    del P
    both = (L_in != 0) & (L_out != 0)
    L2 = torch.where(both, (L_in + L_out) / 2.0, torch.zeros_like(L_in))
    del L_in, L_out
    rows, cols, vals = _dense_nonzero_csr(L2, n)
    two = (_indptr(rows, n), cols.to(torch.int32), _sym_rownorm(rows, cols, vals, n, r, segsum))
    return one, two
