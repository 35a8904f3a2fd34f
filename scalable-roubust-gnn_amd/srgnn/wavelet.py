"""Wavelet basis (graph heat-kernel wavelets) of SpectralModel on the GPU.

The reference (SSRG/models/base_scalable/base_model.py:171-265) builds, for tau in [-s, +s]:
    G = pygsp Graph(nx.adjacency_matrix(nx.Graph(adj)));  L = D - W (combinatorial)
    c = compute_cheby_coeff(Heat(G, tau), m = order);     lmax = G.estimate_lmax()
    phi_tau = cheby_op(G, c, identity blocks of 1000 columns), thresholded at `tolerance`
then L1-normalises each phi row (sklearn normalize).  cheby_op is the Chebyshev recurrence
    T0 = S,  T1 = (L S - a2 S) / a1,  T_{k+1} = (2/a1)(L - a2 I) T_k - T_{k-1},  a1 = a2 = lmax/2
    R = c0/2 T0 + sum_k c_k T_k
Here every Chebyshev order is ONE fused launch of srg_cheby_step_{f64,f32}: the SpMM row-wave
gather plus an epilogue that forms T_{k+1} and accumulates every scale's output R_s in the same
pass (all scales share the T_k panels, so two scales cost one recurrence, not two).  In fp64 (the
reference's precision) the longest rows run as LDS-fed hub workgroups beside the row waves, and panels
that outgrow the Infinity Cache run each order over a column-blocked plan (srg_plan_cheby_step_f64:
one launch per column block, the chains continued through Tn, the same bits).  For fp32 on
large power-law graphs (`split=True`, the default for fp32) each order is instead the
load-balanced SpMM (slice waves, hub workgroups) plus srg_cheby_epilogue_f32 -- bit-identical to
the fused kernel -- and the panel can be filtered in column blocks (`col_block`) so that
billion-edge graphs with d = 256 fit in HBM (R is written in place, no block copies).

pygsp is not available offline: the restatement follows pygsp 0.5.x semantics.  phi and phi^-1 are
bit-identical to the reference's own SpectralModel.preprocess run with pygsp restated
(tests/golden/wav_*.npz) and validated against a dense eigendecomposition.  lmax is an
explicit input (pygsp's ARPACK estimate uses a random start vector); `estimate_lmax` gives the
same estimator (eigsh, tol 5e-3, x1.01) with a fixed start vector.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from .csr import DeviceCSR, _auto_heavy, make_schedule, narrow_heavy


def laplacian_from_adj(adj: sp.spmatrix) -> sp.csr_matrix:
    """L = D - W of nx.Graph(adj): undirected, one weight per node pair (the entry stored last in
    row-major order wins, as networkx overwrites edge data), self-loops kept.  Every diagonal
    entry is stored explicitly (also for isolated nodes), so L - a2*I keeps L's structure."""
    coo = sp.coo_matrix(adj)
    n = coo.shape[0]
    order = np.lexsort((coo.col, coo.row))          # row-major
    r, c, v = coo.row[order].astype(np.int64), coo.col[order].astype(np.int64), coo.data[order].astype(np.float64)
    lo, hi = np.minimum(r, c), np.maximum(r, c)
    key = lo * n + hi
    rk = key[::-1]
    _, first_in_rev = np.unique(rk, return_index=True)
    last = key.size - 1 - first_in_rev               # last occurrence in row-major order
    lo, hi, v = lo[last], hi[last], v[last]
    off = lo != hi
    rows = np.r_[lo, hi[off]]
    cols = np.r_[hi, lo[off]]
    vals = np.r_[v, v[off]]
    W = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    deg = np.asarray(W.sum(axis=1)).ravel()
    return _explicit_diagonal((sp.diags(deg) - W).tocsr())


def _explicit_diagonal(L: sp.csr_matrix) -> sp.csr_matrix:
    """CSR with one stored entry per diagonal slot (value possibly 0), sorted, no duplicates."""
    L = sp.csr_matrix(L, dtype=np.float64, copy=True)
    L.sum_duplicates()
    n = L.shape[0]
    rows = np.repeat(np.arange(n), np.diff(L.indptr))
    have = np.zeros(n, dtype=bool)
    have[rows[L.indices == rows]] = True
    if have.all():
        return L
    add = np.flatnonzero(~have)
    r = np.r_[rows, add]
    c = np.r_[L.indices, add]
    v = np.r_[L.data, np.zeros(add.size)]
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ptr, r + 1, 1)
    return sp.csr_matrix((v, c.astype(np.int32), np.cumsum(ptr)), shape=(n, n))


def estimate_lmax(L: sp.spmatrix) -> float:
    """pygsp Graph.estimate_lmax: largest eigenvalue by ARPACK (tol 5e-3, ncv <= 10) times 1.01,
    with a fixed start vector (a ramp; the constant vector is L's null space) instead of ARPACK's
    random one."""
    n = L.shape[0]
    if n <= 2:
        return float(np.linalg.eigvalsh(L.toarray()).max()) * 1.01
    from scipy.sparse.linalg import eigsh
    lam = eigsh(L.asfptype() if hasattr(L, "asfptype") else L.astype(np.float64), k=1, tol=5e-3,
                ncv=min(n, 10), v0=np.linspace(1.0, 2.0, n), return_eigenvectors=False)
    return float(lam[0]) * 1.01


def heat_cheby_coeffs(tau: float, lmax: float, order: int) -> np.ndarray:
    """pygsp compute_cheby_coeff(filters.Heat(G, tau), m=order): g(x) = exp(-tau x / lmax) sampled
    at the order+1 Chebyshev nodes mapped to [0, lmax]."""
    N = order + 1
    a1 = a2 = lmax / 2.0
    k = np.arange(N)
    nodes = np.cos(np.pi * (k + 0.5) / N)
    g = np.exp(-tau * (a1 * nodes + a2) / lmax)
    return np.array([2.0 / N * np.dot(g, np.cos(np.pi * o * (k + 0.5) / N)) for o in range(order + 1)])


class HeatWaveletFilter:
    """R_s = sum_k c_{s,k} T_k(L~) S for the heat kernels exp(-tau_s x / lmax), every scale at once."""

    def __init__(self, L: sp.spmatrix, taus, order: int = 3, lmax: float | None = None,
                 dtype=torch.float64, device=None, heavy_threshold=None, hub_threshold=None, coeffs=None):
        L = _explicit_diagonal(sp.csr_matrix(L))
        lmax = float(lmax) if lmax is not None else estimate_lmax(L)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._setup(torch.from_numpy(L.indptr.astype(np.int64)).to(dev),
                    torch.from_numpy(L.indices.astype(np.int32)).to(dev),
                    torch.from_numpy(L.data.astype(np.float64)).to(dev), L.shape[0], taus, order, lmax,
                    dtype, heavy_threshold, hub_threshold, coeffs)

    @classmethod
    def from_coefficients(cls, L: sp.spmatrix, coeffs, lmax: float, dtype=torch.float64, device=None):
        """The Chebyshev recurrence of pygsp's cheby_op(G, c, S) with the coefficient rows `coeffs`
        ([n_scales, order + 1], any filter) on the Laplacian L."""
        return cls(L, None, lmax=lmax, dtype=dtype, device=device, coeffs=coeffs)

    @classmethod
    def from_device(cls, indptr: torch.Tensor, indices: torch.Tensor, lvals: torch.Tensor, n: int, taus,
                    order: int = 3, lmax: float = None, dtype=torch.float32, heavy_threshold=None,
                    hub_threshold=None, coeffs=None):
        """From a device CSR of L with every diagonal entry stored (e.g. normalize.laplacian_edges_blocked)
        and an explicit lmax (pygsp's ARPACK estimate is a host computation); `coeffs` instead of
        `taus` / `order`: explicit Chebyshev coefficient rows."""
        if lmax is None:
            raise ValueError("lmax is required for a device-built Laplacian")
        self = cls.__new__(cls)
        self._setup(indptr, indices, lvals, n, taus, order, float(lmax), dtype, heavy_threshold, hub_threshold,
                    coeffs)
        return self

    def _setup(self, indptr, indices, lvals, n, taus, order, lmax, dtype, heavy_threshold, hub_threshold,
               coeffs=None):
        if coeffs is not None:
            coeffs = np.atleast_2d(np.asarray(coeffs, dtype=np.float64))
            order = coeffs.shape[1] - 1
            taus = [None] * coeffs.shape[0]
        if order < 1:
            raise ValueError("order must be >= 1")
        if len(taus) < 1 or len(taus) > 8:
            raise ValueError("1..8 scales")
        if dtype not in (torch.float64, torch.float32):
            raise TypeError("dtype must be float64 or float32")
        self.device = indptr.device
        self.n = int(n)
        self.lmax = lmax
        self.a1 = self.a2 = self.lmax / 2.0
        if coeffs is not None:
            self.taus = taus
            self.coeffs = coeffs
        else:
            self.taus = [float(t) for t in taus]
            self.coeffs = np.stack([heat_cheby_coeffs(t, self.lmax, order) for t in self.taus])
        self.dtype = dtype
        self.indptr, self.indices = indptr, indices
        # F = (2/a1)(L - a2 I), formed in fp64 then rounded (the diagonal is stored explicitly)
        rows = torch.repeat_interleave(torch.arange(self.n, device=self.device),
                                       indptr[1:] - indptr[:-1]) if self.n else indptr[:0]
        diag = indices.to(torch.int64) == rows
        del rows
        l64 = lvals.to(torch.float64)
        self.fvals = ((2.0 / self.a1) * torch.where(diag, l64 - self.a2, l64)).to(dtype)
        del diag, l64
        self.lvals = lvals.to(dtype)
        # the lean epilogue sequence (SRG_CHEBY_INIT_T / STEP_FIRST / NO_T) of the split path and of the fused
        # steps; False runs INIT + STEP epilogues (same bits; set the attribute for A/B runs)
        self.lean_epilogue = True
        self.order, self.n_heavy, self.n_hub = make_schedule(self.indptr, heavy_threshold, hub_threshold)
        self.thresholds = (heavy_threshold, hub_threshold)
        self.n_heavy_narrow = narrow_heavy(self.indptr, self.n_hub) if _auto_heavy(heavy_threshold) else None

    def _coef(self, ct, vals):
        return (ct * len(vals))(*vals)

    def apply(self, S: torch.Tensor, col_block: int | None = None, split: bool | None = None,
              out: torch.Tensor | None = None, fused_epilogue: bool = False) -> torch.Tensor:
        """[n_scales, n, d] filter outputs for the panel S [n, d] (device tensor).  fp32 defaults to
        the split path (load-balanced SpMM + epilogue), in column blocks of `col_block`.
        fused_epilogue (split path): each order is one srg_spmm_cheby_f32 launch writing T_{k+1}
        over T_{k-1}, so a block needs two work panels instead of three.  Same bits either way;
        slower where measured (the epilogue's row accesses follow the schedule's row order instead
        of streaming: products 10.5 vs 9.0 ms per order), so only for when memory is short."""
        if not S.is_cuda or S.shape[0] != self.n or S.dim() != 2:
            raise ValueError("S must be a [n, d] device tensor")
        if split is None:
            split = self.dtype == torch.float32
        if split and self.dtype != torch.float32:
            raise ValueError("the split path is fp32 only")
        if S.dtype != self.dtype or S.stride(1) != 1:
            S = S.to(self.dtype).contiguous()
        n, d = S.shape
        ns = self.coeffs.shape[0]
        R = out if out is not None else torch.empty((ns, n, d), dtype=self.dtype, device=S.device)
        if tuple(R.shape) != (ns, n, d) or R.dtype != self.dtype or R.stride(2) != 1:
            raise ValueError("out must be a [n_scales, n, d] panel stack of the filter dtype")
        if not split:
            if S.stride(0) != d or R.stride(1) != d or R.stride(0) != n * d:
                S = S.contiguous()
                if out is not None:
                    raise ValueError("the fused path needs contiguous S and out")
            return self._apply_fused(S, R)
        cb = d if not col_block else min(int(col_block), d)
        work = [torch.empty((n, cb), dtype=torch.float32, device=S.device)
                for _ in range(self.work_panels(fused_epilogue))]
        for c0 in range(0, d, cb):
            w = min(cb, d - c0)
            self._apply_split(S[:, c0:c0 + w], R[:, :, c0:c0 + w],
                              [t.view(-1)[: n * w].view(n, w) for t in work], fused_epilogue)
        return R

    # fp64 steps over column blocks (srg_plan_cheby_step_f64): None = the planner's rule for the fp64 panel's
    # bytes (blocked from ~512 MiB panels), else forced; whole hub rows of the blocked steps: None = rows
    # longer than hub64_rule(nnz), else an explicit row length (SRG_PLAN_WHOLE_HUBS)
    col_blocks64 = None
    hub64_threshold = None
    # block 0's whole rows of the blocked fp64 steps (None: the planner's 48 entries)
    whole64_max = None

    @staticmethod
    def hub64_rule(nnz: int) -> int:
        """Whole hub rows of the blocked fp64 steps: rows longer than max(2048, nnz / 4096) entries, four times
        as many as the fp32 hops' rule.  An fp64 row wave keeps 8 KiB of 1 KiB rows in flight, so its chain
        is the longer one; products, 16 blocks, one STEP order (profiles/r06i_cheby64_plan_sweep.txt): 17.7 ms
        with the fp32 rule's one hub row, 13.8 with 23 (> 32,768 entries), 14.0 with 252 (> 16,384)."""
        return max(2048, int(nnz) // 4096)

    def _plan64(self, d: int):
        """The column-blocked layout of the fp64 steps over d-column panels (srgnn.plan.NativePlan with
        fp64=True: one plan for L and F, whose entries share positions), or None where the panel stays one
        launch per order."""
        key = (int(d), self.col_blocks64, self.hub64_threshold, self.whole64_max)
        cache = self.__dict__.setdefault("_plans64", {})
        if key not in cache:
            from .plan import NativePlan, query
            A = self._csr(self.fvals)
            cb = int(self.col_blocks64 or 0)
            ht = self.hub64_rule(int(self.indices.numel())) if self.hub64_threshold is None else int(self.hub64_threshold)
            # the run a filter serves: every order of every apply (bench / basis batches reuse it)
            hops = 1 << 20
            wm = (int(self.whole64_max) << _lib.SRG_PLAN_WHOLE_MAX_SHIFT) if self.whole64_max else 0
            _, _, _, B = query(A, 2 * d, hops, cb, False, True, (_lib.SRG_PLAN_WHOLE_HUBS if ht >= 0 else 0) | wm,
                               (ht, _lib.SRG_PLAN_NONE))
            cache[key] = (NativePlan(A, d, hops, col_blocks=cb, fp64=True, hub_threshold=ht, whole_max=self.whole64_max)
                          if B > 1 else None)
        return cache[key]

    def _n_hub64(self) -> int:
        """Hub rows of the one-launch fp64 step: the schedule's first rows longer than hub64_rule(nnz) (the
        fp64 rule; an explicit hub_threshold keeps the schedule's own n_hub).  The schedule lists rows by
        decreasing length, so these are its first n rows."""
        if self.thresholds[1] is not None:
            return self.n_hub
        if "_nh64" not in self.__dict__:
            deg = self.indptr[1:] - self.indptr[:-1]
            self._nh64 = int((deg > self.hub64_rule(int(self.indices.numel()))).sum().item()) if self.n else 0
        return self._nh64

    def order_step(self, vals, Tc, To, Tn, mode, coef_prev, coef, R) -> None:
        """One Chebyshev order over [n, d] panels sharing one row stride (R: [n_scales, n, d] with that row
        stride): srg_cheby_step_f32, or in fp64 srg_plan_cheby_step_f64 over the filter's column-blocked plan
        where the panel is blocked, else srg_cheby_step_hub_f64 with the schedule's hub rows as hub
        workgroups -- the same bits every way.  (Feature chunks of 64 / 32 columns, each its own blocked step,
        measured 9-15 % / 85 % slower: profiles/r06p_products_cheby64_feature_chunks_negative.txt.)"""
        n, d = Tc.shape
        f64 = self.dtype == torch.float64
        ld = Tc.stride(0)
        if any(t is not None and (t.stride(0) != ld or t.stride(1) != 1) for t in (Tc, To, Tn)) or \
                R.stride(1) != ld or R.stride(2) != 1:
            raise ValueError("the step's panels share one row stride")
        ns = self.coeffs.shape[0]
        rs = R.stride(0)
        ct = ctypes.c_double if f64 else ctypes.c_float
        cp = self._coef(ct, coef_prev) if coef_prev is not None else None
        cc = self._coef(ct, coef) if coef is not None else None
        To_p = To.data_ptr() if To is not None else None
        if f64:
            P = self._plan64(d)
            if P is not None:
                P.cheby_step_f64(vals, Tc, To, Tn, ld, d, mode, self.a1, self.a2, cp, cc, ns, R, rs)
                return
            _lib.call(Tc.device, "srg_cheby_step_hub_f64", self.indptr.data_ptr(), self.indices.data_ptr(),
                      vals.data_ptr(), n, self.order.data_ptr(), self._n_hub64(), Tc.data_ptr(), To_p, Tn.data_ptr(), ld, d,
                      mode, self.a1, self.a2, cp, cc, ns, R.data_ptr(), rs, _lib.stream(Tc.device))
            return
        _lib.call(Tc.device, "srg_cheby_step_f32", self.indptr.data_ptr(), self.indices.data_ptr(), vals.data_ptr(), n,
                  self.order.data_ptr(), Tc.data_ptr(), To_p, Tn.data_ptr(), ld, d, mode, self.a1, self.a2, cp, cc, ns,
                  R.data_ptr(), rs, _lib.stream(Tc.device))

    def _apply_fused(self, S, R):
        nc = self.coeffs.shape[1]
        c = self.coeffs

        def launch(vals, Tc, To, Tn, mode, coef_prev, coef):
            self.order_step(vals, Tc, To, Tn, mode, coef_prev, coef, R)

        # the lean sequence (order >= 2): order 1 stores T1 only, order 2 forms R from T0, T1, T2, the last
        # order stores no T -- the same operations in the same order as INIT + STEP..., four panel passes less
        lean = self.lean_epilogue and nc > 2
        # T_{k-1}, T_k and the free panel rotate through three buffers (S itself is never written)
        t_old, t_cur = S, torch.empty_like(S)
        free = [torch.empty_like(S)] if nc > 2 else []
        if lean:
            launch(self.lvals, S, None, t_cur, _lib.SRG_CHEBY_INIT_T, None, None)
        else:
            launch(self.lvals, S, None, t_cur, _lib.SRG_CHEBY_INIT, c[:, 0], c[:, 1])
        for k in range(2, nc):
            t_new = free.pop() if free else torch.empty_like(S)
            last = _lib.SRG_CHEBY_NO_T if lean and k == nc - 1 else 0
            if lean and k == 2:
                launch(self.fvals, t_cur, t_old, t_new, _lib.SRG_CHEBY_STEP_FIRST | last, np.concatenate([c[:, 0], c[:, 1]]),
                       c[:, 2])
            else:
                launch(self.fvals, t_cur, t_old, t_new, _lib.SRG_CHEBY_STEP | last, None, c[:, k])
            if t_old is not S:
                free.append(t_old)
            t_old, t_cur = t_cur, t_new
        return R

    def _csr(self, vals):
        """The operator with values `vals` (L or F), built once per value array so that its column
        blocks (spmm.hop) are cut once."""
        cache = self.__dict__.setdefault("_csr_cache", {})
        if id(vals) not in cache:
            cache[id(vals)] = DeviceCSR(self.indptr, self.indices, vals, self.n, self.n, self.order, self.n_heavy,
                                        self.n_hub, self.n_heavy_narrow, thresholds=self.thresholds)
        return cache[id(vals)]

    def prepare_column_blocks(self, width: int, hops: int) -> int:
        """Lay L and F out (spmm.prepare: the native plan, column blocks when `hops` SpMMs over panels
        `width` columns wide amortise them) for the split path's hops; returns the blocks per SpMM.
        The plans' memory comes from torch's caching allocator (srgnn.plan), so where the panels fill
        the GPU (the RMAT-26 filter bank) the plans reuse the blocks the graph build left cached."""
        from .spmm import prepare
        B = 1
        for vals in (self.lvals, self.fvals):
            B = prepare(self._csr(vals), width, hops)
        return B

    def drop_layouts(self) -> None:
        """Frees L's and F's cached layouts (native plans, column blocks) and the fp64 steps' plans."""
        for vals in (self.lvals, self.fvals):
            self._csr(vals).drop_blocks()
        for P in self.__dict__.pop("_plans64", {}).values():
            if P is not None:
                P.close()

    def work_panels(self, fused_epilogue: bool = False) -> int:
        """[n, column block] work panels the split path needs: T_1 alone for order 1; T_{k-1} and
        T_k with the fused epilogue (T_{k+1} overwrites T_{k-1}); one more for the SpMM's raw
        output without it."""
        return 1 if self.coeffs.shape[1] <= 2 else (2 if fused_epilogue else 3)

    def _apply_split(self, Sb, Rb, work, fused_epilogue: bool = False):
        """One column block: Sb [n, w] and Rb [ns, n, w] may be strided views."""
        from .spmm import hop, spmm_cheby
        n, w = Sb.shape
        ns, nc = self.coeffs.shape
        ct = ctypes.c_float
        stream = _lib.stream(Sb.device)
        Lm, Fm = self._csr(self.lvals), self._csr(self.fvals)
        if fused_epilogue:
            t_old, t_cur = Sb, work[0]
            spmm_cheby(Lm, Sb, t_cur, _lib.SRG_CHEBY_INIT, self.a1, self.a2, None, self.coeffs[:, 0],
                       self.coeffs[:, 1], Rb)
            for k in range(2, nc):
                t_new = work[1] if t_old is Sb else t_old      # T_{k+1} over T_{k-1} (never over S)
                spmm_cheby(Fm, t_cur, t_new, _lib.SRG_CHEBY_STEP, self.a1, self.a2, t_old, None,
                           self.coeffs[:, k], Rb)
                t_old, t_cur = t_cur, t_new
            return

        def epi(Tn, Tc, To, mode, coef_prev, coef):
            cp = self._coef(ct, coef_prev) if coef_prev is not None else None
            cc = self._coef(ct, coef) if coef is not None else None
            _lib.call(Sb.device, "srg_cheby_epilogue_f32", Tn.data_ptr(), Tn.stride(0),
                      Tc.data_ptr() if Tc is not None else None, Tc.stride(0) if Tc is not None else w,
                      To.data_ptr() if To is not None else None, To.stride(0) if To is not None else w, n, w,
                      mode, self.a1, self.a2, cp, cc, ns, Rb.data_ptr(), Rb.stride(1), Rb.stride(0), stream)

        # lean epilogues (order >= 2): order 1 stores T1 only, order 2 forms R from T0, T1, T2 at
        # once, the last order does not store its T -- the same operations in the same order as
        # INIT + STEP..., four panel passes less for order 3
        lean = self.lean_epilogue and nc > 2
        t_old, t_cur = Sb, work[0]
        free = list(work[1:])
        hop(Lm, Sb, t_cur)                 # column-blocked where spmm.auto_col_blocks says so
        if lean:
            epi(t_cur, Sb, None, _lib.SRG_CHEBY_INIT_T, None, None)
        else:
            epi(t_cur, Sb, None, _lib.SRG_CHEBY_INIT, self.coeffs[:, 0], self.coeffs[:, 1])
        for k in range(2, nc):
            t_new = free.pop()
            hop(Fm, t_cur, t_new)
            last = _lib.SRG_CHEBY_NO_T if lean and k == nc - 1 else 0
            if lean and k == 2:
                epi(t_new, t_cur, t_old, _lib.SRG_CHEBY_STEP_FIRST | last,
                    np.concatenate([self.coeffs[:, 0], self.coeffs[:, 1]]), self.coeffs[:, 2])
            else:
                epi(t_new, None, t_old, _lib.SRG_CHEBY_STEP | last, None, self.coeffs[:, k])
            if t_old is not Sb:
                free.append(t_old)
            t_old, t_cur = t_cur, t_new


def wavelet_basis(adj: sp.spmatrix, scale: float = 0.5, order: int = 3, tolerance: float = 1e-4,
                  lmax: float | None = None, batch: int = 1000, device=None):
    """phi (tau = -scale) and phi^-1 (tau = +scale) as L1-row-normalised fp32 CSR matrices, as
    SpectralModel.preprocess builds them (base_model.py:186-193, 236-265, 287-290): identity
    blocks of `batch` columns filtered on the GPU (both scales in one recurrence), entries below
    `tolerance` zeroed."""
    L = laplacian_from_adj(adj)
    filt = HeatWaveletFilter(L, [-scale, scale], order=order, lmax=lmax, device=device)
    n = L.shape[0]
    blocks = [[], []]
    for c0 in range(0, n, batch):
        w = min(batch, n - c0)
        S = torch.zeros((n, w), dtype=torch.float64, device=filt.device)
        S[torch.arange(c0, c0 + w, device=filt.device), torch.arange(w, device=filt.device)] = 1.0
        R = filt.apply(S).cpu().numpy()
        for s in range(2):
            sub = R[s]
            sub[sub < tolerance] = 0
            blocks[s].append(sp.csr_matrix(sub.astype(np.float32)))
    out = []
    for s in range(2):
        phi = sp.hstack(blocks[s]).tocsr()
        out.append(l1_normalize_rows(phi, device=filt.device))
    return out[0], out[1], filt.lmax


def l1_normalize_rows(phi: sp.csr_matrix, device=None) -> sp.csr_matrix:
    """sklearn.preprocessing.normalize(phi, norm='l1', axis=1) (base_model.py:287-290) on the GPU:
    per row, the fp64 sum of |x| left to right (srg_segment_sum_f64), then x / sum in fp64
    rounded to the matrix dtype; all-zero rows left as they are -- sklearn's
    _inplace_csr_row_normalize_l1 arithmetic exactly."""
    from .construct import segment_sum_device
    phi = sp.csr_matrix(phi, copy=True)
    if phi.nnz == 0:
        return phi
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    ip = torch.from_numpy(phi.indptr.astype(np.int64)).to(dev)
    x = torch.from_numpy(phi.data).to(dev)
    sums = segment_sum_device(ip, x.to(torch.float64).abs())
    rows = torch.repeat_interleave(torch.arange(phi.shape[0], device=dev), ip[1:] - ip[:-1])
    den = sums[rows]
    out = torch.where(den == 0, x.to(torch.float64), x.to(torch.float64) / den).to(x.dtype)
    phi.data = out.cpu().numpy()
    return phi


def spectral_features(adj: sp.spmatrix, feature, scale: float = 0.5, order: int = 3, tolerance: float = 1e-4,
                      lmax: float | None = None, batch: int = 1000, device=None):
    """SpectralModel.preprocess's processed_feature (base_model.py:180-219):
    [X | relu(phi phi^-1 X)] as a CPU float32 tensor, with phi / phi^-1 from wavelet_basis.

    The reference forms the product matrix phi phi^-1 with torch_sparse.spspmm and then multiplies
    X; here phi (phi^-1 X) is two exact-chain SpMMs on the GPU (no SpGEMM, no N x N product).
    Same value up to floating-point association: the tests compare against the reference's
    processed_feature (tests/golden/wav_*.npz) within 1e-5 and against a dense fp64 evaluation."""
    from .csr import DeviceCSR
    from .spmm import spmm
    phi, phi_inv, lmax = wavelet_basis(adj, scale, order, tolerance, lmax, batch, device)
    X = torch.as_tensor(np.asarray(feature, dtype=np.float32))
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    A_inv = DeviceCSR.from_scipy(phi_inv, device=dev)
    A_phi = DeviceCSR.from_scipy(phi, device=dev)
    loc = torch.relu(spmm(A_phi, spmm(A_inv, X.to(dev).contiguous())))
    return torch.cat((X, loc.cpu()), dim=1), phi, phi_inv, lmax
