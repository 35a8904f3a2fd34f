"""Device API of the propagation hot path (one hop, K hops) over a `DeviceCSR`.

Every call goes through libsrgnn_hip.so; there is no CPU or torch fallback.  Kernels are enqueued
on torch's current HIP stream of the operand's device, so torch events / synchronisation see them.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .csr import DeviceCSR


_stream = _lib.stream

# K-hop runs and single hops run through the one-GPU planner (srgnn.plan -> srg_plan_build, csrc/
# srg_plan.hip): column blocks for runs of >= SRG_PLAN_MIN_HOPS_TO_CUT hops over panels of >= 512 MiB at
# d >= 64 (one block per ~100 MiB, 12 to 16; 4 from 16 GiB), block 0 as its cut rows' spans and its
# whole rows below 16 GiB, compact launch-ordered copies from SRG_PLAN_MIN_HOPS_TO_COMPACT hops when they
# fit.  The measurements behind every rule are in DESIGN.md §5.1; the rules themselves live in the
# planner only (round 6: the torch formulation of the layout is a test restatement,
# tests/plan_layout_ref.py).
# Test hooks: FORCE_COL_BLOCKS forces a block count for every automatic choice; SPLIT_BLOCK0 forces
# block 0's split on / off (None: the planner's rule).  The same bits whatever they are.
FORCE_COL_BLOCKS = None
SPLIT_BLOCK0 = None


def _forced(col_blocks) -> int:
    return int(col_blocks) if col_blocks is not None else int(FORCE_COL_BLOCKS or 0)


def prepare(A: DeviceCSR, d: int, hops: int, col_blocks=None) -> int:
    """Lays A out for a run of `hops` hops over d-column panels with the native planner (cached on A;
    rebuilt only when a longer run buys a richer layout).  col_blocks: None = automatic, else the
    blocks per hop asked for.  Returns the column blocks per hop that hop() / propagate() then run."""
    from .plan import plan_for
    return plan_for(A, d, hops, _forced(col_blocks), SPLIT_BLOCK0).col_blocks


def auto_col_blocks(A: DeviceCSR, d: int, hops: int | None = None) -> int:
    """Column blocks per hop the planner gives a run of `hops` hops over d-column panels (None: A's
    cached plan for d, or one launch) -- srg_plan_query's resolved choice, nothing built."""
    from .plan import cached, query
    if FORCE_COL_BLOCKS is not None:
        return max(1, int(FORCE_COL_BLOCKS))
    if hops is None:
        P = cached(A, d)
        return P.col_blocks if P is not None else 1
    return query(A, d, hops, 0, None, SPLIT_BLOCK0)[3]


def col_blocks_of(A: DeviceCSR, d: int) -> int:
    """The column blocks per hop hop() runs A in over a d-column panel as A is laid out now (its
    cached plan for d); 1 = the one-launch hop."""
    from .plan import cached
    P = cached(A, d)
    return P.col_blocks if P is not None else 1


def launches_per_hop(A: DeviceCSR, B: int, d: int, agg: bool = False) -> int:
    """k_spmm launches of one hop of A over a d-column panel in B column blocks: the cached plan's (its
    whole hub rows' launch is hub workgroups only, not counted), else what a plan with B blocks would
    run (B, plus one when block 0 runs as its cut spans and its whole rows).  agg: the aggregation epilogue needs no launch of its own where block 0 is split, and
    a separate accumulation pass (not a k_spmm launch) where it is not."""
    from .plan import cached, query
    P = cached(A, d)
    if P is not None and P.col_blocks == B:
        return P.spmm_launches
    if B <= 1:
        return 1
    _, _, ro, rb = query(A, d, _lib.SRG_PLAN_MIN_HOPS_TO_CUT, B, None, SPLIT_BLOCK0)
    return rb + (1 if (ro & _lib.SRG_PLAN_SPLIT_BLOCK0) and rb > 1 else 0)


def hop(A: DeviceCSR, X: torch.Tensor, out: torch.Tensor, nt_store: bool = False, col_blocks=None,
        agg=None, fast: bool = False) -> torch.Tensor:
    """out = A @ X (one hop, exact) through A's plan for X's width (srg_plan_hop_f32): the cached one
    (prepare / propagate laid A out), or a one-launch plan made here; col_blocks forces another block
    count.  Bitwise the same in every layout.  agg = (panel, w, init): the aggregation step
    (0 if init else panel) + w * out fused into the epilogue of the launches where the rows' chains
    end.  fast: SRG_SPMM_FAST for the hub rows (tolerance mode, see spmm); with agg, the step then runs
    as its own accumulation pass."""
    from .plan import cached, plan_for
    d = X.shape[1]
    _check_panel(X, A.n_cols, "X")
    _check_panel(out, A.out_rows, "out", d)
    if agg is not None:
        _check_panel(agg[0], A.out_rows, "agg", d)
    if out.device != A.device or X.device != A.device:
        raise ValueError("A, X and out must be on the same device")
    if X.numel() and X.data_ptr() == out.data_ptr():
        raise ValueError("out must not alias X (its rows are gathered)")
    _no_spans(A, "hop")
    if A.n_rows != A.n_cols:
        # a rectangular operator (a row block): one launch with its own schedule
        if col_blocks not in (None, 1):
            raise ValueError("column blocks take a square operator")
        if agg is None:
            return spmm(A, X, out=out, nt_store=nt_store, fast=fast)
        if fast:
            raise ValueError("fast with agg takes a square operator")
        return spmm_agg(A, X, out, agg[0], agg[1], agg[2], nt_store=nt_store)
    P = cached(A, d)
    if P is None or (col_blocks is not None and int(col_blocks) != P.col_blocks):
        cb = _forced(col_blocks)
        P = plan_for(A, d, _lib.SRG_PLAN_MIN_HOPS_TO_CUT if cb > 1 else 1, cb, SPLIT_BLOCK0)
    flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_FAST if fast else 0)
    if agg is None:
        P.hop(X, out, d, flags)
    elif not fast:
        P.hop(X, out, d, flags, agg[0], agg[1], agg[2])
    else:
        P.hop(X, out, d, flags)
        _lib.call(X.device, "srg_hop_accumulate_f32", agg[0].data_ptr(), agg[0].stride(0), out.data_ptr(),
                  out.stride(0), A.out_rows, d, float(agg[1]), _lib.SRG_ACC_INIT if agg[2] else _lib.SRG_ACC_ADD,
                  _stream(X.device))
    return out


def _check_panel(X: torch.Tensor, rows: int, name: str, d=None):
    if not isinstance(X, torch.Tensor) or not X.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if X.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {X.dtype}")
    if X.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(X.shape)}")
    if X.shape[0] < rows:
        raise ValueError(f"{name} has {X.shape[0]} rows, need {rows}")
    if X.stride(1) != 1:
        raise ValueError(f"{name} must be row-major with unit column stride")
    if X.shape[0] > 1 and X.stride(0) < X.shape[1]:
        raise ValueError(f"{name} rows overlap (stride(0)={X.stride(0)} < {X.shape[1]} columns): "
                         "pass a contiguous tensor, not an expanded / broadcast one")
    if d is not None and X.shape[1] != d:
        raise ValueError(f"{name} has {X.shape[1]} columns, expected {d}")


def spmm(A: DeviceCSR, X: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False,
         nt_store: bool = False, wide_rows: bool = False, hub_w256: bool = False,
         hub_nojoin: bool = False, packed_u2: bool = False, fast: bool = False,
         hub_continue: bool = False) -> torch.Tensor:
    """out[r, :] (+)= A[r, :] @ X  for the rows of A (one hop; exact fma chains in CSR order).
    fast: tolerance mode (SRG_SPMM_FAST): A's hub rows are summed as 64 exact segment chains whose
    partial sums are then added in order -- deterministic, within fp32 re-association error of the
    exact chain, ~64x shorter latency for the longest rows; every other row stays bit-exact.
    wide_rows: diagnostic, one row per wave for every light row (no narrow or packed rows);
    hub_w256: diagnostic, 256-nonzero
    hub windows for any hub launch (same results either way).  hub_nojoin: A's hub rows are left
    running on the library's side stream; the caller must make a stream wait for them
    (srg_hub_join) before reading them.  hub_continue (with hub_nojoin, after an unjoined fork):
    the hub rows are appended to the side stream without a new fork (SRG_SPMM_HUB_CONTINUE)."""
    _check_panel(X, A.n_cols, "X")
    d = X.shape[1]
    if out is None:
        if accumulate:
            raise ValueError("accumulate=True needs an out tensor")
        if A.schedules_subset:
            raise ValueError("this operator (a column block or row group) writes only some rows of a "
                             f"{A.out_rows}-row panel: pass out")
        out = torch.empty((A.n_rows, d), dtype=torch.float32, device=X.device)
    _check_panel(out, A.out_rows, "out", d)
    if out.device != A.device or X.device != A.device:
        raise ValueError("A, X and out must be on the same device")
    flags = (_lib.SRG_SPMM_ACCUMULATE if accumulate else 0) | (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | \
        (_lib.SRG_SPMM_WIDE_ROWS if wide_rows else 0) | (_lib.SRG_SPMM_HUB_W256 if hub_w256 else 0) | \
        (_lib.SRG_SPMM_HUB_NOJOIN if hub_nojoin else 0) | (_lib.SRG_SPMM_PACKED_U2 if packed_u2 else 0) | \
        (_lib.SRG_SPMM_FAST if fast else 0) | (_lib.SRG_SPMM_HUB_CONTINUE if hub_continue else 0)
    if A.is_span:
        _span_call(A, X, out, d, flags, None, 0, 0.0, False)
        return out
    _lib.call(X.device, "srg_spmm_csr_f32", A.indptr.data_ptr(), A.indices.data_ptr(), A.values.data_ptr(),
              A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d), X.data_ptr(),
              X.stride(0), out.data_ptr(), out.stride(0), d, flags, _stream(X.device))
    return out


def _span_call(A: DeviceCSR, X, out, d, flags, agg, lda, w, init):
    """A column block (row spans of a shared CSR): srg_spmm_span_f32, plain or aggregating."""
    _lib.call(X.device, "srg_spmm_span_f32", A.indptr.data_ptr(), A.row_end.data_ptr(), A.indices.data_ptr(),
              A.values.data_ptr(), A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d),
              X.data_ptr(), X.stride(0), out.data_ptr(), out.stride(0), d, flags,
              agg.data_ptr() if agg is not None else None, lda, float(w), 1 if init else 0, _stream(X.device))


def _no_spans(A: DeviceCSR, what: str):
    if A.is_span:
        raise ValueError(f"{what} takes a whole operator, not a column block")


def spmm_agg(A: DeviceCSR, X: torch.Tensor, out: torch.Tensor, agg: torch.Tensor, w: float, init: bool,
             nt_store: bool = False, accumulate: bool = False, packed_u2: bool = False,
             hub_nojoin: bool = False, hub_continue: bool = False) -> torch.Tensor:
    """out = A @ X and, fused into the same kernels' epilogue, agg = (0 if init else agg) + w * out
    (srg_spmm_agg_f32; the arithmetic of spmm followed by one srg_hop_accumulate_f32 step).
    accumulate: the chains continue from out's content (the last block of a column-blocked hop)."""
    _check_panel(X, A.n_cols, "X")
    d = X.shape[1]
    _check_panel(out, A.out_rows, "out", d)
    _check_panel(agg, A.out_rows, "agg", d)
    if not (out.device == X.device == agg.device == A.device):
        raise ValueError("A, X, out and agg must be on the same device")
    flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_ACCUMULATE if accumulate else 0) | \
        (_lib.SRG_SPMM_PACKED_U2 if packed_u2 else 0) | (_lib.SRG_SPMM_HUB_NOJOIN if hub_nojoin else 0) | \
        (_lib.SRG_SPMM_HUB_CONTINUE if hub_continue else 0)
    if A.is_span:
        _span_call(A, X, out, d, flags, agg, agg.stride(0), w, init)
        return out
    _lib.call(X.device, "srg_spmm_agg_f32", A.indptr.data_ptr(), A.indices.data_ptr(), A.values.data_ptr(),
              A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d), X.data_ptr(),
              X.stride(0), out.data_ptr(), out.stride(0), d, flags, agg.data_ptr(), agg.stride(0),
              float(w), 1 if init else 0, _stream(X.device))
    return out


def spmm_cheby(A: DeviceCSR, Tc: torch.Tensor, out: torch.Tensor, mode: int, a1: float, a2: float,
               To: torch.Tensor | None, coef_prev, coef, R: torch.Tensor) -> torch.Tensor:
    """One Chebyshev order in one launch (srg_spmm_cheby_f32): y = A @ Tc becomes, before it is stored,
    INIT: out = (y - a2*Tc) / a1, R[s] = (coef_prev[s]/2)*Tc + coef[s]*out;
    STEP: out = y - To,           R[s] += coef[s]*out
    -- srg_spmm_csr_f32 followed by srg_cheby_epilogue_f32, bit for bit.  `out` may be `To` itself
    (each element of To is read by its owner before it is overwritten).  R: [n_scales, rows, d],
    strided views allowed (row-major rows)."""
    _no_spans(A, "spmm_cheby")
    _check_panel(Tc, A.n_cols, "Tc")
    d = Tc.shape[1]
    _check_panel(out, A.out_rows, "out", d)
    if To is not None:
        _check_panel(To, A.out_rows, "To", d)
    if not isinstance(R, torch.Tensor) or R.dtype != torch.float32 or R.dim() != 3 or R.shape[1] < A.out_rows \
            or R.shape[2] != d or R.stride(2) != 1 or R.device != A.device:
        raise ValueError("R must be a float32 [n_scales, rows, d] tensor with unit column stride on A's device")
    if not (Tc.device == out.device == A.device) or (To is not None and To.device != A.device):
        raise ValueError("A and the panels must be on the same device")
    ns = R.shape[0]
    if len(coef) != ns or (mode == _lib.SRG_CHEBY_INIT and (coef_prev is None or len(coef_prev) != ns)):
        raise ValueError("one coefficient per scale")
    cur = (ctypes.c_float * ns)(*[float(c) for c in coef])
    prev = (ctypes.c_float * ns)(*[float(c) for c in coef_prev]) if coef_prev is not None else None
    _lib.call(Tc.device, "srg_spmm_cheby_f32", A.indptr.data_ptr(), A.indices.data_ptr(), A.values.data_ptr(),
              A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d), Tc.data_ptr(),
              Tc.stride(0), out.data_ptr(), out.stride(0), d, 0, mode, float(a1), float(a2),
              To.data_ptr() if To is not None else None, To.stride(0) if To is not None else 0,
              prev, cur, ns, R.data_ptr(), R.stride(1), R.stride(0), _stream(Tc.device))
    return out


def gather_rows(src: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = src[idx[i]] (srg_gather_rows_f32; the halo exchange's send-side pack), the same rows
    as src.index_select(0, idx).  idx: int64 on src's device, every entry in [0, src.shape[0])."""
    _check_panel(src, 0, "src")
    d = src.shape[1]
    if not isinstance(idx, torch.Tensor) or idx.dtype != torch.int64 or idx.dim() != 1 or idx.device != src.device:
        raise ValueError("idx must be a 1-D int64 tensor on src's device")
    if not idx.is_contiguous():
        idx = idx.contiguous()
    if out is None:
        out = torch.empty((idx.numel(), d), dtype=torch.float32, device=src.device)
    _check_panel(out, idx.numel(), "out", d)
    _lib.call(src.device, "srg_gather_rows_f32", src.data_ptr(), src.stride(0) if src.shape[0] > 1 else d,
              src.shape[0], idx.data_ptr() if idx.numel() else None, idx.numel(), out.data_ptr(),
              out.stride(0) if out.shape[0] > 1 else d, d, _stream(src.device))
    return out


def propagate(A: DeviceCSR, X: torch.Tensor, K: int, panels: list | None = None,
              nt_store: bool = False, col_blocks=None, fast: bool = False) -> list:
    """[X, ÂX, …, Â^K X] as device tensors (panels[0] is X itself, like the reference's list).

    Device-resident form of GraphOp.propagate's hop loop (SSRG/operators/base_operator.py:32-35):
    the K hops run back to back on the GPU with no host round trips, through A's plan for a K-hop run
    (srg_plan_propagate_f32).  fast: tolerance mode for the hub rows (spmm)."""
    _no_spans(A, "propagate")
    if A.n_rows != A.n_cols:
        raise ValueError("propagate needs a square operator")
    _check_panel(X, A.n_rows, "X")
    n, d = A.n_rows, X.shape[1]
    if K < 0:
        raise ValueError("K must be >= 0")
    X0 = X
    if panels is None and X.stride(0) != d:
        X = X.contiguous()          # kernels need one leading dimension for all panels
    if panels is None:
        buf = torch.empty((K, n, d), dtype=torch.float32, device=X.device) if K else None
        panels = [X] + [buf[k] for k in range(K)]
    if len(panels) != K + 1:
        raise ValueError("panels must hold K + 1 tensors")
    ld = panels[0].stride(0)
    for k, p in enumerate(panels):
        _check_panel(p, n, f"panels[{k}]", d)
        if p.stride(0) != ld:
            raise ValueError("all panels must share one leading dimension")
    if K > 0:
        # the native plan (srgnn.plan): layout and hop loop in the library
        from .plan import plan_for
        flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_FAST if fast else 0)
        plan_for(A, d, K, _forced(col_blocks), SPLIT_BLOCK0).propagate(panels, ld, d, K, flags)
    if panels[0] is not X0 and X is not X0:
        panels = [X0] + list(panels[1:])
    return panels
