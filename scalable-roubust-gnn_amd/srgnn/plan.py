"""The one-GPU planner (srg_plan_query / srg_plan_build_in / srg_plan_propagate_f32, csrc/srg_plan.hip) for a
DeviceCSR -- the only layout code of the package (round 6: the torch formulation of the same layout
lives on as a test restatement, tests/plan_layout_ref.py).

srgnn.spmm.prepare / propagate / hop and everything above them (the aggregation and wavelet hop loops,
GraphOp.propagate) run through it: the column blocks, block 0's split, the per-launch schedules, the
hub chain, the spans by slot and the compact launch-ordered copies are built on the device in one pass
(a radix sort of (launch, span length) keys, one scan, one copy).  The plan's memory comes from torch's
caching allocator (srg_plan_query sizes it, srg_plan_build_in builds into it), so a plan competes for
the same cached blocks as the panels instead of sitting beside them; when that memory is short the
layout steps down (compact copies -> spans -> one launch) rather than failing.  C / C++ hosts call the
same entry points (srg_plan_build allocates for them; examples/plan_propagate.c).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


class PlanDesc(ctypes.Structure):
    """srg_plan_desc (include/srgnn_hip.h)."""
    _fields_ = [("n_rows", ctypes.c_int64), ("nnz", ctypes.c_int64), ("device_bytes", ctypes.c_int64),
                ("d", ctypes.c_int32), ("col_blocks", ctypes.c_int32), ("n_launch", ctypes.c_int32),
                ("compact", ctypes.c_int32), ("split_block0", ctypes.c_int32), ("hub_chain", ctypes.c_int32),
                ("device", ctypes.c_int32), ("hub_rows_whole", ctypes.c_int32)]


class HopLaunch(ctypes.Structure):
    """srg_hop_launch (include/srgnn_hip.h)."""
    _fields_ = [("row_beg", ctypes.c_void_p), ("row_end", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("row_order", ctypes.c_void_p), ("n_rows", ctypes.c_int64),
                ("n_hub", ctypes.c_int64), ("n_heavy", ctypes.c_int64), ("flags", ctypes.c_uint32),
                ("slot_beg", ctypes.c_void_p), ("slot_end", ctypes.c_void_p)]


def _opts(compact, split_block0) -> int:
    opts = 0
    if compact is not None:
        opts |= _lib.SRG_PLAN_COMPACT if compact else _lib.SRG_PLAN_SPANS
    if split_block0 is not None:
        opts |= _lib.SRG_PLAN_SPLIT_BLOCK0 if split_block0 else _lib.SRG_PLAN_WHOLE_BLOCK0
    return opts


def _thresholds(A):
    """A's (hub, heavy) thresholds as the planner takes them (None: automatic per launch; negative: no
    such rows)."""
    return tuple(_lib.SRG_PLAN_AUTO if t is None else _lib.SRG_PLAN_NONE if int(t) < 0 else int(t)
                 for t in (A.thresholds[1], A.thresholds[0]))


def query(A, d: int, hops: int, col_blocks: int = 0, compact=None, split_block0=None, extra_opts: int = 0,
          thresholds=None):
    """(keep_bytes, scratch_bytes, resolved opts, resolved column blocks) of a plan for these arguments
    (srg_plan_query: one pass over indptr, nothing allocated); thresholds: (hub, heavy) as the planner takes
    them (default: A's)."""
    kb, sb = ctypes.c_size_t(), ctypes.c_size_t()
    ro, rb = ctypes.c_uint32(), ctypes.c_int32()
    hub_t, heavy_t = _thresholds(A) if thresholds is None else thresholds
    _lib.call(A.device, "srg_plan_query", A.indptr.data_ptr(), A.n_rows, int(d), int(hops), int(col_blocks), hub_t,
              heavy_t, _opts(compact, split_block0) | int(extra_opts), _lib.stream(A.device), ctypes.byref(kb),
              ctypes.byref(sb), ctypes.byref(ro), ctypes.byref(rb))
    return int(kb.value), int(sb.value), int(ro.value), int(rb.value)


def _torch_free(device) -> int:
    """Device memory a new allocation can get: free on the device plus what torch holds cached."""
    free, _ = torch.cuda.mem_get_info(device)
    return int(free) + int(torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device))


class NativePlan:
    """A srg_plan over the arrays of square DeviceCSR `A` for a run of `hops` hops of d-column panels.

    fp64: the layout of fp64 Chebyshev steps (cheby_step_f64): spans of A's arrays without fp32 values, block 0
    split, sized for the fp64 panel; hub_threshold: whole hub rows above this length (SRG_PLAN_WHOLE_HUBS;
    None: A's thresholds, or for fp64 the planner's automatic rule); whole_max: block 0's whole rows at most
    this long (None: the planner's 48).
    col_blocks: 0 = automatic (srg_plan_build's rule), else forced; compact: None = automatic (runs of
    >= SRG_PLAN_MIN_HOPS_TO_COMPACT hops, when the copies and the build's temporaries fit in a quarter
    of the memory torch can still hand out), True / False = always / never; split_block0: None =
    automatic (panels < 16 GiB), True / False.  The plan borrows A's arrays (it keeps references to
    them) and holds its memory -- a torch tensor -- until it is closed or collected.  When torch cannot
    give it that memory (after emptying its cache once), an automatic layout steps down: compact copies
    -> spans of A's arrays -> one launch per hop (the same bits every time)."""

    def __init__(self, A, d: int, hops: int, col_blocks: int = 0, compact=None, split_block0=None, fp64: bool = False,
                 hub_threshold=None, whole_max=None):
        if A.is_span or A.n_rows != A.n_cols:
            raise ValueError("a plan takes a whole square operator")
        self.device = A.device
        self._arrays = (A.indptr, A.indices, A.values)       # borrowed by the plan
        self._p = None
        self._keep = None
        n = A.n_rows
        # A's thresholds, for every launch
        hub_t, heavy_t = _thresholds(A)
        self.fp64 = bool(fp64)
        extra = 0
        if fp64:
            # fp64 Chebyshev steps (cheby_step_f64): spans of A's arrays (the values come with each step), block
            # 0 as two launches, the layout sized for the fp64 panel's bytes; hub rows above an explicit
            # threshold are whole hub rows (automatic: the planner's rule)
            d, compact, split_block0 = 2 * int(d), False, True
            hub_t = _lib.SRG_PLAN_AUTO if hub_threshold is None else int(hub_threshold)
            heavy_t = _lib.SRG_PLAN_NONE
            extra = _lib.SRG_PLAN_WHOLE_HUBS if hub_t >= 0 else 0
        elif hub_threshold is not None:
            # whole hub rows above an explicit length (SRG_PLAN_WHOLE_HUBS) instead of A's per-launch hub rows
            hub_t = int(hub_threshold)
            extra = _lib.SRG_PLAN_WHOLE_HUBS
        if whole_max is not None:
            # block 0's whole rows: at most whole_max entries (SRG_PLAN_WHOLE_MAX; the planner's default 48)
            extra |= int(whole_max) << _lib.SRG_PLAN_WHOLE_MAX_SHIFT
        if compact is None and hops >= _lib.SRG_PLAN_MIN_HOPS_TO_COMPACT:
            # the library's rule (the copies and the build's keys / ids / positions, < 32 B per entry, in a
            # quarter of the free memory) over the memory torch can hand out, cached blocks included
            compact = A.nnz * 32 <= _torch_free(self.device) // 4
        tries = [(int(col_blocks), compact)]
        if compact is not False:
            tries.append((int(col_blocks), False))
        if int(col_blocks) == 0:
            tries.append((1, False))
        last = None
        for cb, cp in tries:
            kb, sb, ro, rb = query(A, d, hops, cb, cp, split_block0, extra, (hub_t, heavy_t))
            try:
                keep, scratch = self._alloc(kb, sb)
            except torch.cuda.OutOfMemoryError as e:     # a smaller layout, the same bits
                last = e
                continue
            p = ctypes.c_void_p()
            _lib.call(self.device, "srg_plan_build_in", A.indptr.data_ptr(),
                      A.indices.data_ptr() if A.indices.numel() else None,
                      A.values.data_ptr() if A.values.numel() and not fp64 else None, n, int(d), int(hops), rb, hub_t,
                      heavy_t,
                      ro, keep.data_ptr() if kb else _dummy(self.device), kb,
                      scratch.data_ptr() if sb else _dummy(self.device), sb, _lib.stream(self.device), ctypes.byref(p))
            del scratch                 # the build has returned (and synchronised): the scratch goes back
            self._p, self._keep = p.value, keep
            break
        else:
            raise last
        self.hops = int(hops)
        self.forced = int(col_blocks) != 0
        desc = PlanDesc()
        _lib.call(self.device, "srg_plan_describe", self._p, ctypes.byref(desc))
        self.desc = desc
        self.col_blocks = int(desc.col_blocks)
        self.n_launch = int(desc.n_launch)
        self.compact = bool(desc.compact)
        self.split_block0 = bool(desc.split_block0)
        self.hub_chain = bool(desc.hub_chain)
        self.hub_rows_whole = int(desc.hub_rows_whole)
        # k_spmm launches per hop: the whole hub rows' launch is hub workgroups only
        self.spmm_launches = self.n_launch - (1 if self.hub_rows_whole else 0)
        self.device_bytes = int(desc.device_bytes)

    def _alloc(self, keep_bytes: int, scratch_bytes: int):
        """The plan's memory and the build's scratch from torch's allocator (one retry after emptying
        its cache)."""
        for attempt in range(2):
            try:
                keep = torch.empty(max(keep_bytes, 1), dtype=torch.uint8, device=self.device)
                scratch = torch.empty(max(scratch_bytes, 1), dtype=torch.uint8, device=self.device)
                return keep, scratch
            except torch.cuda.OutOfMemoryError:
                keep = scratch = None
                if attempt:
                    raise
                torch.cuda.empty_cache()

    def launches(self, d: int):
        """[(srg_hop_launch, join_hub)] of one hop over a d-column panel, as the hops run them."""
        out = []
        for i in range(self.n_launch):
            L, join = HopLaunch(), ctypes.c_int32()
            _lib.call(self.device, "srg_plan_launch", self._p, i, int(d), ctypes.byref(L), ctypes.byref(join),
                      _lib.stream(self.device))
            out.append((L, bool(join.value)))
        return out

    def propagate(self, panels, ld: int, d: int, K: int, flags: int = 0) -> None:
        """K hops: panels[k] = A @ panels[k-1] (device tensors of leading dimension ld, checked by the
        caller)."""
        if self._p is None:
            raise ValueError("the plan is closed")
        arr = (ctypes.c_void_p * (K + 1))(*[p.data_ptr() for p in panels])
        _lib.call(self.device, "srg_plan_propagate_f32", self._p, arr, int(ld), int(d), int(K), int(flags),
                  _lib.stream(self.device))

    def hop(self, X, Y, d: int, flags: int = 0, agg=None, w: float = 0.0, init: bool = False) -> None:
        """One hop Y = A @ X (device tensors with their own row strides, checked by the caller); agg: a
        panel that gets (0 if init else agg) + w * Y in the epilogue where each row's chain ends."""
        if self._p is None:
            raise ValueError("the plan is closed")
        _lib.call(self.device, "srg_plan_hop_f32", self._p, X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0),
                  int(d), int(flags), agg.data_ptr() if agg is not None else None,
                  agg.stride(0) if agg is not None else 0, float(w), 1 if init else 0, _lib.stream(self.device))

    def cheby_step_f64(self, values, Tc, To, Tn, ld: int, d: int, mode: int, a1: float, a2: float, coef_prev, coef,
                       n_scales: int, R, r_stride: int) -> None:
        """One fp64 Chebyshev order through the plan (srg_plan_cheby_step_f64): `values` the operator's fp64
        values, Tc / To / Tn / R device tensors (row stride ld), coef_prev / coef ctypes double arrays."""
        if self._p is None:
            raise ValueError("the plan is closed")
        if not self.fp64:
            raise ValueError("an fp32 plan: build it with fp64=True")
        _lib.call(self.device, "srg_plan_cheby_step_f64", self._p, values.data_ptr() if values.numel() else None,
                  Tc.data_ptr(), To.data_ptr() if To is not None else None, Tn.data_ptr(), int(ld), int(d), int(mode),
                  float(a1), float(a2), coef_prev, coef, int(n_scales), R.data_ptr(), int(r_stride),
                  _lib.stream(self.device))

    def close(self) -> None:
        """Releases the plan: srg_plan_destroy orders itself after every stream the plan's work went to
        and drains the current stream, so its memory returns to torch's cache with nothing reading it."""
        p, self._p = self._p, None
        if p is not None:
            _lib.call(self.device, "srg_plan_destroy", p, _lib.stream(self.device))
        self._keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:      # interpreter shutdown: the library or torch may be gone
            pass


_DUMMIES = {}


def _dummy(device):
    """A valid 256-byte aligned device address for an empty arena (nothing is written to it)."""
    key = str(device)
    if key not in _DUMMIES:
        _DUMMIES[key] = torch.empty(256, dtype=torch.uint8, device=device)
    return _DUMMIES[key].data_ptr()


def hop_class(hops: int) -> int:
    """0: one launch per hop, 1: column blocks, 2: compact copies -- what a run of `hops` hops buys
    (srg_plan_build's SRG_PLAN_MIN_HOPS_TO_CUT / SRG_PLAN_MIN_HOPS_TO_COMPACT)."""
    return (1 if hops >= _lib.SRG_PLAN_MIN_HOPS_TO_CUT else 0) + (1 if hops >= _lib.SRG_PLAN_MIN_HOPS_TO_COMPACT else 0)


def plan_for(A, d: int, hops: int, col_blocks: int = 0, split_block0=None) -> NativePlan:
    """A's cached plan for d-column panels, rebuilt when a longer run (a layout class up: column
    blocks, compact copies), a forced block count or a forced block-0 split asks for another."""
    key = ("native", int(d))
    P = A._blocks.get(key)
    if P is not None and ((col_blocks == 0 and not P.forced) or P.col_blocks == col_blocks) \
            and hop_class(hops) <= hop_class(P.hops) \
            and (split_block0 is None or P.col_blocks == 1 or P.split_block0 == bool(split_block0)):
        return P
    if P is not None:
        P.close()
        A._blocks.pop(key, None)
    P = NativePlan(A, d, hops, col_blocks=col_blocks, split_block0=split_block0)
    A._blocks[key] = P
    return P


def cached(A, d: int):
    return A._blocks.get(("native", int(d)))


__all__ = ["NativePlan", "PlanDesc", "HopLaunch", "plan_for", "cached", "hop_class", "query"]
