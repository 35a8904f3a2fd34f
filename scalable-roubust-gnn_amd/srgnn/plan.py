"""The native one-GPU planner (srg_plan_build / srg_plan_propagate_f32, csrc/srg_plan.hip) for a DeviceCSR.

srgnn.spmm.prepare / propagate run their K-hop loops through it, and spmm.hop (the aggregation and
wavelet hop loops, the host-copy loop of GraphOp.propagate) its single hops, with the aggregation
epilogue where asked (srg_plan_hop_f32): the column blocks, block 0's split, the per-launch schedules,
the hub chain, the spans by slot and the compact launch-ordered copies are built on the device in one
pass (a radix sort of (launch, span length) keys, one scan, one copy) -- the layout
DeviceCSR.column_blocks / compact_column_blocks / split_whole + spmm._hop_plan build with torch (kept
for layout experiments with other constants, and as the layout tests' reference).  C / C++ hosts call
the same entry points (examples/plan_propagate.c).
"""
from __future__ import annotations

import ctypes

from . import _lib


class PlanDesc(ctypes.Structure):
    """srg_plan_desc (include/srgnn_hip.h)."""
    _fields_ = [("n_rows", ctypes.c_int64), ("nnz", ctypes.c_int64), ("device_bytes", ctypes.c_int64),
                ("d", ctypes.c_int32), ("col_blocks", ctypes.c_int32), ("n_launch", ctypes.c_int32),
                ("compact", ctypes.c_int32), ("split_block0", ctypes.c_int32), ("hub_chain", ctypes.c_int32),
                ("device", ctypes.c_int32)]


class HopLaunch(ctypes.Structure):
    """srg_hop_launch (include/srgnn_hip.h)."""
    _fields_ = [("row_beg", ctypes.c_void_p), ("row_end", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("row_order", ctypes.c_void_p), ("n_rows", ctypes.c_int64),
                ("n_hub", ctypes.c_int64), ("n_heavy", ctypes.c_int64), ("flags", ctypes.c_uint32),
                ("slot_beg", ctypes.c_void_p), ("slot_end", ctypes.c_void_p)]


class NativePlan:
    """A srg_plan over the arrays of square DeviceCSR `A` for a run of `hops` hops of d-column panels.

    col_blocks: 0 = automatic (spmm.auto_col_blocks' rule), else forced; compact: None = automatic
    (runs of >= SRG_PLAN_MIN_HOPS_TO_COMPACT hops, if it fits), True / False = always / never;
    split_block0: None = automatic (panels < 16 GiB), True / False.  The plan borrows A's arrays (it
    keeps references to them) and holds device memory until it is closed or collected."""

    def __init__(self, A, d: int, hops: int, col_blocks: int = 0, compact=None, split_block0=None):
        if A.is_span or A.n_rows != A.n_cols:
            raise ValueError("a plan takes a whole square operator")
        opts = 0
        if compact is not None:
            opts |= _lib.SRG_PLAN_COMPACT if compact else _lib.SRG_PLAN_SPANS
        if split_block0 is not None:
            opts |= _lib.SRG_PLAN_SPLIT_BLOCK0 if split_block0 else _lib.SRG_PLAN_WHOLE_BLOCK0
        self.device = A.device
        self._arrays = (A.indptr, A.indices, A.values)       # borrowed by the plan
        self._p = None
        p = ctypes.c_void_p()
        n = A.n_rows
        # A's thresholds (None: automatic per launch; negative: no such rows), for every launch
        hub_t, heavy_t = (_lib.SRG_PLAN_AUTO if t is None else _lib.SRG_PLAN_NONE if int(t) < 0 else int(t)
                          for t in (A.thresholds[1], A.thresholds[0]))
        _lib.call(self.device, "srg_plan_build", A.indptr.data_ptr(), A.indices.data_ptr() if A.indices.numel() else None,
                  A.values.data_ptr() if A.values.numel() else None, n, int(d), int(hops), int(col_blocks), hub_t,
                  heavy_t, opts, _lib.stream(self.device), ctypes.byref(p))
        self._p = p.value
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
        self.device_bytes = int(desc.device_bytes)

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

    def close(self) -> None:
        """Releases the plan's memory in stream order on the device's current stream."""
        p, self._p = self._p, None
        if p is not None:
            _lib.call(self.device, "srg_plan_destroy", p, _lib.stream(self.device))

    def __del__(self):
        try:
            self.close()
        except Exception:      # interpreter shutdown: the library or torch may be gone
            pass


def hop_class(hops: int) -> int:
    """0: one launch per hop, 1: column blocks, 2: compact copies -- what a run of `hops` hops buys."""
    from .spmm import MIN_HOPS_TO_CUT
    return (1 if hops >= MIN_HOPS_TO_CUT else 0) + (1 if hops >= _lib.SRG_PLAN_MIN_HOPS_TO_COMPACT else 0)


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


__all__ = ["NativePlan", "PlanDesc", "HopLaunch", "plan_for", "cached", "hop_class"]
