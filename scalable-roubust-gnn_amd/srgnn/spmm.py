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

# Column-blocked hops (DeviceCSR.column_blocks): B launches per hop, each gathering from one
# contiguous slice of X's rows, so the caches hold a larger share of the rows a launch reads; rows
# of <= csr.BLOCK_WHOLE_MAX nonzeros are not cut (block 0 computes them whole).  Measured
# (profiles/r02t-v_*): products d = 128 7.05 (one launch 7.31) -> 6.67 (B = 2) -> 6.30 ms (B = 4),
# flat over B = 4..6, 6.47 at 8; d = 256 +9 % and papers100M / RMAT-26 +3 / +2 % for B = 4 over 2 / 1;
# arxiv (X 87 MB, already cache-resident) 0.224 vs 0.163 ms at B = 2.  auto_col_blocks: 12 to 16 blocks
# for panels of 512 MiB .. 16 GiB at d >= 64 (4 to 8 before round 5's packed-row kernels) (callers pass col_blocks to force a count; FORCE_COL_BLOCKS
# forces one for every automatic choice, a test hook).
FORCE_COL_BLOCKS = None
# column blocks' launches keep 2 gathers per packed light row in flight (SRG_SPMM_PACKED_U2) for
# d >= 128: products 7.15 -> 7.03 ms per hop, d = 256 +1.3 %, d = 64 -3 % (so not there;
# profiles/r02_ab_col_blocks.txt)
_U2_BLOCKED = True
# column-blocked hops: block b's hub rows continue block b-1's side-stream fork (SRG_SPMM_HUB_CONTINUE)
# instead of a fork, dispatch delay and join per block (profiles/r03_ab_hub_chain_products.txt)
_HUB_CHAIN = True
# span launches of the native plan loop hand the packed light rows their spans by schedule slot
# (DeviceCSR.slot_spans; profiles/r03_ab_slot_spans.txt)
_SLOT_SPANS = True
# block 0 of a column-blocked hop as two launches over the same arrays (DeviceCSR.split_whole): the
# cut rows' first spans, then the rows it computes whole.  Products (1.25 GB panel): 6.21 vs 6.24 ms
# per hop, six alternations; the whole rows first, last or after the cut spans measure the same, and
# beside the blocks on a second stream 6.80 ms.  The HBM-bound giants lose: papers100M (57 GB panel)
# 245.6-246.1 vs 244.1-244.2 ms, RMAT-26 (68 GB) 314.3-315.8 vs 311.5-313.1 ms
# (profiles/r03_ab_split_block0*.txt): split for panels below SPLIT_BLOCK0_MAX_PANEL
SPLIT_BLOCK0_MAX_PANEL = 16 << 30
# None: automatic (tests force it on / off to check both layouts give the same bits)
SPLIT_BLOCK0 = None


def _split_block0(A: DeviceCSR, d: int) -> bool:
    if SPLIT_BLOCK0 is not None:
        return bool(SPLIT_BLOCK0)
    return A.n_cols * d * 4 < SPLIT_BLOCK0_MAX_PANEL


# Cutting an operator into column blocks (row spans: one binary search per row and boundary, plus
# each block's schedule) costs about 3 hops' gain (products: 1.1 ms against 0.42 ms per hop,
# tools/probes/colblock_build_time.py; 21 ms when the blocks were copies of the ids and values):
# it is cut for a run of at least this many hops, or when its blocks already exist.
MIN_HOPS_TO_CUT = 4
# Runs of this many hops copy the blocks' spans into compact arrays in launch order, when the copy fits in
# a quarter of the free memory (= SRG_PLAN_MIN_HOPS_TO_COMPACT of the native planner).  Round 5, the
# native planner (one device pass: profiles/r05_plan_products.json): the compact layout builds in
# ~1.9 ms against ~1.2 ms for spans, and each products hop runs 5.48 instead of ~5.64 ms, so the copy
# pays after ~4-5 hops.  (The torch formulation, DeviceCSR.compact_column_blocks, cost 4.6 ms more
# than spans, round 4: profiles/r04h_one_shot_products.json.)
MIN_HOPS_TO_COMPACT = 6
_COMPACT = True                   # False: spans only (A/B of the round-2 / 3 layouts)


# K-hop runs (prepare / propagate) lay the operator out with the native planner (srgnn.plan,
# csrc/srg_plan.hip: one device pass, the operator's thresholds passed on) when every layout constant
# here and in srgnn.csr has its default value; otherwise (layout experiments) with the torch
# formulation below.  Both give the same layout.
NATIVE_PLAN = True


def _native_ok(A: DeviceCSR) -> bool:
    from . import csr as C
    return (NATIVE_PLAN and _COMPACT and _HUB_CHAIN and _SLOT_SPANS and _U2_BLOCKED and not A.is_span
            and A.n_rows == A.n_cols and C.BLOCK_WHOLE_MAX == 48
            and C.BLOCK_HEAVY_PER == 30000 and C.NARROW_HEAVY_THRESHOLD == 32 and C.DEFAULT_HEAVY_THRESHOLD is None
            and C.DEFAULT_HUB_THRESHOLD is None and SPLIT_BLOCK0_MAX_PANEL == 16 << 30
            and CAP_WAVES_MIN_PANEL == 512 << 20 and MIN_HOPS_TO_CUT == 4
            and MIN_HOPS_TO_COMPACT == _lib.SRG_PLAN_MIN_HOPS_TO_COMPACT)


def prepare(A: DeviceCSR, d: int, hops: int, col_blocks=None) -> int:
    """Lays A out for a run of `hops` hops over d-column panels: column blocks (spans, or compact
    copies in launch order for long runs) or, for one launch per hop and a long run, a launch-ordered
    copy of the whole operator (DeviceCSR.schedule_ordered).  col_blocks: None = automatic, else the
    blocks per hop asked for.  Returns the column blocks per hop that hop() / propagate() then run."""
    if _native_ok(A):
        from .plan import plan_for
        cb = int(col_blocks) if col_blocks is not None else int(FORCE_COL_BLOCKS or 0)
        return plan_for(A, d, hops, cb, SPLIT_BLOCK0).col_blocks
    B = auto_col_blocks(A, d, hops=hops) if col_blocks is None else int(col_blocks)
    if B > 1 and column_blocks_for(A, B, hops=hops):
        return B
    if _COMPACT and hops >= MIN_HOPS_TO_COMPACT and not A.is_span and A.n_rows == A.n_cols:
        free, _ = torch.cuda.mem_get_info(A.device)
        if A.nnz * (A.indices.element_size() + A.values.element_size()) + 24 * A.nnz <= free // 4:
            A.schedule_ordered()
    return 1


def column_blocks_for(A: DeviceCSR, B: int, hops: int | None = None):
    """A's column blocks for a run of `hops` hops: spans, or compact copies for long runs."""
    if _COMPACT and hops is not None and hops >= MIN_HOPS_TO_COMPACT and not A.is_span:
        free, _ = torch.cuda.mem_get_info(A.device)
        # the copies (ids + values of every block: nnz entries) stay; while a block is copied its
        # int64 gather index, the arange added to it and repeat_interleave's output (<= nnz
        # entries each) are alive too
        copies = A.nnz * (A.indices.element_size() + A.values.element_size())
        if copies + 24 * A.nnz <= free // 4:
            return A.compact_column_blocks(B)
    return A.column_blocks(B)


def auto_col_blocks(A: DeviceCSR, d: int, hops: int | None = None) -> int:
    """Column blocks per hop for a panel of d columns (1 = the one-launch hop), if A's blocks exist
    or `hops` hops will amortise cutting it: for panels of >= 512 MiB at d >= 64, one block per
    ~100 MiB of panel, 12 to 16 (round 5, profiles/r05bn_col_blocks_final_kernels.txt: products d = 64
    3.37 -> 3.08 ms per hop at 4 -> 12 blocks, d = 128 5.23 -> 5.15 at 8 -> 12, d = 256 11.73 -> 11.00
    at 8 -> 16); 4 for panels of >= 16 GiB.  Before round 5's packed-row kernels: one per ~150 MiB, 4
    to 8.  Round 4 (slice waves from ~1000-entry spans, rows of <= 48 entries whole): products
    d = 128 5.63 ms at B = 6, 5.60-5.61 at 7 and 8; with 48-entry whole rows 5.58 / 5.53 / 5.51-5.52 at
    6 / 7 / 8 (profiles/r04af_*, r04ag_*, r04ah_*).  Round 3, block 0 in two launches, compact blocks in launch order
    (profiles/r03_ab_col_blocks_round3.txt): products d = 128 (1.25 GB) 5.98 ms at B = 6 against
    6.00-6.01 at 5 and 7, 6.03 at 8, 6.10 at 4; d = 256 (2.5 GB) 12.35 ms at 7-8 against 12.40 at 6
    (before the launch order: 12.55 at 6, 12.67 at 5, 12.70 at 10, 12.91 at 4); d = 64 (0.63 GB) flat
    over 4-5; RMAT-26 (68 GB) 312.8 at 4 against 315.6 at 5, papers100M (57 GB) 242.9 against 242.0."""
    if FORCE_COL_BLOCKS is not None:
        return max(1, int(FORCE_COL_BLOCKS))
    panel = A.n_cols * d * 4
    if d < 64 or panel < (512 << 20):
        B = 1
    elif panel >= SPLIT_BLOCK0_MAX_PANEL:
        B = 4
    else:
        # round 5 (= kAutoBlocksMin / Max of srg_plan.hip): one per ~100 MiB, 12 to 16 blocks
        B = min(16, max(12, int(round(panel / (100 << 20)))))
    if B > 1 and B not in A._blocks and (hops is None or hops < MIN_HOPS_TO_CUT):
        return 1
    return B


def col_blocks_of(A: DeviceCSR, d: int) -> int:
    """The column blocks per hop hop() runs A in over a d-column panel as A is laid out now (its native
    plan for d, or its torch-formulated blocks); 1 = the one-launch hop."""
    if _native_ok(A):
        from .plan import cached
        P = cached(A, d)
        if P is not None:
            return P.col_blocks
    return auto_col_blocks(A, d)


# Hops over panels of at least this many bytes cap the row kernel's occupancy (SRG_SPMM_CAP_WAVES):
# products 5.84 -> 5.81 ms per hop, arxiv (87 MB) 3 % slower capped (profiles/r04x_waves_ab.txt)
CAP_WAVES_MIN_PANEL = 512 << 20


def launches_per_hop(A: DeviceCSR, B: int, d: int, agg: bool = False) -> int:
    """k_spmm launches of one hop of A over a d-column panel in B column blocks (hop()): B, plus
    one when block 0 runs as its cut spans and its whole rows (_split_block0, or the aggregation
    epilogue)."""
    from .plan import cached
    P = cached(A, d) if _native_ok(A) else None
    if P is not None and P.col_blocks == B:
        return P.n_launch
    blocks = A.column_blocks(B) if B > 1 else None
    if not blocks:
        return 1
    return len(blocks) + (1 if (agg or _split_block0(A, d)) and blocks[0].whole_rows is not None else 0)


def _hop_plan(A: DeviceCSR, d: int, B: int, nt_store: bool = False, fast: bool = False, agg: bool = False):
    """The launches of one hop of A over a d-column panel in B column blocks: ([(operator, flags,
    kind)], join) with kind "plain" or "agg" (the launch that carries the aggregation epilogue), and
    join = whether the hub side stream must be joined at the end of the hop."""
    # one launch: a long-lived operator's launch-ordered copy when prepare() made one
    blocks = (A.column_blocks(B) if B > 1 else None) or [A._blocks.get("sched", A) if _COMPACT else A]
    # a block's rows are short: 2 gathers per packed row in flight (d >= 128: 4 or 2 rows per wave;
    # at d = 64, 8 rows per wave, it is 3 % slower)
    u2 = len(blocks) > 1 and d >= 128 and _U2_BLOCKED
    split = blocks[0].split_whole() if (agg or _split_block0(A, d)) and len(blocks) > 1 else None
    # the blocks' hub spans chained on the side stream: one fork (the first block with hub rows),
    # one join at the end of the hop.  X is not written during the hop, and when every block has
    # the same hub rows only the side stream touches them, so nothing else orders them (a row that
    # is a hub in one block only would have spans on both streams: then every block forks and joins)
    # (with block 0 split, the launches over cut rows are split[0] and blocks 1..; split[1]'s rows --
    # whole rows -- are in no other launch, so its hub rows never matter)
    chain = len(blocks) > 1 and not fast and _HUB_CHAIN and \
        _same_hub_rows(A, B, ([split[0]] + blocks[1:]) if split is not None else blocks, agg=split is not None)
    base = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_PACKED_U2 if u2 else 0) | \
        (_lib.SRG_SPMM_CAP_WAVES if A.n_cols * d * 4 >= CAP_WAVES_MIN_PANEL else 0)
    seq = []     # (operator, accumulate, kind)
    for b, Ab in enumerate(blocks):
        if split is not None and b == 0:
            # rows block 0 computes whole finish there: their aggregation runs in that launch
            seq += [(split[0], False, "plain"), (split[1], False, "agg" if agg else "plain")]
        else:
            seq.append((Ab, b > 0, "agg" if agg and b == len(blocks) - 1 else "plain"))
    plan, forked = [], False
    for Ab, acc, kind in seq:
        f = base | (_lib.SRG_SPMM_ACCUMULATE if acc else 0)
        if chain and Ab.n_hub > 0:
            f |= _lib.SRG_SPMM_HUB_NOJOIN | (_lib.SRG_SPMM_HUB_CONTINUE if forked else 0)
            forked = True
        elif fast and kind == "plain":
            f |= _lib.SRG_SPMM_FAST
        plan.append((Ab, f, kind))
    return plan, forked


def hop(A: DeviceCSR, X: torch.Tensor, out: torch.Tensor, nt_store: bool = False, col_blocks=None,
        agg=None, fast: bool = False) -> torch.Tensor:
    """out = A @ X (one hop, exact), column-blocked when auto_col_blocks (or `col_blocks`) says so
    and A's rows allow it; bitwise the same either way.  agg = (panel, w, init): the aggregation
    step fused into the (last) launch's epilogue, as spmm_agg.  fast: SRG_SPMM_FAST for the hub
    rows of every launch (tolerance mode, see spmm)."""
    d = X.shape[1]
    # every launch below writes rows of A's whole row space (the blocks' schedules name them)
    _check_panel(X, A.n_cols, "X")
    _check_panel(out, A.out_rows, "out", d)
    if agg is not None:
        _check_panel(agg[0], A.out_rows, "agg", d)
    if out.device != A.device or X.device != A.device:
        raise ValueError("A, X and out must be on the same device")
    if _native_ok(A) and X.data_ptr() != out.data_ptr() and not (fast and agg is not None):
        # an operator prepared by the native planner: one hop of its plan (srg_plan_hop_f32), the
        # aggregation step in the epilogue of the launches where the rows' chains end
        from .plan import cached
        P = cached(A, d)
        if P is not None and (col_blocks is None or int(col_blocks) == P.col_blocks):
            flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_FAST if fast else 0)
            if agg is None:
                P.hop(X, out, d, flags)
            else:
                P.hop(X, out, d, flags, agg[0], agg[1], agg[2])
            return out
    B = auto_col_blocks(A, d) if col_blocks is None else int(col_blocks)
    plan, join = _hop_plan(A, d, B, nt_store, fast, agg is not None)
    if agg is None and X.stride(0) == out.stride(0) and X.data_ptr() != out.data_ptr():
        # one hop through the native plan loop (the packed rows get their spans by slot there)
        arr = (ctypes.c_void_p * 2)(X.data_ptr(), out.data_ptr())
        _lib.call(X.device, "srg_propagate_plan_f32", _plan_array(plan, d), len(plan), 1 if join else 0, arr,
                  X.stride(0), d, 1, _stream(X.device))
        return out
    for Ab, f, kind in plan:
        if kind == "agg":
            _launch(Ab, X, out, d, f, agg[0], agg[1], agg[2])
        else:
            _launch(Ab, X, out, d, f)
    if join:
        _lib.call(X.device, "srg_hub_join", _stream(X.device))
    return out


def _launch(A: DeviceCSR, X, out, d, flags, agg=None, w=0.0, init=False):
    """One k_spmm launch of a planned hop (operands checked by the caller)."""
    if A.is_span:
        _span_call(A, X, out, d, flags, agg, agg.stride(0) if agg is not None else 0, w, init)
    elif agg is not None:
        _lib.call(X.device, "srg_spmm_agg_f32", A.indptr.data_ptr(), A.indices.data_ptr(), A.values.data_ptr(),
                  A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d), X.data_ptr(),
                  X.stride(0), out.data_ptr(), out.stride(0), d, flags, agg.data_ptr(), agg.stride(0), float(w),
                  1 if init else 0, _stream(X.device))
    else:
        _lib.call(X.device, "srg_spmm_csr_f32", A.indptr.data_ptr(), A.indices.data_ptr(), A.values.data_ptr(),
                  A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d), X.data_ptr(),
                  X.stride(0), out.data_ptr(), out.stride(0), d, flags, _stream(X.device))


class _HopLaunch(ctypes.Structure):
    """srg_hop_launch (include/srgnn_hip.h)."""
    _fields_ = [("row_beg", ctypes.c_void_p), ("row_end", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("row_order", ctypes.c_void_p), ("n_rows", ctypes.c_int64),
                ("n_hub", ctypes.c_int64), ("n_heavy", ctypes.c_int64), ("flags", ctypes.c_uint32),
                ("slot_beg", ctypes.c_void_p), ("slot_end", ctypes.c_void_p)]


def _plan_array(plan, d):
    arr = (_HopLaunch * len(plan))()
    for i, (Ab, f, _) in enumerate(plan):
        sb, se = Ab.slot_spans() if (Ab.is_span and Ab.n_rows and _SLOT_SPANS) else (None, None)
        arr[i] = _HopLaunch(Ab.indptr.data_ptr(), Ab.row_end.data_ptr() if Ab.is_span else None,
                            Ab.indices.data_ptr(), Ab.values.data_ptr(), Ab.order.data_ptr() if Ab.n_rows else None,
                            Ab.n_rows, Ab.n_hub, Ab.heavy(d), f, sb.data_ptr() if sb is not None else None,
                            se.data_ptr() if se is not None else None)
    return arr


HUB_CHAIN_MAX = 256     # = kHubPrefix (csrc/srg_plan.hip)


def _same_hub_rows(A: DeviceCSR, B: int, blocks, agg: bool = False) -> bool:
    """Whether every column block schedules the same set of hub rows (cached per B on A)."""
    key = ("same_hubs", B, agg)
    if key not in A._blocks:
        sets = [torch.sort(b.order[: b.n_hub].to(torch.int64)).values for b in blocks]
        # more than HUB_CHAIN_MAX hub rows in a launch: no chain (the native planner compares that many)
        A._blocks[key] = all(s.numel() <= HUB_CHAIN_MAX for s in sets) and \
            all(s.numel() == sets[0].numel() and bool(torch.equal(s, sets[0])) for s in sets)
    return A._blocks[key]


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
    the K hops run back to back on the GPU with no host round trips (srg_propagate_khop_f32, or
    hop() per hop when the hops are column-blocked).  fast: tolerance mode for the hub rows (spmm)."""
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
    if K > 0 and _native_ok(A):
        # the native plan (srgnn.plan): layout and hop loop in the library
        from .plan import plan_for
        cb = int(col_blocks) if col_blocks is not None else int(FORCE_COL_BLOCKS or 0)
        flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_FAST if fast else 0)
        plan_for(A, d, K, cb, SPLIT_BLOCK0).propagate(panels, ld, d, K, flags)
        if panels[0] is not X0 and X is not X0:
            panels = [X0] + list(panels[1:])
        return panels
    B = auto_col_blocks(A, d, hops=K) if col_blocks is None else int(col_blocks)
    if K > 0 and B > 1 and column_blocks_for(A, B, hops=K):
        # the blocked hop loop runs natively: one call for the K hops (srg_propagate_plan_f32)
        plan, join = _hop_plan(A, d, B, nt_store, fast)
        arr = (ctypes.c_void_p * (K + 1))(*[p.data_ptr() for p in panels])
        _lib.call(X.device, "srg_propagate_plan_f32", _plan_array(plan, d), len(plan), 1 if join else 0, arr,
                  ld, d, K, _stream(X.device))
    elif K > 0 and _COMPACT and "sched" in A._blocks:
        # a long-lived operator's launch-ordered copy (DeviceCSR.schedule_ordered): the one launch
        # per hop as a span operator, through the native plan loop
        S = A._blocks["sched"]
        flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_FAST if fast else 0)
        arr = (ctypes.c_void_p * (K + 1))(*[p.data_ptr() for p in panels])
        _lib.call(X.device, "srg_propagate_plan_f32", _plan_array([(S, flags, "plain")], d), 1, 0, arr, ld, d, K,
                  _stream(X.device))
    else:
        arr = (ctypes.c_void_p * (K + 1))(*[p.data_ptr() for p in panels])
        flags = (_lib.SRG_SPMM_NT_STORE if nt_store else 0) | (_lib.SRG_SPMM_FAST if fast else 0)
        _lib.call(X.device, "srg_propagate_khop_f32", A.indptr.data_ptr(), A.indices.data_ptr(),
                  A.values.data_ptr(), n, A.order.data_ptr() if n else None, A.n_hub, A.heavy(d), arr, ld, d,
                  K, flags, _stream(X.device))
    if panels[0] is not X0 and X is not X0:
        panels = [X0] + list(panels[1:])
    return panels
