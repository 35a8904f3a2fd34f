"""Device-resident CSR operand + its schedule (the "plan").

A `DeviceCSR` holds the normalised adjacency Â of `GraphOp.construct_adj`
(SSRG/operators/base_operator.py:20) in HBM, laid out for the gfx950 kernels:

    indptr  int64 [n_rows + 1]     (nnz may exceed 2^31: papers100M / RMAT-26 scale)
    indices int32 [nnz]            column ids, CSR order preserved exactly (the fma chains follow it)
    values  fp32  [nnz]            Â values, already cast to fp32 as utils.py:39 does
    order   int32 [n_rows]         schedule, each group by decreasing length:
                                     n_hub rows with more than `hub_threshold` nonzeros (one
                                       workgroup per 32-column slice, LDS-staged, side stream),
                                     n_heavy rows with more than `heavy_threshold` (one wave per
                                       32-column slice),
                                     then the rest (row waves: one row per wave, or 64 / S
                                       rows for d <= 32, 512 / d rows for d = 64 / 128 / 256)

The schedule never changes results -- every output element stays one fma chain in CSR order -- it
only decides which wave works on what and when (power-law hubs start first).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib

# Rows longer than the heavy threshold take the slice-wave path; shorter ones the row path (packed
# 512 / d rows per wave at d = 64, 128, 256).  None (default): auto_heavy_threshold(nnz); callers pass
# heavy_threshold to force one.
DEFAULT_HEAVY_THRESHOLD = None
# Narrow panels (d <= 32) run their light rows as 64 / S single-lane-per-column rows per wave, whose
# cost per nonzero is a full dependent gather: they keep the slice waves from 32 up (profiles/
# r02_ab_auto.txt: d = 8 hop 3.34 ms at 32 vs 3.76 at the wide auto threshold; the RMAT-26 wavelet
# in 32-column blocks 63.8 vs 98.9 ms per block).  Used when the wide threshold is automatic.
NARROW_HEAVY_THRESHOLD = 32
# Column blocks: rows of at most this many nonzeros are not cut but computed whole in block 0
# (DeviceCSR.column_blocks); 0 cuts every row.
# Round 4: 48 (products 5.63 -> 5.58 ms per hop at six blocks, 5.53 at seven; 64: the same, 96: 5.62;
# papers100M 236.7 -> 236.1 ms, RMAT-26 307.6 -> 307.1; profiles/r04ag_*, r04ah_*).  Round 2: 32.
BLOCK_WHOLE_MAX = 48             # = kBlockWholeMax of the C halo planner (srg_halo.hip)
# "auto": rows whose slice-wave time (~40 ns per nonzero, measured) would exceed about half of the
# expected hop time (~nnz / 13.5e9 s at the measured hop rate) go to the hub path:
# threshold = nnz // 1024, at least 8192.  Products on 1 GPU -> only the top hub; 1/8 of it -> ~15 K.
# None (default): automatic; callers pass hub_threshold to force one.
DEFAULT_HUB_THRESHOLD = None


def auto_hub_threshold(nnz: int, launches: int = 1) -> int:
    """Row length above which a row goes to the hub workgroups (side stream, beside the main
    launch).  A slice wave needs ~38 ns per nonzero (one dependent gather per 8-nonzero group
    of its row), so a row should be a hub once that latency nears the duration of the launch it
    belongs to: ~nnz * 520 B / 6.5 TB/s at d = 128, split over `launches` back-to-back launches
    (the halo exchange's row groups): nnz / (1024 * launches), floor 2048.  Sweeps
    (profiles/r01_sweep_hub_threshold_*.json): products 123,209 (only the top row) is best;
    arxiv 2,048-4,096 run a hop in 0.208 ms vs 0.236 ms at the former floor of 8,192."""
    return max(2048, int(nnz) // (1024 * max(1, int(launches))))


def auto_heavy_threshold(nnz: int, launches: int = 1) -> int:
    """Row length above which a row is cut into 32-column slice waves instead of running in a packed
    row wave.  A packed row wave costs ~3 instructions per (nonzero, row) against ~13 for the four
    slice waves of a row, but a row's latency grows with its length (one dependent gather round per
    4 nonzeros), so the longest rows must be sliced.  The slice waves are XCD-aware (each XCD's L2
    caches one column slice of the rows they gather), which makes slices cheaper in bytes than
    packed rows.  nnz / (100000 * launches), floor 96.  Sweeps: with XCD-aware slices products is
    flat at 7.18-7.23 ms per hop over 128-1024 and 7.31 at 2102 (profiles/r02_ab_xh*.txt); without
    them it was best at 2048 (7.42 ms vs 7.92 at 96, 8.78 at 16384, where the longest packed rows
    become the tail; r02_packed_sweep_breakdown.jsonl).  arxiv is best at 96-128.  papers100M and
    RMAT-26 are flat over 20000-110000 and slower at 2048 (r02_ab_big.txt, r02_ab_xh2.txt); at
    nnz / 150000 RMAT-26 (d = 256, 14,800) took 331 ms per hop against 318-321 at 20,000-37,000."""
    return max(96, int(nnz) // (100000 * max(1, int(launches))))


def _dev(device):
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError(f"libsrgnn_hip runs on a HIP device, got {device}")
    return device


@dataclass
class DeviceCSR:
    indptr: torch.Tensor
    indices: torch.Tensor
    values: torch.Tensor
    n_rows: int
    n_cols: int
    # the row schedule (order, n_heavy, n_hub, n_heavy_narrow below): None = not built yet -- built
    # from the thresholds on first use (from_tensors leaves it to the first hop that reads it: a K-hop
    # run through the native plan, srgnn.plan, never does)
    _order: torch.Tensor | None
    _n_heavy: int | None
    _n_hub: int | None = 0
    _n_heavy_narrow: int | None = None   # slice-wave rows for d <= 32 (None: n_heavy)
    # row spans (a column block, column_blocks()): row r's entries are [indptr[r], row_end[r]) of
    # indices / values, and indptr holds n_rows starts instead of n_rows + 1 pointers
    row_end: torch.Tensor | None = None
    # column block 0 only: rows this block computes whole (short rows are not cut: the later blocks
    # do not schedule them, so their Y is written once instead of written, read and written again)
    whole_rows: torch.Tensor | None = None
    # rows of the output panel a launch may write: the schedule (`order`) names row ids of the whole
    # operator, so a column block or a row group that schedules a subset of the rows still writes
    # rows up to row_space - 1 (None: n_rows, a schedule that is a permutation of the rows)
    row_space: int | None = None
    # the thresholds the schedule was built with (None = automatic), reused by column blocks
    thresholds: tuple = (None, None)
    _blocks: dict = field(default_factory=dict, repr=False, compare=False)   # column_blocks() cache

    def _schedule(self) -> None:
        heavy_t, hub_t = self.thresholds
        self._order, self._n_heavy, self._n_hub = make_schedule(self.indptr, heavy_t, hub_t)
        self._n_heavy_narrow = narrow_heavy(self.indptr, self._n_hub) if _auto_heavy(heavy_t) else None

    @property
    def order(self) -> torch.Tensor:
        if self._order is None:
            self._schedule()
        return self._order

    @order.setter
    def order(self, v):
        self._order = v

    @property
    def n_heavy(self) -> int:
        if self._order is None:
            self._schedule()
        return self._n_heavy

    @n_heavy.setter
    def n_heavy(self, v):
        self._n_heavy = v

    @property
    def n_hub(self) -> int:
        if self._order is None:
            self._schedule()
        return self._n_hub

    @n_hub.setter
    def n_hub(self, v):
        self._n_hub = v

    @property
    def n_heavy_narrow(self):
        if self._order is None:
            self._schedule()
        return self._n_heavy_narrow

    @n_heavy_narrow.setter
    def n_heavy_narrow(self, v):
        self._n_heavy_narrow = v

    @property
    def out_rows(self) -> int:
        """Rows an output (or aggregation) panel of this operator must have."""
        return self.n_rows if self.row_space is None else int(self.row_space)

    @property
    def schedules_subset(self) -> bool:
        """The schedule covers only some rows of the row space (a column block 1.., a row group)."""
        return self.out_rows != self.n_rows

    def drop_blocks(self) -> None:
        """Frees the cached layouts: column blocks (compact copies hold one more copy of the ids and
        values) and native plans (srgnn.plan; released in stream order)."""
        for v in list(self._blocks.values()):
            if hasattr(v, "close"):
                v.close()
        self._blocks.clear()

    def heavy(self, d: int) -> int:
        """The slice-wave row count for a panel of d columns (same order, a longer prefix of it
        for narrow panels)."""
        return self.n_heavy_narrow if (d <= 32 and self.n_heavy_narrow is not None) else self.n_heavy

    @property
    def nnz(self) -> int:
        if self.row_end is not None:
            return int((self.row_end - self.indptr).sum().item()) if self.n_rows else 0
        return int(self.indices.numel())

    @property
    def is_span(self) -> bool:
        """A column block: rows are spans of a shared CSR (srg_spmm_span_f32)."""
        return self.row_end is not None

    @property
    def device(self):
        return self.indices.device

    # ------------------------------------------------------------------------------------------
    @classmethod
    def from_tensors(cls, indptr, indices, values, n_cols=None, heavy_threshold=None,
                     validate=True, device=None, hub_threshold=None):
        """Build from CSR arrays (numpy or torch, any device); copies to `device` if needed."""
        device = _dev(device if device is not None else
                      (indices.device if isinstance(indices, torch.Tensor) and indices.is_cuda else None))
        # copy in the stored dtypes, convert on the device (host-side conversions of 1e8-entry
        # arrays are single-threaded and slower than the copy)
        ip = torch.as_tensor(indptr).to(device=device).to(torch.int64)
        ix = torch.as_tensor(indices).to(device=device).to(torch.int32)
        vv = torch.as_tensor(values).to(device=device).to(torch.float32)
        n_rows = int(ip.numel()) - 1
        if n_rows < 0:
            raise ValueError("indptr must have n_rows + 1 entries")
        if n_cols is None:
            n_cols = n_rows
        if ix.numel() != vv.numel():
            raise ValueError(f"indices ({ix.numel()}) and values ({vv.numel()}) differ in length")
        ip, ix, vv = ip.contiguous(), ix.contiguous(), vv.contiguous()
        if validate:
            _lib.call(device, "srg_csr_validate", ip.data_ptr(), ix.data_ptr(), n_rows, ix.numel(), n_cols,
                      _lib.stream(device))
        # the schedule is built on first use (DeviceCSR.order)
        return cls(ip, ix, vv, n_rows, int(n_cols), None, None, None, None,
                   thresholds=(heavy_threshold, hub_threshold))

    @classmethod
    def from_scipy(cls, adj, heavy_threshold=None, device=None):
        """From a scipy.sparse.csr_matrix (values cast to fp32 like SSRG/operators/utils.py:39)."""
        return cls.from_tensors(np.asarray(adj.indptr),
                                np.asarray(adj.indices, dtype=np.int32),
                                np.asarray(adj.data),   # cast to fp32 on the device (round to nearest, as astype)
                                n_cols=adj.shape[1], heavy_threshold=heavy_threshold, device=device)

    def column_blocks(self, B: int):
        """B operators over the same rows: block b holds, as a span of each row, the row's entries
        whose column ids lie in [ceil(b * n_cols / B), ceil((b + 1) * n_cols / B)), each block with
        its own schedule (or None for an empty operator or B < 2).

        A hop is then block 0 from +0.0f and blocks 1..B-1 with ACCUMULATE: each output element is
        the same fma chain over the same entries in the same order, continued from the fp32 value
        the previous block stored, so the result is bitwise the one-launch hop.  Â from
        construct_adj has sorted column ids (utils.py:81-93 builds a canonical transpose), so a
        block is one span of every row: the blocks share indices / values and hold only their
        split points (srg_csr_col_splits, one binary search per row and boundary; an n_rows int64
        array per boundary).  Rows with unsorted ids still split into spans that partition them in
        CSR order -- exact, only without the locality.  Cached per B (compact blocks, once made by
        compact_column_blocks, are returned instead)."""
        B = int(B)
        if B in self._blocks:
            return self._blocks[B]
        if self.is_span:
            raise ValueError("column_blocks of a column block")
        if B < 2 or self.n_rows == 0 or self.nnz == 0:
            self._blocks[B] = None
            return None
        ip, n = self.indptr, self.n_cols
        dev = ip.device
        splits = torch.empty((B - 1, self.n_rows), dtype=torch.int64, device=dev)
        _lib.call(dev, "srg_csr_col_splits", ip.data_ptr(), self.indices.data_ptr(), self.n_rows, n, B,
                  splits.data_ptr(), _lib.stream(dev))
        whole = (ip[1:] - ip[:-1]) <= BLOCK_WHOLE_MAX if BLOCK_WHOLE_MAX > 0 else None
        if whole is not None:
            # short rows run whole in block 0: their later spans are empty and not scheduled
            splits = torch.where(whole.unsqueeze(0), ip[1:].unsqueeze(0), splits)
            later = torch.nonzero(~whole).squeeze(1)
        bounds = [ip[:-1]] + [splits[b] for b in range(B - 1)] + [ip[1:]]
        heavy_t, hub_t = self.thresholds
        auto_narrow = self.n_heavy_narrow is not None      # the parent's narrow split is automatic
        out = []
        for b in range(B):
            beg, end = bounds[b], bounds[b + 1]
            deg = end - beg
            nnz_b = int(deg.sum().item())
            sel = deg[later] if (b > 0 and whole is not None) else deg
            order, n_heavy, n_hub = schedule_from_degrees(sel, nnz_b, heavy_t, hub_t, block=True)
            if b > 0 and whole is not None:
                order = later[order.to(torch.int64)].to(torch.int32)
            narrow = narrow_heavy_degrees(sel, n_hub) if auto_narrow else None
            out.append(DeviceCSR(beg, self.indices, self.values, int(sel.numel()), n, order, n_heavy, n_hub, narrow,
                                 row_end=end, whole_rows=whole if b == 0 else None, row_space=self.n_rows,
                                 thresholds=self.thresholds))
        self._blocks[B] = out
        return out

    def split_whole(self):
        """Column block 0 as two schedules over the same arrays: (the cut rows' first spans, the
        rows it computes whole) -- for a hop whose aggregation epilogue must run in the launch
        that finishes each row (srgnn.spmm.hop with agg).  Cached."""
        if self.whole_rows is None:
            return None
        if "split" not in self._blocks:
            parts = []
            for sel in (~self.whole_rows, self.whole_rows):
                rows = torch.nonzero(sel).squeeze(1)
                ip = self.indptr
                deg = ((self.row_end - ip) if self.is_span else (ip[1:] - ip[:-1]))[rows]
                heavy_t, hub_t = self.thresholds
                order, n_heavy, n_hub = schedule_from_degrees(deg, int(deg.sum().item()), heavy_t, hub_t,
                                                              block=True)
                order = rows[order.to(torch.int64)].to(torch.int32)
                narrow = narrow_heavy_degrees(deg, n_hub) if self.n_heavy_narrow is not None else None
                parts.append(DeviceCSR(self.indptr, self.indices, self.values, int(rows.numel()), self.n_cols, order,
                                       n_heavy, n_hub, narrow, row_end=self.row_end, row_space=self.out_rows,
                                       thresholds=self.thresholds))
            self._blocks["split"] = tuple(parts)
        return self._blocks["split"]

    def slot_spans(self):
        """(beg, end) int64 [n_rows]: the span of the row in each schedule slot (span operators).
        Cached."""
        if "slots" not in self._blocks:
            o = self.order.to(torch.int64)
            self._blocks["slots"] = (self.indptr[o].contiguous(), self.row_end[o].contiguous())
        return self._blocks["slots"]

    def _copy_in_order(self, rows: torch.Tensor):
        """(beg, end, indices, values): the entries of `rows` (int64 row ids) copied out one row after
        the other in that order, row r's at [beg[r], end[r]) of the copies (rows not listed: empty)."""
        ip = self.indptr
        dev = ip.device
        b0 = ip[rows]
        deg = (self.row_end[rows] if self.is_span else ip[rows + 1]) - b0
        pos = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(deg, 0, out=pos[1:])
        nnz = int(pos[-1].item())
        beg = torch.zeros(self.out_rows, dtype=torch.int64, device=dev)
        end = torch.zeros(self.out_rows, dtype=torch.int64, device=dev)
        if self.indices.dtype != torch.int32 or self.values.dtype != torch.float32:
            # entry e of the copy is entry b0[i] + (e - pos[i]) of row i of the list
            idx = torch.repeat_interleave(b0 - pos[:-1], deg, output_size=nnz)
            idx += torch.arange(nnz, dtype=torch.int64, device=dev)
            beg[rows] = pos[:-1]
            end[rows] = pos[1:]
            return beg, end, self.indices[idx], self.values[idx]
        ix = torch.empty(nnz, dtype=self.indices.dtype, device=dev)
        v = torch.empty(nnz, dtype=self.values.dtype, device=dev)
        # srg_csr_copy_spans: one pass over the spans (the torch formulation, an int64 gather index of
        # nnz entries built with repeat_interleave, took 4.6 ms more on products' six blocks)
        order = rows.to(torch.int32).contiguous()
        row_end = self.row_end if self.is_span else ip[1:]
        _lib.call(dev, "srg_csr_copy_spans", order.data_ptr(), order.numel(), ip.data_ptr(), row_end.data_ptr(),
                  self.indices.data_ptr(), self.values.data_ptr(), pos.data_ptr(), ix.data_ptr(), v.data_ptr(),
                  beg.data_ptr(), end.data_ptr(), _lib.stream(dev))
        return beg, end, ix, v

    def schedule_ordered(self) -> "DeviceCSR":
        """This operator with its entries copied out in the order its launch takes the rows (its
        schedule): a span operator over the copy, the same entries in the same order per row, so the
        same bits.  For a long-lived one-launch operator (spmm.propagate), as compact_column_blocks
        is for blocked ones.  Cached."""
        if "sched" not in self._blocks:
            beg, end, ix, v = self._copy_in_order(self.order.to(torch.int64))
            self._blocks["sched"] = DeviceCSR(beg, ix, v, self.n_rows, self.n_cols, self.order, self.n_heavy, self.n_hub,
                                              self.n_heavy_narrow, row_end=end, row_space=self.out_rows,
                                              thresholds=self.thresholds)
        return self._blocks["sched"]

    def compact_column_blocks(self, B: int):
        """column_blocks(B) with each block's entries copied into arrays of its own, laid out in the
        order its launches take the rows: block b's schedule, and for block 0 the schedule of its
        cut rows' spans followed by that of its whole rows (its two launches, split_whole()).  One
        more copy of the ids and values (1 GB on products), for operators that serve many hops
        (spmm.MIN_HOPS_TO_COMPACT): no cache line of the id / value streams is read by two launches
        (45.4 -> 44.9 GB per hop on products, round 2), and the consecutive rows a wave takes read
        consecutive entries (round 3, tools/whole_rows_probe.py --sched: the whole-row launch 0.898
        -> 0.862 ms, block 0's cut spans 1.339 -> 1.301, a later block 1.399 -> 1.384).  Each block
        is a span operator over its copy; the same entries in the same order per row, so the same
        bits as the spans."""
        B = int(B)
        key = ("compact", B)
        blocks = self.column_blocks(B)
        if not blocks or self._blocks.get(key):
            return blocks
        out = []
        for blk in blocks:
            parts = blk.split_whole() if blk.whole_rows is not None else None
            rows = torch.cat([parts[0].order, parts[1].order]) if parts else blk.order
            beg, end, ix, v = blk._copy_in_order(rows.to(torch.int64))
            nb = DeviceCSR(beg, ix, v, blk.n_rows, self.n_cols, blk.order, blk.n_heavy, blk.n_hub, blk.n_heavy_narrow,
                           row_end=end, whole_rows=blk.whole_rows, row_space=blk.row_space, thresholds=blk.thresholds)
            if parts:
                nb._blocks["split"] = tuple(
                    DeviceCSR(beg, ix, v, p.n_rows, self.n_cols, p.order, p.n_heavy, p.n_hub, p.n_heavy_narrow,
                              row_end=end, row_space=p.row_space, thresholds=p.thresholds) for p in parts)
            out.append(nb)
            del beg, end, ix, v
        self._blocks[B] = out
        self._blocks[key] = True
        return out

    def rows(self, r0: int, r1: int, heavy_threshold=None, hub_threshold=None) -> "DeviceCSR":
        """Row block [r0, r1) with rebased row pointers (global column ids kept)."""
        if self.is_span:
            raise ValueError("rows() of a column block")
        ip = self.indptr[r0:r1 + 1]
        base = int(ip[0].item())
        end = int(ip[-1].item())
        ip = ip - base
        order, n_heavy, n_hub = make_schedule(ip, heavy_threshold, hub_threshold)
        return DeviceCSR(ip.contiguous(), self.indices[base:end], self.values[base:end],
                         r1 - r0, self.n_cols, order, n_heavy, n_hub,
                         narrow_heavy(ip, n_hub) if _auto_heavy(heavy_threshold) else None,
                         thresholds=(heavy_threshold, hub_threshold))


def _auto_heavy(heavy_threshold) -> bool:
    return heavy_threshold is None and DEFAULT_HEAVY_THRESHOLD is None


def narrow_heavy(indptr: torch.Tensor, n_hub: int, threshold: int | None = None) -> int:
    """Slice-wave rows of the schedule for narrow panels: rows longer than NARROW_HEAVY_THRESHOLD,
    hubs excluded (they lead the same decreasing-length order)."""
    return narrow_heavy_degrees(indptr[1:] - indptr[:-1], n_hub, threshold)


def narrow_heavy_degrees(deg: torch.Tensor, n_hub: int, threshold: int | None = None) -> int:
    """narrow_heavy from the row lengths."""
    t = NARROW_HEAVY_THRESHOLD if threshold is None else threshold
    return max(0, int((deg > t).sum().item()) - int(n_hub)) if deg.numel() else 0


def make_schedule(indptr: torch.Tensor, heavy_threshold=None, hub_threshold=None):
    """(order int32, n_heavy, n_hub) for a CSR with row pointers `indptr`: rows sorted by
    decreasing length; the first n_hub have more than hub_threshold nonzeros, the next n_heavy
    more than heavy_threshold.  A negative threshold disables that group."""
    return schedule_from_degrees(indptr[1:] - indptr[:-1], int(indptr[-1]) if indptr.numel() else 0,
                                 heavy_threshold, hub_threshold)


# Column blocks' spans take the slice waves above nnz_b / BLOCK_HEAVY_PER entries.  Round 3 (five
# blocks): 300-500 best, 6.13 ms per hop; 160: 6.43, 600: 6.19 (profiles/r03_ab_heavy_threshold_B5.txt).
# Round 4, with the slice waves' id prefetch and the occupancy cap, longer packed spans pay: products
# (six blocks, nnz_b ~ 19 M) 5.79 ms at 60000 (~320 entries), 5.62-5.64 at 30000 / 20000 / 15000
# (650-1300; 2000+ entries: 6.84); papers100M 239.0 -> 237.4 ms, RMAT-26 307.7 -> 306.2
# (profiles/r04ab_*, r04ac_*, r04ad_*).  At eight blocks (nnz_b ~ 14.5 M, shorter launches) the cliff
# comes sooner: 5.51 ms at 30000 and 20000 (~485 / ~730 entries), 7.04 at 12000 (~1200;
# r04ap_*), so 30000 keeps the margin.
BLOCK_HEAVY_PER = 30000


def schedule_from_degrees(deg: torch.Tensor, nnz: int, heavy_threshold=None, hub_threshold=None,
                          block: bool = False):
    """make_schedule from the row lengths `deg` (nnz = their sum, for the automatic thresholds);
    block: the lengths are a column block's spans (BLOCK_HEAVY_PER for the automatic heavy split)."""
    if heavy_threshold is None:
        heavy_threshold = DEFAULT_HEAVY_THRESHOLD
    if heavy_threshold is None:
        heavy_threshold = max(96, int(nnz) // BLOCK_HEAVY_PER) if block else auto_heavy_threshold(nnz)
    if hub_threshold is None:
        hub_threshold = DEFAULT_HUB_THRESHOLD
    if hub_threshold is None:
        hub_threshold = auto_hub_threshold(nnz)
    n = int(deg.numel())
    if n == 0:
        return torch.zeros(0, dtype=torch.int32, device=deg.device), 0, 0
    order = torch.sort(deg, descending=True, stable=True).indices.to(torch.int32)
    n_hub = int((deg > hub_threshold).sum().item()) if hub_threshold >= 0 else 0
    n_big = int((deg > heavy_threshold).sum().item()) if heavy_threshold >= 0 else 0
    n_heavy = max(0, n_big - n_hub)
    return order.contiguous(), n_heavy, n_hub
