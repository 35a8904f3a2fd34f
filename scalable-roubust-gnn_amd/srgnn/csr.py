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
# Column blocks of the halo partition's row chunks (srgnn.dist.HaloPartitionedOperator.chunk_blocks):
# rows of at most this many nonzeros are not cut but computed whole in block 0; 0 cuts every row.  The
# one-GPU plan's rule (kWholeMax, csrc/srg_plan.hip) and the C halo planner's (kBlockWholeMax,
# srg_halo.hip) are the same 48 (round 4: products 5.63 -> 5.58 ms per hop at six blocks, 5.53 at seven;
# 64: the same, 96: 5.62; profiles/r04ag_*, r04ah_*).
BLOCK_WHOLE_MAX = 48
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
    # row spans (a column block of the halo partition's row chunks, srgnn.dist): row r's entries are
    # [indptr[r], row_end[r]) of indices / values, and indptr holds n_rows starts instead of n_rows + 1
    # pointers
    row_end: torch.Tensor | None = None
    # rows of the output panel a launch may write: the schedule (`order`) names row ids of the whole
    # operator, so a column block or a row group that schedules a subset of the rows still writes
    # rows up to row_space - 1 (None: n_rows, a schedule that is a permutation of the rows)
    row_space: int | None = None
    # the thresholds the schedule was built with (None = automatic), reused by column blocks
    thresholds: tuple = (None, None)
    _blocks: dict = field(default_factory=dict, repr=False, compare=False)   # cached plans (srgnn.plan)

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
        """Frees the cached layouts: the native plans (srgnn.plan; compact ones hold one more copy of
        the ids and values), released after every stream their work went to."""
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


def schedule_from_degrees(deg: torch.Tensor, nnz: int, heavy_threshold=None, hub_threshold=None):
    """make_schedule from the row lengths `deg` (nnz = their sum, for the automatic thresholds)."""
    if heavy_threshold is None:
        heavy_threshold = DEFAULT_HEAVY_THRESHOLD
    if heavy_threshold is None:
        heavy_threshold = auto_heavy_threshold(nnz)
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
