"""Multi-GPU propagation: 1-D row partition of Â, one process per GPU (torch.distributed; the
"nccl" backend is RCCL over xGMI; gloo on CPU for tests).  SURVEY.md §8(e).

Rank p owns the contiguous row block [starts[p], starts[p+1]) of Â (blocks balanced by nonzeros)
and the same rows of every hop panel.  Two exchanges:

* HaloPartitionedOperator (default): each rank receives only the remote rows its own rows
  reference, group by group (nnz-balanced row chunks + the hub rows), with one asynchronous
  all_to_all_single per group issued as soon as that group's kernel is done -- RCCL runs it on its
  own stream while the later groups compute.  Low-degree halo rows whose neighbours are all local ("ghost rows") are
  computed on the rank that needs them instead of received (the same CSR row, so the same bits):
  a pair of GPUs shares one xGMI link, and on power-law graphs most of the halo is such rows.
  HaloWaveletFilter runs the wavelet basis' Chebyshev recurrence on the same plan (one exchange per
  order, no ghost rows).
* RowPartitionedOperator: one padded all_gather_into_tensor of the whole panel per hop.

In both, the local operator's column ids are remapped into the local panel layout with every
row's entries kept in their CSR order, so each output element is the same fma chain as on one
GPU: the multi-GPU results are bitwise equal to the single-GPU ones.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist


def balanced_row_starts(indptr: torch.Tensor, parts: int):
    """Row boundaries [0 = s_0 <= ... <= s_P = n] splitting the nonzeros as evenly as rows allow (the
    halo planner's rule too: srg_halo.hip balanced()).  Weighting long rows more (so the rank holding a
    giant row gets fewer others) was measured and dropped (profiles/r01_giant_weight_sweep.json)."""
    ip = indptr.to(torch.int64).cpu()
    n = ip.numel() - 1
    nnz = int(ip[-1])
    targets = torch.tensor([(nnz * p) // parts for p in range(parts + 1)], dtype=torch.int64)
    starts = torch.searchsorted(ip, targets, right=False).clamp_(0, n)
    starts[0], starts[-1] = 0, n
    for p in range(1, parts + 1):            # monotone
        starts[p] = max(int(starts[p]), int(starts[p - 1]))
    return [int(s) for s in starts]


def remap_columns(indices: torch.Tensor, starts, max_rows: int) -> torch.Tensor:
    st = torch.tensor(starts[:-1], dtype=torch.int64, device=indices.device)
    c = indices.to(torch.int64)
    q = torch.searchsorted(st, c, right=True) - 1
    return (q * max_rows + (c - st[q])).to(torch.int32)


class RowPartitionedOperator:
    """This rank's share of Â plus the buffers of the per-hop exchange.

    `local_spmm(A_local, X_full, out)` computes out = A_local @ X_full; by default the HIP kernel
    (srgnn.spmm.spmm).  Tests on CPU ranks inject the oracle there to exercise the partition and
    exchange logic with gloo."""

    def __init__(self, indptr, indices, values, n: int, group=None, local_spmm=None,
                 heavy_threshold=None, device=None, rank=None, world=None):
        self.group = group
        # rank / world may be given explicitly to build one share without a process group
        # (simulate_propagate: P virtual ranks in one process, e.g. on a single GPU)
        self.virtual = rank is not None
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.n = n
        self.starts = balanced_row_starts(indptr, self.world)
        self.max_rows = max(self.starts[p + 1] - self.starts[p] for p in range(self.world))
        r0, r1 = self.starts[self.rank], self.starts[self.rank + 1]
        self.r0, self.r1 = r0, r1
        self.rows = r1 - r0
        dev = torch.device(device) if device is not None else indices.device
        ip = indptr[r0:r1 + 1].to(torch.int64)
        base, end = int(ip[0]), int(ip[-1])
        ip = (ip - base).to(dev)
        ix = remap_columns(indices[base:end].to(dev), self.starts, self.max_rows)
        vv = values[base:end].to(dev)
        self.nnz_local = end - base
        self.nnz_total = int(indptr[-1])
        if local_spmm is None:
            from .csr import DeviceCSR
            from .spmm import spmm
            self.A = DeviceCSR.from_tensors(ip, ix, vv, n_cols=self.world * self.max_rows,
                                            heavy_threshold=heavy_threshold, device=dev)
            self._spmm = lambda A, X, out: spmm(A, X, out=out)
        else:
            self.A = (ip, ix, vv)
            self._spmm = local_spmm
        self.device = dev
        self._full = None

    def _gather(self, block: torch.Tensor) -> torch.Tensor:
        d = block.shape[1]
        if self._full is None or self._full.shape[1] != d:
            self._full = torch.empty((self.world * self.max_rows, d), dtype=block.dtype, device=block.device)
        if self.world == 1:
            self._full.copy_(block)
        elif self.virtual:
            raise RuntimeError("virtual shares exchange through simulate_propagate()")
        elif dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self._full, block, group=self.group)
        else:
            dist.all_gather(list(self._full.split(self.max_rows)), block, group=self.group)
        return self._full

    def new_panel(self, d: int) -> torch.Tensor:
        return torch.zeros((self.max_rows, d), dtype=torch.float32, device=self.device)

    def propagate(self, x_local: torch.Tensor, K: int, panels=None):
        """[X, ÂX, …, Â^K X] restricted to this rank's rows (each [max_rows, d], first `rows` valid).
        x_local: this rank's rows of X ([rows, d] or a padded [max_rows, d] panel)."""
        d = x_local.shape[1]
        if panels is None:
            panels = [self.new_panel(d) for _ in range(K + 1)]
        if x_local.shape[0] != self.max_rows or x_local.data_ptr() != panels[0].data_ptr():
            panels[0][: self.rows].copy_(x_local[: self.rows])
        for k in range(1, K + 1):
            full = self._gather(panels[k - 1])
            self._spmm(self.A, full, panels[k][: self.rows])
        return panels


def simulate_propagate(indptr, indices, values, n: int, x: torch.Tensor, K: int, world: int,
                       heavy_threshold=None, device=None):
    """P virtual ranks in ONE process: every share computes its rows of each hop from the padded
    full panel assembled exactly as all_gather_into_tensor would lay it out.  Returns the K+1 full
    [n, d] panels.  Exercises partition, column remap and padded layout on one device."""
    shares = [RowPartitionedOperator(indptr, indices, values, n, heavy_threshold=heavy_threshold,
                                     device=device, rank=p, world=world) for p in range(world)]
    d = x.shape[1]
    mr = shares[0].max_rows
    panels = [[s.new_panel(d) for _ in range(K + 1)] for s in shares]
    for s, pp in zip(shares, panels):
        pp[0][: s.rows].copy_(x[s.r0:s.r1])
    full = torch.empty((world * mr, d), dtype=torch.float32, device=panels[0][0].device)
    for k in range(1, K + 1):
        for p in range(world):
            full[p * mr:(p + 1) * mr].copy_(panels[p][k - 1])
        for s, pp in zip(shares, panels):
            s._spmm(s.A, full, pp[k][: s.rows])
    return [torch.cat([pp[k][: s.rows] for s, pp in zip(shares, panels)]) for k in range(K + 1)]


# ================================================================================================
# Halo exchange: each rank receives only the remote X rows its rows reference, group by group,
# overlapped with the computation of the later groups.
# ================================================================================================

# The plan of a rank's share (row blocks, chunks + hub group, halos, ghost rows, sends, local CSR,
# schedules) is built by the library's planner, srg_halo_plan_build (csrc/srg_halo.hip), for this
# package and for C hosts alike.  Its automatic ghost cap minimises the modelled hop: max over ranks
# of max(SpMM bytes incl. ghost rows at 8.4e12 B/s -- products at P = 2: 63.1 M nonzeros x 512 B in
# 3.85 ms --, busiest peer link at the link rate); a row is 4d bytes on both sides, so d cancels.
# The rate: this group's all_to_all, measured (measure_link_bps), or, without a group, one peer
# link's rate per direction assumed here (half of the ~153 GB/s xGMI link figure, minus RCCL overhead).
GHOST_LINK_BPS = 64e9


def measure_link_bps(group=None, device=None, mbytes_per_peer: int = 32, reps: int = 3) -> float:
    """Per-link rate of this process group's all_to_all: every rank sends `mbytes_per_peer` to every
    peer at once (as the halo exchange does), timed over `reps` calls after one warm-up; the
    minimum over ranks (all_reduce), so every rank gets the same number.  Bytes per second per
    peer link and direction."""
    import time
    P = dist.get_world_size(group)
    n = max(1, mbytes_per_peer * (1 << 20) // 4)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    send = torch.ones(P * n, dtype=torch.float32, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_to_all_single(recv, send, group=group)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    rate = torch.tensor([n * 4 * reps / max(time.perf_counter() - t0, 1e-9)], dtype=torch.float64, device=dev)
    dist.all_reduce(rate, op=dist.ReduceOp.MIN, group=group)
    return float(rate.item())


# The row chunks' slice waves take rows above max(192, nnz_local / (100000 C)) entries (the planner's
# kHaloHeavyMin).  Products at P = 8 (where the second term is below 96): per-rank hop 1.149-1.152 ms at
# 96, 1.123-1.129 at 128, 1.110-1.112 at 160-200, 1.131 at 256, 1.165 at 300 (round 4, with the slice
# waves' id prefetch; profiles/r04ak_*, r04al_halo_heavy_ab.txt).  papers100M / RMAT-26 ranks are above it.

# column blocks per row-chunk launch of the halo path for large local panels (1 = off; the
# operator's col_blocks argument forces a count).  Bitwise the same hops either way.  Default: 8 for
# local panels of >= 8 GiB at d >= 256 (RMAT-26 at P = 8, 23.8 GB of [own | halo] rows of 1 KiB: per-rank
# hop 46.4 ms at B = 1, 43.6 at 4, 40.7 at 8, 41.3 at 12, 43.6 at 32), else 1 (papers100M at d = 128 is
# flat over B = 1..16, products at P = 8 slower; profiles/r04_halo_col_blocks_p8.txt)
WIDE_HALO_COL_BLOCKS = 8
WIDE_HALO_PANEL = 8 << 30
# Measured and removed (round 5: they cost time at every setting; DESIGN.md §7 keeps the numbers): the
# hub group in column blocks (profiles/r03_halo_hub_blocks_negative.txt, r04n_*), the groups launched
# from launch-ordered copies (r03_halo_launch_order_negative.txt), medium hub rows as column spans in
# the chunks (r04_halo_medium_spans_negative.txt), long rows moved into the first chunk
# (r03_halo_p8_early_rows_negative.txt) and the halo pack fused into the SpMM epilogue
# (r01_halo_ranks_products_fused_pack_probe.json).


class HaloPartitionedOperator:
    """Rank p's share of Â for the halo-exchange multi-GPU propagation.

    Setup (deterministic from the GLOBAL operator, identical on every rank, no messages):
      * rows: the nnz-balanced block [starts[p], starts[p+1]);
      * groups: the block's rows are split into `chunks` contiguous ranges balanced by nonzeros
        (hub rows excluded), plus one group of hub rows (more than the owner's hub threshold);
        exchange order = chunk 0 .. chunk C-1, then hubs (the hub kernel finishes last);
      * every rank q's needs from every source s: the distinct columns of q's rows owned by s,
        by (group on s, source, id) -- so sends and receives are known without negotiation;
      * ghost rows: a halo row whose own neighbours all lie in this rank's rows or halo, with at
        most `ghost_max_degree` nonzeros, is computed here every hop (the same CSR row, the same
        fma chain, so the same bits) instead of received -- on a power-law graph most of the halo
        is such low-degree rows, and a pair of GPUs shares one xGMI link (the planner's cost model, above);
      * local panel layout: [own rows | received halo rows by (group, source, id) | ghost rows by
        (source, id)], and the local operator (own rows and ghost rows) with its column ids
        remapped into it (each row's entries keep their CSR order, so every output element is the
        same fma chain as on one GPU).
    Per hop k, all on the launch stream: the hub group's workgroups are forked onto the library's
    hub side stream, the row chunks write the own part of panel k+1, and after each chunk its rows
    that peers need are packed and sent with an asynchronous all_to_all_single (RCCL, overlapping
    the next chunks and the ghost rows' kernel); the hub group is joined and exchanged last, and
    the stream waits for the collectives.  Only X's first exchange also carries the ghost rows.
    """

    def __init__(self, indptr, indices, values, n: int, group=None, chunks: int = 4,
                 heavy_threshold=None, hub_threshold=None, device=None, rank=None, world=None,
                 local_spmm=None, ghost_max_degree=None, calibrate_link: bool = True, fast: bool = False,
                 col_blocks=None):
        from . import _lib
        from .comm import HaloPlan
        from .csr import DEFAULT_HEAVY_THRESHOLD, DEFAULT_HUB_THRESHOLD, NARROW_HEAVY_THRESHOLD
        self._narrow_heavy = NARROW_HEAVY_THRESHOLD
        self.group = group
        # tolerance mode for the hub group (SRG_SPMM_FAST: each hub row as 64 exact segment chains
        # plus their ordered sum; the other rows stay bit-exact)
        self.fast = bool(fast)
        # column blocks of the row chunks' launches (None: the automatic rule of _col_blocks_for)
        self.col_blocks = col_blocks
        self._cb = {}
        self.virtual = rank is not None
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        P, p = self.world, self.rank
        dev = torch.device(device) if device is not None else indices.device
        self.device = dev
        self.n = n
        C = max(1, int(chunks))
        self.C = C
        self.n_groups = C + 1
        G = self.n_groups
        # --- the plan: the library's planner (srg_halo_plan_build, csrc/srg_halo.hip) over the host
        # copy of the global CSR, identical on every rank (no messages); the ghost cap from its link-rate
        # model at the rate this group's all_to_all measures (the minimum over ranks, so every rank
        # passes the same rate and gets the same cap), or the assumed GHOST_LINK_BPS
        ip_h = indptr.detach().to("cpu", torch.int64).contiguous().numpy()
        ix_h = indices.detach().to("cpu", torch.int32).contiguous().numpy()
        self.link_bps = GHOST_LINK_BPS
        if ghost_max_degree is None and calibrate_link and P > 1 and not self.virtual and dist.is_initialized():
            self.link_bps = measure_link_bps(group, dev)
        if hub_threshold is None:
            hub_threshold = DEFAULT_HUB_THRESHOLD
        hub_c = _lib.SRG_HALO_AUTO if hub_threshold is None else (int(hub_threshold) if hub_threshold >= 0
                                                                 else _lib.SRG_HALO_NONE)
        if heavy_threshold is None:
            heavy_threshold = DEFAULT_HEAVY_THRESHOLD
        if heavy_threshold is not None and heavy_threshold < 0:
            raise ValueError("heavy_threshold must be >= 0 (None: automatic)")
        auto_heavy = heavy_threshold is None
        self._auto_heavy = auto_heavy
        self._heavy_explicit = heavy_threshold
        plan = HaloPlan(ip_h, ix_h, n, P, p, chunks=C, hub_threshold=hub_c,
                        heavy_threshold=_lib.SRG_HALO_AUTO if auto_heavy else int(heavy_threshold),
                        ghost_max_degree=_lib.SRG_HALO_AUTO if ghost_max_degree is None else int(ghost_max_degree),
                        link_bps=self.link_bps)
        info = plan.info
        self.ghost_max_degree = int(info["ghost_max_degree"])
        self.starts = [int(v) for v in plan.array(_lib.SRG_HALO_STARTS)]
        cr = plan.array(_lib.SRG_HALO_CHUNK_RANGES)
        self.chunk_ranges = [(int(cr[c]), int(cr[c + 1])) for c in range(C)]
        self.nnz_total = int(ip_h[-1]) if ip_h.size else 0
        r0, rows = int(info["row0"]), int(info["n_rows"])
        r1 = r0 + rows
        self.r0, self.r1, self.rows = r0, r1, rows
        b0, b1 = int(ip_h[r0]), int(ip_h[r1])
        self._b0, self._b1 = b0, b1
        self.nnz_local = b1 - b0
        self.n_recv, self.n_ghost, self.halo = int(info["n_recv"]), int(info["n_ghost"]), int(info["halo"])
        self.recv_counts = [[int(v) for v in plan.array(_lib.SRG_HALO_RECV_COUNTS, g)] for g in range(G)]
        self.ghost_recv_counts = [int(v) for v in plan.array(_lib.SRG_HALO_GHOST_RECV_COUNTS)]
        self.group_offsets = [int(v) for v in plan.array(_lib.SRG_HALO_GROUP_OFFSETS)]

        def dev64(a):
            return torch.from_numpy(a.astype("int64", copy=False)).to(dev)

        def split_peers(cat, counts):
            """A concatenation over the peers q != p (ascending) -> per-peer pieces (None for p)."""
            out, off = [None] * P, 0
            for q in range(P):
                if q == p:
                    continue
                out[q] = cat[off:off + counts[q]]
                off += counts[q]
            return out

        # --- my sends: for every peer q, my rows q receives, per group, in q's receive order, and
        # (first exchange only) my rows q computes as ghosts, by id
        self.send_counts = [[int(v) for v in plan.array(_lib.SRG_HALO_SEND_COUNTS, g)] for g in range(G)]
        self.send_cat = [dev64(plan.array(_lib.SRG_HALO_SEND_ROWS, g)) for g in range(G)]
        self.send_idx = [split_peers(self.send_cat[g], self.send_counts[g]) for g in range(G)]
        self.ghost_send_counts = [int(v) for v in plan.array(_lib.SRG_HALO_GHOST_SEND_COUNTS)]
        self.ghost_send_cat = dev64(plan.array(_lib.SRG_HALO_GHOST_SEND))
        self.ghost_send_idx = split_peers(self.ghost_send_cat, self.ghost_send_counts)
        # --- local operator over the panel rows [own | received (empty rows) | ghosts], columns
        # remapped into the same layout
        self._halo_ids = dev64(plan.array(_lib.SRG_HALO_HALO_IDS))
        self._ghost_pos = dev64(plan.array(_lib.SRG_HALO_GHOST_POSITIONS))
        lip = dev64(plan.array(_lib.SRG_HALO_LOCAL_INDPTR))
        lix = torch.from_numpy(plan.array(_lib.SRG_HALO_LOCAL_INDICES)).to(dev).contiguous()
        # the entries' GLOBAL column ids (sorted within each row, as Â's are): the column blocks
        # of the chunks' launches split every row where these cross the global block bounds
        if dev.type == "cuda":
            gix = indices.to(dev)
            self._lix_glob = torch.cat([gix[b0:b1].to(torch.int32), gix[self._ghost_pos].to(torch.int32)]).contiguous()
        else:
            self._lix_glob = None
        lvv = self._local_values(values)
        self.ncols_local = self.rows + self.halo
        # --- per-group row schedules (local row ids; long rows first), then the ghost rows' launch
        self.views = []
        narrow = []           # slice-wave rows of each view for narrow panels (d <= 32), automatic only
        for v in range(G + 1):
            order = torch.from_numpy(plan.array(_lib.SRG_HALO_VIEW_ORDER, v)).to(dev).contiguous()
            n_g, n_hub, n_heavy, n_narrow = (int(x) for x in plan.array(_lib.SRG_HALO_VIEW_META, v))
            if v < G:
                self.views.append((order, n_g, n_heavy, n_hub))
            else:
                self.ghost_view = (order, n_g, n_heavy, 0)
            narrow.append(n_narrow if auto_heavy and v != C else None)
        plan.destroy()
        self._lip, self._lix, self._lvv = lip, lix, lvv
        if local_spmm is None:
            from .csr import DeviceCSR
            from .spmm import spmm
            # the groups write own rows of the panel, the ghost launch the ghost slots of its halo
            spaces = [self.rows] * len(self.views) + [self.rows + self.halo]
            self._A = [DeviceCSR(lip, lix, lvv, n_g, self.ncols_local, order, n_heavy, n_hub, nn, row_space=rs)
                       for (order, n_g, n_heavy, n_hub), nn, rs in zip(self.views + [self.ghost_view], narrow, spaces)]
            self._spmm = lambda A, X, out: spmm(A, X, out=out)
        else:
            self._A = [(lip, lix, lvv, order) for (order, _, _, _) in self.views + [self.ghost_view]]
            self._spmm = local_spmm
        self._hip = local_spmm is None and dev.type == "cuda"      # the HIP kernels

    # ------------------------------------------------------------------------------------------
    def new_panel(self, d: int) -> torch.Tensor:
        """[own rows | halo] panel for this rank."""
        return torch.zeros((self.rows + self.halo, d), dtype=torch.float32, device=self.device)

    def with_values(self, values: torch.Tensor) -> "HaloPartitionedOperator":
        """The same partition, halo plan and schedules for an operator with the same structure and
        other values (e.g. the Chebyshev F = (2/a1)(L - a2 I) next to L); `values` is global."""
        import copy
        other = copy.copy(self)
        lvv = self._local_values(values)
        other._lvv = lvv
        other._cb = {}                 # column blocks hold the values: rebuilt for `other` on use
        if isinstance(self._A[0], tuple):
            other._A = [(a[0], a[1], lvv, a[3]) for a in self._A]
        else:
            from .csr import DeviceCSR
            other._A = [DeviceCSR(a.indptr, a.indices, lvv, a.n_rows, a.n_cols, a.order, a.n_heavy, a.n_hub,
                                  a.n_heavy_narrow, row_space=a.row_space)
                        for a in self._A]
        return other

    def _col_blocks_for(self, d: int) -> int:
        """Column blocks per row-chunk launch for a panel of d columns: `col_blocks` if given, else
        WIDE_HALO_COL_BLOCKS for local panels ([own | halo] rows) of >= WIDE_HALO_PANEL at d >= 256,
        else 1 (HIP ranks only; the C planner's srg_halo_col_blocks is the same rule)."""
        if not self._hip:
            return 1
        if self.col_blocks is not None:
            return max(1, int(self.col_blocks))
        panel = (self.rows + self.halo) * d * 4
        return WIDE_HALO_COL_BLOCKS if d >= 256 and panel >= WIDE_HALO_PANEL else 1

    def chunk_blocks(self, d: int):
        """The row chunks' column blocks for a panel of d columns: per chunk, B DeviceCSRs over row
        spans of the local operator (block b of a row: its entries whose GLOBAL column ids lie in
        [ceil(b n / B), ceil((b+1) n / B)), each block with its own schedule), or None for one
        launch per chunk.  Block 0 runs from +0.0f and blocks 1.. continue every chain with
        ACCUMULATE, so each row is the same fma chain in the same order: bitwise the unblocked
        chunk.  Rows of <= csr.BLOCK_WHOLE_MAX entries are computed whole in block 0.  Each launch
        gathers from 1 / B of the global columns, so the caches hold B times as many of the rows
        it reads (one GPU: the plan's column blocks, srg_plan_build).  Cached per B."""
        B = self._col_blocks_for(d)
        if B < 2:
            return None
        if B in self._cb:
            return self._cb[B]
        from .csr import DeviceCSR, auto_heavy_threshold, narrow_heavy_degrees, schedule_from_degrees
        bounds, whole = self._block_bounds(B)
        heavy_t = auto_heavy_threshold(self.nnz_local, launches=self.C * B) if self._auto_heavy \
            else self._heavy_explicit
        per_chunk = []
        for c in range(self.C):
            rows_c = self.views[c][0].to(torch.int64)
            if rows_c.numel() == 0:
                per_chunk.append(None)
                continue
            cut = rows_c[~whole[rows_c]]
            blocks = []
            for b in range(B):
                beg, end = bounds[b], bounds[b + 1]
                sel = rows_c if b == 0 else cut
                dsel = (end - beg)[sel]
                order, n_heavy, _ = schedule_from_degrees(dsel, int(dsel.sum()) if dsel.numel() else 0, heavy_t, -1)
                order = sel[order.to(torch.int64)].to(torch.int32).contiguous()
                narrow = narrow_heavy_degrees(dsel, 0) if self._auto_heavy else None
                blocks.append(DeviceCSR(beg, self._lix, self._lvv, int(sel.numel()), self.ncols_local, order,
                                        n_heavy, 0, narrow, row_end=end, row_space=self.rows))
            per_chunk.append(blocks)
        self._cb[B] = per_chunk
        return per_chunk

    def _block_bounds(self, B: int):
        """Per local row, the CSR positions where its entries' GLOBAL column ids cross the bounds
        ceil(b n / B) (srg_csr_col_splits): B + 1 position vectors, and the mask of the rows of
        <= csr.BLOCK_WHOLE_MAX entries, which stay whole in block 0 (their later spans empty).
        Cached per B."""
        key = ("bounds", B)
        if key in self._cb:
            return self._cb[key]
        from . import _lib
        from .csr import BLOCK_WHOLE_MAX
        dev = self.device
        nloc = self.rows + self.halo
        lip = self._lip
        splits = torch.empty((B - 1, nloc), dtype=torch.int64, device=dev)
        if nloc:
            _lib.call(dev, "srg_csr_col_splits", lip.data_ptr(), self._lix_glob.data_ptr() if self._lix_glob.numel() else None,
                      nloc, self.n, B, splits.data_ptr(), _lib.stream(dev))
        deg = lip[1:] - lip[:-1]
        whole = (deg <= BLOCK_WHOLE_MAX) if BLOCK_WHOLE_MAX > 0 else torch.zeros_like(deg, dtype=torch.bool)
        splits = torch.where(whole.unsqueeze(0), lip[1:].unsqueeze(0), splits)
        self._cb[key] = ([lip[:-1]] + [splits[b] for b in range(B - 1)] + [lip[1:]], whole)
        return self._cb[key]

    def _hub_launch(self, src: torch.Tensor, out: torch.Tensor):
        """The hub group forked onto the library's hub side stream (joined by the caller)."""
        from .spmm import spmm
        spmm(self._A[self.C], src, out=out, hub_nojoin=True, fast=self.fast)

    def _chunk_spmm(self, c: int, src: torch.Tensor, out: torch.Tensor, blocks=None):
        """Row chunk c's launch(es): one, or its column blocks in order (bitwise the same)."""
        if blocks is not None and blocks[c] is not None:
            from .spmm import spmm
            u2 = src.shape[1] >= 128
            for b, Ab in enumerate(blocks[c]):
                spmm(Ab, src, out=out, accumulate=b > 0, packed_u2=u2)
        else:
            self._spmm(self._A[c], src, out)

    def _local_values(self, values: torch.Tensor) -> torch.Tensor:
        """The local operator's values: the own rows' slice, then the ghost rows' entries."""
        own = values[self._b0:self._b1].to(self.device)
        if self.n_ghost:
            own = torch.cat([own, values[self._ghost_pos.to(values.device)].to(self.device)])
        return own.contiguous()

    def _exchange_group(self, panel: torch.Tensor, g: int, async_op: bool = False):
        """all_to_all of group g's rows, gathered from the panel's own rows here (on the current
        stream).  async_op: returns (work, send) -- the caller waits on the work before the halo is
        read."""
        P, p = self.world, self.rank
        off = self.rows + self.group_offsets[g]
        out_splits = [self.recv_counts[g][q] for q in range(P)]
        in_splits = [self.send_counts[g][q] for q in range(P)]
        total_in = sum(out_splits)
        if P == 1 or (total_in == 0 and sum(in_splits) == 0 and not dist.is_initialized()):
            return None
        recv = panel[off:off + total_in]
        if self.send_cat[g].numel():
            if self._hip and panel.dtype == torch.float32:   # srg_gather_rows_f32: 16-byte row chunks, 12-15 % faster than index_select
                from .spmm import gather_rows
                send = gather_rows(panel[: self.rows], self.send_cat[g])
            else:
                send = panel[: self.rows].index_select(0, self.send_cat[g])
        else:
            send = panel.new_zeros((0, panel.shape[1]))
        if self.virtual:
            raise RuntimeError("virtual shares exchange through simulate_halo_propagate()")
        work = dist.all_to_all_single(recv, send, out_splits, in_splits, group=self.group, async_op=async_op)
        return (work, send) if async_op else None

    def _exchange_ghosts(self, panel: torch.Tensor):
        """all_to_all of the ghost rows (X's first exchange only: later hops compute them)."""
        P = self.world
        if P == 1 or self.ghost_max_degree == 0:       # the cap is global: every rank skips alike
            return
        off = self.rows + self.n_recv
        recv = panel[off:off + self.n_ghost]
        if self.ghost_send_cat.numel():
            if self._hip and panel.dtype == torch.float32:
                from .spmm import gather_rows
                send = gather_rows(panel[: self.rows], self.ghost_send_cat)
            else:
                send = panel[: self.rows].index_select(0, self.ghost_send_cat)
        else:
            send = panel.new_zeros((0, panel.shape[1]))
        if self.virtual:
            raise RuntimeError("virtual shares exchange through simulate_halo_propagate()")
        dist.all_to_all_single(recv, send, list(self.ghost_recv_counts), list(self.ghost_send_counts),
                               group=self.group)

    def exchange(self, panel: torch.Tensor, ghosts: bool = False):
        """The whole halo of `panel` from its owners: the received rows, group by group, and with
        ghosts=True (the first panel, X) the ghost rows too."""
        for g in range(self.n_groups):
            self._exchange_group(panel, g)
        if ghosts:
            self._exchange_ghosts(panel)

    def _launch_groups(self, src: torch.Tensor, dst: torch.Tensor, ghosts: bool = True, after_group=None):
        """dst[:rows] = local Â rows @ src, everything on the current stream: the hub group's
        workgroups forked onto the library's hub side stream (srg_spmm_csr_f32 with
        SRG_SPMM_HUB_NOJOIN; they run beside the chunks), the row chunks in order, the ghost rows
        into their halo slots of dst (ghosts=True), then the join of the hub side stream.
        after_group(g) is called right after group g's launch (chunks in order, the hub group after
        its join): the hop issues group g's exchange there.
        No other stream is used: a second torch stream may share a hardware queue with this one,
        and its waits would then stall the chunks behind the hub (measured: chunks + hub instead
        of the longer of the two)."""
        gA = self._A[self.n_groups]
        C = self.C
        out = dst[: self.rows]
        if self.device.type != "cuda":
            for g in list(range(C)) + [C]:
                if self.views[g][1]:
                    self._spmm(self._A[g], src, out)
            if ghosts and self.n_ghost:
                self._spmm(gA, src, dst)
            if after_group is not None:
                for g in list(range(C)) + [C]:
                    after_group(g)
            return
        from . import _lib
        fork = bool(self.views[C][1] and self.views[C][3] and self._hip)
        if self.views[C][1]:
            if fork:
                self._hub_launch(src, out)
            else:
                self._spmm(self._A[C], src, out)
        blocks = self.chunk_blocks(src.shape[1])
        for c in range(C):
            if self.views[c][1]:
                self._chunk_spmm(c, src, out, blocks)
            if after_group is not None:
                after_group(c)
        if ghosts and self.n_ghost:
            self._spmm(gA, src, dst)
        if fork:
            _lib.call(self.device, "srg_hub_join", _lib.stream(self.device))
        if after_group is not None:
            after_group(C)

    def compute(self, src: torch.Tensor, dst: torch.Tensor, ghosts: bool = True):
        """dst[:rows] = local Â rows @ src (all groups, no exchange) and, with ghosts, the ghost
        rows of dst's halo; ordered on the current stream."""
        self._launch_groups(src, dst, ghosts=ghosts)

    def hop(self, src: torch.Tensor, dst: torch.Tensor, exchange: bool = True):
        """One hop: dst own rows from src, then (unless exchange=False, e.g. the last hop, whose halo
        no later hop reads) dst's halo, group by group: each group's rows are packed on the current
        stream right after its kernel and sent with an asynchronous all_to_all_single (RCCL runs it
        on its own stream while the later groups compute); the current stream waits for all of
        them at the end of the hop."""
        if not exchange or self.world == 1 or self.device.type != "cuda":
            self._launch_groups(src, dst, ghosts=exchange)   # no later hop reads the last ghosts
            if exchange:
                self.exchange(dst)
            return
        pending = []
        self._launch_groups(src, dst, ghosts=True,
                            after_group=lambda g: pending.append(self._exchange_group(dst, g, async_op=True)))
        for item in pending:
            if item is not None:
                item[0].wait()        # the current stream waits for RCCL's stream (the CPU does not)

    def hop_with_epilogue(self, src: torch.Tensor, dst: torch.Tensor, epilogue):
        """One exchange step whose own rows are finished by epilogue(a, b), an element-wise function
        of rows [a, b) of the SpMM output (the Chebyshev recurrence of HaloWaveletFilter), before
        peers receive them.  On the launch stream: the hub group forked (joined after chunk 0's
        kernel, which it runs beside), then per chunk c its kernel, the epilogue over its row range
        (hub rows in it included), its pack and an asynchronous all_to_all; the hub group's
        exchange last; the stream waits for the collectives at the end.  GPU ranks with the HIP
        kernels (no ghost rows: the epilogue covers own rows only)."""
        if not (self._hip and self.world > 1 and not self.virtual) or self.n_ghost:
            raise RuntimeError("hop_with_epilogue needs real GPU ranks with the HIP kernels and no ghost rows")
        from . import _lib
        from .spmm import spmm
        out = dst[: self.rows]
        C = self.C
        fork = bool(self.views[C][1] and self.views[C][3])
        if self.views[C][1]:
            if fork:
                self._hub_launch(src, out)
            else:
                self._spmm(self._A[C], src, out)
        pending = []
        blocks = self.chunk_blocks(src.shape[1])
        for c in range(C):
            if self.views[c][1]:
                self._chunk_spmm(c, src, out, blocks)
            if c == 0 and fork:
                _lib.call(self.device, "srg_hub_join", _lib.stream(self.device))
            a, b = self.chunk_ranges[c]
            if b > a:
                epilogue(a, b)
            pending.append(self._exchange_group(dst, c, async_op=True))
        pending.append(self._exchange_group(dst, C, async_op=True))
        for item in pending:
            if item is not None:
                item[0].wait()

    def halo_ids(self) -> torch.Tensor:
        """Global row ids of the panel's halo rows, in panel order (received, then ghosts)."""
        return self._halo_ids

    def propagate(self, x_local: torch.Tensor, K: int, panels=None, x_full: torch.Tensor | None = None):
        """[X, ÂX, …, Â^K X] on this rank's rows: K+1 panels [rows + halo, d] (first `rows` are
        this rank's rows in natural order).  x_full: the whole feature matrix [n, d] when this rank
        holds it (as GraphOp.propagate's `feature` is given whole): hop 0's halo is then gathered
        from it locally instead of exchanged; the results are the same bits."""
        d = x_local.shape[1]
        if panels is None:
            panels = [self.new_panel(d) for _ in range(K + 1)]
        if x_full is not None:
            if x_full.shape[0] != self.n or x_full.shape[1] != d:
                raise ValueError(f"x_full must be [{self.n}, {d}], got {tuple(x_full.shape)}")
            panels[0][: self.rows].copy_(x_full[self.r0:self.r1])
            if self.halo:
                if self._hip:
                    from .spmm import gather_rows
                    gather_rows(x_full, self._halo_ids, out=panels[0][self.rows:self.rows + self.halo])
                else:
                    panels[0][self.rows:self.rows + self.halo] = x_full.index_select(0, self._halo_ids)
        elif x_local.data_ptr() != panels[0].data_ptr():
            panels[0][: self.rows].copy_(x_local[: self.rows])
        if K > 0 and x_full is None:
            self.exchange(panels[0], ghosts=True)
        for k in range(1, K + 1):
            self.hop(panels[k - 1], panels[k], exchange=k < K)    # the last hop's halo is never read
        return panels


def _virtual_exchange(shares, panels, ghosts: bool = False):
    """all_to_all of P virtual shares emulated by copies: panels[q] is share q's [rows + halo, d]."""
    for g in range(shares[0].n_groups):
        for q, sq in enumerate(shares):             # receiver
            off = sq.rows + sq.group_offsets[g]
            for s, ss in enumerate(shares):         # source, in receive order
                cnt = sq.recv_counts[g][s]
                if cnt:
                    idx = ss.send_idx[g][q]
                    panels[q][off:off + cnt].copy_(panels[s][: ss.rows].index_select(0, idx))
                off += cnt
    if ghosts:
        for q, sq in enumerate(shares):
            off = sq.rows + sq.n_recv
            for s, ss in enumerate(shares):
                cnt = sq.ghost_recv_counts[s]
                if cnt:
                    panels[q][off:off + cnt].copy_(panels[s][: ss.rows].index_select(0, ss.ghost_send_idx[q]))
                off += cnt


def simulate_halo_propagate(indptr, indices, values, n: int, x: torch.Tensor, K: int, world: int,
                            chunks: int = 3, heavy_threshold=None, hub_threshold=None, device=None,
                            ghost_max_degree=None, shares=None, col_blocks=None, **kw):
    """P virtual halo-exchange ranks in ONE process (all_to_all emulated by copies); returns the
    K+1 full [n, d] panels.  Exercises the group split, ghost rows, halo layout and column remap
    on a device."""
    if shares is None:
        shares = [HaloPartitionedOperator(indptr, indices, values, n, chunks=chunks, heavy_threshold=heavy_threshold,
                                          hub_threshold=hub_threshold, device=device, rank=q, world=world,
                                          ghost_max_degree=ghost_max_degree, col_blocks=col_blocks, **kw)
                  for q in range(world)]
    d = x.shape[1]
    panels = [[s.new_panel(d) for _ in range(K + 1)] for s in shares]
    for s, pp in zip(shares, panels):
        pp[0][: s.rows].copy_(x[s.r0:s.r1])
    _virtual_exchange(shares, [pp[0] for pp in panels], ghosts=True)
    for k in range(1, K + 1):
        for s, pp in zip(shares, panels):
            s.compute(pp[k - 1], pp[k])
        _virtual_exchange(shares, [pp[k] for pp in panels])
    return [torch.cat([pp[k][: s.rows] for s, pp in zip(shares, panels)]) for k in range(K + 1)]


# ----------------------------------------------------------------------------------------------
# the wavelet basis' Chebyshev filter bank over the halo partition
# ----------------------------------------------------------------------------------------------
def _epilogue_device(Tn, Tc, To, mode, a1, a2, coef_prev, coef, R):
    import ctypes
    from . import _lib
    ns = R.shape[0]
    n, w = Tn.shape
    ct = ctypes.c_float
    cp = (ct * len(coef_prev))(*coef_prev) if coef_prev is not None else None
    cc = (ct * ns)(*coef) if coef is not None else None
    _lib.call(Tn.device, "srg_cheby_epilogue_f32", Tn.data_ptr(), Tn.stride(0),
              Tc.data_ptr() if Tc is not None else None, Tc.stride(0) if Tc is not None else w,
              To.data_ptr() if To is not None else None, To.stride(0) if To is not None else w, n, w, mode,
              a1, a2, cp, cc, ns, R.data_ptr(), R.stride(1), R.stride(0), _lib.stream(Tn.device))


# fp64 halo orders on GPU ranks: the hub group's rows above this many entries run as hub workgroups
HUB_GROUP64_MIN = 8192


class HaloWaveletFilter:
    """HeatWaveletFilter's fp32 split path (wavelet.py) over the halo-exchange partition: every
    Chebyshev order is the local SpMM of this rank's rows (L for order 1, F = (2/a1)(L - a2 I)
    after), the element-wise epilogue on the own rows, and one halo exchange of the new T_k --
    the same arithmetic per element as one GPU, so the result is bitwise equal to it.
    SpectralModel's operator at the RMAT-26 configuration (BASELINE.json) on P GPUs.
    dtype=torch.float64 (pygsp cheby_op's own precision, base_model.py:236-265): every order is one
    fused srg_cheby_step_hub_f64 launch over this rank's rows (the longest as hub workgroups beside
    the row waves, the lean epilogue sequence), its halo exchanged as fp64 rows -- bitwise the one-GPU
    fp64 filter and the oracle's cheby_op."""

    def __init__(self, indptr, indices, lvals, n: int, taus, order: int = 3, lmax: float = None,
                 group=None, chunks: int = 4, heavy_threshold=None, hub_threshold=None, device=None,
                 rank=None, world=None, local_spmm=None, epilogue=None, dtype=torch.float32):
        from .wavelet import heat_cheby_coeffs
        if lmax is None:
            raise ValueError("lmax is required")
        dev = torch.device(device) if device is not None else indices.device
        ip = indptr.to(dev, torch.int64)
        lv64 = lvals.to(dev, torch.float64)
        rows = torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1])
        diag = indices.to(dev).to(torch.int64) == rows
        del rows
        self.lmax = float(lmax)
        self.a1 = self.a2 = self.lmax / 2.0
        fvals = ((2.0 / self.a1) * torch.where(diag, lv64 - self.a2, lv64)).to(torch.float32)
        del diag
        self.opL = HaloPartitionedOperator(ip, indices, lvals.to(dev, torch.float32), n, group=group, chunks=chunks,
                                           heavy_threshold=heavy_threshold, hub_threshold=hub_threshold,
                                           device=dev, rank=rank, world=world, local_spmm=local_spmm,
                                           ghost_max_degree=0)   # the epilogue runs on own rows only
        self.opF = self.opL.with_values(fvals)
        self.taus = [float(t) for t in taus]
        self.coeffs = np.stack([heat_cheby_coeffs(t, self.lmax, order) for t in self.taus])
        self.rows, self.r0, self.r1 = self.opL.rows, self.opL.r0, self.opL.r1
        self._epi = epilogue or _epilogue_device
        self.overlap = True      # real GPU ranks: each order's exchange overlapped chunk by chunk
        if dtype not in (torch.float32, torch.float64):
            raise TypeError("dtype must be float32 or float64")
        self.dtype = dtype
        if dtype == torch.float64:
            from .wavelet import HeatWaveletFilter
            rows64 = torch.repeat_interleave(torch.arange(n, device=dev), ip[1:] - ip[:-1])
            diag64 = indices.to(dev).to(torch.int64) == rows64
            del rows64
            # F in fp64 (the one-GPU filter's values, not rounded), both at the local entry positions
            self._v64 = {"L": self.opL._local_values(lv64),
                         "F": self.opL._local_values((2.0 / self.a1) * torch.where(diag64, lv64 - self.a2, lv64))}
            del diag64
            # own rows by decreasing length (stable), the longest as hub rows (the one-GPU fp64 rule on
            # this rank's entries; an explicit hub_threshold holds as given)
            lip = self.opL._lip
            deg = lip[1:self.rows + 1] - lip[:self.rows]
            self._sched64 = torch.sort(deg, descending=True, stable=True).indices.to(torch.int32).contiguous()
            t = HeatWaveletFilter.hub64_rule(int(deg.sum().item())) if hub_threshold is None else int(hub_threshold)
            self._hub64_t = t
            self._n_hub64 = int((deg > t).sum().item()) if t >= 0 else 0
            # the same per exchange group of the halo plan, for the orders overlapped with their exchange: the
            # hub group's launch first, its fp64 hub rows left running on the hub side stream
            # (SRG_CHEBY_HUB_NOJOIN: they carry every fp64 hub row), then each chunk's other rows beside them,
            # every chunk's group sent right after its launch, the hub group's after the join
            # The hub group's rows above HUB_GROUP64_MIN entries run as hub workgroups too (the rank's longest
            # rows: as row waves on the stream they would hold the chunks behind them -- RMAT-26 P = 8, 334
            # such rows of up to 67 K entries: 32.2 ms per order against 24.8 for one launch, profiles/r06ap_*;
            # every hub-group row, products P = 8's 1,070 of them (all > 2,048 entries): 3.16 against 2.51 with
            # its 194 rows > 3,850 only, r06aq_*, r06ar_*).
            self._sched64_groups = []
            C = self.opL.C
            for g in [C] + list(range(C)):
                order_g, n_g = self.opL.views[g][0], self.opL.views[g][1]
                rows_g = order_g[:n_g].to(torch.int64)
                dg = deg[rows_g]
                og = rows_g[torch.sort(dg, descending=True, stable=True).indices].to(torch.int32).contiguous()
                tg = min(t, HUB_GROUP64_MIN) if g == C else t
                nh = int((dg > tg).sum().item()) if t >= 0 else 0
                self._sched64_groups.append((g, (og, nh)))
        del lv64

    def new_panel(self, d):
        if self.dtype == torch.float64:
            return torch.zeros((self.rows + self.opL.halo, d), dtype=torch.float64, device=self.opL.device)
        return self.opL.new_panel(d)

    # the local fp64 steps over column blocks: 1 = one launch per order (the default: faster on every rank share
    # measured -- products P=4 max 5.67 ms one launch vs 6.14 planner-blocked (15 blocks), P=8 2.73 vs 4.33 (12);
    # profiles/r06ae_*, r06af_*), None = the planner's rule for the rank's [rows + halo] fp64 panel, else forced
    col_blocks64 = 1

    def _plan64(self, d: int):
        """The rank's column-blocked fp64 layout (srgnn.plan.NativePlan, fp64): a plan over the local operator as
        a square one on the panel's rows -- own rows, then the halo's empty rows (their epilogue results land in
        halo slots the exchange overwrites, and in rows of an internal R that are dropped) -- or None for one
        launch per order."""
        cache = self.__dict__.setdefault("_plans64", {})
        key = (int(d), self.col_blocks64)
        if key not in cache:
            from . import _lib
            from .csr import DeviceCSR
            from .plan import NativePlan, query
            op = self.opL
            m = self.rows + op.halo
            A = DeviceCSR.from_tensors(op._lip, op._lix, self._v64["F"], n_cols=m, device=op.device, validate=False)
            cb = int(self.col_blocks64 or 0)
            t = self._hub64_t
            _, _, _, B = query(A, 2 * d, 1 << 20, cb, False, True, _lib.SRG_PLAN_WHOLE_HUBS if t >= 0 else 0,
                               (t, _lib.SRG_PLAN_NONE))
            cache[key] = NativePlan(A, d, 1 << 20, col_blocks=cb, fp64=True, hub_threshold=t) if B > 1 else None
        return cache[key]

    def drop_layouts(self) -> None:
        for P in self.__dict__.pop("_plans64", {}).values():
            if P is not None:
                P.close()

    def _order64(self, which, Tc, To, Tn, mode, coef_prev, coef, R, sched=None):
        """One fp64 order over this rank's rows: Tc gathered through the local operator (own rows and halo),
        Tn and R written on the own rows (over the rank's column-blocked plan: every panel row, R then
        [n_scales, rows + halo, d]).  sched = (rows by decreasing length, hub rows among them): one launch
        over those rows only (an exchange group of the overlapped orders)."""
        from . import _lib
        op = self.opL
        d = Tc.shape[1]
        ns = self.coeffs.shape[0]
        ct = ctypes.c_double
        cp = (ct * len(coef_prev))(*coef_prev) if coef_prev is not None else None
        cc = (ct * len(coef))(*coef) if coef is not None else None
        P = self._plan64(d) if sched is None else None
        if P is not None:
            P.cheby_step_f64(self._v64[which], Tc, To, Tn, d, d, mode, self.a1, self.a2, cp, cc, ns, R, R.stride(0))
            return
        order, n_hub = (self._sched64, self._n_hub64) if sched is None else sched
        if order.numel() == 0:
            return
        _lib.call(op.device, "srg_cheby_step_hub_f64", op._lip.data_ptr(), op._lix.data_ptr() if op._lix.numel() else None,
                  self._v64[which].data_ptr() if self._v64[which].numel() else None, order.numel(), order.data_ptr(),
                  n_hub, Tc.data_ptr(), To.data_ptr() if To is not None else None, Tn.data_ptr(), d, d, mode,
                  self.a1, self.a2, cp, cc, ns, R.data_ptr(), self.rows * d, _lib.stream(op.device))

    def _order64_overlapped(self, which, Tc, To, Tn, mode, coef_prev, coef, R, exchange: bool = True):
        """One fp64 order on real GPU ranks with its exchange overlapped (HaloPartitionedOperator.
        hop_with_epilogue's pattern): per exchange group of the halo plan one launch over its rows (the
        recurrence fused, so they are final) -- the hub group first with its hub rows left running beside
        the row chunks, each chunk's rows packed and sent with an asynchronous all_to_all right after its
        launch while the next chunks compute, the hub group's after the join; the stream waits for all of
        them.  exchange=False: the launches alone (tools/probes/halo_cheby64_ranks.py times them)."""
        from . import _lib
        op = self.opL
        pending = []
        (gh, hub_sched), chunks = self._sched64_groups[0], self._sched64_groups[1:]
        self._order64(which, Tc, To, Tn, mode | _lib.SRG_CHEBY_HUB_NOJOIN, coef_prev, coef, R, sched=hub_sched)
        for g, sched in chunks:
            self._order64(which, Tc, To, Tn, mode, coef_prev, coef, R, sched=sched)
            if exchange:
                pending.append(op._exchange_group(Tn, g, async_op=True))
        _lib.call(op.device, "srg_hub_join", _lib.stream(op.device))
        if exchange:
            pending.append(op._exchange_group(Tn, gh, async_op=True))
        for item in pending:
            if item is not None:
                item[0].wait()

    def _overlap64(self, d: int) -> bool:
        op = self.opL
        return bool(self.overlap and op._hip and op.world > 1 and not op.virtual and self._plan64(d) is None)

    def _steps64(self, S_panel, work, R):
        """steps() in fp64: the lean sequence of fused one-launch orders; yields each T_k whose halo the
        caller exchanges (all but the last order's; real GPU ranks exchange their own, overlapped chunk by
        chunk, and yield nothing)."""
        from . import _lib
        ns, nc = self.coeffs.shape
        cf = self.coeffs
        lean = nc > 2
        R_out = R
        if self._plan64(S_panel.shape[1]) is not None:
            # the plan's launches write every panel row: R over the panel's rows, the own rows copied out last
            R = torch.empty((ns, self.rows + self.opL.halo, S_panel.shape[1]), dtype=torch.float64, device=R.device)
        t_old, t_cur = S_panel, work[0]
        free = list(work[1:])
        overlap = self._overlap64(S_panel.shape[1])

        def order(exchange, *args):
            """One order; whether the caller still has to exchange its T (not when it was overlapped)."""
            if exchange and overlap:
                self._order64_overlapped(*args)
                return False
            self._order64(*args)
            return exchange
        if lean:
            more = order(nc > 2, "L", S_panel, None, t_cur, _lib.SRG_CHEBY_INIT_T, None, None, R)
        else:
            more = order(nc > 2, "L", S_panel, None, t_cur, _lib.SRG_CHEBY_INIT, cf[:, 0], cf[:, 1], R)
        if more:
            yield t_cur
        for k in range(2, nc):
            t_new = free.pop()
            last = _lib.SRG_CHEBY_NO_T if k == nc - 1 else 0
            if k == 2:
                more = order(k + 1 < nc, "F", t_cur, t_old, t_new, _lib.SRG_CHEBY_STEP_FIRST | last,
                             np.concatenate([cf[:, 0], cf[:, 1]]), cf[:, 2], R)
            else:
                more = order(k + 1 < nc, "F", t_cur, t_old, t_new, _lib.SRG_CHEBY_STEP | last, None, cf[:, k], R)
            if t_old is not S_panel:
                free.append(t_old)
            t_old, t_cur = t_cur, t_new
            if more:
                yield t_cur
        if R is not R_out:
            R_out.copy_(R[:, :self.rows])

    def _order(self, op, src, dst, epi, exchange: bool) -> bool:
        """One Chebyshev order: dst = op @ src on the own rows, finished by epi(a, b) over row
        ranges.  Real GPU ranks overlap it with dst's halo exchange chunk by chunk
        (hop_with_epilogue); otherwise the whole epilogue runs after the SpMM and the caller
        exchanges.  Returns whether the caller still has to exchange dst's halo."""
        if exchange and op._hip and op.world > 1 and not op.virtual and self.overlap:
            op.hop_with_epilogue(src, dst, epi)
            return False
        op.compute(src, dst)
        epi(0, self.rows)
        return exchange

    def steps(self, S_panel, work, R):
        """Generator over the orders: yields after an order's local compute + epilogue with the
        panel whose halo the caller must exchange next (on real GPU ranks the orders exchange
        their own halo, overlapped, and nothing is yielded).  S_panel's halo must already be
        filled; work = three [rows + halo, d] panels; R = [ns, rows, d]."""
        if self.dtype == torch.float64:
            yield from self._steps64(S_panel, work, R)
            return
        ns, nc = self.coeffs.shape
        t_old, t_cur = S_panel, work[0]
        free = list(work[1:])
        a1, a2, cf = self.a1, self.a2, self.coeffs
        # the lean epilogue sequence of HeatWaveletFilter's split path (same bits): order 1 stores
        # T1 only, order 2 forms R from T0, T1, T2, the last order stores no T (its halo is never
        # exchanged)
        lean = nc > 2

        def epi_first(a, b, t=t_cur):
            if lean:
                self._epi(t[a:b], S_panel[a:b], None, 2, a1, a2, None, None, R[:, a:b])
            else:
                self._epi(t[a:b], S_panel[a:b], None, 0, a1, a2, cf[:, 0], cf[:, 1], R[:, a:b])
        if self._order(self.opL, S_panel, t_cur, epi_first, exchange=nc > 2):
            yield t_cur
        for k in range(2, nc):
            t_new = free.pop()

            def epi_k(a, b, t=t_new, o=t_old, c=t_cur, k=k):
                last = 0x10 if k == nc - 1 else 0
                if k == 2:
                    self._epi(t[a:b], c[a:b], o[a:b], 3 | last, a1, a2, np.concatenate([cf[:, 0], cf[:, 1]]),
                              cf[:, 2], R[:, a:b])
                else:
                    self._epi(t[a:b], None, o[a:b], 1 | last, a1, a2, None, cf[:, k], R[:, a:b])
            more = self._order(self.opF, t_cur, t_new, epi_k, exchange=k + 1 < nc)
            if t_old is not S_panel:
                free.append(t_old)
            t_old, t_cur = t_cur, t_new
            if more:
                yield t_cur

    def apply(self, S_local: torch.Tensor) -> torch.Tensor:
        """[n_scales, rows, d] filter outputs for this rank's rows of the panel S (real ranks)."""
        d = S_local.shape[1]
        S_panel = self.new_panel(d)
        S_panel[: self.rows].copy_(S_local[: self.rows])
        self.opL.exchange(S_panel)
        R = torch.empty((self.coeffs.shape[0], self.rows, d), dtype=self.dtype, device=S_panel.device)
        work = [self.new_panel(d) for _ in range(3)]
        for panel in self.steps(S_panel, work, R):
            self.opL.exchange(panel)
        return R


def simulate_halo_wavelet(indptr, indices, lvals, n: int, S: torch.Tensor, taus, order: int, lmax: float,
                          world: int, chunks: int = 3, heavy_threshold=None, hub_threshold=None, device=None,
                          dtype=torch.float32, col_blocks64=1):
    """P virtual HaloWaveletFilter ranks in one process; returns the full [n_scales, n, d] output
    (col_blocks64: each fp64 rank's column blocks, 1 = one launch per order, None = the planner's rule)."""
    shares = [HaloWaveletFilter(indptr, indices, lvals, n, taus, order, lmax, chunks=chunks,
                                heavy_threshold=heavy_threshold, hub_threshold=hub_threshold, device=device,
                                rank=q, world=world, dtype=dtype) for q in range(world)]
    for f in shares:
        f.col_blocks64 = col_blocks64
    d = S.shape[1]
    ops = [f.opL for f in shares]
    S_p = [f.new_panel(d) for f in shares]
    for f, sp_ in zip(shares, S_p):
        sp_[: f.rows].copy_(S[f.r0:f.r1])
    _virtual_exchange(ops, S_p)
    Rs = [torch.empty((len(taus), f.rows, d), dtype=dtype, device=S_p[0].device) for f in shares]
    gens = [f.steps(sp_, [f.new_panel(d) for _ in range(3)], R) for f, sp_, R in zip(shares, S_p, Rs)]
    while True:
        outs = [next(g, None) for g in gens]
        if outs[0] is None:
            break
        _virtual_exchange(ops, outs)
    return torch.cat(Rs, dim=1)
