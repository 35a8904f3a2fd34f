"""Test infrastructure: the halo-exchange plan restated in torch -- the planner srgnn/dist.py used
before round 5, when HaloPartitionedOperator planned with torch (the product now runs the library's
srg_halo_plan_build for Python and C hosts alike).  tests/test_halo_capi_cpu.py checks the library's
plan against this restatement array for array: row blocks, chunks and hub group, halos by (group,
owner, id), the ghost rows and the automatic ghost cap (the link-rate cost model), sends, the
remapped local CSR and the schedules.  Not imported by the product."""
import torch

from srgnn.csr import NARROW_HEAVY_THRESHOLD, auto_heavy_threshold, auto_hub_threshold
from srgnn.dist import balanced_row_starts

HALO_HEAVY_MIN = 192
GHOST_SCAN_MAX = 64
GHOST_CAPS = (0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64)
GHOST_GATHER_BPS = 8.4e12


def _chunk_bounds(indptr_local: torch.Tensor, chunks: int):
    """Contiguous local row ranges with about equal nonzeros (like balanced_row_starts)."""
    return balanced_row_starts(indptr_local, chunks)


def _row_positions(gip: torch.Tensor, rows: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    """Global nonzero ids of `rows` (their CSR ranges, concatenated in the given row order)."""
    total = int(lens.sum()) if lens.numel() else 0
    if total == 0:
        return torch.zeros(0, dtype=torch.int64, device=gip.device)
    starts = torch.repeat_interleave(gip[rows], lens)
    first = torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
    return starts + (torch.arange(total, device=gip.device) - first)


def _ghost_candidates(gip, gix, deg, halo, s0: int, s1: int, n: int, max_degree: int) -> torch.Tensor:
    """Mask over `halo` (rank q's full halo; q owns rows [s0, s1)): rows with at most `max_degree`
    nonzeros whose every column is one of q's own rows or halo rows -- q can compute them from its
    own panel, so it need not receive them."""
    ok = torch.zeros(halo.numel(), dtype=torch.bool, device=halo.device)
    if max_degree <= 0 or halo.numel() == 0:
        return ok
    cand = torch.nonzero(deg[halo] <= max_degree).flatten()
    if cand.numel() == 0:
        return ok
    rows = halo[cand]
    lens = deg[rows]
    mark = torch.zeros(n, dtype=torch.bool, device=halo.device)
    mark[s0:s1] = True
    mark[halo] = True
    pos = _row_positions(gip, rows, lens)
    seg = torch.repeat_interleave(torch.arange(rows.numel(), device=halo.device), lens)
    bad = torch.zeros(rows.numel(), dtype=torch.int64, device=halo.device)
    bad.index_add_(0, seg, (~mark[gix[pos].to(torch.int64)]).to(torch.int64))
    ok[cand[bad == 0]] = True
    return ok



def ghost_plan(halos, elig, deg, owner, gip, starts, caps=GHOST_CAPS, link_bps=64e9):
    """The ghost degree cap minimising the modelled hop time max over ranks q of
    max(q's SpMM incl. ghosts, q's busiest peer link), with the rates GHOST_GATHER_BPS and
    `link_bps`.  Returns (cap, {cap: modelled seconds per byte of row}).
    Deterministic from the global plan and the rates, so every rank picks the same cap."""
    link_bps = float(link_bps)
    P = len(halos)
    model = {}
    for c in caps:
        worst = 0.0
        for q in range(P):
            h, e = halos[q], elig[q]
            dh = deg[h]
            gmask = e & (dh <= c)
            nnz_q = int(gip[starts[q + 1]] - gip[starts[q]]) + int(dh[gmask].sum())
            recv = torch.bincount(owner[h[~gmask]], minlength=P)
            link = int(recv.max()) if recv.numel() else 0
            worst = max(worst, nnz_q / GHOST_GATHER_BPS, link / link_bps)
        model[c] = worst
    best = min(caps, key=lambda c: (model[c], c))
    return best, model


class PyHaloPlan:
    """Rank p's share as the torch planner built it (CPU tensors): the attributes
    HaloPartitionedOperator had (starts, chunk_ranges, r0 / rows, n_recv / n_ghost / halo, views,
    ghost_view, recv / send counts and lists, group_offsets, _lip, _lix, _ghost_pos, halo_ids,
    ghost_max_degree)."""

    def __init__(self, indptr, indices, n, world, rank, chunks=4, hub_threshold=None, heavy_threshold=None,
                 ghost_max_degree=None, link_bps=64e9):
        P, p = world, rank
        dev = torch.device("cpu")
        self.n = n
        gip = torch.as_tensor(indptr).to(dev, torch.int64)
        gix = torch.as_tensor(indices).to(dev)
        self.starts = balanced_row_starts(gip, P)
        st = torch.tensor(self.starts, dtype=torch.int64, device=dev)
        self.nnz_total = int(gip[-1])
        deg = gip[1:] - gip[:-1]
        owner = torch.bucketize(torch.arange(n, device=dev), st[1:], right=True)   # owner rank of each row
        # hub flags: each owner's threshold (auto from its own nonzero count unless given)
        thr = torch.empty(P, dtype=torch.int64, device=dev)
        for q in range(P):
            nnz_q = int(gip[self.starts[q + 1]] - gip[self.starts[q]])
            thr[q] = auto_hub_threshold(nnz_q, launches=max(1, int(chunks))) if hub_threshold is None else (
                hub_threshold if hub_threshold >= 0 else (1 << 62))
        is_hub = deg > thr[owner]
        # chunk of every row (contiguous nnz-balanced ranges inside each owner's block)
        C = max(1, int(chunks))
        self.C = C
        grp = torch.empty(n, dtype=torch.int64, device=dev)
        for q in range(P):
            s0, s1 = self.starts[q], self.starts[q + 1]
            lip = gip[s0:s1 + 1] - gip[s0]
            cb = _chunk_bounds(lip, C)
            for c in range(C):
                grp[s0 + cb[c]:s0 + cb[c + 1]] = c
            if q == p:
                # local row range of each chunk (its hub rows included: they belong to group C)
                self.chunk_ranges = [(cb[c], cb[c + 1]) for c in range(C)]
        grp[is_hub] = C
        self.n_groups = C + 1
        G = self.n_groups
        r0, r1 = self.starts[p], self.starts[p + 1]
        self.r0, self.r1, self.rows = r0, r1, r1 - r0
        b0, b1 = int(gip[r0]), int(gip[r1])
        self._b0, self._b1 = b0, b1
        self.nnz_local = b1 - b0

        def needs_of(q):
            """q's full halo (distinct remote columns of its rows), sorted by (group, source, id)."""
            q0, q1 = int(gip[self.starts[q]]), int(gip[self.starts[q + 1]])
            cols = torch.unique(gix[q0:q1].to(torch.int64))
            cols = cols[(cols < self.starts[q]) | (cols >= self.starts[q + 1])]
            key = (grp[cols] * P + owner[cols]) * n + cols          # sort by (group, source, id)
            return cols[torch.argsort(key)]

        # --- every rank's halo and its ghost candidates (identical on all ranks: sends follow)
        halos, elig = [], []
        for q in range(P):
            hq = needs_of(q)
            halos.append(hq)
            elig.append(_ghost_candidates(gip, gix, deg, hq, self.starts[q], self.starts[q + 1], n,
                                          GHOST_SCAN_MAX if ghost_max_degree is None else ghost_max_degree))
        self.link_bps = link_bps
        if ghost_max_degree is None:
            ghost_max_degree = ghost_plan(halos, elig, deg, owner, gip, self.starts, link_bps=self.link_bps)[0]
        self.ghost_max_degree = int(ghost_max_degree)
        ghosts = [e & (deg[h] <= self.ghost_max_degree) for h, e in zip(halos, elig)]
        need = halos[p][~ghosts[p]]                                  # received: (group, source, id)
        gh = halos[p][ghosts[p]]
        gh = gh[torch.argsort(owner[gh] * n + gh)]                   # ghosts: (source, id)
        ng, ns = grp[need], owner[need]
        counts = torch.zeros((G, P), dtype=torch.int64, device=dev)
        counts.index_put_((ng, ns), torch.ones_like(need), accumulate=True)
        self.recv_counts = counts.cpu().tolist()                 # [group][source]
        self.ghost_recv_counts = torch.bincount(owner[gh], minlength=P).cpu().tolist()
        self.n_recv = int(need.numel())
        self.n_ghost = int(gh.numel())
        self.halo = self.n_recv + self.n_ghost
        self.group_offsets = []                                  # start of each group's halo region
        off = 0
        for g in range(G):
            self.group_offsets.append(off)
            off += sum(self.recv_counts[g])
        # --- my sends: for every peer q, my rows q receives, per group, in q's receive order, and
        # (first exchange only) my rows q computes as ghosts, by id
        self.send_idx = [[None] * P for _ in range(G)]
        self.send_counts = [[0] * P for _ in range(G)]
        self.ghost_send_idx = [None] * P
        self.ghost_send_counts = [0] * P
        for q in range(P):
            if q == p:
                continue
            hq = halos[q]
            from_me = owner[hq] == p
            mine = hq[from_me & ~ghosts[q]]                      # already sorted by (group, id)
            gm = grp[mine]
            for g in range(G):
                sel = mine[gm == g] - r0
                self.send_idx[g][q] = sel
                self.send_counts[g][q] = int(sel.numel())
            gq = torch.sort(hq[from_me & ghosts[q]]).values - r0
            self.ghost_send_idx[q] = gq
            self.ghost_send_counts[q] = int(gq.numel())
        del halos, elig, ghosts
        self.send_cat = []
        for g in range(G):
            parts = [self.send_idx[g][q] for q in range(P) if q != p and self.send_counts[g][q] > 0]
            self.send_cat.append(torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=dev))
        parts = [self.ghost_send_idx[q] for q in range(P) if q != p and self.ghost_send_counts[q] > 0]
        self.ghost_send_cat = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=dev)
        # --- local operator over the panel rows [own | received (empty rows) | ghosts], columns
        # remapped into the same layout
        self._halo_ids = torch.cat([need, gh]).contiguous()
        g2l = torch.full((n,), -1, dtype=torch.int64, device=dev)
        g2l[r0:r1] = torch.arange(self.rows, device=dev)
        g2l[need] = self.rows + torch.arange(self.n_recv, device=dev)
        g2l[gh] = self.rows + self.n_recv + torch.arange(self.n_ghost, device=dev)
        gdeg = deg[gh]
        self._ghost_pos = _row_positions(gip, gh, gdeg)              # global nnz ids of the ghost rows
        glob = torch.cat([gix[b0:b1].to(torch.int64), gix[self._ghost_pos].to(torch.int64)])
        lix = g2l[glob]
        del glob
        if bool((lix < 0).any()):
            raise RuntimeError("halo layout misses a referenced column")
        lens = torch.cat([deg[r0:r1], torch.zeros(self.n_recv, dtype=torch.int64, device=dev), gdeg])
        lip = torch.zeros(self.rows + self.halo + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=lip[1:])
        lix = lix.to(torch.int32).contiguous()
        self.ncols_local = self.rows + self.halo
        # --- per-group row schedules (local row ids; long rows first)
        lgrp = grp[r0:r1]
        ldeg = deg[r0:r1]
        # per launch: the rank's nonzeros split over its row chunks, as for the hub threshold
        auto_heavy = heavy_threshold is None
        heavy_t = max(HALO_HEAVY_MIN, auto_heavy_threshold(int(lip[self.rows]), launches=C)) if auto_heavy \
            else heavy_threshold
        self.views = []
        narrow = []           # slice-wave rows of each view for narrow panels (d <= 32), automatic only
        for g in range(G):
            rows_g = torch.nonzero(lgrp == g).flatten()
            rows_g = rows_g[torch.sort(ldeg[rows_g], descending=True, stable=True).indices]
            n_g = int(rows_g.numel())
            if g == C:
                n_hub, n_heavy = n_g, 0
            else:
                n_hub = 0
                n_heavy = int((ldeg[rows_g] > heavy_t).sum()) if heavy_t >= 0 else 0
            self.views.append((rows_g.to(torch.int32).contiguous(), n_g, n_heavy, n_hub))
            narrow.append(int((ldeg[rows_g] > NARROW_HEAVY_THRESHOLD).sum()) if auto_heavy and g != C else None)
        # the ghost rows: one more launch (no exchange), panel rows rows + n_recv + i
        gsort = torch.sort(gdeg, descending=True, stable=True)
        g_rows = (self.rows + self.n_recv + gsort.indices).to(torch.int32).contiguous()
        g_heavy = int((gsort.values > heavy_t).sum()) if heavy_t >= 0 else 0
        self.ghost_view = (g_rows, self.n_ghost, g_heavy, 0)
        narrow.append(int((gsort.values > NARROW_HEAVY_THRESHOLD).sum()) if auto_heavy else None)
        self.narrow = narrow
        self._lip, self._lix = lip, lix

    def halo_ids(self):
        return self._halo_ids
