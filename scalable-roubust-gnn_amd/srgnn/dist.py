"""Multi-GPU propagation: 1-D row partition of Â, one process per GPU, one all-gather per hop.

SURVEY.md §8(e).  Rank p owns the contiguous row block [starts[p], starts[p+1]) of Â (blocks
balanced by nonzeros) and the same rows of every hop panel.  Before each hop the ranks all-gather
their current panel blocks into a full panel (RCCL over xGMI with the "nccl" backend; gloo on CPU
for tests), then each rank computes its rows of the next hop with the local kernel.

Layout: blocks are gathered into a PADDED full panel [P * max_rows, d] (one fixed-size collective,
no re-packing), so the local operator's column ids are remapped once, at partition time, from
global id c (in block q) to q * max_rows + (c - starts[q]).  The remap is monotone, so every row's
nonzeros keep their CSR order and each output element is the same fma chain as on one GPU: the
multi-GPU result is bitwise equal to the single-GPU one.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def balanced_row_starts(indptr: torch.Tensor, parts: int):
    """Row boundaries [0 = s_0 <= ... <= s_P = n] splitting the nonzeros as evenly as rows allow."""
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
