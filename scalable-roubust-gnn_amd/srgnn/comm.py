"""Python handle on the C-ABI communicator entries (srg_comm_*, srg_dist_propagate_khop_f32; include/
srgnn_hip.h): the RCCL row-partitioned K-hop propagation a C / C++ host would call, usable from Python
for testing and for single-process multi-GPU runs.  The torch.distributed path (srgnn.dist) is the
package's own multi-GPU driver; both are bitwise the one-GPU hops."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .csr import DeviceCSR


class ShardF32(ctypes.Structure):
    """srg_shard_f32 (include/srgnn_hip.h)."""
    _fields_ = [("device", ctypes.c_int), ("indptr", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("row0", ctypes.c_int64), ("n_rows", ctypes.c_int64),
                ("row_order", ctypes.c_void_p), ("n_hub", ctypes.c_int64), ("n_heavy", ctypes.c_int64),
                ("x_full", ctypes.c_void_p), ("panels", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _lib.call_host("srg_comm_unique_id", buf)
    return buf.raw


class Comm:
    """srg_comm: init_all(devices) for one process driving several GPUs, init_rank(...) for one
    rank per process (the id from unique_id() on rank 0, shared out of band)."""

    def __init__(self, handle, devices, first_rank: int = 0):
        self._h = handle
        self.devices = list(devices)
        self._first_rank = first_rank        # global rank of local rank 0

    @classmethod
    def init_all(cls, devices):
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        _lib.call_host("srg_comm_init_all", len(devices), devs, ctypes.byref(h))
        return cls(h, devices)

    @classmethod
    def init_rank(cls, nranks: int, uid: bytes, rank: int, device: int):
        h = ctypes.c_void_p()
        _lib.call_host("srg_comm_init_rank", nranks, ctypes.c_char_p(uid), rank, device, ctypes.byref(h))
        return cls(h, [device], first_rank=rank)

    @property
    def size(self) -> int:
        return _lib.query("srg_comm_size", self._h)

    def destroy(self):
        if self._h:
            _lib.call_host("srg_comm_destroy", self._h)
            self._h = None

    def propagate(self, blocks: list[DeviceCSR], row_starts: list[int], x_blocks: list[torch.Tensor], K: int,
                  panels: list[list[torch.Tensor]] | None = None):
        """panels[i][k] (k = 0..K) of local rank i: the rank's rows of Â^k X.  blocks[i] is the
        rank's row block (rebased indptr, global column ids), x_blocks[i] its rows of X."""
        n = int(row_starts[-1])
        d = int(x_blocks[0].shape[1])
        shards = (ShardF32 * len(blocks))()
        keep = []
        out = []
        for i, (A, xb) in enumerate(zip(blocks, x_blocks)):
            dev = xb.device
            ps = panels[i] if panels is not None else [xb] + [torch.empty_like(xb) for _ in range(K)]
            if any(p.stride(0) != d or not p.is_contiguous() for p in ps):
                raise ValueError("panels must be contiguous [rows, d] tensors")
            x_full = torch.empty((n, d), dtype=torch.float32, device=dev)
            arr = (ctypes.c_void_p * (K + 1))(*[p.data_ptr() for p in ps])
            keep += [x_full, arr]
            shards[i] = ShardF32(dev.index, A.indptr.data_ptr(), A.indices.data_ptr() if A.nnz else None,
                                 A.values.data_ptr() if A.nnz else None, int(row_starts[self._rank_of(i)]),
                                 A.n_rows, A.order.data_ptr() if A.n_rows else None, A.n_hub, A.heavy(d),
                                 x_full.data_ptr(), ctypes.cast(arr, ctypes.c_void_p),
                                 torch.cuda.current_stream(dev).cuda_stream)
            out.append(ps)
        starts = (ctypes.c_int64 * len(row_starts))(*[int(s) for s in row_starts])
        _lib.call_host("srg_dist_propagate_khop_f32", self._h, shards, len(blocks), starts, d, d, K)
        for dev in {xb.device for xb in x_blocks}:
            torch.cuda.synchronize(dev)
        del keep
        return out

    def _rank_of(self, i: int) -> int:
        return self._first_rank + i


# ------------------------------------------------------------------------------------------------
# the halo-exchange partition through the C-ABI (srg_halo_*): the plan a C / C++ host builds, its
# device shares, and the hop loop over RCCL or the loopback transport
# ------------------------------------------------------------------------------------------------
_HALO_DTYPES = {_lib.SRG_HALO_STARTS: ctypes.c_int64, _lib.SRG_HALO_LOCAL_INDPTR: ctypes.c_int64,
                _lib.SRG_HALO_LOCAL_INDICES: ctypes.c_int32, _lib.SRG_HALO_GHOST_POSITIONS: ctypes.c_int64,
                _lib.SRG_HALO_HALO_IDS: ctypes.c_int64, _lib.SRG_HALO_GROUP_OFFSETS: ctypes.c_int64,
                _lib.SRG_HALO_GHOST_SEND: ctypes.c_int64, _lib.SRG_HALO_GHOST_SEND_COUNTS: ctypes.c_int64,
                _lib.SRG_HALO_GHOST_RECV_COUNTS: ctypes.c_int64, _lib.SRG_HALO_CHUNK_RANGES: ctypes.c_int64,
                _lib.SRG_HALO_HUB_THRESHOLDS: ctypes.c_int64, _lib.SRG_HALO_VIEW_ORDER: ctypes.c_int32,
                _lib.SRG_HALO_VIEW_META: ctypes.c_int64, _lib.SRG_HALO_SEND_ROWS: ctypes.c_int64,
                _lib.SRG_HALO_SEND_COUNTS: ctypes.c_int64, _lib.SRG_HALO_RECV_COUNTS: ctypes.c_int64}


class HaloPlan:
    """srg_halo_plan: rank `rank`'s share of the halo partition, built by the library's host planner
    from the global CSR (numpy / CPU arrays).  Needs no device.  ghost_max_degree: a cap, or
    SRG_HALO_AUTO for the link-rate cost model at `link_bps` (<= 0: 64e9)."""

    def __init__(self, indptr, indices, n: int, nranks: int, rank: int, chunks: int = 4,
                 hub_threshold: int = _lib.SRG_HALO_AUTO, heavy_threshold: int = _lib.SRG_HALO_AUTO,
                 ghost_max_degree: int = 0, link_bps: float = 0.0):
        import numpy as np
        self._ip = np.ascontiguousarray(np.asarray(indptr), dtype=np.int64)
        self._ix = np.ascontiguousarray(np.asarray(indices), dtype=np.int32)
        # the planner reads indptr[0 .. n] and indices[0 .. indptr[n]): short arrays would be host
        # over-reads, so their sizes are checked here (the C side validates their contents)
        if self._ip.ndim != 1 or self._ip.size != int(n) + 1:
            raise ValueError(f"indptr must have n + 1 = {int(n) + 1} entries, got {self._ip.size}")
        if self._ix.ndim != 1 or self._ix.size != int(self._ip[-1]):
            raise ValueError(f"indices must have indptr[n] = {int(self._ip[-1])} entries, got {self._ix.size}")
        self.nnz = int(self._ip[-1])
        h = ctypes.c_void_p()
        _lib.call_host("srg_halo_plan_build", self._ip.ctypes.data, self._ix.ctypes.data if self._ix.size else None,
                       int(n), int(nranks), int(rank), int(chunks), int(hub_threshold), int(heavy_threshold),
                       int(ghost_max_degree), float(link_bps), ctypes.byref(h))
        self._h = h
        info = _lib.HaloInfo()
        _lib.call_host("srg_halo_plan_info", self._h, ctypes.byref(info))
        self.info = {k: getattr(info, k) for k, _ in _lib.HaloInfo._fields_}

    def array(self, what: int, index: int = 0):
        """A copy of one of the plan's arrays (numpy)."""
        import numpy as np
        data, count = ctypes.c_void_p(), ctypes.c_int64()
        _lib.call_host("srg_halo_plan_array", self._h, int(what), int(index), ctypes.byref(data), ctypes.byref(count))
        ct = _HALO_DTYPES[what]
        if count.value == 0:
            return np.zeros(0, dtype=np.int64 if ct is ctypes.c_int64 else np.int32)
        return np.ctypeslib.as_array(ctypes.cast(data, ctypes.POINTER(ct)), shape=(count.value,)).copy()

    def destroy(self):
        if self._h:
            _lib.call_host("srg_halo_plan_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001
            pass


class HaloShare:
    """srg_halo_share: a plan's device arrays on `device` (values: the GLOBAL fp32 values, host)."""

    def __init__(self, plan: HaloPlan, values, device: int, d_max: int):
        import numpy as np
        v = np.ascontiguousarray(np.asarray(values), dtype=np.float32)
        if v.ndim != 1 or v.size != plan.nnz:
            raise ValueError(f"values must hold the global CSR's {plan.nnz} entries, got {v.size}")
        h = ctypes.c_void_p()
        _lib.call_host("srg_halo_share_create", plan._h, v.ctypes.data if v.size else None, int(device), int(d_max),
                       ctypes.byref(h))
        self._h, self.plan, self.device = h, plan, torch.device("cuda", int(device))
        self.rows, self.halo = plan.info["n_rows"], plan.info["halo"]

    def col_blocks(self, n_blocks: int = _lib.SRG_HALO_AUTO):
        """srg_halo_share_col_blocks: the row chunks in n_blocks column blocks (1: unblocked) for every
        d, or the automatic rule per d (SRG_HALO_AUTO)."""
        _lib.call_host("srg_halo_share_col_blocks", self._h, int(n_blocks))
        return self

    def new_panel(self, d: int) -> torch.Tensor:
        return torch.zeros((self.rows + self.halo, d), dtype=torch.float32, device=self.device)

    def check_panel(self, p: torch.Tensor, d: int, what: str):
        """A [rows + halo, d] float32 contiguous panel on the share's device (the C side trusts it)."""
        if not isinstance(p, torch.Tensor) or p.dtype != torch.float32 or p.device != self.device or \
                tuple(p.shape) != (self.rows + self.halo, d) or not p.is_contiguous():
            raise ValueError(f"{what} must be a contiguous float32 [{self.rows + self.halo}, {d}] tensor on "
                             f"{self.device}, got {getattr(p, 'dtype', None)} {tuple(getattr(p, 'shape', ()))} "
                             f"on {getattr(p, 'device', None)}")

    def fill_x_halo(self, X: torch.Tensor, panel0: torch.Tensor):
        """Panel 0 from the whole X: own rows, then the halo rows gathered by global id."""
        d = int(X.shape[1]) if isinstance(X, torch.Tensor) and X.dim() == 2 else -1
        if d < 0 or X.dtype != torch.float32 or X.device != self.device or X.stride(1) != 1 or \
                X.shape[0] != int(self.plan._ip.size - 1):
            raise ValueError("X must be the whole float32 [n, d] feature matrix (unit column stride) on the "
                             "share's device")
        self.check_panel(panel0, d, "panel0")
        _lib.call(self.device, "srg_halo_fill_x_halo", self._h, X.data_ptr(), X.stride(0), panel0.data_ptr(),
                  panel0.stride(0), X.shape[1], _lib.stream(self.device))

    def destroy(self):
        if self._h:
            _lib.call_host("srg_halo_share_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001
            pass


def loopback(nranks: int, device: int = 0) -> Comm:
    """srg_comm_init_loopback: nranks virtual ranks in this process on one device."""
    h = ctypes.c_void_p()
    _lib.call_host("srg_comm_init_loopback", int(nranks), int(device), ctypes.byref(h))
    return Comm(h, [device] * nranks)


def halo_propagate(comm: Comm, shares: list[HaloShare], panels: list[list[torch.Tensor]], K: int,
                   x_halo_filled: bool = False, streams=None):
    """srg_halo_propagate_f32 over the local shares (loopback: every rank, in order); panels[i][k]
    [rows + halo, d] of share i; asynchronous on each share's stream (torch's current one by
    default)."""
    n = len(shares)
    if n == 0 or len(panels) != n:
        raise ValueError(f"one panel list per share: {len(panels)} lists for {n} shares")
    if K < 0:
        raise ValueError("K must be >= 0")
    d = int(panels[0][0].shape[1])
    for i, (s, ps) in enumerate(zip(shares, panels)):
        if len(ps) != K + 1:
            raise ValueError(f"share {i}: K + 1 = {K + 1} panels needed, got {len(ps)}")
        for k, p in enumerate(ps):
            s.check_panel(p, d, f"panels[{i}][{k}]")
    arrs = [(ctypes.c_void_p * (K + 1))(*[p.data_ptr() for p in ps]) for ps in panels]
    parr = (ctypes.c_void_p * n)(*[ctypes.cast(a, ctypes.c_void_p) for a in arrs])
    sh = (ctypes.c_void_p * n)(*[s._h for s in shares])
    strm = (ctypes.c_void_p * n)(*[(streams[i] if streams else torch.cuda.current_stream(s.device).cuda_stream)
                                   for i, s in enumerate(shares)])
    # every panel is contiguous [rows + halo, d]: its leading dimension is d
    _lib.call_host("srg_halo_propagate_f32", comm._h, sh, n, parr, panels[0][0].stride(0), d, int(K),
                   _lib.SRG_HALO_X_HALO_FILLED if x_halo_filled else 0, strm)
