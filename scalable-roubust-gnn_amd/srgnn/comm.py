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
