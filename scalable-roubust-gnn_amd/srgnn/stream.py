"""The light rows of a launch as LDS-DMA entry streams (srg_stream.hip, include/srgnn_hip.h).

A `StreamLayout` copies the light part of one span launch of a hop -- the rows its schedule runs after
the hub and slice-wave rows -- into one contiguous stream of (column id, value) pairs in schedule
order, cut into per-wave runs of about `wave_entries` entries.  `srg_spmm_stream_f32` then computes
those rows with every wave streaming its run's X rows into an LDS ring by LDS-DMA: the same fma chains
over the same entries in the same order as the span launch, so the same bits.  An accumulating launch
(the later column blocks of a hop) gets a pseudo entry per row that reads the row's partial sum from
the output panel (fma(1, y, -0) == y).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib

# default run length of a wave (entries); see srg_stream.hip
WAVE_ENTRIES = 512
STREAM_WIDTHS = (64, 128, 256)


@dataclass
class StreamLayout:
    ent: torch.Tensor       # int32 [entries, 2]
    end: torch.Tensor       # int64 [n]
    row: torch.Tensor       # int32 [n]
    wave: torch.Tensor      # int32 [waves + 1]
    n: int
    entries: int
    waves: int
    wave_entries: int
    accumulate: bool

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.ent, self.end, self.row, self.wave))


def build(order: torch.Tensor, beg: torch.Tensor, end: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
          accumulate: bool, wave_entries: int = WAVE_ENTRIES) -> StreamLayout:
    """The stream of rows order[i] (int32) whose entries are [beg[r], end[r]) (int64, row-indexed) of
    indices (int32) / values (fp32), all on one device."""
    dev = indices.device
    order = order.to(torch.int32).contiguous()
    n = int(order.numel())
    if beg.dtype != torch.int64 or end.dtype != torch.int64:
        raise TypeError("beg / end must be int64")
    if indices.dtype != torch.int32 or values.dtype != torch.float32:
        raise TypeError("indices must be int32 and values float32")
    ents, waves = ctypes.c_int64(0), ctypes.c_int64(0)
    s = _lib.stream(dev)
    _lib.call(dev, "srg_stream_layout_size", order.data_ptr() if n else None, n, beg.data_ptr(), end.data_ptr(),
              1 if accumulate else 0, int(wave_entries), ctypes.byref(ents), ctypes.byref(waves), s)
    E, W = int(ents.value), int(waves.value)
    ent = torch.empty((max(E, 1), 2), dtype=torch.int32, device=dev)
    st_end = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    st_row = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    st_wave = torch.empty(W + 1, dtype=torch.int32, device=dev)
    _lib.call(dev, "srg_stream_layout_build", order.data_ptr() if n else None, n, beg.data_ptr(), end.data_ptr(),
              indices.data_ptr(), values.data_ptr(), 1 if accumulate else 0, int(wave_entries), E, W,
              ent.data_ptr(), st_end.data_ptr(), st_row.data_ptr(), st_wave.data_ptr(), s)
    return StreamLayout(ent, st_end, st_row, st_wave, n, E, W, int(wave_entries), bool(accumulate))


def run(L: StreamLayout, X: torch.Tensor, Y: torch.Tensor, nt_store: bool = False) -> torch.Tensor:
    """Y[L.row[i]] = stream row i * X (accumulating into Y's rows when the layout does)."""
    d = X.shape[1]
    if Y.shape[1] != d or X.dtype != torch.float32 or Y.dtype != torch.float32 or X.stride(1) != 1 or \
            Y.stride(1) != 1 or X.device != L.ent.device or Y.device != L.ent.device:
        raise ValueError("X and Y must be float32 row-major panels of the same width on the layout's device")
    flags = (_lib.SRG_SPMM_ACCUMULATE if L.accumulate else 0) | (_lib.SRG_SPMM_NT_STORE if nt_store else 0)
    _lib.call(X.device, "srg_spmm_stream_f32", L.ent.data_ptr(), L.end.data_ptr(), L.row.data_ptr(),
              L.wave.data_ptr(), L.waves, L.wave_entries, X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), d,
              flags, _lib.stream(X.device))
    return Y
