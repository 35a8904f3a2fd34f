"""Reference-compatible operator base classes (mirror of SSRG/operators/base_operator.py).

`GraphOp.propagate` keeps the reference's signature, checks, error messages and return type (a list
of K+1 CPU float32 tensors, hop 0 being the caller's feature array) -- SSRG/operators/
base_operator.py:19-36 -- but the K hops run back to back on the GPU: Â and X are uploaded once,
the hop loop is `srgnn.spmm.propagate` (libsrgnn_hip.so, exact fma chains, bit-identical to the
reference's FloatCSRMulDenseOMP), and the K result panels come back in one batch of copies.

`propagate_device` is the performance entry: same computation, device tensors in and out.

`propagate_aggregate(adj, feature, msg_op)` is `msg_op.aggregate(self.propagate(adj, feature))` --
the non-learnable branch of BaseSGModel.preprocess (SSRG/models/base_scalable/base_model.py:34-44)
-- without the hop list: srgnn.aggregate folds each hop into the result as it is produced, in the
reference's own summation order (bit-identical), so only 4-5 panels are ever resident.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn as nn
from torch import Tensor

from operators.utils import csr_sparse_dense_matmul, cuda_csr_sparse_dense_matmul  # noqa: F401
from srgnn.csr import DeviceCSR
from srgnn.spmm import propagate as _device_propagate


def _hops_to_host(A, X, K, ring=3):
    """Hops 1..K of A on the device panel X, each copied to pinned host memory on a copy stream
    while the next hop runs (the D2H of the reference-shaped list overlaps the kernels); device
    memory holds a ring of `ring` hop panels.  Returns the K host tensors."""
    from srgnn.spmm import spmm
    dev = A.device
    main = torch.cuda.current_stream(dev)
    copy_s = torch.cuda.Stream(dev)
    R = max(1, min(K, ring))
    bufs = [torch.empty_like(X) for _ in range(R)]
    host = [torch.empty(tuple(X.shape), dtype=torch.float32, pin_memory=True) for _ in range(K)]
    copied = []
    prev = X
    for k in range(1, K + 1):
        buf = bufs[(k - 1) % R]
        if k > R:
            main.wait_event(copied[k - 1 - R])      # the ring slot's previous hop is on the host
        spmm(A, prev, out=buf)
        done = torch.cuda.Event()
        done.record(main)
        copy_s.wait_event(done)
        with torch.cuda.stream(copy_s):
            host[k - 1].copy_(buf, non_blocking=True)
        c = torch.cuda.Event()
        c.record(copy_s)
        copied.append(c)
        prev = buf
    copy_s.synchronize()
    main.synchronize()
    return host


class GraphOp:
    def __init__(self, prop_steps):
        self.prop_steps = prop_steps
        self._adj, self._adj_dev = None, None

    # The reference keeps Â as self.adj (a scipy matrix).  When Â is built on the device
    # (construct_adj_device) the host copy is made on first access only.
    @property
    def adj(self):
        if self._adj is None and self._adj_dev is not None:
            from srgnn.construct import to_scipy
            self._adj = to_scipy(*self._adj_dev)
        return self._adj

    @adj.setter
    def adj(self, value):
        self._adj, self._adj_dev = value, None

    def construct_adj(self, adj):
        raise NotImplementedError

    def construct_adj_device(self, adj, device):
        """(indptr, indices, values fp64) device tensors of construct_adj(adj), bit-identical, or
        None when the operator has no device form (the host construct_adj is used then)."""
        return None

    def _build_operator(self, adj, device=None):
        """construct_adj on the device when the operator has a device form and adj is a square CSR
        (SURVEY.md §8(f) item 2); otherwise the host construct_adj, with its own errors."""
        if isinstance(adj, sp.csr_matrix) and adj.shape[0] == adj.shape[1]:
            dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            built = self.construct_adj_device(adj, dev)
            if built is not None:
                ip, ix, v64 = built
                self._adj, self._adj_dev = None, (ip, ix, v64, adj.shape[0])
                return DeviceCSR.from_tensors(ip, ix, v64.to(torch.float32), n_cols=adj.shape[0], device=dev)
        self.adj = self.construct_adj(adj)
        return None

    def _checked_inputs(self, adj, feature, device=None):
        """The reference's checks, in its order (base_operator.py:20-30); returns the feature array
        and the device operator (None when Â was built on the host)."""
        A = self._build_operator(adj, device)
        if not isinstance(adj, sp.csr_matrix):
            raise TypeError("The adjacency matrix must be a scipy csr sparse matrix!")
        elif not isinstance(feature, np.ndarray):
            if isinstance(feature, Tensor):
                feature = feature.numpy()
            else:
                raise TypeError("The feature matrix must be a numpy.ndarray!")
        elif (adj.shape[0] if A is not None else self.adj.shape[1]) != feature.shape[0]:
            raise ValueError("Dimension mismatch detected for the adjacency and the feature matrix!")
        if self.prop_steps > 0 and feature.dtype != np.float32:
            # the reference's first hop hands the array to an ndpointer(float32) (utils.py:29-34)
            raise ctypes.ArgumentError("argument 5: TypeError: array must have data type float32")
        return feature, A

    def _operator(self, device=None):
        adj = self.adj if isinstance(self.adj, sp.csr_matrix) else sp.csr_matrix(self.adj)
        return DeviceCSR.from_scipy(adj, device=device)

    def propagate(self, adj, feature):
        feature, A = self._checked_inputs(adj, feature)
        if self.prop_steps <= 0:
            return [torch.FloatTensor(feature)]
        A = A if A is not None else self._operator()
        X = torch.from_numpy(np.ascontiguousarray(feature)).to(A.device)
        return [torch.FloatTensor(feature)] + _hops_to_host(A, X, self.prop_steps)

    def propagate_device(self, adj, feature, device=None):
        """Same as propagate() but returns device tensors (hop 0 = the feature on the device)."""
        if isinstance(feature, Tensor) and feature.is_cuda:
            A = self._build_operator(adj, feature.device)
            if not isinstance(adj, sp.csr_matrix):
                raise TypeError("The adjacency matrix must be a scipy csr sparse matrix!")
            if adj.shape[0] != feature.shape[0]:
                raise ValueError("Dimension mismatch detected for the adjacency and the feature matrix!")
            A = A if A is not None else self._operator(feature.device)
            X = feature.to(torch.float32)
        else:
            feature, A = self._checked_inputs(adj, feature, device)
            A = A if A is not None else self._operator(device)
            X = torch.from_numpy(np.ascontiguousarray(feature)).to(A.device)
        return _device_propagate(A, X, self.prop_steps)

    def propagate_aggregate(self, adj, feature, msg_op, device=None, to_host=True):
        """msg_op.aggregate(self.propagate(adj, feature)) for msg_op in last / sum / mean /
        simple_weighted, computed on the GPU without materialising the K+1 hops.  Same checks
        and errors as propagate(); learnable message ops raise ValueError (they need the list)."""
        from srgnn.aggregate import fused_combine
        if isinstance(feature, Tensor) and feature.is_cuda:
            A = self._build_operator(adj, feature.device)
            if not isinstance(adj, sp.csr_matrix):
                raise TypeError("The adjacency matrix must be a scipy csr sparse matrix!")
            if adj.shape[0] != feature.shape[0]:
                raise ValueError("Dimension mismatch detected for the adjacency and the feature matrix!")
            A = A if A is not None else self._operator(feature.device)
            X = feature.to(torch.float32).contiguous()
        else:
            feature, A = self._checked_inputs(adj, feature, device)
            A = A if A is not None else self._operator(device)
            X = torch.from_numpy(np.ascontiguousarray(feature)).to(A.device, torch.float32)
        out = fused_combine(A, X, max(self.prop_steps, 0), msg_op)
        return out.cpu() if to_host else out


# Might include training parameters
class MessageOp(nn.Module):
    def __init__(self, start=None, end=None):
        super(MessageOp, self).__init__()
        self.aggr_type = None
        self.start, self.end = start, end

    def aggr_type(self):
        return self.aggr_type

    def combine(self, feat_list):
        return NotImplementedError

    def aggregate(self, feat_list):
        if not isinstance(feat_list, list):
            return TypeError("The input must be a list consists of feature matrices!")
        for feat in feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The feature matrices must be tensors!")
        return self.combine(feat_list)


def ada_platform_one_step_propagation(adj, x):
    """One hop with host arrays (base_operator.py:309-314).  The reference takes its C kernel on
    Linux and scipy's adj.dot elsewhere; this build is gfx950/Linux only, so it is always the GPU
    SpMM (csr_sparse_dense_matmul -> libsrgnn_hip), with no CPU path to fall back to."""
    return csr_sparse_dense_matmul(adj, x)
