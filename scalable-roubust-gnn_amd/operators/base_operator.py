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
    memory holds a ring of `ring` hop panels.  Returns the K host tensors.  The hops are
    column-blocked where srgnn.spmm.auto_col_blocks says so (bitwise the one-launch hop)."""
    from srgnn.spmm import hop, prepare
    dev = A.device
    B = prepare(A, X.shape[1], K)
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
        hop(A, prev, buf, col_blocks=B)
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


# ----------------------------------------------------------------------------------------------
# The other operator families of SSRG/operators/base_operator.py:62-307 (two-order PPR
# approximation, complex / magnetic, un/in/out directed).  Their construct_adj implementations
# (subclasses in the reference's graph_operator/) need torch_scatter / torch_geometric, absent
# here; these bases take any subclass' construct_adj and run every hop on the GPU with the same
# per-hop product as the reference (bit-identical; pinned by tests/golden/fam_*.npz).
# ----------------------------------------------------------------------------------------------
def _checked_family(adjs, adj, feature, prop_steps):
    """The families' input checks, in the reference's order (base_operator.py:74-83 etc.)."""
    if not isinstance(adj, sp.csr_matrix):
        raise TypeError("The adjacency matrix must be a scipy csr sparse matrix!")
    elif not isinstance(feature, np.ndarray):
        if isinstance(feature, Tensor):
            feature = feature.numpy()
        else:
            raise TypeError("The feature matrix must be a numpy.ndarray!")
    elif any(a.shape[1] != feature.shape[0] for a in adjs):
        raise ValueError("Dimension mismatch detected for the adjacency and the feature matrix!")
    if prop_steps > 0 and feature.dtype != np.float32:
        raise ctypes.ArgumentError("argument 5: TypeError: array must have data type float32")
    return feature


def _device_op(a):
    a = a if isinstance(a, sp.csr_matrix) else sp.csr_matrix(a)
    return DeviceCSR.from_scipy(a)


class TwoOrderPprApproxGraphOp:
    """Two operators, K hops each (base_operator.py:60-93)."""

    def __init__(self, prop_steps):
        self.prop_steps = prop_steps
        self.one_adj = None
        self.two_adj = None

    def construct_adj(self, adj):
        raise NotImplementedError

    def propagate(self, adj, feature):
        self.one_adj, self.two_adj = self.construct_adj(adj)
        feature = _checked_family((self.one_adj, self.two_adj), adj, feature, self.prop_steps)
        out = []
        for a in (self.one_adj, self.two_adj):
            hops = []
            if self.prop_steps > 0:
                A = _device_op(a)
                hops = _hops_to_host(A, torch.from_numpy(np.ascontiguousarray(feature)).to(A.device), self.prop_steps)
            out.append([torch.FloatTensor(feature)] + hops)
        return out[0], out[1]


class TwoOrderPprApproxMessageOp(nn.Module):
    def __init__(self, start=None, end=None):
        super(TwoOrderPprApproxMessageOp, self).__init__()
        self.aggr_type = None
        self.start, self.end = start, end

    def aggr_type(self):
        return self.aggr_type

    def combine(self, one_feat_list, two_feat_list):
        return NotImplementedError

    def aggregate(self, one_feat_list, two_feat_list):
        if not isinstance(one_feat_list, list) or not isinstance(two_feat_list, list):
            return TypeError("The input must be a list consists of feature matrices!")
        for feat in one_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The one order feature matrices must be tensors!")
        for feat in two_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The two order feature matrices must be tensors!")
        return self.combine(one_feat_list, two_feat_list)


class calculator:
    """A term of the complex expansion (base_operator.py:124-140): value and its real / imaginary
    step counts."""

    def __init__(self, value, r_step=0, i_step=0):
        self.value = value
        self.r_step = r_step
        self.i_step = i_step

    def prop_step(self):
        return self.r_step + self.i_step

    def reversal(self):
        if self.i_step & 1 == 0 and self.i_step != 0:
            self.value = -self.value

    def set_variable(self, value, r=False, i=False):
        self.value = value
        if r:
            self.r_step += 1
        elif i:
            self.i_step += 1


def calculate_real_imag_feat(tmp_prop_feat_calculator_out_list):
    """base_operator.py:315-338, including its in-place accumulation into the FIRST real and
    imaginary terms' own value arrays (those terms carry the sums into the next step)."""
    real_feat_list = []
    imag_feat_list = []
    for k in range(len(tmp_prop_feat_calculator_out_list)):
        tmp_calculator = tmp_prop_feat_calculator_out_list[k]
        if tmp_calculator.i_step & 1 == 0 and tmp_calculator.i_step != 0:
            real_feat_list.append(tmp_calculator.value)
        elif tmp_calculator.i_step == 0:
            real_feat_list.append(tmp_calculator.value)
        else:
            imag_feat_list.append(tmp_calculator.value)
    if len(real_feat_list) != len(imag_feat_list):
        raise RuntimeError("Something wrong!")
    for k in range(len(real_feat_list)):
        if k == 0:
            real_feat = real_feat_list[k]
            imag_feat = imag_feat_list[k]
        else:
            real_feat += real_feat_list[k]           # in place, as the reference's numpy +=
            imag_feat += imag_feat_list[k]
    return real_feat, imag_feat


class ComGraphOp:
    """Complex (magnetic) propagation (base_operator.py:143-202): the 2^k-term expansion over the
    real and imaginary operators, every term's product on the GPU (device tensors play the role of
    the reference's numpy arrays, in-place accumulation included)."""

    def __init__(self, prop_steps):
        self.prop_steps = prop_steps
        self.real_adj = None
        self.imag_adj = None

    def construct_adj(self, adj):
        raise NotImplementedError

    def propagate(self, adj, feature):
        from srgnn.spmm import spmm
        self.real_adj, self.imag_adj = self.construct_adj(adj)
        feature = _checked_family((self.real_adj, self.imag_adj), adj, feature, self.prop_steps)
        if self.prop_steps <= 0:
            return [torch.FloatTensor(feature)], [torch.FloatTensor(feature)]
        Ar, Ai = _device_op(self.real_adj), _device_op(self.imag_adj)
        X = torch.from_numpy(np.ascontiguousarray(feature)).to(Ar.device)
        init_real_calculator = calculator(X)
        init_imag_calculator = calculator(X)
        real_prop_feat_list = [init_real_calculator.value]
        imag_prop_feat_list = [init_imag_calculator.value]
        tmp_in, tmp_out = [], []
        for steps in range(self.prop_steps):
            if steps == 0:
                init_real_calculator.set_variable(spmm(Ar, real_prop_feat_list[-1]), r=True)
                tmp_in.append(init_real_calculator)
                real_prop_feat_list.append(init_real_calculator.value)
                init_imag_calculator.set_variable(spmm(Ai, imag_prop_feat_list[-1]), i=True)
                tmp_in.append(init_imag_calculator)
                imag_prop_feat_list.append(init_imag_calculator.value)
            else:
                for tmp_calculator in tmp_in:
                    new_calculator = calculator(tmp_calculator.value, tmp_calculator.r_step, tmp_calculator.i_step)
                    new_calculator.set_variable(spmm(Ar, tmp_calculator.value), r=True)
                    tmp_out.append(new_calculator)
                for tmp_calculator in tmp_in:
                    new_calculator = calculator(tmp_calculator.value, tmp_calculator.r_step, tmp_calculator.i_step)
                    new_calculator.set_variable(spmm(Ai, tmp_calculator.value), i=True)
                    new_calculator.reversal()
                    tmp_out.append(new_calculator)
                real_feat, imag_feat = calculate_real_imag_feat(tmp_out)
                real_prop_feat_list.append(real_feat)
                imag_prop_feat_list.append(imag_feat)
                tmp_in, tmp_out = tmp_out, []
        host_r = [torch.FloatTensor(feature)] + [t.cpu() for t in real_prop_feat_list[1:]]
        host_i = [torch.FloatTensor(feature)] + [t.cpu() for t in imag_prop_feat_list[1:]]
        return host_r, host_i


class ComMessageOp(nn.Module):
    def __init__(self, start=None, end=None):
        super(ComMessageOp, self).__init__()
        self.aggr_type = None
        self.start, self.end = start, end

    def aggr_type(self):
        return self.aggr_type

    def combine(self, real_feat_list, imag_feat_list):
        return NotImplementedError

    def aggregate(self, real_feat_list, imag_feat_list):
        if not isinstance(real_feat_list, list) or not isinstance(imag_feat_list, list):
            return TypeError("The input must be a list consists of feature matrices!")
        for feat in real_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The real feature matrices must be tensors!")
        for feat in imag_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The imag feature matrices must be tensors!")
        return self.combine(real_feat_list, imag_feat_list)


class TwoDirGraphOp:
    """Undirected / in / out operators, K hops each (base_operator.py:226-265)."""

    def __init__(self, prop_steps):
        self.prop_steps = prop_steps
        self.un_adj = None
        self.in_adj = None
        self.out_adj = None

    def construct_adj(self, adj):
        raise NotImplementedError

    def propagate(self, adj, feature):
        self.un_adj, self.in_adj, self.out_adj = self.construct_adj(adj)
        feature = _checked_family((self.un_adj, self.in_adj, self.out_adj), adj, feature, self.prop_steps)
        out = []
        for a in (self.un_adj, self.in_adj, self.out_adj):
            hops = []
            if self.prop_steps > 0:
                A = _device_op(a)
                hops = _hops_to_host(A, torch.from_numpy(np.ascontiguousarray(feature)).to(A.device), self.prop_steps)
            out.append([torch.FloatTensor(feature)] + hops)
        return out[0], out[1], out[2]


class TwoDirMessageOp(nn.Module):
    def __init__(self, start=None, end=None):
        super(TwoDirMessageOp, self).__init__()
        self.aggr_type = None
        self.start, self.end = start, end

    def aggr_type(self):
        return self.aggr_type

    def combine(self, un_feat_list, in_feat_list, out_feat_list):
        return NotImplementedError

    def aggregate(self, un_feat_list, in_feat_list, out_feat_list):
        if not isinstance(un_feat_list, list) or not isinstance(in_feat_list, list) or not isinstance(out_feat_list, list):
            return TypeError("The input must be a list consists of feature matrices!")
        for feat in un_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The un direction feature matrices must be tensors!")
        for feat in in_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The in direction feature matrices must be tensors!")
        for feat in out_feat_list:
            if not isinstance(feat, Tensor):
                raise TypeError("The out direction feature matrices must be tensors!")
        return self.combine(un_feat_list, in_feat_list, out_feat_list)


def ada_platform_one_step_propagation(adj, x):
    """One hop with host arrays (base_operator.py:309-314).  The reference takes its C kernel on
    Linux and scipy's adj.dot elsewhere; this build is gfx950/Linux only, so it is always the GPU
    SpMM (csr_sparse_dense_matmul -> libsrgnn_hip), with no CPU path to fall back to."""
    return csr_sparse_dense_matmul(adj, x)
