"""The C-ABI communicator path (srg_comm_*, srg_dist_propagate_khop_f32: RCCL grouped send/recv of
every rank's row block, then the rank's rows on the gathered panel).  On a one-GPU box: one rank, via
srg_comm_init_all and via srg_comm_init_rank, bitwise equal to the one-GPU K-hop propagate; argument
checks.  Several ranks need a multi-GPU node (tools/comm_capi_check.py)."""
import ctypes

import numpy as np
import pytest
import torch

from srgnn import _lib

pytestmark = pytest.mark.gpu


def _graph(n=6000, e=60000, d=64, seed=3):
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.normalize import sym_norm_binary
    u, v = synth.rmat_undirected_t(n, e, seed=seed, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    X = synth.uniform_features_t(n, d, device="cuda")
    return DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda"), X


@pytest.mark.parametrize("how", ["init_all", "init_rank"])
def test_one_rank_equals_one_gpu_propagate(how):
    from srgnn.comm import Comm, unique_id
    from srgnn.spmm import propagate
    A, X = _graph()
    K = 4
    want = propagate(A, X, K)
    comm = Comm.init_all([0]) if how == "init_all" else Comm.init_rank(1, unique_id(), 0, 0)
    try:
        assert comm.size == 1
        out = comm.propagate([A], [0, A.n_rows], [X.clone()], K)
        for k in range(K + 1):
            assert torch.equal(out[0][k], want[k]), f"hop {k}"
    finally:
        comm.destroy()


def test_argument_checks():
    from srgnn.comm import Comm
    L = _lib.lib()
    starts = (ctypes.c_int64 * 2)(0, 10)
    assert L.srg_dist_propagate_khop_f32(None, None, 0, starts, 4, 4, 1) == _lib.SRG_ERR_INVALID
    A, X = _graph(n=500, e=3000, d=8)
    comm = Comm.init_all([0])
    try:
        with pytest.raises(_lib.SrgError, match="row_starts block"):
            comm.propagate([A], [0, A.n_rows - 1], [X], 2)
        with pytest.raises(_lib.SrgError, match="shards for"):
            comm.propagate([A, A], [0, A.n_rows], [X, X], 2)
    finally:
        comm.destroy()
