"""Synthetic workload generator: numpy == torch bit for bit, determinism, graph invariants."""
import numpy as np
import torch

from srgnn import synth


def test_features_numpy_equals_torch():
    a = synth.uniform_features_np(257, 33, seed=5)
    b = synth.uniform_features_t(257, 33, seed=5).numpy()
    np.testing.assert_array_equal(a, b)
    assert a.min() >= -1.0 and a.max() < 1.0 and a.dtype == np.float32


def test_rmat_candidates_numpy_equals_torch():
    s1, d1 = synth.rmat_candidates_np(2023, 17, 5000, 14)
    s2, d2 = synth.rmat_candidates_t(2023, 17, 5000, 14)
    np.testing.assert_array_equal(s1, s2.numpy())
    np.testing.assert_array_equal(d1, d2.numpy())


def test_rmat_graph_invariants():
    n, e = 3000, 20000
    u, v = synth.rmat_undirected_t(n, e, seed=9)
    assert u.numel() == e
    assert bool((u != v).all())
    key = torch.minimum(u, v) * n + torch.maximum(u, v)
    assert torch.unique(key).numel() == e                         # each pair once
    ip, ix = synth.symmetric_csr_t(n, u, v)
    assert int(ip[-1]) == 2 * e
    rows = torch.repeat_interleave(torch.arange(n), ip[1:] - ip[:-1])
    fwd = set(zip(rows.tolist(), ix.tolist()))
    assert all((c, r) in fwd for r, c in list(fwd)[:2000])       # symmetric
    for r in range(0, n, 97):                                      # sorted rows
        seg = ix[ip[r]:ip[r + 1]]
        assert bool((seg[1:] > seg[:-1]).all())


def test_rmat_deterministic_and_skewed():
    u1, v1 = synth.rmat_undirected_t(4096, 30000, seed=1)
    u2, v2 = synth.rmat_undirected_t(4096, 30000, seed=1)
    assert torch.equal(u1, u2) and torch.equal(v1, v2)
    deg = torch.bincount(torch.cat([u1, v1]), minlength=4096)
    assert int(deg.max()) > 20 * float(deg.float().mean())      # power-law hubs present


def test_blocked_builders_equal_reference_builders():
    """The bounded-temporary builders (billion-edge configs) give the same graph and Â."""
    import torch
    from srgnn import normalize
    for n, m, batch, buckets in [(3000, 20000, 5000, 4), (20000, 90000, 1 << 14, 16), (257, 2000, 999, 3)]:
        u0, v0 = synth.rmat_undirected_t(n, m, seed=5)
        u1, v1 = synth.rmat_undirected_blocked_t(n, m, seed=5, batch=batch, buckets=buckets)
        assert torch.equal(u0, u1) and torch.equal(v0, v1)
        ip, ix = synth.symmetric_csr_t(n, u0, v0)
        ref = normalize.sym_norm_binary(ip, ix, n, 0.5)
        for blk in (1 << 12, 1 << 30):
            got = normalize.sym_norm_edges_blocked(u0.to(torch.int32), v0.to(torch.int32), n, 0.5, block_nnz=blk)
            for a, b in zip(got, ref):
                assert torch.equal(a, b)
