"""Benchmark workloads of BASELINE.json / SURVEY.md §8: synthetic power-law graphs with the
node / edge counts of the OGB graphs, normalised by construct_adj (r = 0.5), plus U[-1,1) features.
Built on the device (deterministic: the same seed gives the same graph on every rank and on CPU)."""
from __future__ import annotations

import torch

from . import synth
from .normalize import sym_norm_binary, sym_norm_edges_blocked

# above this many undirected edges the bounded-temporary builders are used (same graph)
BLOCKED_EDGES = 1 << 27


def build(config: str, device, r: float = 0.5, n=None, n_edges=None, d=None, seed=synth.RMAT_SEED,
          blocked=None):
    """Returns (indptr int64, indices int32, values fp32, n, d, K) on `device`."""
    cfg = dict(synth.CONFIGS[config]) if config in synth.CONFIGS else {}
    n = n or cfg["n"]
    n_edges = n_edges or cfg["n_edges"]
    d = d or cfg["d"]
    k = cfg.get("k", 3)
    if blocked is None:
        blocked = n_edges > BLOCKED_EDGES
    if blocked:
        u, v = synth.rmat_undirected_blocked_t(n, n_edges, seed=seed, device=device)
        if n < 2 ** 31:
            u, v = u.to(torch.int32), v.to(torch.int32)
        torch.cuda.empty_cache() if torch.device(device).type == "cuda" else None
        ip, ix, vals = sym_norm_edges_blocked(u, v, n, r)
        del u, v
    else:
        u, v = synth.rmat_undirected_t(n, n_edges, seed=seed, device=device)
        ip, ix = synth.symmetric_csr_t(n, u, v)
        del u, v
        ip, ix, vals = sym_norm_binary(ip, ix, n, r)
    torch.cuda.empty_cache() if torch.device(device).type == "cuda" else None
    return ip, ix, vals, n, d, k


def build_laplacian(config: str, device, n=None, n_edges=None, d=None, seed=synth.RMAT_SEED):
    """The wavelet basis' operator for a synthetic config: L = D - A of the same binary symmetric
    graph as build(), with every diagonal entry stored (wavelet.laplacian_from_adj's layout), fp32
    values (exact: -1 and integer degrees < 2^24).  Returns (indptr, indices, lvals, n, d, lmax)
    with lmax = 2 * max degree, the Gershgorin bound of L's spectrum (pygsp's ARPACK estimate is a
    host computation; the Chebyshev cost does not depend on it)."""
    cfg = dict(synth.CONFIGS[config]) if config in synth.CONFIGS else {}
    n = n or cfg["n"]
    n_edges = n_edges or cfg["n_edges"]
    d = d or cfg["d"]
    u, v = synth.rmat_undirected_blocked_t(n, n_edges, seed=seed, device=device)
    if n < 2 ** 31:
        u, v = u.to(torch.int32), v.to(torch.int32)
    torch.cuda.empty_cache() if torch.device(device).type == "cuda" else None
    ip, ix, lv = sym_norm_edges_blocked(u, v, n, kind="laplacian")
    del u, v
    torch.cuda.empty_cache() if torch.device(device).type == "cuda" else None
    lmax = 2.0 * float((ip[1:] - ip[:-1]).max()) if n else 0.0
    return ip, ix, lv, n, d, lmax
