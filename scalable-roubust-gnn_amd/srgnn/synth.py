"""Deterministic synthetic inputs for the propagation path (SURVEY.md §8(d) "Synthetic inputs").

Everything here is driven by a counter-based hash (splitmix64 of (seed, stream, counter)), written
twice: once in numpy (uint64) and once in torch (int64 two's-complement, which wraps exactly like
uint64 for +, *, ^ and masked shifts).  The same seed therefore produces bit-identical graphs and
feature panels on the host and on the GPU, which is what lets the small parity configurations be
generated on the CPU and the bench-sized ones on the device.

Graphs are Graph500-style R-MAT (a, b, c, d) = (0.57, 0.19, 0.19, 0.05) at scale ceil(log2 N):
ids >= N and self-loops are dropped, undirected duplicates are removed keeping first occurrence,
the first `n_edges` unique edges (in generation order) are kept, node ids are relabelled by a
seeded random permutation, and the result is symmetrised.  The reference's datasets are stored the
same way before `construct_adj` adds the self-loops (SSRG/data_process.py:52-53 stores one triangle;
the models see the symmetric adjacency).
"""
from __future__ import annotations

import math

import numpy as np

try:  # torch is plumbing only; the numpy path works without it
    import torch
except ImportError:  # pragma: no cover
    torch = None

_GOLDEN = 0x9E3779B97F4A7C15
_M1 = 0xBF58476D1CE4E5B9
_M2 = 0x94D049BB133111EB
_U64 = (1 << 64) - 1

RMAT_ABCD = (0.57, 0.19, 0.19, 0.05)
RMAT_SEED = 2023       # SSRG/configs/training_config.py:7
FEATURE_SEED = 7

# ----------------------------------------------------------------------------------------------
# numpy implementation (uint64)
# ----------------------------------------------------------------------------------------------


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(_GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_M2)
        return z ^ (z >> np.uint64(31))


def _stream_key(seed: int, stream: int) -> int:
    """Python-int key for (seed, stream); identical in both implementations."""
    def sm(v):
        v = (v + _GOLDEN) & _U64
        v = ((v ^ (v >> 30)) * _M1) & _U64
        v = ((v ^ (v >> 27)) * _M2) & _U64
        return v ^ (v >> 31)
    return sm((sm(seed & _U64) + (stream & _U64)) & _U64)


def hash_np(seed: int, stream: int, counter: np.ndarray) -> np.ndarray:
    key = np.uint64(_stream_key(seed, stream))
    with np.errstate(over="ignore"):
        return splitmix64_np(np.asarray(counter, dtype=np.uint64) + key)


def uniform_features_np(n: int, d: int, seed: int = FEATURE_SEED) -> np.ndarray:
    """X ~ U[-1, 1) fp32, row-major n x d; each value = top 24 hash bits * 2^-23 - 1 (exact)."""
    h = hash_np(seed, 1, np.arange(n * d, dtype=np.uint64))
    u = (h >> np.uint64(40)).astype(np.int64)
    return (u.astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1.0)).reshape(n, d)


def binary_rownorm_features_np(n: int, d: int, per_row: int = 18, seed: int = FEATURE_SEED):
    """Planetoid-like bag-of-words features: `per_row` ones per row (collisions merge), then
    row-normalised (SSRG/sparsity_datasets/simhomo/planetoid.py:99-107 normalises feature rows).
    Row sums are computed in fp32 left to right; empty rows stay zero.
    Returns a dense fp32 n x d array."""
    cols = (hash_np(seed, 2, np.arange(n * per_row, dtype=np.uint64)) % np.uint64(d)).astype(np.int64)
    X = np.zeros((n, d), dtype=np.float32)
    rows = np.repeat(np.arange(n), per_row)
    X[rows, cols] = 1.0
    s = X.sum(axis=1, dtype=np.float32)
    s[s == 0] = 1.0
    return (X / s[:, None]).astype(np.float32)


def _rmat_thresholds(abcd=RMAT_ABCD):
    a, b, c, _ = abcd
    t = [int(round(a * (1 << 24))), int(round((a + b) * (1 << 24))), int(round((a + b + c) * (1 << 24)))]
    return t


def rmat_candidates_np(seed: int, first: int, count: int, scale: int, abcd=RMAT_ABCD):
    """Candidate directed edges [first, first+count) of the R-MAT stream (before filtering)."""
    t0, t1, t2 = _rmat_thresholds(abcd)
    e = np.arange(first, first + count, dtype=np.uint64)
    src = np.zeros(count, dtype=np.int64)
    dst = np.zeros(count, dtype=np.int64)
    for lvl in range(scale):
        # counter = edge * 64 + level  (scale <= 40 always fits)
        h = hash_np(seed, 3, e * np.uint64(64) + np.uint64(lvl))
        p = (h >> np.uint64(40)).astype(np.int64)
        sbit = (p >= t1).astype(np.int64)                    # quadrants c, d -> src bit 1
        dbit = (((p >= t0) & (p < t1)) | (p >= t2)).astype(np.int64)   # quadrants b, d
        src = (src << 1) | sbit
        dst = (dst << 1) | dbit
    return src, dst


# ----------------------------------------------------------------------------------------------
# torch implementation (int64, any device) -- bit-identical to the numpy one
# ----------------------------------------------------------------------------------------------


def _to_i64(v: int) -> int:
    v &= _U64
    return v - (1 << 64) if v >= (1 << 63) else v


def _srl(x, s: int):
    """Logical right shift of int64 tensor viewed as uint64."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def splitmix64_t(x):
    z = x + _to_i64(_GOLDEN)
    z = (z ^ _srl(z, 30)) * _to_i64(_M1)
    z = (z ^ _srl(z, 27)) * _to_i64(_M2)
    return z ^ _srl(z, 31)


def hash_t(seed: int, stream: int, counter):
    return splitmix64_t(counter + _to_i64(_stream_key(seed, stream)))


def uniform_features_t(n: int, d: int, seed: int = FEATURE_SEED, device="cpu", chunk: int = 1 << 26):
    out = torch.empty(n * d, dtype=torch.float32, device=device)
    for s in range(0, n * d, chunk):
        e = min(n * d, s + chunk)
        c = torch.arange(s, e, dtype=torch.int64, device=device)
        u = _srl(hash_t(seed, 1, c), 40)
        out[s:e] = u.to(torch.float32) * (2.0 ** -23) - 1.0
    return out.view(n, d)


def rmat_candidates_t(seed: int, first: int, count: int, scale: int, abcd=RMAT_ABCD, device="cpu"):
    t0, t1, t2 = _rmat_thresholds(abcd)
    e = torch.arange(first, first + count, dtype=torch.int64, device=device) * 64
    src = torch.zeros(count, dtype=torch.int64, device=device)
    dst = torch.zeros(count, dtype=torch.int64, device=device)
    for lvl in range(scale):
        p = _srl(hash_t(seed, 3, e + lvl), 40)
        sbit = (p >= t1).to(torch.int64)
        dbit = (((p >= t0) & (p < t1)) | (p >= t2)).to(torch.int64)
        src = (src << 1) | sbit
        dst = (dst << 1) | dbit
    return src, dst


def rmat_undirected_t(n: int, n_edges: int, seed: int = RMAT_SEED, device="cpu", abcd=RMAT_ABCD,
                      batch: int | None = None):
    """First `n_edges` unique undirected edges (u < v after relabelling is NOT implied) of the
    filtered R-MAT stream, relabelled by a seeded permutation.  Returns (u, v) int64 tensors with
    u != v, each unordered pair once."""
    scale = max(1, math.ceil(math.log2(max(n, 2))))
    keys = torch.empty(0, dtype=torch.int64, device=device)
    firstpos = torch.empty(0, dtype=torch.int64, device=device)
    produced = 0
    if batch is None:
        batch = max(1024, int(n_edges * 1.35))
    while True:
        s, d = rmat_candidates_t(seed, produced, batch, scale, abcd, device)
        ok = (s < n) & (d < n) & (s != d)
        lo = torch.minimum(s, d)[ok]
        hi = torch.maximum(s, d)[ok]
        pos = torch.arange(produced, produced + batch, dtype=torch.int64, device=device)[ok]
        produced += batch
        k = torch.cat([keys, lo * n + hi])
        p = torch.cat([firstpos, pos])
        uk, inv = torch.unique(k, sorted=True, return_inverse=True)
        fp = torch.full((uk.numel(),), produced, dtype=torch.int64, device=device)
        fp = fp.scatter_reduce(0, inv, p, reduce="amin", include_self=True)
        keys, firstpos = uk, fp
        if keys.numel() >= n_edges:
            break
        batch = max(1024, int((n_edges - keys.numel()) * 1.6) + 1024)
    order = torch.argsort(firstpos)[:n_edges]
    sel = keys[order]
    lo, hi = sel // n, sel % n
    perm = relabel_permutation_t(n, seed, device)
    return perm[lo], perm[hi]


def nonzero_chunked(mask, chunk: int = 1 << 30):
    """torch.nonzero(mask) of a 1-D bool tensor in < 2^31-element pieces (ascending positions)."""
    parts = [torch.nonzero(mask[i:i + chunk]).squeeze(1) + i for i in range(0, mask.numel(), chunk)]
    if not parts:
        return torch.empty(0, dtype=torch.int64, device=mask.device)
    return parts[0] if len(parts) == 1 else torch.cat(parts)


def _first_occurrence(keys, buckets: int):
    """Bool mask, True where keys[i] is the first occurrence of its value.  Keys are split into
    hash buckets (equal keys share one) so that no sort exceeds ~numel/buckets elements."""
    first = torch.zeros(keys.numel(), dtype=torch.bool, device=keys.device)
    bits = max(1, (buckets - 1).bit_length())
    shift = 64 - bits
    for b in range(1 << bits):
        h = _srl(keys * _to_i64(_GOLDEN), shift)
        idx = nonzero_chunked(h == b)
        del h
        if idx.numel() == 0:
            continue
        k = keys[idx]
        sk, perm = torch.sort(k, stable=True)
        del k
        newrun = torch.ones(sk.numel(), dtype=torch.bool, device=keys.device)
        newrun[1:] = sk[1:] != sk[:-1]
        first[idx[perm[newrun]]] = True
    return first


def rmat_undirected_blocked_t(n: int, n_edges: int, seed: int = RMAT_SEED, device="cpu", abcd=RMAT_ABCD,
                              batch: int = 1 << 27, buckets: int = 64):
    """The same edge list as rmat_undirected_t (first `n_edges` unique undirected edges of the
    stream, relabelled), built with bounded temporaries for billion-edge graphs: candidates in
    batches, duplicates found per hash bucket, no sort larger than ~1/buckets of the stream."""
    scale = max(1, math.ceil(math.log2(max(n, 2))))
    chunks, produced = [], 0
    target = max(1024, int(n_edges * 1.35))
    while True:
        while produced < target:
            b = min(batch, target - produced)
            s, d = rmat_candidates_t(seed, produced, b, scale, abcd, device)
            ok = (s < n) & (d < n) & (s != d)
            chunks.append((torch.minimum(s, d) * n + torch.maximum(s, d))[ok])
            del s, d, ok
            produced += b
        keys = chunks[0] if len(chunks) == 1 else torch.cat(chunks)
        chunks = [keys]
        first = _first_occurrence(keys, buckets)
        cnt = int(first.sum())
        if cnt >= n_edges:
            break
        del first
        target = produced + max(1024, int((n_edges - cnt) * 1.6) + 1024)
    pos = nonzero_chunked(first)[:n_edges]
    del first
    sel = keys[pos]
    del keys, chunks, pos
    perm = relabel_permutation_t(n, seed, device)
    return perm[sel // n], perm[sel % n]


def relabel_permutation_t(n: int, seed: int, device="cpu"):
    """new_id[old_id]: rank of hash(seed, 4, old_id) (ties broken by id; stable sort)."""
    h = hash_t(seed, 4, torch.arange(n, dtype=torch.int64, device=device))
    h = _srl(h, 1)  # non-negative, order-preserving within the top 63 bits
    order = torch.sort(h, stable=True).indices
    new_id = torch.empty(n, dtype=torch.int64, device=device)
    new_id[order] = torch.arange(n, dtype=torch.int64, device=device)
    return new_id


def symmetric_csr_t(n: int, u, v, device=None):
    """Symmetric binary adjacency (no self-loops) as CSR (indptr int64, indices int32), sorted."""
    device = device or u.device
    rows = torch.cat([u, v])
    cols = torch.cat([v, u])
    key = torch.sort(rows * n + cols).values
    rows = key // n
    cols = (key % n).to(torch.int32)
    counts = torch.bincount(rows, minlength=n)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr, cols


# Shapes from SURVEY.md §8 header (E_undirected from sparsity_dataset.py:24-33 for the OGB graphs).
CONFIGS = {
    "arxiv": dict(n=169_343, n_edges=1_157_799, d=128, k=5),
    "products": dict(n=2_449_029, n_edges=61_859_012, d=128, k=10),
    "papers100M": dict(n=111_059_956, n_edges=1_615_685_872, d=128, k=5),
    "rmat26": dict(n=1 << 26, n_edges=1 << 30, d=256, k=8),
}
