"""HIP kernels vs the reference (golden fixtures) and vs the CPU oracle.  Run on the MI355X box.

Bar: exact mode is BIT-IDENTICAL to the reference's FloatCSRMulDenseOMP (one fp32 fma chain per
output element in CSR order), so hops are compared by SHA-256 of their bytes.  Each case runs
through every path of the kernel: row waves only, column-slice waves for every row, hub workgroups
(LDS producer/consumer) for every row, the default split, and a mixed three-way split.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import golden_cases as G

pytestmark = pytest.mark.gpu

# (heavy_threshold, hub_threshold)
THRESHOLDS = [(-1, -1), (0, -1), (0, 0), (None, None), (4, 64)]


def _csr(c, thr):
    from srgnn.csr import DeviceCSR
    ip, ix, v = c.ahat()
    heavy, hub = thr if isinstance(thr, tuple) else (thr, None)
    return DeviceCSR.from_tensors(ip, ix, v, n_cols=c.n, heavy_threshold=heavy, hub_threshold=hub,
                                  device="cuda")


@pytest.mark.parametrize("thr", THRESHOLDS)
@pytest.mark.parametrize("name", G.names("norm"))
def test_khop_bit_exact_vs_reference(name, thr):
    from srgnn.spmm import propagate
    c = G.Case(name)
    A = _csr(c, thr)
    X = torch.from_numpy(c.x()).cuda()
    hops = propagate(A, X, c.k)
    torch.cuda.synchronize()
    assert hops[0] is X
    for k in range(1, c.k + 1):
        c.check_hop(k, hops[k].cpu().numpy())


@pytest.mark.parametrize("thr", THRESHOLDS)
@pytest.mark.parametrize("name", G.names("raw"))
def test_one_hop_raw_bit_exact(name, thr):
    """Unsorted rows, duplicate entries and F-order inputs: the chain follows STORED order."""
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    c = G.Case(name)
    a = c.adj()
    A = DeviceCSR.from_tensors(a.indptr, a.indices, a.data.astype(np.float32), n_cols=c.n,
                               heavy_threshold=thr[0], hub_threshold=thr[1], device="cuda")
    y = spmm(A, torch.from_numpy(c.x()).cuda())
    c.check_hop(1, y.cpu().numpy())


@pytest.mark.parametrize("name", G.names("raw") + ["rand_d7_r03", "rand_d130_r1"])
def test_drop_in_host_entry_bit_exact(name):
    """operators.utils.csr_sparse_dense_matmul -> libsrgnn_hip FloatCSRMulDenseOMP (host buffers)."""
    from operators.utils import csr_sparse_dense_matmul
    c = G.Case(name)
    if c.meta["op"] == "raw_spmm":
        adj, x = c.adj(), c.x()
        c.check_hop(1, csr_sparse_dense_matmul(adj, x))
    else:
        ip, ix, v = c.ahat()
        adj = sp.csr_matrix((v, ix, ip.astype(np.int32)), shape=(c.n, c.n))
        h = c.x()
        for k in range(1, c.k + 1):
            h = csr_sparse_dense_matmul(adj, h)
            c.check_hop(k, h)


def test_cuda_compat_entry_overwrites():
    from operators.utils import cuda_csr_sparse_dense_matmul
    c = G.Case("raw_dups_d128")
    c.check_hop(1, cuda_csr_sparse_dense_matmul(c.adj(), c.x()))


@pytest.mark.parametrize("name", ["cora_sym_k3", "cora_asstored_k3", "rand_d36_ppr", "rand_d1_r05"])
def test_graphop_propagate_end_to_end(name):
    """The reference API (operators.graph_operator.*) end to end: construct_adj + K hops + list."""
    from operators.graph_operator.symmetrical_simgraph_laplacian_operator import SymLaplacianGraphOp
    from operators.graph_operator.symmetrical_simgraph_ppr_operator import PprGraphOp
    c = G.Case(name)
    op = (PprGraphOp(c.k, r=c.meta["r"], alpha=c.meta["alpha"]) if c.meta["op"] == "ppr"
          else SymLaplacianGraphOp(c.k, r=c.meta["r"]))
    x = c.x()
    out = op.propagate(c.adj(), x)
    assert len(out) == c.k + 1 and all(isinstance(t, torch.Tensor) and t.dtype == torch.float32 for t in out)
    np.testing.assert_array_equal(out[0].numpy(), x)
    np.testing.assert_array_equal(op.adj.data, c["ahat_data64"])
    for k in range(1, c.k + 1):
        c.check_hop(k, out[k].numpy())
    dev = op.propagate_device(c.adj(), torch.from_numpy(x).cuda())
    for k in range(1, c.k + 1):
        c.check_hop(k, dev[k].cpu().numpy())


def test_graphop_error_behaviour_matches_reference():
    import ctypes
    from operators.graph_operator.symmetrical_simgraph_laplacian_operator import SymLaplacianGraphOp
    from operators.graph_operator.symmetrical_simgraph_ppr_operator import PprGraphOp
    errs = G.manifest()["_errors"]
    c = G.Case("rand_d7_r03")
    adj, x = c.adj(), c.x()

    def outcome(fn):
        try:
            fn()
            return "ok"
        except ctypes.ArgumentError:
            return "ArgumentError"
        except Exception as e:  # noqa: BLE001
            return type(e).__name__

    got = {
        "coo_adj": outcome(lambda: SymLaplacianGraphOp(2).propagate(adj.tocoo(), x)),
        "float64_feature": outcome(lambda: SymLaplacianGraphOp(2).propagate(adj, x.astype(np.float64))),
        "dim_mismatch": outcome(lambda: SymLaplacianGraphOp(2).propagate(adj, x[:-1])),
        "list_feature": outcome(lambda: SymLaplacianGraphOp(2).propagate(adj, x.tolist())),
        "tensor_feature": outcome(lambda: SymLaplacianGraphOp(2).propagate(adj, torch.from_numpy(x))),
        "ppr_dense_adj": outcome(lambda: PprGraphOp(2).propagate(adj.toarray(), x)),
        "k0": outcome(lambda: SymLaplacianGraphOp(0).propagate(adj, x)),
    }
    assert got == errs


def test_accumulate_and_nt_store_flags(oracle_mod):
    from srgnn.spmm import spmm
    c = G.Case("rand_d128_r05")
    A = _csr(c, None)
    x = c.x()
    X = torch.from_numpy(x).cuda()
    y0 = np.random.default_rng(0).standard_normal((c.n, x.shape[1])).astype(np.float32)
    Y = torch.from_numpy(y0.copy()).cuda()
    spmm(A, X, out=Y, accumulate=True)
    ref = oracle_mod.spmm(*c.ahat(), x, out=y0.copy(), accumulate=True)
    np.testing.assert_array_equal(Y.cpu().numpy(), ref)
    Z = spmm(A, X, nt_store=True)
    np.testing.assert_array_equal(Z.cpu().numpy(), oracle_mod.spmm(*c.ahat(), x))
    # accumulate through the hub and slice paths too
    for thr in ((0, 0), (0, -1)):
        Ah = _csr(c, thr)
        Y = torch.from_numpy(y0.copy()).cuda()
        spmm(Ah, X, out=Y, accumulate=True)
        np.testing.assert_array_equal(Y.cpu().numpy(), ref, err_msg=str(thr))


@pytest.mark.parametrize("thr", THRESHOLDS)
@pytest.mark.parametrize("name", ["rand_d128_r05", "cora_sym_k3", "rand_d7_r03"])
def test_column_blocked_chain_continuation(name, thr):
    """ACCUMULATE continues a row's fma chain from the stored fp32 value: Â's columns are sorted
    (utils.py:81-93), so running the entries of B column blocks in ascending order (block 0 from
    +0.0f, the rest with ACCUMULATE) is bitwise the one-pass hop and so the reference's product
    (tools/colblock_probe.py measures this form at full size)."""
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    c = G.Case(name)
    ip, ix, v = (np.asarray(a) for a in c.ahat())
    assert all(np.all(np.diff(ix[ip[i]:ip[i + 1]]) > 0) for i in range(c.n))
    X = torch.from_numpy(c.x()).cuda()
    heavy, hub = thr
    row = np.repeat(np.arange(c.n), np.diff(ip))
    for B in (2, 3, 7):
        blk = (ix.astype(np.int64) * B) // c.n
        Y = torch.empty_like(X)
        for b in range(B):
            m = blk == b
            bip = np.concatenate([[0], np.cumsum(np.bincount(row[m], minlength=c.n))])
            Ab = DeviceCSR.from_tensors(bip, ix[m], v[m], n_cols=c.n, heavy_threshold=heavy,
                                        hub_threshold=hub, device="cuda")
            spmm(Ab, X, out=Y, accumulate=b > 0)
        torch.cuda.synchronize()
        c.check_hop(1, Y.cpu().numpy())


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("B,whole_max", [(2, 0), (2, 8), (3, 0), (3, 8), (5, 0), (5, 8), (4, 0), (4, 32)])
@pytest.mark.parametrize("name", G.names("norm"))
def test_propagate_column_blocked_bit_exact(name, B, compact, whole_max):
    """Column-blocked hops through the library's plan loop (srg_propagate_plan_f32: span launches,
    ACCUMULATE, slot spans, the hub chain) over layouts the planner itself does not pick -- every row
    cut (whole_max 0) or short rows whole up to 8 / 32 entries, spans or compact copies; built by the
    test restatement tests/plan_layout_ref.py -- and the product path's own plan for B blocks
    (propagate(col_blocks=B), hop(col_blocks=B)): the reference's hops, bit for bit."""
    import plan_layout_ref as R
    from srgnn.spmm import hop, propagate
    c = G.Case(name)
    A = _csr(c, (None, None))
    blocks = (R.compact_column_blocks if compact else R.column_blocks)(A, B, whole_max)
    assert blocks is not None and len(blocks) == B and sum(b.nnz for b in blocks) == A.nnz
    assert all(b.is_span for b in blocks)
    # compact blocks hold copies of their entries (laid out in launch order), spans share A's arrays
    assert all((b.indices.data_ptr() != A.indices.data_ptr()) == compact for b in blocks)
    X = torch.from_numpy(c.x()).cuda()
    for hops in (R.propagate(A, X, c.k, B, compact=compact, split=True, whole_max=whole_max),
                 R.propagate(A, X, c.k, B, compact=compact, split=False, whole_max=whole_max),
                 propagate(A, X, c.k, col_blocks=B)):
        torch.cuda.synchronize()
        for k in range(1, c.k + 1):
            c.check_hop(k, hops[k].cpu().numpy())
    one = hop(A, X, torch.empty_like(X), col_blocks=B)
    c.check_hop(1, one.cpu().numpy())


@pytest.mark.parametrize("name", ["rand_d128_r05", "rand_d36_ppr", "cora_sym_k3"])
def test_block0_split_launches_bit_exact(monkeypatch, name):
    """Block 0 of a column-blocked hop as two launches (its cut spans, then its whole rows; the
    default below 16 GiB panels) or one (spmm.SPLIT_BLOCK0 = False): the same bits as the reference
    either way, and launches_per_hop counts B + 1 or B launches."""
    from srgnn import spmm as spmm_mod
    c = G.Case(name)
    X = torch.from_numpy(c.x()).cuda()
    d = X.shape[1]
    for split in (True, False):
        monkeypatch.setattr(spmm_mod, "SPLIT_BLOCK0", split)
        A = _csr(c, (None, None))
        assert spmm_mod.launches_per_hop(A, 4, d) == (5 if split else 4)
        hops = spmm_mod.propagate(A, X, c.k, col_blocks=4)
        torch.cuda.synchronize()
        assert spmm_mod.launches_per_hop(A, 4, d) == (5 if split else 4)
        for k in range(1, c.k + 1):
            c.check_hop(k, hops[k].cpu().numpy())
    monkeypatch.setattr(spmm_mod, "SPLIT_BLOCK0", None)
    A = _csr(c, (None, None))
    assert spmm_mod.launches_per_hop(A, 1, d) == 1
    assert spmm_mod.launches_per_hop(A, 4, d) == 5        # "auto": a small panel is split


@pytest.mark.parametrize("name", G.names("raw"))
def test_column_blocks_exact_for_unordered_rows(name):
    """Column blocks are spans of each row (one binary search per row and boundary), and the split
    points of any row -- sorted or not -- lie in the row and never decrease, so the spans partition it
    in CSR order: the blocked hop is the one-launch hop bit for bit even where the ids are unsorted
    (those rows only lose the blocks' locality)."""
    import plan_layout_ref as R
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import hop
    c = G.Case(name)
    a = c.adj()
    ip, ix = np.asarray(a.indptr), np.asarray(a.indices)
    A = DeviceCSR.from_tensors(ip, ix, a.data.astype(np.float32), n_cols=c.n, device="cuda")
    X = torch.from_numpy(c.x()).cuda()
    want = hop(A, X, torch.empty((c.n, X.shape[1]), device="cuda"), col_blocks=1).cpu().numpy()
    assert A.n_rows == A.n_cols
    for B in (2, 3):
        blocks = R.column_blocks(A, B)
        assert blocks is not None and sum(b.nnz for b in blocks) == A.nnz
        for Y in (hop(A, X, torch.empty((c.n, X.shape[1]), device="cuda"), col_blocks=B),
                  R.propagate(A, X, 1, B, split=True)[1], R.propagate(A, X, 1, B, compact=True)[1]):
            np.testing.assert_array_equal(Y.cpu().numpy(), want)
    c.check_hop(1, want)


@pytest.mark.parametrize("whole_max", [0, 16])
def test_column_block_spans_are_lower_bounds(whole_max):
    """srg_csr_col_splits on a host-checkable CSR: for sorted rows each split is the first entry
    whose id reaches ceil(b n / B); every split lies in its row and is monotone in b (any row).
    Rows of <= whole_max entries end in block 0 (every later split at the row's end)."""
    import plan_layout_ref as R
    from srgnn.csr import DeviceCSR
    rng = np.random.default_rng(5)
    n, deg = 997, rng.integers(0, 40, 997)
    deg[3], deg[10] = 3000, 0
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.integers(0, n, k)) for k in deg]).astype(np.int32)
    shuffled = ix.copy()
    shuffled[ip[5]:ip[6]] = shuffled[ip[5]:ip[6]][::-1]
    for ids, sorted_rows in ((ix, True), (shuffled, False)):
        # an explicit hub threshold: the 3000-entry row stays a cut row (automatic hub rows this long would
        # be whole hub rows, cut nowhere)
        A = DeviceCSR.from_tensors(ip, ids, np.ones(ids.size, np.float32), n_cols=n, hub_threshold=100000,
                                   device="cuda")
        for B in (2, 3, 7):
            blocks = R.column_blocks(A, B, whole_max)
            starts = [b.indptr.cpu().numpy() for b in blocks] + [blocks[-1].row_end.cpu().numpy()]
            assert np.array_equal(starts[0], ip[:-1]) and np.array_equal(starts[-1], ip[1:])
            for b in range(1, B):
                assert np.all(starts[b] >= starts[b - 1])
                assert np.array_equal(blocks[b - 1].row_end.cpu().numpy(), starts[b])
                short = np.diff(ip) <= whole_max
                assert np.array_equal(starts[b][short], ip[1:][short])
                if sorted_rows:
                    bound = -(-b * n // B)
                    want = np.array([ip[r] + np.searchsorted(ids[ip[r]:ip[r + 1]], bound) for r in range(n)])
                    assert np.array_equal(starts[b][~short], want[~short])


def test_strided_panels_and_row_blocks(oracle_mod):
    """Leading dimensions > d and a row block with rebased indptr (the multi-GPU layout)."""
    from srgnn.spmm import spmm
    c = G.Case("rand_d128_r05")
    A = _csr(c, None)
    x = c.x()
    big = torch.zeros((c.n, 160), device="cuda")
    big[:, :128] = torch.from_numpy(x).cuda()
    out = torch.full((c.n, 136), 7.0, device="cuda")
    spmm(A, big[:, :128], out=out[:, :128])
    want = oracle_mod.spmm(*c.ahat(), x)
    np.testing.assert_array_equal(out[:, :128].cpu().numpy(), want)
    assert bool((out[:, 128:] == 7.0).all())
    blk = A.rows(50, 140)
    yb = spmm(blk, torch.from_numpy(x).cuda())
    np.testing.assert_array_equal(yb.cpu().numpy(), want[50:140])
    hub_blk = A.rows(50, 140, heavy_threshold=2, hub_threshold=5)
    assert hub_blk.n_hub > 0
    yh = spmm(hub_blk, torch.from_numpy(x).cuda())
    np.testing.assert_array_equal(yh.cpu().numpy(), want[50:140])


def test_edge_cases_empty_and_special_values(oracle_mod):
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    # all-empty matrix
    A = DeviceCSR.from_tensors(np.zeros(6, np.int64), np.zeros(0, np.int32), np.zeros(0, np.float32),
                               n_cols=5, device="cuda")
    y = spmm(A, torch.ones((5, 64), device="cuda"))
    assert bool((y == 0).all())
    # -0.0, inf and nan propagate exactly as the fma chain does
    ip = np.array([0, 2, 3, 5], np.int64)
    ix = np.array([0, 1, 2, 0, 2], np.int32)
    v = np.array([1.0, -1.0, 2.0, -0.0, 1.0], np.float32)
    x = np.zeros((3, 128), np.float32)
    x[0, 0], x[1, 0], x[2, 1], x[2, 2] = -0.0, 0.0, np.inf, np.nan
    x[0, 3] = -0.0
    A = DeviceCSR.from_tensors(ip, ix, v, n_cols=3, device="cuda")
    got = spmm(A, torch.from_numpy(x).cuda()).cpu().numpy()
    want = oracle_mod.spmm(ip, ix, v, x)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_validate_rejects_bad_ids():
    from srgnn import SrgError
    from srgnn.csr import DeviceCSR
    with pytest.raises(SrgError):
        DeviceCSR.from_tensors(np.array([0, 2], np.int64), np.array([0, 9], np.int32),
                               np.ones(2, np.float32), n_cols=3, device="cuda")
    with pytest.raises(SrgError):
        DeviceCSR.from_tensors(np.array([0, 3, 2], np.int64), np.array([0, 1, 2], np.int32),
                               np.ones(3, np.float32), n_cols=3, device="cuda")


@pytest.mark.parametrize("d", [1, 4, 36, 64, 96, 128, 200, 256, 512])
def test_rmat_many_widths_bit_exact(oracle_mod, d):
    """Power-law R-MAT graph (hubs, empty rows) at assorted widths, both wave roles."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    n = 6000
    u, v = synth.rmat_undirected_t(n, 40000, seed=3)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = synth.uniform_features_np(1, int(ix.numel()), seed=99)[0] * 0.5 + 0.5
    x = synth.uniform_features_np(n, d, seed=4)
    want = oracle_mod.spmm(ip.numpy(), ix.numpy(), vals, x)
    for thr in ((-1, -1), (0, -1), (16, -1), (0, 0), (16, 300)):
        A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=thr[0], hub_threshold=thr[1],
                                   device="cuda")
        got = spmm(A, torch.from_numpy(x).cuda()).cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg=f"d={d} thr={thr}")


@pytest.mark.parametrize("world", [2, 3, 8])
def test_row_partitioned_virtual_ranks_bitwise(world):
    """The multi-GPU layout (nnz-balanced row blocks, remapped ids, padded gathered panel) on one
    device: bitwise equal to the single-device propagation."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.dist import simulate_propagate
    from srgnn.normalize import sym_norm_binary
    from srgnn.spmm import propagate
    n = 20000
    u, v = synth.rmat_undirected_t(n, 150000, seed=21, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 128, device="cuda")
    want = propagate(DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda"), x, 3)
    got = simulate_propagate(ip, ix, vals, n, x, 3, world, device="cuda")
    for k in range(1, 4):
        assert torch.equal(got[k], want[k]), f"hop {k} differs with {world} virtual ranks"


def test_products_scale_sampled_rows_bit_exact(oracle_mod):
    """Full products-shaped graph (126 M nonzeros): each hop checked bit for bit on 3000 sampled
    rows (plus every heavy row's first slice owner) against the oracle fed with the GPU's previous
    hop -- a size-independent check of every launch."""
    from srgnn import graphs, synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import propagate
    ip, ix, vals, n, d, _ = graphs.build("products", "cuda")
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda", hub_threshold=4096)
    assert A.n_hub > 0 and A.n_heavy > 0
    x = synth.uniform_features_t(n, d, device="cuda")
    hops = propagate(A, x, 2)
    ipn, ixn, vn = ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy()
    deg = np.diff(ipn)
    rng = np.random.default_rng(5)
    rows = np.unique(np.r_[rng.choice(n, 3000, replace=False), np.argsort(-deg)[:50]])
    sub_ptr = np.r_[0, np.cumsum(deg[rows])]
    sub_ix = np.concatenate([ixn[ipn[r]:ipn[r + 1]] for r in rows])
    sub_v = np.concatenate([vn[ipn[r]:ipn[r + 1]] for r in rows])
    for k in (1, 2):
        prev = hops[k - 1].cpu().numpy()
        want = oracle_mod.spmm(sub_ptr, sub_ix, sub_v, prev)
        got = hops[k][torch.from_numpy(rows).cuda()].cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg=f"hop {k}")
    # size-independent property: Â is symmetric-normalised with r = 0.5 -> Â 1-vector scaled by
    # D^(1/2) is an eigenvector with eigenvalue 1: Â (D^(1/2) 1) = D^(1/2) 1 (up to rounding)
    # every term is positive, so the sequential fp32 chain of row i is within (deg_i + 8) * 2^-24
    # relative of the exact value (deg_i roundings of the sum, ~3 per term, 1 for the reference)
    dh = torch.from_numpy(np.sqrt(deg.astype(np.float64)).astype(np.float32)).cuda()
    y = propagate(A, dh.view(-1, 1).expand(n, 4).contiguous(), 1)[1]
    rel = ((y[:, 0].double() - dh.double()).abs() / dh.double())
    bound = (torch.from_numpy(deg).cuda().double() + 8) * 2.0 ** -24
    assert bool((rel <= bound).all()), float((rel / bound).max())
    assert bool((y[:, 1:] == y[:, :1]).all())


@pytest.mark.parametrize("world,chunks,ghost,cb", [(2, 3, None, None), (8, 4, None, None), (2, 3, 0, None),
                                                  (4, 2, 64, None), (8, 3, 8, None), (2, 3, None, 2),
                                                  (8, 4, None, 3), (4, 2, 64, 4), (8, 4, None, 2)])
def test_halo_virtual_ranks_bitwise(world, chunks, ghost, cb):
    """The halo-exchange multi-GPU layout (groups, remapped columns, hub group, ghost rows
    computed into the halo, the row chunks' column blocks split by GLOBAL column ids) on one
    device with the real kernels: bitwise equal to the single-device propagation."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.dist import simulate_halo_propagate
    from srgnn.normalize import sym_norm_binary
    from srgnn.spmm import propagate
    n = 20000
    u, v = synth.rmat_undirected_t(n, 150000, seed=22, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 128, device="cuda")
    want = propagate(DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda"), x, 3)
    got = simulate_halo_propagate(ip, ix, vals, n, x, 3, world, chunks=chunks, hub_threshold=300,
                                  device="cuda", ghost_max_degree=ghost, col_blocks=cb)
    for k in range(1, 4):
        assert torch.equal(got[k], want[k]), f"hop {k} differs with {world} virtual halo ranks"


def test_launch_chunking_beyond_2e32_lanes(oracle_mod):
    """More rows than one dispatch can hold (2^25 + rows -> > 2^31 lanes at 64 per row, chunked
    launches with a block base): every row of a banded CSR checked, for the SpMM and Chebyshev."""
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    n, d = (1 << 25) + 4099, 4
    r = torch.arange(n, device="cuda", dtype=torch.int64)
    # row i: columns i and (i + 7) mod n -> indptr 2i, stored sorted
    c0, c1 = r, (r + 7) % n
    cols = torch.stack([torch.minimum(c0, c1), torch.maximum(c0, c1)], 1).reshape(-1).to(torch.int32)
    ip = torch.arange(0, 2 * n + 1, 2, device="cuda", dtype=torch.int64)
    vals = ((r % 13).to(torch.float32) * 0.25 - 1.0).repeat_interleave(2)
    vals[1::2] = 0.5
    A = DeviceCSR.from_tensors(ip, cols, vals, n_cols=n, device="cuda", heavy_threshold=-1, hub_threshold=-1)
    X = (torch.arange(n * d, device="cuda", dtype=torch.int64) % 1021).to(torch.float32).view(n, d) * 0.125
    Y = spmm(A, X)
    a0 = vals[0::2].view(n, 1)
    x0 = X[cols[0::2].long()]
    x1 = X[cols[1::2].long()]
    want = torch.addcmul(torch.zeros_like(Y), a0, x0)       # 0 + a*x, then fma with 0.5*x1 (exact)
    want = want + 0.5 * x1
    assert torch.equal(Y, want)


@pytest.mark.parametrize("name", G.names("norm"))
def test_device_construct_adj_bit_exact(name):
    """construct_adj on the GPU (srgnn.construct: sorts, sequential fp64 segment sums, host
    np.power) == the reference's scipy Â stored in the fixture, bit for bit (fp64 values)."""
    from srgnn import construct as C
    c = G.Case(name)
    a = c.adj()
    if c.meta["op"] == "ppr":
        ip, ix, v = C.ppr_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"], c.meta["alpha"], device="cuda")
    else:
        ip, ix, v = C.sym_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"], device="cuda")
    np.testing.assert_array_equal(ip.cpu().numpy(), c["ahat_indptr"])
    np.testing.assert_array_equal(ix.cpu().numpy(), c["ahat_indices"])
    np.testing.assert_array_equal(v.cpu().numpy(), c["ahat_data64"])


def test_device_construct_weighted_duplicates_equal_oracle(oracle_mod):
    from srgnn import construct as C
    rng = np.random.default_rng(4)
    n, m = 5000, 60000
    r, c = rng.integers(0, n, m), rng.integers(0, n, m)
    v = rng.random(m) * 3
    order = np.lexsort((rng.random(m), r))
    r, c, v = r[order], c[order], v[order]
    ptr = np.r_[0, np.cumsum(np.bincount(r, minlength=n))]
    ip, ix, vals = C.sym_norm(ptr, c.astype(np.int32), v, n, 0.4, device="cuda")
    want = oracle_mod.sym_norm(ptr, c, v, n, 0.4)
    for got, w in zip((ip, ix, vals), want):
        np.testing.assert_array_equal(got.cpu().numpy(), w)
    e = np.stack([r, c]).astype(np.int64)
    ip, ix, vals = C.edge_index_to_adj(torch.from_numpy(e), n, symmetric=True, device="cuda")
    want = sp.csr_matrix((np.ones(2 * m), (np.r_[r, c], np.r_[c, r])), shape=(n, n))
    np.testing.assert_array_equal(ip.cpu().numpy(), want.indptr)
    np.testing.assert_array_equal(ix.cpu().numpy(), want.indices)
    np.testing.assert_array_equal(vals.cpu().numpy(), want.data)


@pytest.mark.parametrize("thr", [(-1, -1), (None, None), (4, 64)])
@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 8, 13, 16, 17, 31, 32])
def test_narrow_rows_per_wave_bit_exact(oracle_mod, thr, d):
    """d <= 32: 64/S rows per wave (narrow path) == one row per wave == the oracle, bit for bit,
    including ACCUMULATE, the fused aggregation epilogue and strided panels."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm, spmm_agg
    n = 2500
    u, v = synth.rmat_undirected_t(n, 20000, seed=30 + d)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = torch.from_numpy(np.random.default_rng(d).random(ix.numel()).astype(np.float32))
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=thr[0], hub_threshold=thr[1], device="cuda")
    wide = torch.from_numpy(np.random.default_rng(2).standard_normal((n, d + 5)).astype(np.float32)).cuda()
    X = wide[:, 2:2 + d]                                   # strided panel (ld = d + 5)
    y = spmm(A, X)
    np.testing.assert_array_equal(y.cpu().numpy(),
                                  oracle_mod.spmm(ip.numpy(), ix.numpy(), vals.numpy(), X.cpu().numpy()))
    assert torch.equal(spmm(A, X, wide_rows=True), y)
    y2 = y.clone()
    spmm(A, X, out=y2, accumulate=True)
    y3 = y.clone()
    spmm(A, X, out=y3, accumulate=True, wide_rows=True)
    assert torch.equal(y2, y3)
    agg = torch.ones_like(y)
    out = torch.empty_like(y)
    spmm_agg(A, X, out, agg, 0.25, False)
    assert torch.equal(out, y) and torch.equal(agg, 1.0 + 0.25 * y)


@pytest.mark.parametrize("thr", [(-1, -1), (None, None), (4, 64)])
@pytest.mark.parametrize("d,ld", [(64, 64), (128, 128), (128, 132), (256, 256), (192, 192), (96, 100), (200, 200)])
def test_packed_light_rows_bit_exact(oracle_mod, thr, d, ld):
    """Wide panels: 4 light rows per wave (packed path; d = 64 / 128 / 256 with 16-byte aligned
    rows, the others fall back) == one row per wave == the oracle, bit for bit, including
    ACCUMULATE, the fused aggregation and halo-pack epilogues and strided panels."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm, spmm_agg
    n = 3000
    u, v = synth.rmat_undirected_t(n, 24000, seed=50 + d)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = torch.from_numpy(np.random.default_rng(d).random(ix.numel()).astype(np.float32) - 0.5)
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=thr[0], hub_threshold=thr[1], device="cuda")
    wide = torch.from_numpy(np.random.default_rng(3).standard_normal((n, ld)).astype(np.float32)).cuda()
    X = wide[:, :d]
    y = spmm(A, X)
    np.testing.assert_array_equal(y.cpu().numpy(),
                                  oracle_mod.spmm(ip.numpy(), ix.numpy(), vals.numpy(), X.cpu().numpy()))
    assert torch.equal(spmm(A, X, wide_rows=True), y)
    y2, y3 = y.clone(), y.clone()
    spmm(A, X, out=y2, accumulate=True)
    spmm(A, X, out=y3, accumulate=True, wide_rows=True)
    assert torch.equal(y2, y3)
    agg = torch.full_like(y, 2.0)
    out = torch.empty_like(y)
    spmm_agg(A, X, out, agg, -0.5, False)
    assert torch.equal(out, y) and torch.equal(agg, 2.0 + (-0.5) * y)


def test_papers100M_scale_sampled_rows_bit_exact(oracle_mod):
    """The papers100M-shaped graph on one GPU (111 M rows, 3.34e9 nonzeros: indptr beyond 2^31,
    launches chunked beyond 2^32 lanes): one hop checked bit for bit on 2000 sampled rows plus the
    longest rows, against the oracle on the compacted sub-problem (the rows' own column lists and
    the X rows they gather)."""
    from srgnn import graphs, synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    free, _ = torch.cuda.mem_get_info()
    if free < 200e9:
        pytest.skip("needs a full MI355X (200 GB free)")
    ip, ix, vals, n, d, _ = graphs.build("papers100M", "cuda")
    assert int(ip[-1]) > 2 ** 31
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
    x = synth.uniform_features_t(n, d, device="cuda")
    y = spmm(A, x)
    deg = ip[1:] - ip[:-1]
    g = torch.Generator(device="cpu").manual_seed(9)
    rows = torch.unique(torch.cat([torch.randint(0, n, (2000,), generator=g).cuda(),
                                   torch.sort(deg, descending=True).indices[:20]]))
    beg, cnt = ip[rows], deg[rows]
    pos = torch.repeat_interleave(beg - torch.cumsum(cnt, 0) + cnt, cnt) + torch.arange(int(cnt.sum()), device="cuda")
    cols, vv = ix[pos].long(), vals[pos]
    ucols, inv = torch.unique(cols, return_inverse=True)
    sub_ip = np.r_[0, np.cumsum(cnt.cpu().numpy())]
    want = oracle_mod.spmm(sub_ip, inv.to(torch.int32).cpu().numpy(), vv.cpu().numpy(), x[ucols].cpu().numpy())
    np.testing.assert_array_equal(y[rows].cpu().numpy(), want)


@pytest.mark.parametrize("d", [1, 3, 7, 36, 128, 256, 1433])
def test_gather_rows_equals_index_select(d):
    """srg_gather_rows_f32 (the halo exchange's send-side pack): the rows of index_select, for every
    vector width / lanes-per-row variant, strided panels, duplicate indices and an empty list."""
    from srgnn.spmm import gather_rows
    g = torch.Generator(device="cuda").manual_seed(d)
    n = 5003
    big = torch.rand((n, d + 5), generator=g, device="cuda")
    for src in (big[:, :d].contiguous(), big[:, :d]):
        for m in (0, 1, 17, 4099):
            idx = torch.randint(0, n, (m,), generator=g, device="cuda")
            got = gather_rows(src, idx)
            torch.cuda.synchronize()
            assert torch.equal(got, src.index_select(0, idx)), f"d={d} m={m} ld={src.stride(0)}"
    out = torch.full((3, d + 2), 7.0, device="cuda")[:, :d]
    gather_rows(big[:, :d], torch.tensor([2, 0, 2], device="cuda"), out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, big[[2, 0, 2], :d])


@pytest.mark.parametrize("world,ghost", [(2, None), (4, 0), (8, 16)])
def test_halo_whole_x_hop0_gather(world, ghost):
    """propagate(x_full=X) on each virtual rank (K = 1: no exchange at all): hop 0's halo, ghost
    rows included, is gathered from the whole X on the GPU, and hop 1's own rows (ghost kernels
    included in the launch) are bitwise the single-device hop."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.dist import HaloPartitionedOperator
    from srgnn.normalize import sym_norm_binary
    from srgnn.spmm import propagate
    n = 20000
    u, v = synth.rmat_undirected_t(n, 150000, seed=24, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 64, device="cuda")
    want = propagate(DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda"), x, 1)
    for q in range(world):
        op = HaloPartitionedOperator(ip, ix, vals, n, chunks=3, hub_threshold=300, device="cuda", rank=q,
                                     world=world, ghost_max_degree=ghost)
        panels = op.propagate(x[op.r0:op.r1], 1, x_full=x)
        torch.cuda.synchronize()
        assert torch.equal(panels[0][op.rows:], x.index_select(0, op.halo_ids()))
        assert torch.equal(panels[1][: op.rows], want[1][op.r0:op.r1]), f"rank {q}/{world}"


@pytest.mark.parametrize("name", ["rand_d128_r05", "rand_d36_ppr", "cora_sym_k3"])
def test_hub_window_256_bit_exact(name, oracle_mod):
    """Hub workgroups with 256-nonzero windows (two per CU; the default once a launch has more hub
    workgroups than CUs) and with 512: every
    row a hub row, all bit-identical to the reference."""
    from srgnn.spmm import spmm
    c = G.Case(name)
    A = _csr(c, (0, 0))
    assert A.n_hub == A.n_rows
    x = c.x()
    if x.shape[1] % 4:
        # hub workgroups take panels of d % 4 == 0 (others go to slice waves): Cora's 1433
        # columns -> its first 1432 against the oracle
        x = np.ascontiguousarray(x[:, : x.shape[1] // 4 * 4])
        want = oracle_mod.spmm(*c.ahat(), x)
    X = torch.from_numpy(x).cuda()
    for w256 in (True, False):
        y = spmm(A, X, hub_w256=w256)
        if x.shape[1] != c.x().shape[1]:
            np.testing.assert_array_equal(y.cpu().numpy(), want)
        else:
            c.check_hop(1, y.cpu().numpy())
    # rows longer than one window (several 256-windows and a partial one)
    from srgnn.csr import DeviceCSR
    n, deg = 40, 1500
    rng = np.random.default_rng(5)
    ip = np.arange(n + 1, dtype=np.int64) * deg
    ix = rng.integers(0, 3000, n * deg).astype(np.int32)
    vv = rng.standard_normal(n * deg).astype(np.float32)
    x = rng.standard_normal((3000, 64)).astype(np.float32)
    B = DeviceCSR.from_tensors(ip, ix, vv, n_cols=3000, heavy_threshold=0, hub_threshold=0, device="cuda")
    want = None
    for w256 in (True, False):
        y = spmm(B, torch.from_numpy(x).cuda(), hub_w256=w256).cpu().numpy()
        want = y if want is None else want
        assert np.array_equal(y, want)
    assert np.array_equal(want, oracle_mod.spmm(ip, ix, vv, x))


def test_blocked_hop_rejects_undersized_out_and_agg():
    """Column blocks 1.. and the split parts of block 0 schedule a subset of the rows but write rows
    of the whole operator: hop / spmm / spmm_agg check out and agg against the full row count
    (ValueError, nothing launched), and a block refuses to allocate its own out."""
    import plan_layout_ref as R
    from srgnn.spmm import hop, spmm, spmm_agg
    c = G.Case("rand_d128_r05")
    A = _csr(c, (None, None))
    X = torch.from_numpy(c.x()).cuda()
    blocks = R.column_blocks(A, 4)
    assert any(b.schedules_subset for b in blocks[1:])
    small = torch.empty((c.n - 1, X.shape[1]), device="cuda")
    full = torch.empty_like(X)
    with pytest.raises(ValueError):
        hop(A, X, small, col_blocks=4)
    with pytest.raises(ValueError):
        hop(A, X, full, col_blocks=4, agg=(small, 1.0, True))
    sub = next(b for b in blocks[1:] if b.schedules_subset)
    with pytest.raises(ValueError):
        spmm(sub, X)
    with pytest.raises(ValueError):
        spmm(sub, X, out=torch.empty((sub.n_rows, X.shape[1]), device="cuda"))
    with pytest.raises(ValueError):
        spmm_agg(sub, X, full, small, 1.0, True)
    hop(A, X, full, col_blocks=4)
    torch.cuda.synchronize()
    c.check_hop(1, full.cpu().numpy())


def test_hub_side_streams_bounded():
    """Hub rows fork onto a library side stream per (device, caller stream); callers that make a
    new stream per call do not grow the set without bound (at most 8 per device, LRU), and results
    stay bit-exact on every stream."""
    from srgnn import _lib
    from srgnn.spmm import spmm
    c = G.Case("rand_d128_r05")
    A = _csr(c, (0, 0))
    assert A.n_hub > 0
    X = torch.from_numpy(c.x()).cuda()
    for i in range(24):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            y = spmm(A, X)
        st.synchronize()
        if i % 8 == 0:
            c.check_hop(1, y.cpu().numpy())
        assert _lib.query("srg_hub_side_streams") <= 8 * torch.cuda.device_count()


def test_column_blocks_keep_explicit_thresholds():
    """An operator built with explicit thresholds has its column blocks (and block 0's split parts)
    scheduled with the same thresholds and no automatic narrow split -- in the native plan, launch by
    launch, as in the test restatement; the automatic operator's blocks keep the narrow split.  Same
    bits either way."""
    import plan_layout_ref as R
    from srgnn.plan import NativePlan
    from srgnn.spmm import hop
    c = G.Case("rand_d128_r05")
    A = _csr(c, (5, 60))
    assert A.n_heavy_narrow is None and A.thresholds == (5, 60)
    X = torch.from_numpy(c.x()).cuda()
    for blk in R.column_blocks(A, 3):
        assert blk.thresholds == (5, 60) and blk.n_heavy_narrow is None
        deg = (blk.row_end - blk.indptr)[blk.order.long()]
        assert blk.n_hub == int((deg > 60).sum()) and blk.n_hub + blk.n_heavy == int((deg > 5).sum())
    for part in R.split_whole(R.column_blocks(A, 3)[0]) or ():
        assert part.n_heavy_narrow is None
    P = NativePlan(A, 16, hops=4, col_blocks=3, split_block0=True)
    plan_py, _ = R.hop_plan(A, 16, 3, compact=False, split=True)
    for (L, _), (Ab, _, _) in zip(P.launches(16), plan_py):
        assert (L.n_hub, L.n_heavy) == (Ab.n_hub, Ab.heavy(16))     # d = 16: the narrow count is n_heavy
    P.close()
    auto = _csr(c, (None, None))
    assert all(b.n_heavy_narrow is not None for b in R.column_blocks(auto, 3))
    y = hop(A, X, torch.empty_like(X), col_blocks=3, agg=(torch.zeros_like(X), 1.0, True))
    torch.cuda.synchronize()
    c.check_hop(1, y.cpu().numpy())


@pytest.mark.parametrize("mode", ["mixed", "same"])
def test_blocked_hop_hub_rows_chained_or_forked_bit_exact(oracle_mod, mode):
    """Column-blocked hops chain the blocks' hub spans on the side stream only when every block has
    the same hub rows (then no other launch touches them); when a row is a hub in some blocks only,
    every block forks and joins.  Both are bitwise the one-launch hop, repeated hops included."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.normalize import sym_norm_binary
    import plan_layout_ref as R
    from srgnn.plan import cached
    from srgnn.spmm import hop, spmm
    n = 30000
    u, v = synth.rmat_undirected_t(n, 400000, seed=51, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 128, device="cuda")
    # on this graph the block spans of the rows longer than 300 all exceed 300 (121 hub rows in each
    # of the 3 blocks: the same set), while at 150 the sets differ (207 / 169 / 142 rows)
    thr = 150 if mode == "mixed" else 300
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, hub_threshold=thr, device="cuda")
    want = spmm(A, x)
    blocks = R.column_blocks(A, 3)
    assert any(b.n_hub for b in blocks)
    assert R._same_hub_rows([R.split_whole(blocks[0])[0]] + blocks[1:]) == (mode == "same")
    y = torch.empty_like(x)
    for _ in range(3):
        hop(A, x, y, col_blocks=3)
        torch.cuda.synchronize()
        assert torch.equal(y, want), mode
    # the native plan chains exactly when the restatement does
    assert cached(A, 128).hub_chain == (mode == "same")
    # with the aggregation step fused (the split block 0 and the aggregating last block in the chain)
    agg = torch.empty_like(x)
    for _ in range(2):
        hop(A, x, y, col_blocks=3, agg=(agg, 0.5, True))
        torch.cuda.synchronize()
        assert torch.equal(y, want) and torch.equal(agg, 0.0 + 0.5 * want), mode


def test_propagate_plan_entry_rejects_bad_launches():
    """srg_propagate_plan_f32 (the native blocked hop loop) validates every launch before the first
    kernel: a schedule with hub / heavy rows but no row_order, a null panel, negative K."""
    import ctypes
    import plan_layout_ref as R
    from srgnn import _lib
    c = G.Case("rand_d128_r05")
    A = _csr(c, (None, None))
    X = torch.from_numpy(c.x()).cuda()
    Y = torch.empty_like(X)
    d = X.shape[1]
    plan, join = R.hop_plan(A, d, 2, compact=False, split=True)
    arr = R.launch_array(plan, d)
    panels = (ctypes.c_void_p * 2)(X.data_ptr(), Y.data_ptr())
    _lib.call(X.device, "srg_propagate_plan_f32", arr, len(plan), int(join), panels, d, d, 1, _lib.stream(X.device))
    torch.cuda.synchronize()
    c.check_hop(1, Y.cpu().numpy())
    bad = R.launch_array(plan, d)
    bad[0].n_heavy, bad[0].row_order = max(1, bad[0].n_heavy), None
    with pytest.raises(RuntimeError):
        _lib.call(X.device, "srg_propagate_plan_f32", bad, len(plan), int(join), panels, d, d, 1, _lib.stream(X.device))
    if any(Ab.is_span for Ab, _, _ in plan):
        half = R.launch_array(plan, d)
        i = next(j for j, (Ab, _, _) in enumerate(plan) if Ab.is_span)
        half[i].slot_end = None                   # slot spans come in pairs
        with pytest.raises(RuntimeError):
            _lib.call(X.device, "srg_propagate_plan_f32", half, len(plan), int(join), panels, d, d, 1,
                      _lib.stream(X.device))
    nulls = (ctypes.c_void_p * 2)(X.data_ptr(), None)
    with pytest.raises(RuntimeError):
        _lib.call(X.device, "srg_propagate_plan_f32", arr, len(plan), int(join), nulls, d, d, 1, _lib.stream(X.device))
    with pytest.raises(RuntimeError):
        _lib.call(X.device, "srg_propagate_plan_f32", arr, len(plan), int(join), panels, d, d, -1, _lib.stream(X.device))
    # unjoined hub forks over several hops would race the next hop's reads: rejected
    Ah = _csr(c, (16, 64))
    hplan = [(Ah, _lib.SRG_SPMM_HUB_NOJOIN, "plain")]
    assert Ah.n_hub > 0
    nj = R.launch_array(hplan, d)
    Z = torch.empty_like(X)
    three = (ctypes.c_void_p * 3)(X.data_ptr(), Y.data_ptr(), Z.data_ptr())
    with pytest.raises(RuntimeError, match="join_hub"):
        _lib.call(X.device, "srg_propagate_plan_f32", nj, 1, 0, three, d, d, 2, _lib.stream(X.device))
    _lib.call(X.device, "srg_propagate_plan_f32", nj, 1, 1, three, d, d, 2, _lib.stream(X.device))
    torch.cuda.synchronize()
    c.check_hop(1, Y.cpu().numpy())
    c.check_hop(2, Z.cpu().numpy())


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("name", ["rand_d128_r05", "rand_d36_ppr", "cora_sym_k3"])
def test_schedule_ordered_one_launch_bit_exact(name, native):
    """A long-lived one-launch operator's launch-ordered copy (spmm.prepare for runs of >=
    SRG_PLAN_MIN_HOPS_TO_COMPACT hops: the native plan's compact copy; or the test restatement's
    schedule_ordered, run through the plan loop): propagate and hop through it == the reference, bit
    for bit."""
    import plan_layout_ref as R
    from srgnn import spmm as spmm_mod
    from srgnn.plan import cached
    c = G.Case(name)
    A = _csr(c, (None, None))
    X = torch.from_numpy(c.x()).cuda()
    if native:
        assert spmm_mod.prepare(A, X.shape[1], hops=1000) == 1
        P = cached(A, X.shape[1])
        assert P.compact and P.n_launch == 1 and P.col_blocks == 1
        hops = spmm_mod.propagate(A, X, c.k)
    else:
        S = R.schedule_ordered(A)
        assert S.is_span and S.nnz == A.nnz and S.indices.data_ptr() != A.indices.data_ptr()
        hops = R.propagate(A, X, c.k, 1, compact=True)
    torch.cuda.synchronize()
    for k in range(1, c.k + 1):
        c.check_hop(k, hops[k].cpu().numpy())
    c.check_hop(1, spmm_mod.hop(A, X, torch.empty_like(X), col_blocks=1).cpu().numpy())
