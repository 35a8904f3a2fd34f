"""Fused hop aggregation on the GPU vs the reference's MessageOp.combine on the full hop list.

Expected values: the hop list from the oracle (bit-exact to the reference, pinned by the golden
fixtures) combined by oracle.combine (the reference's own torch CPU operations).  Bar: bit-exact.
"""
import numpy as np
import pytest
import torch

import golden_cases as G

pytestmark = pytest.mark.gpu


class _Msg:
    def __init__(self, aggr, start=None, end=None, combination_type=None, alpha=None, weight_list=None):
        self.aggr_type, self.start, self.end = aggr, start, end
        self.combination_type, self.alpha, self.weight_list = combination_type, alpha, weight_list


def _ops(K):
    return [
        _Msg("last"), _Msg("sum", 0, K + 1), _Msg("mean", 1, K + 1), _Msg("mean", 0, K + 2),
        _Msg("simple_weighted", 0, K + 1, "alpha", alpha=0.15),
        _Msg("simple_weighted", 2, K, "alpha", alpha=0.5),
        _Msg("simple_weighted", 1, 3, "hand_crafted", weight_list=torch.FloatTensor([0.7, -0.3])),
    ]


def _expected(oracle_mod, msg, hops):
    feats = [torch.from_numpy(h) for h in hops]
    return oracle_mod.combine(msg.aggr_type, feats, msg.start, msg.end, alpha=msg.alpha,
                              weight_list=msg.weight_list).numpy()


@pytest.mark.parametrize("K", [3, 10, 20])
@pytest.mark.parametrize("name", ["cora_sym_k3", "pubmed_sym_k3", "rand_d1_r05", "rand_d130_r1",
                                  "rand_d36_ppr", "rand_d1433_r05"])
def test_fused_combine_bit_exact(oracle_mod, name, K):
    from srgnn.aggregate import fused_combine
    from srgnn.csr import DeviceCSR
    c = G.Case(name)
    ip, ix, v = c.ahat()
    x = c.x()
    hops = oracle_mod.propagate(ip, ix, v, x, K)
    for k in range(1, min(K, c.k) + 1):            # the oracle's hops are the reference's
        c.check_hop(k, hops[k])
    A = DeviceCSR.from_tensors(ip, ix, v, n_cols=c.n, device="cuda")
    X = torch.from_numpy(x).cuda()
    for msg in _ops(K):
        got = fused_combine(A, X, K, msg).cpu().numpy()
        want = _expected(oracle_mod, msg, hops)
        np.testing.assert_array_equal(got, want, err_msg=f"{name} K={K} {msg.aggr_type} {msg.start}:{msg.end}")


@pytest.mark.parametrize("B", [2, 3])
@pytest.mark.parametrize("name", ["cora_sym_k3", "rand_d130_r1", "rand_d36_ppr"])
def test_propagate_aggregate_column_blocked_bit_exact(oracle_mod, name, B):
    """Column-blocked hops in the fused aggregation (the plan's hops, srg_plan_hop_f32: blocks with
    ACCUMULATE, the aggregation epilogue in the launch that finishes each row -- the last block's, or
    block 0's whole-row launch for the short rows) == the reference's combine, bit for bit."""
    from srgnn.aggregate import combine_plan, combine_steps, propagate_aggregate
    from srgnn.csr import DeviceCSR
    c = G.Case(name)
    ip, ix, v = c.ahat()
    x = c.x()
    K = 5
    hops = oracle_mod.propagate(ip, ix, v, x, K)
    A = DeviceCSR.from_tensors(ip, ix, v, n_cols=c.n, device="cuda")
    X = torch.from_numpy(x).cuda()
    for msg in _ops(K):
        mode, terms, div = combine_plan(msg, K + 1)
        if mode == "last":
            got = propagate_aggregate(A, X, K, last_only=True, col_blocks=B)
        else:
            got = propagate_aggregate(A, X, K, combine_steps(mode, terms, div), col_blocks=B)
        np.testing.assert_array_equal(got.cpu().numpy(), _expected(oracle_mod, msg, hops),
                                      err_msg=f"{name} B={B} {msg.aggr_type} {msg.start}:{msg.end}")


@pytest.mark.parametrize("whole", [(0, False), (4, False), (16, True), (1 << 30, False)])
@pytest.mark.parametrize("B", [2, 3])
@pytest.mark.parametrize("name", ["cora_sym_k3", "rand_d130_r1", "rand_d36_ppr"])
def test_aggregation_epilogue_over_restated_layouts(name, B, whole):
    """The aggregation epilogue in layouts the planner does not pick (tests/plan_layout_ref.py: every
    row cut, short rows whole up to 4 / 16 entries or every row whole, spans or compact copies):
    out and agg == the one-launch srg_spmm_agg_f32, bit for bit."""
    import plan_layout_ref as R
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm_agg
    c = G.Case(name)
    ip, ix, v = c.ahat()
    A = DeviceCSR.from_tensors(ip, ix, v, n_cols=c.n, device="cuda")
    blocks = (R.compact_column_blocks if whole[1] else R.column_blocks)(A, B, whole[0])
    assert blocks is not None and sum(b.nnz for b in blocks) == A.nnz
    if whole[0]:
        assert blocks[0].whole_rows is not None and R.split_whole(blocks[0]) is not None
    X = torch.from_numpy(c.x()).cuda()
    prev = torch.from_numpy(np.random.default_rng(3).standard_normal(X.shape).astype(np.float32)).cuda()
    y_ref, agg_ref = torch.empty_like(X), prev.clone()
    spmm_agg(A, X, y_ref, agg_ref, 0.37, False)
    y, agg = torch.empty_like(X), prev.clone()
    R.hop(A, X, y, B, compact=whole[1], split=True, whole_max=whole[0], agg=(agg, 0.37, False))
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int32), y_ref.view(torch.int32))
    assert torch.equal(agg.view(torch.int32), agg_ref.view(torch.int32))


def test_graphop_propagate_aggregate_matches_aggregate_of_propagate():
    """operators API: GraphOp.propagate_aggregate(adj, x, msg) == msg.aggregate(GraphOp.propagate(adj, x))."""
    from operators.graph_operator.symmetrical_simgraph_laplacian_operator import SymLaplacianGraphOp
    from operators.message_operator.last_message_op import LastMessageOp
    from operators.message_operator.mean_message_op import MeanMessageOp
    from operators.message_operator.simple_weighted_message_op import SimpleWeightedMessageOp
    from operators.message_operator.sum_message_op import SumMessageOp
    c = G.Case("cora_sym_k3")
    x = c.x()
    for K in (2, 12):
        op = SymLaplacianGraphOp(K, r=0.5)
        feats = op.propagate(c.adj(), x)
        for msg in (LastMessageOp(), SumMessageOp(0, K + 1), MeanMessageOp(1, K + 1),
                    SimpleWeightedMessageOp(0, K + 1, "alpha", 0.1),
                    SimpleWeightedMessageOp(1, 3, "hand_crafted", [0.25, 0.75])):
            want = msg.aggregate(feats).numpy()
            got = op.propagate_aggregate(c.adj(), x, msg)
            assert isinstance(got, torch.Tensor) and got.dtype == torch.float32 and not got.is_cuda
            np.testing.assert_array_equal(got.numpy(), want, err_msg=f"K={K} {msg.aggr_type}")
    op = SymLaplacianGraphOp(3, r=0.5)
    with pytest.raises(TypeError):
        op.propagate_aggregate(c.adj().tocoo(), x, SumMessageOp(0, 4))
    with pytest.raises(ValueError):
        op.propagate_aggregate(c.adj(), x[:-1], SumMessageOp(0, 4))


def test_products_scale_weighted_bit_exact():
    """Full products-shaped graph, K = 10, GBP-style alpha weights: the fused result equals the
    reference's one_dim_weighted_add of the hop list (hops from the GPU, bit-exact by the hop tests)."""
    from srgnn import graphs, synth
    from srgnn.aggregate import fused_combine
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import propagate
    import oracle.oracle as O
    ip, ix, vals, n, d, K = graphs.build("products", "cuda")
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
    del ip, ix, vals
    x = synth.uniform_features_t(n, d, device="cuda")
    msg = _Msg("simple_weighted", 0, K + 1, "alpha", alpha=0.15)
    got = fused_combine(A, x, K, msg).cpu()
    hops = [h.cpu() for h in propagate(A, x, K)]
    want = O.combine("simple_weighted", hops, 0, K + 1, alpha=0.15)
    assert torch.equal(got, want)
    got = fused_combine(A, x, K, _Msg("mean", 0, K + 1)).cpu()
    assert torch.equal(got, O.combine("mean", hops, 0, K + 1))


@pytest.mark.parametrize("thr", [(-1, -1), (0, -1), (0, 0), (None, None), (4, 64)])
@pytest.mark.parametrize("d", [1, 7, 64, 128, 130])
def test_spmm_agg_epilogue_equals_separate_steps(thr, d):
    """srg_spmm_agg_f32 (aggregation fused into the row-wave, slice-wave and hub epilogues) ==
    srg_spmm_csr_f32 followed by srg_hop_accumulate_f32, bit for bit, INIT and ADD."""
    from srgnn import _lib, synth
    from srgnn.aggregate import _DeviceSteps
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm, spmm_agg
    n = 3000
    u, v = synth.rmat_undirected_t(n, 30000, seed=3)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = torch.from_numpy(np.random.default_rng(d).random(ix.numel()).astype(np.float32))
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=thr[0], hub_threshold=thr[1], device="cuda")
    X = torch.from_numpy(np.random.default_rng(1).standard_normal((n, d)).astype(np.float32)).cuda()
    prev = torch.from_numpy(np.random.default_rng(2).standard_normal((n, d)).astype(np.float32)).cuda()
    ex = _DeviceSteps(n, d, X.device)
    for init in (True, False):
        y_ref = spmm(A, X)
        agg_ref = prev.clone()
        ex._acc(agg_ref, y_ref, 0.37, _lib.SRG_ACC_INIT if init else _lib.SRG_ACC_ADD)
        y = torch.empty_like(y_ref)
        agg = prev.clone()
        spmm_agg(A, X, y, agg, 0.37, init)
        assert torch.equal(y, y_ref) and torch.equal(agg, agg_ref)
    with pytest.raises(Exception):
        spmm_agg(A, X, y, y, 0.5, True)            # agg aliasing Y is refused


@pytest.mark.parametrize("name", G.names("aggregate"))
def test_fused_combine_equals_reference_message_ops(name):
    """Device construct_adj + fused hops/aggregation == the reference's own message operators
    (fixtures from make_golden.py), for every message operator of the fixture."""
    from srgnn import construct as C
    from srgnn.aggregate import fused_combine
    from srgnn.csr import DeviceCSR
    c = G.Case(name)
    a = c.adj()
    ip, ix, v64 = C.sym_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"], device="cuda")
    A = DeviceCSR.from_tensors(ip, ix, v64.to(torch.float32), n_cols=c.n, device="cuda")
    X = torch.from_numpy(c.x()).cuda()
    for key, spec in G.agg_specs(c.k).items():
        c.check_output(key, fused_combine(A, X, c.k, G.Msg(*spec)).cpu().numpy())


def test_degenerate_inputs():
    """K = 0, empty graphs, rows without entries, zero-width panels: same results as the reference
    combine on the (trivial) hop lists, no launches on empty shapes."""
    import scipy.sparse as sp
    from srgnn import construct as C
    from srgnn.aggregate import fused_combine
    from srgnn.csr import DeviceCSR
    import oracle.oracle as O
    # K = 0: the hop list is [X]
    n, d = 50, 9
    adj = sp.random(n, n, density=0.1, format="csr", random_state=0)
    ip, ix, v = C.sym_norm(adj.indptr, adj.indices, adj.data, n, 0.5, device="cuda")
    A = DeviceCSR.from_tensors(ip, ix, v.to(torch.float32), n_cols=n, device="cuda")
    X = torch.from_numpy(np.random.default_rng(0).standard_normal((n, d)).astype(np.float32))
    for spec in G.agg_specs(0).values():
        m = G.Msg(*spec)
        if m.aggr_type == "simple_weighted" and m.combination_type == "hand_crafted":
            continue                                  # needs 2 hops in its slice
        if m.aggr_type != "last" and not range(1)[slice(m.start, m.end)]:
            continue                                  # the reference fails on an empty slice too
        want = O.combine(m.aggr_type, [X], m.start, m.end, alpha=m.alpha, weight_list=m.weight_list)
        assert torch.equal(fused_combine(A, X.cuda(), 0, m).cpu(), want)
    # empty graph (n = 0) and an edgeless graph
    ip, ix, v = C.sym_norm(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0), 0, 0.5, device="cuda")
    assert ip.tolist() == [0] and ix.numel() == 0
    A0 = DeviceCSR.from_tensors(ip, ix, v.to(torch.float32), n_cols=0, device="cuda")
    out = fused_combine(A0, torch.zeros((0, 4), device="cuda"), 3, G.Msg("sum", 0, 4, None, None, None))
    assert out.shape == (0, 4)
    e = C.edge_index_to_adj(torch.zeros((2, 0), dtype=torch.int64), 5, device="cuda")
    assert e[0].tolist() == [0] * 6 and e[1].numel() == 0
    ip, ix, v = C.sym_norm(*(t.cpu().numpy() for t in e), 5, 0.5, device="cuda")
    assert ip.tolist() == list(range(6)) and torch.equal(v.cpu(), torch.ones(5, dtype=torch.float64))


@pytest.mark.parametrize("thr", [(-1, -1), (0, -1), (0, 0), (None, None), (4, 64)])
@pytest.mark.parametrize("d", [1, 7, 64, 128, 130, 256])
def test_span_blocks_every_path(thr, d):
    """Column blocks as row spans (srg_spmm_span_f32) through every worker kind the thresholds
    select -- hub workgroups (0, 0), slice waves, packed / narrow / whole light rows -- plain and
    with the aggregation epilogue in the last block: bitwise the one-launch srg_spmm_csr_f32 and
    srg_spmm_agg_f32.  The spans come from srg_csr_col_splits on a CSR with sorted rows."""
    from srgnn.csr import DeviceCSR, narrow_heavy_degrees, schedule_from_degrees
    from srgnn.spmm import spmm, spmm_agg
    n = 3000
    ip, ix = synth_graph(n)
    vals = torch.from_numpy(np.random.default_rng(d).random(ix.numel()).astype(np.float32))
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=thr[0], hub_threshold=thr[1], device="cuda")
    X = torch.from_numpy(np.random.default_rng(1).standard_normal((n, d)).astype(np.float32)).cuda()
    prev = torch.from_numpy(np.random.default_rng(2).standard_normal((n, d)).astype(np.float32)).cuda()
    y_ref = spmm(A, X)
    agg_ref = prev.clone()
    spmm_agg(A, X, torch.empty_like(y_ref), agg_ref, 0.37, False)
    import plan_layout_ref as R
    for B in (2, 3):
        spans = R.column_blocks(A, B)
        blocks = []
        for s in spans:        # the same spans, scheduled with the test's thresholds
            deg = s.row_end - s.indptr
            order, n_heavy, n_hub = schedule_from_degrees(deg, int(deg.sum()), thr[0], thr[1])
            blocks.append(DeviceCSR(s.indptr, s.indices, s.values, n, n, order, n_heavy, n_hub,
                                    narrow_heavy_degrees(deg, n_hub) if thr == (None, None) else None,
                                    row_end=s.row_end))
        if thr == (0, 0):
            assert any(b.n_hub > 0 for b in blocks)
        y = torch.empty_like(y_ref)
        agg = prev.clone()
        for b, Ab in enumerate(blocks):
            if b == B - 1:
                spmm_agg(Ab, X, y, agg, 0.37, False, accumulate=True)
            else:
                spmm(Ab, X, out=y, accumulate=b > 0)
        assert torch.equal(y, y_ref) and torch.equal(agg, agg_ref)


def synth_graph(n):
    from srgnn import synth
    u, v = synth.rmat_undirected_t(n, 30000, seed=3)
    return synth.symmetric_csr_t(n, u, v)
