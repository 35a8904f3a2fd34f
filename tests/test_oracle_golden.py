"""Pin the CPU oracle against the reference's own outputs (tests/golden/, made by running the
reference's operators) and against the reference's matmul.c compiled from source (oracle/_ref)."""
import numpy as np
import pytest

import golden_cases as G


@pytest.mark.parametrize("name", G.names("norm"))
def test_sym_norm_matches_reference(oracle_mod, name):
    c = G.Case(name)
    a = c.adj()
    if c.meta["op"] == "ppr":
        ip, ix, v = oracle_mod.ppr_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"], c.meta["alpha"])
    else:
        ip, ix, v = oracle_mod.sym_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"])
    np.testing.assert_array_equal(ip, c["ahat_indptr"])
    np.testing.assert_array_equal(ix, c["ahat_indices"])
    np.testing.assert_array_equal(v, c["ahat_data64"])          # fp64, bit for bit
    np.testing.assert_array_equal(v.astype(np.float32), c["ahat_data"])


@pytest.mark.parametrize("name", G.names("norm"))
def test_propagate_matches_reference(oracle_mod, name):
    c = G.Case(name)
    hops = oracle_mod.propagate(*c.ahat(), c.x(), c.k)
    for k in range(1, c.k + 1):
        c.check_hop(k, hops[k])


@pytest.mark.parametrize("name", G.names("raw"))
def test_raw_spmm_matches_reference(oracle_mod, name):
    c = G.Case(name)
    a = c.adj()
    y = oracle_mod.spmm(a.indptr, a.indices, a.data.astype(np.float32), c.x())
    c.check_hop(1, y)


@pytest.mark.parametrize("name", G.names("raw") + ["rand_d128_r05", "rand_d7_r03", "cora_sym_k3"])
def test_oracle_equals_reference_build(oracle_mod, name):
    if oracle_mod.ref_lib() is None:
        pytest.skip("oracle/_ref/libmatmul_ref.so not built (reference sources absent)")
    c = G.Case(name)
    if c.meta["op"] == "raw_spmm":
        a = c.adj()
        ip, ix, v = a.indptr, a.indices, a.data.astype(np.float32)
    else:
        ip, ix, v = c.ahat()
    x = c.x()
    np.testing.assert_array_equal(oracle_mod.spmm(ip, ix, v, x), oracle_mod.ref_spmm(ip, ix, v, x))


def test_error_manifest_present():
    errs = G.manifest()["_errors"]
    assert errs["coo_adj"] == "TypeError"
    assert errs["float64_feature"] == "ArgumentError"
    assert errs["dim_mismatch"] == "ValueError"


@pytest.mark.parametrize("name", G.names("aggregate"))
def test_oracle_combine_equals_reference_message_ops(oracle_mod, name):
    """oracle.combine on the oracle's hops == the reference's own message operators (fixtures)."""
    import torch
    c = G.Case(name)
    a = c.adj()
    ip, ix, v64 = oracle_mod.sym_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"])
    hops = oracle_mod.propagate(ip, ix, v64.astype(np.float32), c.x(), c.k)
    feats = [torch.from_numpy(h) for h in hops]
    for key, (aggr, s, e, ct, alpha, wl) in G.agg_specs(c.k).items():
        out = oracle_mod.combine(aggr, feats, s, e, alpha=alpha, weight_list=wl)
        c.check_output(key, out.numpy())


@pytest.mark.parametrize("name", G.names("aggregate"))
def test_aggregation_plan_equals_reference_message_ops(oracle_mod, name):
    """srgnn.aggregate's planned step order, executed in numpy fp32, == the reference's combine."""
    from srgnn import aggregate as AG
    from test_aggregate_cpu import run_steps_np
    c = G.Case(name)
    a = c.adj()
    ip, ix, v64 = oracle_mod.sym_norm(a.indptr, a.indices, a.data, c.n, c.meta["r"])
    hops = oracle_mod.propagate(ip, ix, v64.astype(np.float32), c.x(), c.k)
    for key, spec in G.agg_specs(c.k).items():
        mode, terms, div = AG.combine_plan(G.Msg(*spec), c.k + 1)
        if mode == "last":
            out = hops[-1]
        else:
            out = run_steps_np(AG.combine_steps(mode, terms, div), hops, c.n, hops[0].shape[1])
        c.check_output(key, out)


@pytest.mark.parametrize("name", ["rand_d128_r05", "cora_sym_k3", "rand_d7_r03"])
def test_column_blocked_chain_continuation_oracle(oracle_mod, name):
    """The exactness argument behind tools/colblock_probe.py, on the reference's own hops: with
    sorted columns, B ascending column-block passes (the first from +0.0f, the rest accumulating
    into the stored fp32 partial) reproduce the reference's one-pass product bit for bit."""
    c = G.Case(name)
    ip, ix, v = (np.asarray(a) for a in c.ahat())
    x = c.x()
    row = np.repeat(np.arange(c.n), np.diff(ip))
    for B in (2, 5):
        blk = (ix.astype(np.int64) * B) // c.n
        y = None
        for b in range(B):
            m = blk == b
            bip = np.concatenate([[0], np.cumsum(np.bincount(row[m], minlength=c.n))])
            y = oracle_mod.spmm(bip, ix[m], v[m].astype(np.float32), x, out=y, accumulate=b > 0)
        c.check_hop(1, y)
