"""Tolerance mode SRG_SPMM_FAST (EXACT, FAST, ACCUMULATE): hub rows summed as 64
exact segment chains plus their ordered sum.  Bar (north_star: fp32 within 1e-5 relative of the
reference path; matmul.c:23-40 is the exact chain):
  * every row that is not a hub row of the launch: bit-identical to exact mode;
  * hub rows: every element within the fp32 forward-error bound gamma_{len+65} * sum |a||x| of
    the exact (fp64) product -- the bound the exact chain itself obeys -- and, normwise per row,
    within 1e-5 of the exact chain where the row has no heavy cancellation;
  * deterministic: two runs give the same bits."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bound_check(oracle_mod, ip, ix, v, x, got, rows, what):
    sub_ip = np.r_[0, np.cumsum(np.diff(ip)[rows])]
    sub_ix = np.concatenate([ix[ip[r]:ip[r + 1]] for r in rows])
    sub_v = np.concatenate([v[ip[r]:ip[r + 1]] for r in rows]).astype(np.float64)
    exact = oracle_mod.spmm64(sub_ip, sub_ix, sub_v, x.astype(np.float64))
    mag = oracle_mod.spmm64(sub_ip, sub_ix, np.abs(sub_v), np.abs(x).astype(np.float64))
    n_ops = np.diff(sub_ip).astype(np.float64)[:, None] + 65
    gamma = n_ops * 2.0 ** -24 / (1 - n_ops * 2.0 ** -24)
    err = np.abs(got[rows].astype(np.float64) - exact)
    assert (err <= gamma * mag).all(), f"{what}: beyond the fp32 bound, worst ratio {float((err / (gamma * mag)).max()):.3g}"
    return exact


@pytest.mark.parametrize("d", [64, 128, 36])
def test_fast_hub_rows_within_bound_others_exact(oracle_mod, d):
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    n = 8000
    u, v = synth.rmat_undirected_t(n, 120000, seed=41)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = synth.uniform_features_np(1, int(ix.numel()), seed=42)[0] * 0.5 + 0.5
    x = synth.uniform_features_np(n, d, seed=43)
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, hub_threshold=200, device="cuda")
    assert A.n_hub > 0
    X = torch.from_numpy(x).cuda()
    exact = spmm(A, X).cpu().numpy()
    fast = spmm(A, X, fast=True).cpu().numpy()
    again = spmm(A, X, fast=True).cpu().numpy()
    assert np.array_equal(fast.view(np.uint32), again.view(np.uint32)), "FAST is not deterministic"
    hub = A.order[: A.n_hub].long().cpu().numpy()
    other = np.setdiff1d(np.arange(n), hub)
    np.testing.assert_array_equal(fast[other], exact[other])
    ipn, ixn = ip.numpy(), ix.numpy()
    _bound_check(oracle_mod, ipn, ixn, vals, x, fast, hub, "fast hub rows")
    _bound_check(oracle_mod, ipn, ixn, vals, x, exact, hub, "exact hub rows (the same bound)")
    # normwise per row within 1e-5 of the exact chain
    rel = np.linalg.norm(fast[hub] - exact[hub], axis=1) / np.linalg.norm(exact[hub], axis=1)
    assert rel.max() <= 1e-5, rel.max()
    # ACCUMULATE: the partial sums added to Y's content
    y0 = torch.from_numpy(synth.uniform_features_np(n, d, seed=44)).cuda()
    ye = spmm(A, X, out=y0.clone(), accumulate=True).cpu().numpy()
    yf = spmm(A, X, out=y0.clone(), accumulate=True, fast=True).cpu().numpy()
    np.testing.assert_array_equal(yf[other], ye[other])
    rel = np.linalg.norm(yf[hub] - ye[hub], axis=1) / np.linalg.norm(ye[hub], axis=1)
    assert rel.max() <= 1e-5, rel.max()


def test_fast_blocked_hops_and_khop(oracle_mod):
    """FAST through the column-blocked hop (row spans: each block's hub rows segmented) and the
    device K-hop loop: within tolerance of the exact hops, rows that are no block's hub exact."""
    from srgnn import synth
    from srgnn.csr import DeviceCSR
    from srgnn.normalize import sym_norm_binary
    from srgnn.spmm import hop, propagate
    n = 20000
    u, v = synth.rmat_undirected_t(n, 250000, seed=45, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    x = synth.uniform_features_t(n, 128, device="cuda")
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, hub_threshold=300, device="cuda")
    exact = propagate(A, x, 3)
    fast = propagate(A, x, 3, fast=True)
    for k in (1, 2, 3):
        rel = (fast[k] - exact[k]).norm(dim=1) / exact[k].norm(dim=1).clamp_min(1e-30)
        assert float(rel.max()) <= 1e-5, (k, float(rel.max()))
    hub = set(A.order[: A.n_hub].tolist())
    B = 3
    ye = hop(A, x, torch.empty_like(x), col_blocks=B)
    yf = hop(A, x, torch.empty_like(x), col_blocks=B, fast=True)
    import plan_layout_ref as R
    blocks = R.column_blocks(A, B)        # the plan's blocks, restated: their hub rows run FAST
    hubs = set()
    for blk in blocks:
        hubs |= set(blk.order[: blk.n_hub].tolist())
    assert hubs
    plain = torch.tensor(sorted(set(range(n)) - hubs - hub), device="cuda")
    assert torch.equal(yf[plain], ye[plain])
    rel = (yf - ye).norm(dim=1) / ye.norm(dim=1).clamp_min(1e-30)
    assert float(rel.max()) <= 1e-5
    _bound_check(oracle_mod, ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy(), x.cpu().numpy(),
                 yf.cpu().numpy(), np.array(sorted(hubs)), "blocked fast hub rows")


def test_fast_products_top_row_latency_and_bound(oracle_mod):
    """The products-shaped graph's 155,868-entry top row: FAST within the fp32 bound of the exact
    product, and its side-stream work much shorter than the exact chain's (timed alone)."""
    from srgnn import graphs, synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    ip, ix, vals, n, d, _ = graphs.build("products", "cuda")
    deg = ip[1:] - ip[:-1]
    top = int(torch.argmax(deg))
    one = DeviceCSR.from_tensors(ip[top:top + 2] - ip[top], ix[int(ip[top]):int(ip[top + 1])],
                                 vals[int(ip[top]):int(ip[top + 1])], n_cols=n, hub_threshold=0,
                                 heavy_threshold=0, device="cuda")
    assert one.n_hub == 1
    x = synth.uniform_features_t(n, d, device="cuda")
    times = {}
    for fast in (False, True):
        spmm(one, x, fast=fast)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(5):
            y = spmm(one, x, fast=fast)
        ev[1].record()
        torch.cuda.synchronize()
        times[fast] = ev[0].elapsed_time(ev[1]) / 5
    assert times[True] < 0.5 * times[False], times
    cols = ix[int(ip[top]):int(ip[top + 1])].long()
    _bound_check(oracle_mod, np.array([0, cols.numel()]), np.arange(cols.numel(), dtype=np.int32),
                 vals[int(ip[top]):int(ip[top + 1])].cpu().numpy(), x[cols].cpu().numpy(),
                 y.cpu().numpy(), np.array([0]), "products top row")
