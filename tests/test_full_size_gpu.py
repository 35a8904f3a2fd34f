"""The benchmark configurations of BASELINE.json at full size, in the layouts bench.py times.

Each hop is checked against the CPU oracle (oracle/srg_oracle.c: one fp32 fma chain per output
element in CSR order, matmul.c:23-40) fed with the GPU's previous hop: bit for bit on every row
where the oracle finishes in seconds (arxiv), on sampled rows plus the longest rows elsewhere --
the rows' own entries with their columns renumbered over the X rows they gather, so the check
needs only those rows of the previous panel.  The wavelet filter's fp32 orders are checked the
same way against the oracle's fp32 chain and within 1e-5 against an fp64 evaluation of the same
recurrence step (pygsp cheby_op, base_model.py:236-265).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_gb():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return torch.cuda.mem_get_info()[0] / 1e9


def _sample(ip, ix, vals, n, n_random, n_top, seed):
    """(rows, sub-CSR over renumbered columns, the X rows it gathers) -- device-side extraction."""
    deg = ip[1:] - ip[:-1]
    g = torch.Generator(device="cpu").manual_seed(seed)
    pick = [torch.randint(0, n, (n_random,), generator=g).cuda(), torch.sort(deg, descending=True).indices[:n_top]]
    rows = torch.unique(torch.cat(pick))
    beg, cnt = ip[rows], deg[rows]
    tot = int(cnt.sum())
    pos = torch.repeat_interleave(beg - torch.cumsum(cnt, 0) + cnt, cnt, output_size=tot) + \
        torch.arange(tot, device="cuda")
    ucols, inv = torch.unique(ix[pos].long(), return_inverse=True)
    sub = (np.r_[0, np.cumsum(cnt.cpu().numpy())].astype(np.int64), inv.to(torch.int32).cpu().numpy(),
           vals[pos].cpu().numpy())
    return rows, sub, ucols


def _check_rows(oracle_mod, rows, sub, ucols, prev, got, what):
    want = oracle_mod.spmm(*sub, prev[ucols].cpu().numpy())
    have = got[rows].cpu().numpy()
    bad = np.flatnonzero((have.view(np.uint32) != want.view(np.uint32)).any(axis=1))
    assert bad.size == 0, f"{what}: {bad.size} of {rows.numel()} sampled rows differ (first row {int(rows[bad[0]])})"


@pytest.mark.timeout(600)
def test_products_timed_layout_every_hop_bit_exact(oracle_mod):
    """The operator bench.py times on the headline config: products-shaped graph (126 M nonzeros),
    K = 10, d = 128, default thresholds, the native plan's twelve COMPACT column blocks (>= 6 hops; block 0 in two
    launches, its cut spans then its whole rows; compact copies in launch order, packed rows reading
    their spans by schedule slot), short rows (<= BLOCK_WHOLE_MAX = 48) whole in block 0, 2 gathers
    per packed row (PACKED_U2) -- EVERY row of every hop (2,449,029 x 128 per hop) checked bit for
    bit against the oracle fed with the GPU's previous hop (~1-3 s of host time per hop)."""
    from srgnn import csr as csr_mod, graphs, spmm as spmm_mod, synth
    from srgnn.csr import DeviceCSR
    from srgnn.plan import cached
    from srgnn.spmm import auto_col_blocks, prepare, propagate
    assert csr_mod.DEFAULT_HEAVY_THRESHOLD is None and csr_mod.DEFAULT_HUB_THRESHOLD is None
    ip, ix, vals, n, d, K = graphs.build("products", "cuda")
    assert K == 10 and d == 128
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
    hops = K * 25                                   # the driver's 20 steps + 5 warm-up
    assert auto_col_blocks(A, d, hops=hops) == 12
    assert prepare(A, d, hops) == 12                # bench.py's call: the native plan
    P = cached(A, d)
    # the top row (155,868 entries) is a whole hub row: one hub launch forked first, then 13 k_spmm launches
    assert P.compact and P.split_block0 and P.hub_rows_whole >= 1 and P.n_launch == 14
    assert spmm_mod.launches_per_hop(A, 12, d) == 13
    launches = P.launches(d)
    assert launches[0][0].n_hub == P.hub_rows_whole and launches[0][1]
    x = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device="cuda")
    panels = propagate(A, x, K)                     # through the cached plan
    torch.cuda.synchronize()
    ipn, ixn, vn = ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy()
    del ip, ix, vals
    prev = panels[0].cpu().numpy()
    want = np.empty_like(prev)
    for k in range(1, K + 1):
        oracle_mod.spmm(ipn, ixn, vn, prev, out=want)
        got = panels[k].cpu().numpy()
        bad = np.flatnonzero((got.view(np.uint32) != want.view(np.uint32)).any(axis=1))
        assert bad.size == 0, f"products hop {k}: {bad.size} of {n} rows differ (first row {int(bad[0])})"
        prev = got


@pytest.mark.timeout(600)
def test_products_wavelet_f64_blocked_two_columns_every_row(oracle_mod):
    """The fp64 filter bank bench.py --op wavelet --dtype f64 times (pygsp cheby_op's precision): the
    products-shaped Laplacian (126 M entries), d = 128, order 3, two scales, through the automatic
    column-blocked plan (16 blocks, the whole hub rows above max(2048, nnz / 4096) entries as hub
    workgroups, the lean epilogue sequence) -- every row of both scales' outputs in two columns against
    the oracle's cheby_op over the whole graph, bit for bit."""
    from srgnn import graphs, synth
    from srgnn import wavelet as W
    ip, ix, lv, n, d, lmax = graphs.build_laplacian("products", torch.device("cuda"))
    assert d == 128
    filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float64)
    S = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device="cuda").to(torch.float64)
    R = filt.apply(S)
    P = filt._plan64(d)
    assert P is not None and P.col_blocks == 16 and P.hub_rows_whole >= 1 and not P.compact
    torch.cuda.synchronize()
    cols = [0, d - 1]
    want = oracle_mod.cheby_op((ip.cpu().numpy(), ix.cpu().numpy(), lv.to(torch.float64).cpu().numpy()), filt.coeffs,
                               S[:, cols].cpu().numpy(), lmax)
    got = R[:, :, cols].cpu().numpy()
    for s in range(2):
        bad = np.flatnonzero((got[s].view(np.uint64) != want[s].view(np.uint64)).any(axis=1))
        assert bad.size == 0, f"scale {s}: {bad.size} of {n} rows differ (first row {int(bad[0])})"
    filt.drop_layouts()


def test_arxiv_k5_every_row_bit_exact(oracle_mod):
    """arxiv-shaped graph (169 K nodes, 2.48 M nonzeros), K = 5, d = 128 (BASELINE configs[1]):
    every row of every hop equals the oracle's own 5-hop chain from X, bit for bit."""
    from srgnn import graphs, synth
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import auto_col_blocks, propagate
    ip, ix, vals, n, d, K = graphs.build("arxiv", "cuda")
    assert K == 5 and d == 128
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
    assert auto_col_blocks(A, d, hops=K * 25) == 1          # X is cache-resident: one launch per hop
    x = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device="cuda")
    panels = propagate(A, x, K)
    torch.cuda.synchronize()
    want = oracle_mod.propagate(ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy(), x.cpu().numpy(), K)
    for k in range(1, K + 1):
        got = panels[k].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want[k].view(np.uint32)), f"arxiv hop {k}"


@pytest.mark.timeout(900)
def test_rmat26_d256_k8_blocked_sampled_rows_bit_exact(oracle_mod):
    """RMAT-26 (67 M nodes, 2.2e9 nonzeros: int64 row pointers), d = 256, K = 8 in bench.py's
    layout for it (two ping-pong panels, four column blocks of the native plan): every hop checked on
    1500 random rows plus the 5 longest against the oracle fed with the GPU's previous hop."""
    from srgnn import graphs, synth
    from srgnn.csr import DeviceCSR
    from srgnn.plan import cached
    from srgnn.spmm import hop, prepare
    if _free_gb() < 235:
        pytest.skip("needs a full MI355X (235 GB free)")
    ip, ix, vals, n, d, K = graphs.build("rmat26", "cuda")
    assert d == 256 and K == 8 and int(ip[-1]) > 2 ** 31
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda", validate=False)
    # bench.py's call: the operator laid out once for every warm-up and timed step's hops, by the
    # native planner (srg_plan_build): the layout the bench times, past 2^31 entries
    B = prepare(A, d, K * 25)
    assert B == 4 and cached(A, d) is not None and cached(A, d).col_blocks == 4
    rows, sub, ucols = _sample(ip, ix, vals, n, 1500, 5, seed=32)
    del ip, ix, vals
    cur = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device="cuda")
    bufs = [torch.empty_like(cur), torch.empty_like(cur)]
    for k in range(1, K + 1):
        nxt = bufs[k % 2]
        hop(A, cur, nxt, col_blocks=B)
        torch.cuda.synchronize()
        _check_rows(oracle_mod, rows, sub, ucols, cur, nxt, f"rmat26 hop {k}")
        cur = nxt


@pytest.mark.timeout(900)
def test_papers100M_blocked_hop_sampled_rows_bit_exact(oracle_mod):
    """papers100M-shaped graph (111 M nodes, 3.34e9 nonzeros), d = 128, in the four-column-block
    layout bench.py times it in (prepare -> the native plan, srg_plan_build): all K = 5 hops, each checked on 1500 random rows plus the 10
    longest against the oracle fed with the GPU's previous hop."""
    from srgnn import graphs, synth
    from srgnn.csr import DeviceCSR
    from srgnn.plan import cached
    from srgnn.spmm import hop, prepare
    if _free_gb() < 180:
        pytest.skip("needs a full MI355X (180 GB free)")
    ip, ix, vals, n, d, K = graphs.build("papers100M", "cuda")
    assert int(ip[-1]) > 2 ** 31
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda", validate=False)
    B = prepare(A, d, K * 25)          # bench.py's layout call: the native planner's plan
    assert B == 4 and cached(A, d) is not None and cached(A, d).col_blocks == 4
    rows, sub, ucols = _sample(ip, ix, vals, n, 1500, 10, seed=33)
    del ip, ix, vals
    cur = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device="cuda")
    nxt = torch.empty_like(cur)
    assert K == 5
    for k in range(1, K + 1):
        hop(A, cur, nxt, col_blocks=B)
        torch.cuda.synchronize()
        _check_rows(oracle_mod, rows, sub, ucols, cur, nxt, f"papers100M hop {k}")
        cur, nxt = nxt, cur


@pytest.mark.timeout(1100)
def test_papers100M_p8_partition_sampled_rows_bit_exact(oracle_mod):
    """VERDICT r5 "do this" 8: the halo partition bench.py runs at N = 8 (HaloPartitionedOperator, 6 row
    chunks + the hub group, ghost rows at the automatic cap, each rank's local operator with its
    columns remapped into [own | received | ghost] panel rows) on the papers100M-shaped graph (111 M
    rows, 3.34e9 entries), all 8 ranks' shares built on ONE GPU one after another.  Each rank's panel
    gets its own rows and its halo from the global previous hop (the rows the exchange would deliver,
    at the positions the plan assigns them), runs its local hop (compute: chunks, hub group on the side
    stream, ghost rows), and hands its own rows back.  Two hops; every rank's rows of every hop are
    checked on sampled rows (the 16 longest of the graph and ~300 random rows per rank) against the
    oracle fed with the previous hop, bit for bit -- so the first real 8-GPU run is not the first time
    the partition meets 111 M rows."""
    from srgnn import graphs, synth
    from srgnn.dist import HaloPartitionedOperator
    from srgnn.spmm import gather_rows
    if _free_gb() < 220:
        pytest.skip("needs a full MI355X (220 GB free)")
    ip, ix, vals, n, d, K = graphs.build("papers100M", "cuda")
    P, hops = 8, 2
    rows, sub, ucols = _sample(ip, ix, vals, n, 300 * P, 16, seed=35)
    from conftest import progress
    shares = []
    for q in range(P):
        shares.append(HaloPartitionedOperator(ip, ix, vals, n, chunks=6, device="cuda", rank=q, world=P))
        torch.cuda.synchronize()
        progress(f"papers100M P=8: share {q} built (rows {shares[-1].rows}, halo {shares[-1].halo})")
    assert shares[0].starts[-1] == n and sum(s.rows for s in shares) == n
    assert any(s.n_ghost for s in shares) and any(s.views[s.C][3] for s in shares)   # ghost rows, hub rows
    del ip, ix, vals
    torch.cuda.empty_cache()
    prev = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device="cuda")
    for k in range(1, hops + 1):
        last = k == hops
        nxt = None if last else torch.empty_like(prev)
        got = torch.empty((rows.numel(), d), dtype=torch.float32, device="cuda")
        for q, s in enumerate(shares):
            src, dst = s.new_panel(d), s.new_panel(d)
            src[: s.rows].copy_(prev[s.r0:s.r1])
            if s.halo:
                gather_rows(prev, s.halo_ids(), out=src[s.rows:s.rows + s.halo])
            s.compute(src, dst)
            mine = (rows >= s.r0) & (rows < s.r1)
            got[mine] = dst[rows[mine] - s.r0]
            if not last:
                nxt[s.r0:s.r1].copy_(dst[: s.rows])
            del src, dst
        torch.cuda.synchronize()
        progress(f"papers100M P=8: hop {k} computed on every rank")
        want = oracle_mod.spmm(*sub, prev[ucols].cpu().numpy())
        have = got.cpu().numpy()
        bad = np.flatnonzero((have.view(np.uint32) != want.view(np.uint32)).any(axis=1))
        per_rank = [int(((rows >= s.r0) & (rows < s.r1)).sum()) for s in shares]
        assert min(per_rank) > 100, per_rank
        assert bad.size == 0, f"papers100M P=8 hop {k}: {bad.size} of {rows.numel()} sampled rows differ " \
                              f"(first row {int(rows[bad[0]])})"
        del prev
        prev = nxt
        torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_rmat26_wavelet_orders_sampled_rows(oracle_mod):
    """The RMAT-26 heat-wavelet filter bank (bench.py --op wavelet): L and F = (2/a1)(L - a2 I) in
    four column blocks, a 64-column block of the panel, Chebyshev order 3, two scales, fp32.  Per
    order, on 1500 random rows plus the 5 longest:
      * the SpMM equals the oracle's fp32 chain bit for bit (fed with the GPU's previous T);
      * T_{k+1} and every scale's output R agree with the fp64 evaluation of the same step (pygsp's
        arithmetic, base_model.py:236-265) within the fp32 forward-error bound of the step,
        gamma_{deg+c} * (sum of |terms|), gamma_n = n u / (1 - n u), u = 2^-24, element by element;
      * rows of degree <= 64 (the bulk of the graph) within 1e-5 normwise.
    Rows with ~10^5-10^6 nonzeros accumulate fp32 rounding over their chains (the fp64 entry,
    srg_cheby_step_f64, is the reference's precision at twice the bytes)."""
    from srgnn import _lib, graphs, synth
    from srgnn import wavelet as W
    from srgnn.spmm import hop
    if _free_gb() < 200:
        pytest.skip("needs a full MI355X (200 GB free)")
    ip, ix, lv, n, d, lmax = graphs.build_laplacian("rmat26", "cuda")
    filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=3, lmax=lmax, dtype=torch.float32)
    cb = 64
    B = filt.prepare_column_blocks(cb, hops=3 * 4 * 2)
    assert B == 4
    rows, subL, ucols = _sample(ip, ix, filt.lvals, n, 1500, 5, seed=34)
    deg = torch.from_numpy(np.diff(subL[0])).cuda().double().unsqueeze(1)
    subF = (subL[0], subL[1], filt.fvals[_positions(ip, rows)].cpu().numpy())
    lv64 = lv.to(torch.float64)[_positions(ip, rows)].cpu().numpy()
    f64 = ((2.0 / filt.a1) * np.where(ucols.cpu().numpy()[subL[1]] == np.repeat(rows.cpu().numpy(), np.diff(subL[0])),
                                      lv64 - filt.a2, lv64))
    del ip, ix, lv
    S = synth.uniform_features_t(n, cb, seed=synth.FEATURE_SEED, device="cuda")
    Lm, Fm = filt._csr(filt.lvals), filt._csr(filt.fvals)
    T = [S]

    def prod64(vals, P, absolute=False):
        x = P[ucols].double().cpu().numpy()
        out = _spmm64(subL[0], subL[1], np.abs(vals) if absolute else vals, np.abs(x) if absolute else x)
        return torch.from_numpy(out).cuda()
    # order 1: y = L S (checked), then the INIT_T epilogue turns it into T1 = (y - a2 S) / a1 in place
    y = torch.empty_like(S)
    hop(Lm, S, y, col_blocks=B)
    torch.cuda.synchronize()
    _check_rows(oracle_mod, rows, subL, ucols, S, y, "rmat26 wavelet L @ S")
    _lib.call(S.device, "srg_cheby_epilogue_f32", y.data_ptr(), cb, S.data_ptr(), cb, None, cb, n, cb,
              _lib.SRG_CHEBY_INIT_T, filt.a1, filt.a2, None, None, 2, None, cb, n * cb, _lib.stream(S.device))
    torch.cuda.synchronize()
    s_abs = filt.a2 * S[rows].double().abs()
    _within_fp32(y[rows].double(), (prod64(lv64, S) - filt.a2 * S[rows].double()) / filt.a1,
                 (prod64(lv64, S, True) + s_abs) / filt.a1, deg + 3, deg, "T1")
    T.append(y)
    for k in (2, 3):
        y = torch.empty_like(S)
        hop(Fm, T[-1], y, col_blocks=B)
        torch.cuda.synchronize()
        _check_rows(oracle_mod, rows, subF, ucols, T[-1], y, f"rmat26 wavelet F @ T{k - 1}")
        y.sub_(T[-2])                        # the STEP epilogue's T_{k+1} = F T_k - T_{k-1} (fp32)
        _within_fp32(y[rows].double(), prod64(f64, T[-1]) - T[-2][rows].double(),
                     prod64(f64, T[-1], True) + T[-2][rows].double().abs(), deg + 2, deg, f"T{k}")
        T.append(y)
    # R from the lean split path (what the bench times) against the fp64 sums of the GPU's T's
    R = filt.apply(S, col_block=cb)
    torch.cuda.synchronize()
    c = filt.coeffs
    for s in range(2):
        terms = [(c[s, 0] / 2) * T[0][rows].double()] + [c[s, k] * T[k][rows].double() for k in (1, 2, 3)]
        _within_fp32(R[s][rows].double(), sum(terms), sum(t.abs() for t in terms), torch.full_like(deg, 8.0), deg,
                     f"R scale {s}")


def _within_fp32(got, want, abs_terms, n_ops, deg, what, tol=1e-5, bulk_degree=64):
    """Element-wise |got - want| <= gamma_{n_ops} * abs_terms (the fp32 forward-error bound of a
    chain of n_ops roundings over terms whose magnitudes sum to abs_terms), and rows of degree <=
    bulk_degree within `tol` normwise."""
    u = 2.0 ** -24
    gamma = n_ops * u / (1 - n_ops * u)
    err = (got - want).abs()
    over = err > gamma * abs_terms
    assert not bool(over.any()), f"{what}: {int(over.any(dim=1).sum())} rows beyond the fp32 error bound, " \
                                 f"worst ratio {float((err / (gamma * abs_terms).clamp_min(1e-300)).max()):.3g}"
    bulk = deg.squeeze(1) <= bulk_degree
    rel = (got - want).norm(dim=1) / want.norm(dim=1).clamp_min(1e-30)
    worst = float(rel[bulk].max()) if bool(bulk.any()) else 0.0
    assert worst <= tol, f"{what}: rows of degree <= {bulk_degree}: max normwise relative error {worst:.3g} > {tol}"


def _positions(ip, rows):
    deg = ip[1:] - ip[:-1]
    beg, cnt = ip[rows], deg[rows]
    tot = int(cnt.sum())
    return torch.repeat_interleave(beg - torch.cumsum(cnt, 0) + cnt, cnt, output_size=tot) + \
        torch.arange(tot, device=ip.device)


def _spmm64(ip, ix, v, X):
    """fp64 product of the sampled sub-CSR (numpy; scipy's order: products added left to right)."""
    import scipy.sparse as sp
    A = sp.csr_matrix((v, ix, ip), shape=(ip.size - 1, X.shape[0]))
    return np.asarray(A @ X)




# ------------------------------------------------------------------------------------------------
# int64 offsets: EVERY row of a hop whose entry offsets pass 2^31, against a closed form
# ------------------------------------------------------------------------------------------------
_I64_N = 1 << 25


def _closed_form_csr(N=_I64_N):
    """A CSR with N rows of 33..120 entries (nnz ~2.57e9 > 2^31: the entry offsets of the later rows,
    their column-block span pointers and their compact-copy / slot-span positions all need 64 bits).
    Row r's entries are the arithmetic progression c_j = start_r + j * step_r (sorted, spread over
    the column blocks), with values ((r + j) % 3) + 1; every quantity is an integer, so any chain
    order gives the same exactly representable sums."""
    dev = "cuda"
    r = torch.arange(N, device=dev, dtype=torch.int64)
    lens = 33 + (r * 40503 + 12345) % 88
    steps = 1 + (r * 69069 + 7) % (N // 256)
    starts = ((r * 2654435761) % 4294967291) % (N - lens * steps)
    ip = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=ip[1:])
    nnz = int(ip[-1])
    ix = torch.empty(nnz, dtype=torch.int32, device=dev)
    vals = torch.empty(nnz, dtype=torch.float32, device=dev)
    for r0 in range(0, N, 1 << 20):
        r1 = min(N, r0 + (1 << 20))
        e0, e1 = int(ip[r0]), int(ip[r1])
        rows = torch.repeat_interleave(r[r0:r1], lens[r0:r1], output_size=e1 - e0)
        j = torch.arange(e0, e1, device=dev, dtype=torch.int64) - ip[rows]
        ix[e0:e1] = (starts[rows] + j * steps[rows]).to(torch.int32)
        vals[e0:e1] = ((rows + j) % 3 + 1).to(torch.float32)
    return ip, ix, vals, lens


def _closed_form_x(N, d):
    c = torch.arange(N, device="cuda", dtype=torch.int64).unsqueeze(1) * 3 + torch.arange(d, device="cuda")
    return (c % 5 - 2).to(torch.float32)


@pytest.fixture(scope="module")
def int64_operator():
    from srgnn.csr import DeviceCSR
    if _free_gb() < 120:
        pytest.skip("needs a full MI355X (120 GB free)")
    ip, ix, vals, lens = _closed_form_csr()
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=_I64_N, device="cuda")
    yield A, lens
    A.drop_blocks()
    del A, ip, ix, vals
    torch.cuda.empty_cache()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("d", [4, 64, 128])
def test_int64_offsets_every_row_closed_form(int64_operator, d):
    """VERDICT r4 "weak" #1 / r5 "do this" 2: past 2^31 entries only sampled rows were checked, and
    then only in the torch-built twin of the layout.  Here nnz ~2.57e9 and a hop through the NATIVE
    plan (srg_plan_build: k_plan_splits / k_plan_items / k_plan_spans / k_plan_copy and the slot-span
    and copy positions they write) in the bench's column-block layout -- 4 compact blocks in launch
    order, block 0 in two launches, slot spans, hub / slice / packed or narrow rows -- is compared on
    EVERY row with the exact integer result (int64 slips in span, slot or copy offsets would move
    whole ranges of rows)."""
    from srgnn.plan import NativePlan
    A, lens = int64_operator
    N = _I64_N
    assert A.nnz > 2 ** 31
    P = NativePlan(A, d, hops=8, col_blocks=4, compact=True, split_block0=True)
    assert P.col_blocks == 4 and P.compact and P.split_block0 and P.n_launch == 5
    X = _closed_form_x(N, d)
    Y = torch.full((N, d), float("nan"), device="cuda")
    P.hop(X, Y, d)
    P.close()
    want = torch.zeros_like(Y)
    ip = A.indptr
    r = torch.arange(N, device="cuda", dtype=torch.int64)
    step = max(1, (1 << 23) // (d * 80))
    for r0 in range(0, N, step):
        r1 = min(N, r0 + step)
        e0, e1 = int(ip[r0]), int(ip[r1])
        rows = torch.repeat_interleave(r[r0:r1] - r0, lens[r0:r1], output_size=e1 - e0)
        contrib = A.values[e0:e1].unsqueeze(1) * X[A.indices[e0:e1].long()]
        want[r0:r1].index_add_(0, rows, contrib)
    torch.cuda.synchronize()
    bad = torch.nonzero((Y != want).any(dim=1)).squeeze(1)
    assert bad.numel() == 0, f"d={d}: {bad.numel()} of {N} rows differ (first row {int(bad[0])}, " \
                             f"entries from {int(ip[bad[0]])})"
