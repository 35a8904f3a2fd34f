"""The native one-GPU planner (srg_plan_build / srg_plan_propagate_f32, csrc/srg_plan.hip) against the
test-side torch restatement of the same layout (tests/plan_layout_ref.py: column blocks, compact copies,
block 0's split, the hop plan's flags) launch by launch -- schedules, hub / slice-wave counts, flags, the
entries every slot span points at -- and its hops against the reference's (golden fixtures) bit for bit."""
import ctypes

import numpy as np
import pytest
import torch

import golden_cases as G

pytestmark = pytest.mark.gpu

_hip = None


def _read(ptr, count, dtype):
    """A device array the library owns, copied into a torch tensor (hipMemcpy device to device)."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = torch.empty(int(count), dtype=dtype, device="cuda")
    if count:
        torch.cuda.synchronize()
        assert _hip.hipMemcpy(out.data_ptr(), ptr, out.numel() * out.element_size(), 3) == 0
    return out


def _power_law(n=40000, hubs=(30000, 9000), seed=3, unsorted_rows=0):
    rng = np.random.default_rng(seed)
    deg = np.minimum(rng.zipf(1.9, n), 1500).astype(np.int64)
    deg[rng.integers(0, n, 200)] = 0
    for i, h in enumerate(hubs):
        deg[17 + 1000 * i] = h
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) if k else np.zeros(0, np.int64)
                         for k in deg]).astype(np.int32)
    for r in range(unsorted_rows):
        a, b = ip[100 + r], ip[101 + r]
        ix[a:b] = ix[a:b][::-1]
    v = (rng.standard_normal(ix.size) * 0.3).astype(np.float32)
    return ip, ix, v, n


def _csr(ip, ix, v, n):
    from srgnn.csr import DeviceCSR
    return DeviceCSR.from_tensors(ip, ix, v, n_cols=n, device="cuda")


def _spans(beg, end):
    """Flattened entry positions of the spans [beg[i], end[i]) (int64 tensors), in slot order."""
    lens = (end - beg).to(torch.int64)
    tot = int(lens.sum().item())
    start = torch.repeat_interleave(beg.to(torch.int64), lens, output_size=tot)
    off = torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens, output_size=tot)
    return start + torch.arange(tot, dtype=torch.int64, device=beg.device) - off


def _python_layout(A, d, B, compact, split, monkeypatch=None):
    """The restatement's launches for a forced layout: [(operator, flags)], join (split None: the
    planner's automatic choice for these small panels, split)."""
    import plan_layout_ref as R
    if B > 1:
        plan, join = R.hop_plan(A, d, B, compact, True if split is None else bool(split))
        return [(Ab, f) for Ab, f, _ in plan], join
    if compact:
        return [(R.schedule_ordered(A), 0)], False
    return [(A, 0)], False


def _check_layout(A, P, d, py, join_py):
    """The native plan's launches == the torch formulation's, entry for entry."""
    launches = P.launches(d)
    assert len(launches) == len(py)
    for (L, join), (Ab, f) in zip(launches, py):
        assert join == join_py
        assert L.n_rows == Ab.n_rows
        assert L.n_hub == Ab.n_hub and L.n_heavy == Ab.heavy(d)
        assert L.flags == f, (hex(L.flags), hex(f))
        if not L.n_rows:
            continue
        order = _read(L.row_order, L.n_rows, torch.int32)
        assert torch.equal(order, Ab.order)
        o = Ab.order.to(torch.int64)
        if Ab.is_span:
            pb, pe = Ab.indptr[o], Ab.row_end[o]
        else:
            pb, pe = Ab.indptr[o], Ab.indptr[o + 1]
        if L.slot_beg:
            nb, ne = _read(L.slot_beg, L.n_rows, torch.int64), _read(L.slot_end, L.n_rows, torch.int64)
        else:
            assert not Ab.is_span and not L.row_end
            ip = _read(L.row_beg, A.n_rows + 1, torch.int64)
            nb, ne = ip[o], ip[o + 1]
        assert torch.equal(ne - nb, pe - pb)
        pos_n, pos_p = _spans(nb, ne), _spans(pb, pe)
        nnz = int(A.indices.numel())
        ix_n = _read(L.indices, nnz, torch.int32)
        v_n = _read(L.values, nnz, torch.float32)
        assert torch.equal(ix_n[pos_n], Ab.indices[pos_p])
        assert torch.equal(v_n[pos_n].view(torch.int32), Ab.values[pos_p].view(torch.int32))
        if L.row_end:
            # the slice / hub waves read the row-indexed spans: the same spans
            rb = _read(L.row_beg, A.n_rows, torch.int64)[o]
            re = _read(L.row_end, A.n_rows, torch.int64)[o]
            assert torch.equal(rb, nb) and torch.equal(re, ne)


LAYOUTS = [(1, False, None), (1, True, None), (3, False, True), (3, True, True), (3, False, False),
           (6, True, True), (6, True, False), (2, False, True)]


@pytest.mark.parametrize("d", [16, 64, 128])
@pytest.mark.parametrize("B,compact,split", LAYOUTS)
def test_native_layout_matches_torch_formulation(monkeypatch, B, compact, split, d):
    from srgnn.plan import NativePlan
    ip, ix, v, n = _power_law(unsorted_rows=3)
    A = _csr(ip, ix, v, n)
    P = NativePlan(A, d, hops=3, col_blocks=B, compact=compact, split_block0=split)
    assert P.col_blocks == B and P.compact == compact
    # B launches, one more for block 0's split, one more for the whole hub rows (blocked plans)
    assert P.n_launch == (B + 1 if (B > 1 and split) else B) + (1 if B > 1 else 0)
    # the hops first (a compact plan at 64 / 128 columns has row-indexed spans for its hub and
    # slice-wave rows only until srg_plan_launch completes them): the one-launch hops, bit for bit
    from srgnn.spmm import spmm
    X = torch.randn(n, d, device="cuda")
    panels = [X] + [torch.empty_like(X) for _ in range(3)]
    P.propagate(panels, X.stride(0), d, 3)
    ref = X
    for k in range(1, 4):
        ref = spmm(A, ref)
        assert torch.equal(panels[k].view(torch.int32), ref.view(torch.int32)), k
    py, join = _python_layout(A, d, B, compact, split, monkeypatch)
    _check_layout(A, P, d, py, join)
    if B > 1:
        # the two hubs are longer than max(2048, nnz / 1024): the whole hub rows' launch, first, forked
        assert P.hub_rows_whole == 2 and not P.hub_chain and join
        L0, _ = P.launches(d)[0]
        assert L0.n_rows == L0.n_hub == 2 and L0.n_heavy == 0
    P.close()


@pytest.mark.parametrize("thresholds", [(40, 400), (-1, 3000), (200, -1), (0, 0)])
@pytest.mark.parametrize("B,compact,split", [(1, False, None), (1, True, None), (3, True, True), (3, False, False)])
def test_native_layout_with_explicit_thresholds(monkeypatch, B, compact, split, thresholds):
    """An operator built with its own heavy / hub thresholds (negative: no such rows): the native plan
    schedules every launch with them, as the torch formulation's blocks do; the hops bit for bit."""
    from srgnn.csr import DeviceCSR
    from srgnn.plan import NativePlan
    from srgnn.spmm import spmm
    ip, ix, v, n = _power_law(seed=21, unsorted_rows=2)
    heavy_t, hub_t = thresholds
    A = DeviceCSR.from_tensors(ip, ix, v, n_cols=n, heavy_threshold=heavy_t, hub_threshold=hub_t, device="cuda")
    for d in (16, 64):
        P = NativePlan(A, d, hops=3, col_blocks=B, compact=compact, split_block0=split)
        X = torch.randn(n, d, device="cuda")
        panels = [X] + [torch.empty_like(X) for _ in range(2)]
        P.propagate(panels, d, d, 2)
        assert torch.equal(panels[2].view(torch.int32), spmm(A, spmm(A, X)).view(torch.int32))
        py, join = _python_layout(A, d, B, compact, split, monkeypatch)
        _check_layout(A, P, d, py, join)
        P.close()


@pytest.mark.parametrize("d_run", [8, 36, 64, 256])
def test_compact_plan_other_widths(d_run):
    """A compact plan built for 128 columns keeps row-indexed spans for its hub and slice-wave rows
    only; a run over a width whose light rows read them (not 64 / 128 / 256) completes them first.
    Every width: the one-launch hops, bit for bit."""
    from srgnn.plan import NativePlan
    from srgnn.spmm import spmm
    ip, ix, v, n = _power_law(seed=5)
    A = _csr(ip, ix, v, n)
    P = NativePlan(A, 128, hops=2, col_blocks=4, compact=True)
    X = torch.randn(n, d_run, device="cuda")
    panels = [X, torch.empty_like(X), torch.empty_like(X)]
    P.propagate(panels, d_run, d_run, 2)
    ref = spmm(A, spmm(A, X))
    assert torch.equal(panels[2].view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("B,compact,split", LAYOUTS)
@pytest.mark.parametrize("name", G.names("norm"))
def test_native_plan_bit_exact_vs_reference(name, B, compact, split):
    from srgnn.plan import NativePlan
    c = G.Case(name)
    ip, ix, v = c.ahat()
    A = _csr(ip, ix, v, c.n)
    X = torch.from_numpy(np.ascontiguousarray(c.x())).cuda()
    d = X.shape[1]
    P = NativePlan(A, d, hops=c.k, col_blocks=B, compact=compact, split_block0=split)
    panels = [X] + [torch.empty_like(X) for _ in range(c.k)]
    P.propagate(panels, X.stride(0), d, c.k)
    torch.cuda.synchronize()
    for k in range(1, c.k + 1):
        c.check_hop(k, panels[k].cpu().numpy())


@pytest.mark.parametrize("name", G.names("raw"))
def test_native_plan_unsorted_rows_bit_exact(name):
    """Raw operators (unsorted rows, duplicates): the spans still partition each row in CSR order."""
    from srgnn.csr import DeviceCSR
    from srgnn.plan import NativePlan
    c = G.Case(name)
    a = c.adj()
    if a.shape[0] != a.shape[1]:
        pytest.skip("a plan takes a square operator")
    A = DeviceCSR.from_tensors(a.indptr, a.indices, a.data.astype(np.float32), n_cols=c.n, device="cuda")
    X = torch.from_numpy(np.ascontiguousarray(c.x())).cuda()
    d = X.shape[1]
    for B, compact in ((3, False), (3, True), (1, True)):
        P = NativePlan(A, d, hops=1, col_blocks=B, compact=compact)
        Y = torch.empty_like(X)
        P.propagate([X, Y], X.stride(0), d, 1)
        torch.cuda.synchronize()
        c.check_hop(1, Y.cpu().numpy())


def test_khop_without_schedule_plans_itself():
    """srg_propagate_khop_f32 given no schedule builds a plan for its hops (and frees it after them):
    the same bits as the scheduled one-launch hops."""
    from srgnn import _lib
    ip, ix, v, n = _power_law(seed=7)
    A = _csr(ip, ix, v, n)
    for d in (8, 64):
        X = torch.randn(n, d, device="cuda")
        outs = []
        for sched in (True, False):
            panels = [X] + [torch.empty_like(X) for _ in range(4)]
            arr = (ctypes.c_void_p * 5)(*[p.data_ptr() for p in panels])
            _lib.call(X.device, "srg_propagate_khop_f32", A.indptr.data_ptr(), A.indices.data_ptr(),
                      A.values.data_ptr(), n, A.order.data_ptr() if sched else None, A.n_hub if sched else 0,
                      A.heavy(d) if sched else 0, arr, d, d, 4, 0, _lib.stream(X.device))
            outs.append(panels)
        torch.cuda.synchronize()
        for k in range(1, 5):
            assert torch.equal(outs[0][k].view(torch.int32), outs[1][k].view(torch.int32))


def test_khop_without_schedule_fast_stays_exact():
    """srg_propagate_khop_f32 without a schedule never had hub rows, so SRG_SPMM_FAST (which
    re-associates hub rows only) changed no bit; its implicit plan is built without hub rows under
    FAST, so the call stays exact -- bitwise the unscheduled exact call, on a graph with long rows."""
    from srgnn import _lib
    ip, ix, v, n = _power_law(seed=23)
    A = _csr(ip, ix, v, n)
    X = torch.randn(n, 64, device="cuda")
    outs = []
    for flags in (0, _lib.SRG_SPMM_FAST):
        panels = [X] + [torch.empty_like(X) for _ in range(3)]
        arr = (ctypes.c_void_p * 4)(*[p.data_ptr() for p in panels])
        _lib.call(X.device, "srg_propagate_khop_f32", A.indptr.data_ptr(), A.indices.data_ptr(), A.values.data_ptr(),
                  n, None, 0, 0, arr, 64, 64, 3, flags, _lib.stream(X.device))
        outs.append(panels)
    torch.cuda.synchronize()
    for k in range(1, 4):
        assert torch.equal(outs[0][k].view(torch.int32), outs[1][k].view(torch.int32)), k


def test_native_plan_edge_cases():
    """No entries; every row whole (the cut launches are empty); a hub in one block only (no chain)."""
    from srgnn.plan import NativePlan
    from srgnn.spmm import spmm
    # no entries: one empty launch, zero output
    ip = np.zeros(6, np.int64)
    A = _csr(ip, np.zeros(0, np.int32), np.zeros(0, np.float32), 5)
    P = NativePlan(A, 8, hops=20, col_blocks=4)
    assert P.col_blocks == 1 and P.n_launch == 1
    X = torch.randn(5, 8, device="cuda")
    Y = torch.full_like(X, 7.0)
    P.propagate([X, Y], 8, 8, 1)
    assert torch.equal(Y, torch.zeros_like(Y))
    # no rows at all: a plan with no launches, every call a no-op
    A0 = _csr(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.float32), 0)
    P0 = NativePlan(A0, 16, hops=20, col_blocks=3)
    assert P0.n_launch == 0 and P0.device_bytes == 0
    E = torch.zeros(0, 16, device="cuda")
    P0.propagate([E, torch.zeros(0, 16, device="cuda")], 16, 16, 1)
    # more blocks than rows and columns: empty spans everywhere but the hops are exact
    ipt = np.array([0, 2, 3, 3, 6], np.int64)
    ixt = np.array([0, 3, 1, 0, 1, 2], np.int32)
    At = _csr(ipt, ixt, np.arange(1, 7, dtype=np.float32), 4)
    Xt = torch.randn(4, 64, device="cuda")
    for compact in (False, True):
        Pt = NativePlan(At, 64, hops=3, col_blocks=9, compact=compact, split_block0=True)
        pt = [Xt, torch.empty_like(Xt), torch.empty_like(Xt)]
        Pt.propagate(pt, 64, 64, 2)
        assert torch.equal(pt[2].view(torch.int32), spmm(At, spmm(At, Xt)).view(torch.int32))
    # every row short: block 0 computes all of them, the later launches schedule no row
    rng = np.random.default_rng(1)
    n = 3000
    deg = rng.integers(0, 40, n)
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) for k in deg]).astype(np.int32)
    A = _csr(ip, ix, rng.standard_normal(ix.size).astype(np.float32), n)
    X = torch.randn(n, 32, device="cuda")
    for compact in (False, True):
        P = NativePlan(A, 32, hops=2, col_blocks=4, compact=compact, split_block0=True)
        Ls = P.launches(32)
        assert [L.n_rows for L, _ in Ls] == [0, n, 0, 0, 0]
        panels = [X, torch.empty_like(X), torch.empty_like(X)]
        P.propagate(panels, 32, 32, 2)
        ref = spmm(A, spmm(A, X))
        assert torch.equal(panels[2].view(torch.int32), ref.view(torch.int32))
    # a hub row whose entries all lie in block 0: block 0's launch has a hub the others lack -> no chain
    # (an explicit hub threshold: automatic ones would make this row a whole hub row, below)
    from srgnn.csr import DeviceCSR
    ip2, ix2, v2, n2 = _power_law(hubs=(), seed=11)
    deg = np.diff(ip2)
    deg[5] = 6000
    ip2 = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    rows = [np.sort(rng.choice(n2, k, replace=False)) if r != 5 else np.arange(6000) for r, k in enumerate(deg)]
    ix2 = np.concatenate(rows).astype(np.int32)
    vv2 = rng.standard_normal(ix2.size).astype(np.float32)
    # automatic: the 6000-entry row is a whole hub row (> max(2048, nnz / 1024)): its own launch, first
    Aa = _csr(ip2, ix2, vv2, n2)
    Pa = NativePlan(Aa, 64, hops=2, col_blocks=4, split_block0=True)
    assert Pa.hub_rows_whole == 1 and not Pa.hub_chain and Pa.n_launch == 6
    A = DeviceCSR.from_tensors(ip2, ix2, vv2, n_cols=n2, hub_threshold=2048, device="cuda")
    P = NativePlan(A, 64, hops=2, col_blocks=4, split_block0=True)
    assert not P.hub_chain and P.hub_rows_whole == 0
    Ls = P.launches(64)
    assert Ls[0][0].n_hub == 1 and all(L.n_hub == 0 for L, _ in Ls[2:])
    X = torch.randn(n2, 64, device="cuda")
    for plan in (P, Pa):
        panels = [X, torch.empty_like(X), torch.empty_like(X)]
        plan.propagate(panels, 64, 64, 2)
        ref = spmm(A, spmm(A, X))
        assert torch.equal(panels[2].view(torch.int32), ref.view(torch.int32))


def test_native_plan_automatic_choices_match_prepare(monkeypatch):
    """At a size where the automatic rules cut (a 600 MB panel): prepare() lays the operator out with the
    native plan (12 compact blocks, block 0 split, 13 launches, launch for launch the test restatement's
    layout); propagate() runs through it."""
    from srgnn import spmm as S
    from srgnn.plan import NativePlan, cached
    rng = np.random.default_rng(2)
    n = 1_200_000
    deg = np.minimum(rng.zipf(2.0, n), 2000).astype(np.int64) + 3
    deg[12345] = 60000
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    # sorted ids per row without a per-row Python loop: sort (row, id) keys
    rows = np.repeat(np.arange(n, dtype=np.int64), deg)
    ids = rng.integers(0, n, int(ip[-1]), dtype=np.int64)
    ix = (np.sort(rows * n + ids) - rows * n).astype(np.int32)
    A = _csr(ip, ix, np.ones(ix.size, np.float32), n)
    d = 128
    B = S.prepare(A, d, hops=40)
    P = cached(A, d)
    assert P is not None and B == P.col_blocks == 12 and P.split_block0 and P.compact
    assert S.launches_per_hop(A, B, d) == B + 1
    # the test restatement of the same layout on a second operator over the same arrays
    import plan_layout_ref as R
    from srgnn.csr import DeviceCSR
    A2 = DeviceCSR.from_tensors(A.indptr, A.indices, A.values, n_cols=n, device="cuda")
    plan_py, join = R.hop_plan(A2, d, B, compact=True, split=True)
    _check_layout(A, P, d, [(Ab, f) for Ab, f, _ in plan_py], join)
    X = torch.randn(n, d, device="cuda")
    out = S.propagate(A, X, 1, col_blocks=B)
    ref = S.spmm(A, X)
    assert torch.equal(out[1].view(torch.int32), ref.view(torch.int32))
    assert isinstance(P, NativePlan) and P.device_bytes > A.indices.numel() * 8


def test_repeated_plan_calls_replay_a_graph_bitwise():
    """srg_plan_propagate_f32 repeated with the same arguments on a non-null stream replays the K hops
    as a HIP graph from the second call on: every call's hops stay the one-launch hops, bit for bit,
    for one launch per hop and for column blocks with the hub chain; a changed panel list re-plans."""
    from srgnn.plan import NativePlan
    from srgnn.spmm import spmm
    ip, ix, v, n = _power_law(seed=9)
    A = _csr(ip, ix, v, n)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for B in (1, 3):
            P = NativePlan(A, 64, hops=4, col_blocks=B)
            X = torch.randn(n, 64, device="cuda")
            ref = [X]
            for _ in range(4):
                ref.append(spmm(A, ref[-1]))
            for trial in range(2):
                panels = [X] + [torch.empty_like(X) for _ in range(4)]
                for _ in range(4):
                    for p in panels[1:]:
                        p.fill_(float("nan"))
                    P.propagate(panels, 64, 64, 4)
                    st.synchronize()
                    for k in range(1, 5):
                        assert torch.equal(panels[k].view(torch.int32), ref[k].view(torch.int32)), (B, trial, k)
            P.close()


AGG_LAYOUTS = [(1, False, None), (1, True, None), (3, True, True), (3, False, True), (3, True, False),
               (6, True, True)]


@pytest.mark.parametrize("B,compact,split", AGG_LAYOUTS)
@pytest.mark.parametrize("d", [64, 128, 36])
def test_plan_hop_strided_and_aggregating(B, compact, split, d):
    """srg_plan_hop_f32: one hop between panels of different leading dimensions (X a column slice of
    a wider panel), bitwise the one-launch hop; with the aggregation epilogue (INIT, then ADD) bitwise
    the hop followed by srg_hop_accumulate_f32 -- fused where block 0 is split or the hop is one launch,
    a separate pass where block 0 is one launch (split False)."""
    from srgnn import _lib
    from srgnn.plan import NativePlan
    from srgnn.spmm import spmm
    ip, ix, v, n = _power_law(seed=13, unsorted_rows=2)
    A = _csr(ip, ix, v, n)
    P = NativePlan(A, d, hops=8, col_blocks=B, compact=compact, split_block0=split)
    wide = torch.randn(n, d + 40, device="cuda")
    X = wide[:, 8:8 + d]                       # ld d + 40, 32-byte offset
    ref = spmm(A, X.contiguous())
    Y = torch.full((n, d), float("nan"), device="cuda")
    P.hop(X, Y, d)
    assert torch.equal(Y.view(torch.int32), ref.view(torch.int32))
    # the aggregation epilogue: agg = 0 + w * Y, then agg += w2 * Y2
    agg = torch.full((n, d + 4), float("nan"), device="cuda")[:, :d]
    ref_agg = torch.empty((n, d), device="cuda")
    st = _lib.stream(X.device)
    Y1 = torch.empty((n, d), device="cuda")
    P.hop(X, Y1, d, 0, agg, 0.375, True)
    _lib.call(X.device, "srg_hop_accumulate_f32", ref_agg.data_ptr(), d, ref.data_ptr(), d, n, d, 0.375,
              _lib.SRG_ACC_INIT, st)
    assert torch.equal(Y1.view(torch.int32), ref.view(torch.int32))
    assert torch.equal(agg.view(torch.int32), ref_agg.view(torch.int32))
    Y2 = torch.empty((n, d), device="cuda")
    P.hop(Y1, Y2, d, _lib.SRG_SPMM_NT_STORE, agg, -1.25, False)
    ref2 = spmm(A, ref)
    _lib.call(X.device, "srg_hop_accumulate_f32", ref_agg.data_ptr(), d, ref2.data_ptr(), d, n, d, -1.25,
              _lib.SRG_ACC_ADD, st)
    assert torch.equal(Y2.view(torch.int32), ref2.view(torch.int32))
    assert torch.equal(agg.view(torch.int32), ref_agg.view(torch.int32))
    # argument checks before any launch
    for bad in (dict(flags=_lib.SRG_SPMM_ACCUMULATE), dict(flags=_lib.SRG_SPMM_FAST, agg=agg)):
        with pytest.raises(_lib.SrgError):
            P.hop(X, Y, d, bad.get("flags", 0), bad.get("agg"), 1.0, True)
    with pytest.raises(_lib.SrgError):
        P.hop(Y, Y, d)


def test_aggregation_loop_runs_the_native_plan(monkeypatch):
    """spmm.prepare lays the operator out with the native plan; propagate_aggregate's fused hops then
    run through it (srg_plan_hop_f32, the aggregation in the epilogue): the same bits as the
    aggregation over one-launch hops."""
    from srgnn.aggregate import combine_plan, combine_steps, propagate_aggregate
    from srgnn.plan import cached
    ip, ix, v, n = _power_law(seed=17)
    d, K = 128, 6

    class _Msg:
        aggr_type, start, end, combination_type, alpha, weight_list = "simple_weighted", 0, K + 1, "alpha", 0.15, None
    steps = combine_steps(*combine_plan(_Msg(), K + 1))
    X = torch.randn(n, d, device="cuda")
    outs = []
    calls = []
    from srgnn import plan as PL
    orig = PL.NativePlan.hop

    def spy(self, *a, **k):
        calls.append((self.col_blocks, a[4] if len(a) > 4 else k.get("agg")))
        return orig(self, *a, **k)
    monkeypatch.setattr(PL.NativePlan, "hop", spy)
    for B in (3, 1):
        A = _csr(ip, ix, v, n)
        outs.append(propagate_aggregate(A, X, K, steps, col_blocks=B))
        assert cached(A, d) is not None and cached(A, d).col_blocks == B
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    assert len(calls) == 2 * K and any(agg is not None for B, agg in calls if B == 3)


@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("B,compact", [(1, True), (1, False), (3, True), (4, False)])
def test_packed_row_id_chunks_at_every_length(oracle_mod, d, B, compact):
    """The packed light rows take their (id, value) entries S at a time (S = 8 / 16 / 32 lanes per row at
    d = 64 / 128 / 256) and, in column blocks, pipeline their gathers one step ahead:
    rows of every length 0..3S+1 (chunk and step boundaries on both sides), in waves that mix lengths,
    plus a few long rows, against the CPU oracle bit for bit -- one launch (U = 4) and column blocks
    (U = 2), spans and compact copies."""
    from srgnn.plan import NativePlan
    rng = np.random.default_rng(d + 7 * B)
    n = 3000
    S = {64: 8, 128: 16, 256: 32}[d]
    lens = np.concatenate([np.arange(0, 3 * S + 2), rng.integers(0, 3 * S + 2, n - 3 * S - 2 - 6),
                           [400, 700, 1200, 1600, 2500, 2999]])[:n]
    rng.shuffle(lens)
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) if k else np.zeros(0, np.int64)
                         for k in lens]).astype(np.int32)
    v = (rng.standard_normal(ix.size) * 0.5).astype(np.float32)
    A = _csr(ip, ix, v, n)
    x = rng.standard_normal((n, d)).astype(np.float32)
    X = torch.from_numpy(x).cuda()
    P = NativePlan(A, d, hops=8, col_blocks=B, compact=compact, split_block0=True if B > 1 else None)
    panels = [X, torch.full_like(X, float("nan")), torch.full_like(X, float("nan"))]
    P.propagate(panels, d, d, 2)
    torch.cuda.synchronize()
    h1 = oracle_mod.spmm(ip, ix, v, x)
    np.testing.assert_array_equal(panels[1].cpu().numpy(), h1)
    np.testing.assert_array_equal(panels[2].cpu().numpy(), oracle_mod.spmm(ip, ix, v, h1))
