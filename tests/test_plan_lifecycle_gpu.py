"""The one-GPU plan's lifecycle through the C-ABI ("do this" 1): a plan is built, its hops run
(with the hub rows chained on the side stream, replayed as a HIP graph, on several streams), it is
released with work possibly still in flight, and a new plan is built over the same memory -- every hop
bitwise the CPU oracle's.

Round 5 saw a memory-access fault and two hangs in this sequence (examples/plan_propagate, plan memory
from the stream-ordered pool).  srg_plan_destroy now joins every stream the plan's work went to (an
event per stream, recorded after the hub side stream was joined into it) into its own stream, drains
that, and only then destroys the executable graphs and frees the memory; a graph replaced by a new key
is retired until its last launch completes.  The sequences below release plans without
any host synchronisation of their own, so they only pass if that ordering holds."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(n=40000, seed=11):
    """A power-law CSR with sorted rows and two hubs long enough to be hub rows in every column block."""
    rng = np.random.default_rng(seed)
    deg = np.minimum(rng.zipf(1.9, n), 1500).astype(np.int64)
    deg[rng.integers(0, n, 300)] = 0
    deg[17], deg[1017] = 30000, 9000
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) if k else np.zeros(0, np.int64)
                         for k in deg]).astype(np.int32)
    v = (rng.standard_normal(ix.size) * 0.3).astype(np.float32)
    return ip, ix, v, n


@pytest.fixture(scope="module")
def case(oracle_mod):
    from srgnn import _lib
    ip, ix, v, n = _graph()
    d, K = 64, 3
    x = np.random.default_rng(5).uniform(-1, 1, (n, d)).astype(np.float32)
    want = oracle_mod.propagate(ip, ix, v, x, K)
    dev = torch.device("cuda", 0)
    arrays = tuple(torch.from_numpy(a).to(dev) for a in (ip, ix, v))
    return dict(lib=_lib, n=n, d=d, K=K, x=torch.from_numpy(x).to(dev), want=want, arrays=arrays, dev=dev)


def _build(c, stream, hops=20, col_blocks=4, opts=None, hub=1000):
    L = c["lib"]
    ip, ix, v = c["arrays"]
    p = ctypes.c_void_p()
    if opts is None:
        opts = L.SRG_PLAN_COMPACT | L.SRG_PLAN_SPLIT_BLOCK0
    # hub rows: > 1000 entries in a launch -> both hubs, in every block (a chained hub side stream); automatic
    # (SRG_PLAN_AUTO): both are whole hub rows, one launch of their own forked first in every hop
    L.call(c["dev"], "srg_plan_build", ip.data_ptr(), ix.data_ptr(), v.data_ptr(), c["n"], c["d"], hops, col_blocks,
           hub, L.SRG_PLAN_AUTO, opts, stream.cuda_stream, ctypes.byref(p))
    return p.value


def _desc(c, p):
    from srgnn.plan import PlanDesc
    desc = PlanDesc()
    c["lib"].call(c["dev"], "srg_plan_describe", p, ctypes.byref(desc))
    return desc


def _panels(c):
    buf = torch.empty((c["K"], c["n"], c["d"]), dtype=torch.float32, device=c["dev"])
    return [c["x"]] + [buf[k] for k in range(c["K"])]


def _propagate(c, p, panels, stream):
    arr = (ctypes.c_void_p * len(panels))(*[t.data_ptr() for t in panels])
    c["lib"].call(c["dev"], "srg_plan_propagate_f32", p, arr, c["d"], c["d"], c["K"], 0, stream.cuda_stream)


def _destroy(c, p, stream):
    c["lib"].call(c["dev"], "srg_plan_destroy", p, stream.cuda_stream)


def _check(c, panels, what):
    torch.cuda.synchronize()
    for k in range(1, c["K"] + 1):
        got = panels[k].cpu().numpy()
        assert np.array_equal(got.view(np.int32), c["want"][k].view(np.int32)), f"{what}: hop {k} differs"


@pytest.mark.parametrize("hub", ["chained", "whole"])
def test_build_hop_release_build_hop_bitwise(case, hub):
    c = case
    L = c["lib"]
    ht = 1000 if hub == "chained" else L.SRG_PLAN_AUTO
    s1 = torch.cuda.Stream(device=c["dev"])
    s1.wait_stream(torch.cuda.current_stream())
    A, B = _panels(c), _panels(c)
    # 1. chained hub spans (or the whole hub rows' launch), eager then captured and replayed; released
    # right behind the replay
    p1 = _build(c, s1, hub=ht)
    d1 = _desc(c, p1)
    assert d1.col_blocks == 4 and d1.compact == 1 and d1.split_block0 == 1
    assert (d1.hub_chain, d1.hub_rows_whole) == ((1, 0) if hub == "chained" else (0, 2))
    for _ in range(3):                   # call 1 eager, call 2 captured + replayed, call 3 replayed
        _propagate(c, p1, A, s1)
    _destroy(c, p1, s1)                  # no host synchronisation before: destroy must order itself
    # 2. a new plan over (most likely) the same memory, its hops into other panels
    p2 = _build(c, s1, hub=ht)
    _propagate(c, p2, B, s1)
    _destroy(c, p2, s1)
    _check(c, A, "first plan (graph replay, released in flight)")
    _check(c, B, "second plan (built after the first was released)")


def test_release_joins_other_streams_and_retired_graphs(case):
    c = case
    L = c["lib"]
    s1, s2 = torch.cuda.Stream(device=c["dev"]), torch.cuda.Stream(device=c["dev"])
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream())
    A, B, C = _panels(c), _panels(c), _panels(c)
    p = _build(c, s1)
    s2.wait_stream(s1)
    # one hop on s2 (its hub rows on s2's side stream) ...
    Y = torch.empty_like(c["x"])
    L.call(c["dev"], "srg_plan_hop_f32", p, c["x"].data_ptr(), c["d"], Y.data_ptr(), c["d"], c["d"], 0, None, 0,
           0.0, 0, s2.cuda_stream)
    # ... a graph captured and replayed on s1, then replaced by another key while it may still run ...
    for _ in range(3):
        _propagate(c, p, A, s1)
    _propagate(c, p, B, s1)              # key change: the panels-A graph is retired, not destroyed
    for _ in range(2):
        _propagate(c, p, C, s1)          # eager, then captured
    # ... and the plan released on s1 with s2's hop and both graphs possibly in flight
    _destroy(c, p, s1)
    p2 = _build(c, s1)                   # reuses the memory
    D = _panels(c)
    _propagate(c, p2, D, s1)
    _destroy(c, p2, s1)
    torch.cuda.synchronize()
    assert np.array_equal(Y.cpu().numpy().view(np.int32), c["want"][1].view(np.int32)), "hop on the second stream"
    for name, P in (("A", A), ("B", B), ("C", C), ("D", D)):
        _check(c, P, f"panels {name}")


def test_implicit_plans_back_to_back(case):
    """srg_propagate_khop_f32 without a schedule plans its own hops and releases the plan after them:
    two calls back to back on one stream, no synchronisation between them."""
    c = case
    L = c["lib"]
    ip, ix, v = c["arrays"]
    s1 = torch.cuda.Stream(device=c["dev"])
    s1.wait_stream(torch.cuda.current_stream())
    outs = []
    for _ in range(2):
        P = _panels(c)
        arr = (ctypes.c_void_p * len(P))(*[t.data_ptr() for t in P])
        L.call(c["dev"], "srg_propagate_khop_f32", ip.data_ptr(), ix.data_ptr(), v.data_ptr(), c["n"], None, 0, 0, arr,
               c["d"], c["d"], c["K"], 0, s1.cuda_stream)
        outs.append(P)
    for i, P in enumerate(outs):
        _check(c, P, f"implicit plan {i}")


def test_plan_in_caller_memory(case):
    """srg_plan_query + srg_plan_build_in: the plan in torch-allocated memory, the same hops bitwise;
    undersized memory is refused before anything is built."""
    c = case
    L = c["lib"]
    ip, ix, v = c["arrays"]
    s1 = torch.cuda.Stream(device=c["dev"])
    s1.wait_stream(torch.cuda.current_stream())
    kb, sb = ctypes.c_size_t(), ctypes.c_size_t()
    ro, rb = ctypes.c_uint32(), ctypes.c_int32()
    L.call(c["dev"], "srg_plan_query", ip.data_ptr(), c["n"], c["d"], 20, 4, 1000, L.SRG_PLAN_AUTO,
           L.SRG_PLAN_SPLIT_BLOCK0, s1.cuda_stream,
           ctypes.byref(kb), ctypes.byref(sb), ctypes.byref(ro), ctypes.byref(rb))
    assert rb.value == 4 and (ro.value & L.SRG_PLAN_SPLIT_BLOCK0)
    keep = torch.empty(kb.value, dtype=torch.uint8, device=c["dev"])
    scratch = torch.empty(sb.value, dtype=torch.uint8, device=c["dev"])
    p = ctypes.c_void_p()
    with pytest.raises(L.SrgError, match="caller memory"):
        L.call(c["dev"], "srg_plan_build_in", ip.data_ptr(), ix.data_ptr(), v.data_ptr(), c["n"], c["d"], 20, 4, 1000,
               L.SRG_PLAN_AUTO, ro.value, keep.data_ptr(), kb.value - 256, scratch.data_ptr(), sb.value, s1.cuda_stream,
               ctypes.byref(p))
    L.call(c["dev"], "srg_plan_build_in", ip.data_ptr(), ix.data_ptr(), v.data_ptr(), c["n"], c["d"], 20, 4, 1000,
           L.SRG_PLAN_AUTO, ro.value, keep.data_ptr(), kb.value, scratch.data_ptr(), sb.value, s1.cuda_stream,
           ctypes.byref(p))
    del scratch                          # the build has returned: the scratch may go
    desc = _desc(c, p.value)
    assert desc.device_bytes == kb.value and desc.col_blocks == 4
    A = _panels(c)
    for _ in range(3):
        _propagate(c, p.value, A, s1)
    _destroy(c, p.value, s1)
    del keep
    _check(c, A, "plan in caller memory")
