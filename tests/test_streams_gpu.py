"""Streams, devices and host threads around the C-ABI (device guard, per-stream hub
fork/join events, overlapping row strides).  Results must stay bit-identical to the oracle."""
import threading

import numpy as np
import pytest
import torch

import golden_cases as G

pytestmark = pytest.mark.gpu


def _hub_csr(c):
    from srgnn.csr import DeviceCSR
    ip, ix, v = c.ahat()
    A = DeviceCSR.from_tensors(ip, ix, v, n_cols=c.n, heavy_threshold=2, hub_threshold=8, device="cuda")
    assert A.n_hub > 0 and A.n_heavy > 0
    return A


def test_spmm_on_a_side_torch_stream_bit_exact(oracle_mod):
    """A non-default caller stream: the library resolves its device from the stream and forks the
    hub rows from THAT stream (its own side stream and events)."""
    from srgnn.spmm import propagate, spmm
    c = G.Case("rand_d128_r05")
    A = _hub_csr(c)
    x = c.x()
    X = torch.from_numpy(x).cuda()
    want = oracle_mod.propagate(*c.ahat(), x, 3)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        hops = propagate(A, X, 3)
        y = spmm(A, X)
    s.synchronize()
    for k in (1, 2, 3):
        np.testing.assert_array_equal(hops[k].cpu().numpy(), want[k])
    np.testing.assert_array_equal(y.cpu().numpy(), want[1])


def test_hub_nojoin_then_join_per_stream(oracle_mod):
    """SRG_SPMM_HUB_NOJOIN on two caller streams in turn: each srg_hub_join waits on its own
    stream's hub launch."""
    from srgnn import _lib
    from srgnn.spmm import spmm
    c = G.Case("rand_d128_r05")
    A = _hub_csr(c)
    x = c.x()
    X = torch.from_numpy(x).cuda()
    want = oracle_mod.spmm(*c.ahat(), x)
    outs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        with torch.cuda.stream(s):
            outs.append(spmm(A, X, hub_nojoin=True))
    for s in streams:
        with torch.cuda.stream(s):
            _lib.call(X.device, "srg_hub_join", _lib.stream(X.device))
            outs.append(outs.pop(0).clone())      # read after the join, on the same stream
    torch.cuda.synchronize()
    for y in outs:
        np.testing.assert_array_equal(y.cpu().numpy(), want)


def test_two_host_threads_two_streams(oracle_mod):
    """Two host threads issue hub-forking hops concurrently on their own streams."""
    from srgnn.spmm import propagate
    c = G.Case("rand_d128_r05")
    A = _hub_csr(c)
    x = c.x()
    want = oracle_mod.propagate(*c.ahat(), x, 4)
    errors, results = [], [None, None]

    def work(i):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                X = torch.from_numpy(x).cuda()
                for _ in range(20):
                    hops = propagate(A, X, 4)
                results[i] = [h.cpu() for h in hops]
            s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for r in results:
        for k in range(1, 5):
            np.testing.assert_array_equal(r[k].numpy(), want[k])


def test_expanded_panels_rejected():
    """An expanded (stride(0) == 0) source would make the kernel read past its allocation."""
    from srgnn.spmm import gather_rows
    src = torch.ones((1, 16), device="cuda").expand(8, 16)
    with pytest.raises(ValueError, match="overlap"):
        gather_rows(src, torch.zeros(4, dtype=torch.int64, device="cuda"))
    one = torch.ones((1, 16), device="cuda")
    out = gather_rows(one, torch.zeros(3, dtype=torch.int64, device="cuda"))
    assert bool((out == 1).all())
