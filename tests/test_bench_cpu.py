"""bench.py host-side pieces on the CPU: argument defaults (the driver runs `python bench.py` with no
flags) and the cpu_baseline leg (the reference's matmul.c build, and the int64 port fallback)."""
import importlib.util
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_defaults(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert a.gpus == 1 and a.config == "products" and a.op == "khop" and a.exchange == "halo"
    assert a.steps >= 1 and a.warmup >= 0


@pytest.mark.parametrize("force_port", [False, True])
def test_cpu_baseline_leg(oracle_mod, monkeypatch, force_port):
    from srgnn import synth
    b = _bench()
    n = 3000
    u, v = synth.rmat_undirected_t(n, 20000, seed=2)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = np.full(ix.numel(), 0.25, dtype=np.float32)
    x = synth.uniform_features_np(n, 16, seed=1)
    if force_port:
        monkeypatch.setattr(oracle_mod, "ref_lib", lambda: None)
    res = b.cpu_baseline(ip.numpy(), ix.numpy(), vals, x, n, 16, 0.3)
    assert res["value"] > 0 and res["cores"] >= 1 and res["unit"] == "propagated edges/s"
    assert res["kind"] == ("port" if force_port else ("reference" if oracle_mod.ref_lib() else "port"))
    assert "cpu_model" in res and "sample" in res
