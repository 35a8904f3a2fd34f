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


_WORKER = r"""
import json, os, sys
import torch
import torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
if dist.get_rank() == 0:
    print(json.dumps({"n_gpus": dist.get_world_size(), "sum": float(t), "argv": sys.argv[1:],
                      "addr": os.environ["MASTER_ADDR"]}), flush=True)
dist.destroy_process_group()
"""


def test_rank_launcher_spawns_workers(tmp_path):
    """bench.py --gpus N without torchrun spawns N workers with torchrun's environment (127.0.0.1
    rendezvous) and forwards rank 0's line; a failing worker ends the others and its code is returned."""
    import json
    import subprocess
    script = tmp_path / "worker.py"
    script.write_text(_WORKER)
    code = ("import sys, importlib.util; spec = importlib.util.spec_from_file_location('b', %r); "
            "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b); "
            "sys.exit(b.launch_ranks(3, ['--x', '1'], script=%r))" % (os.path.join(REPO, "bench.py"), str(script)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line == {"n_gpus": 3, "sum": 6.0, "argv": ["--x", "1"], "addr": "127.0.0.1"}
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(7)\ntime.sleep(60)\n")
    code2 = code.replace(str(script), str(bad))
    r = subprocess.run([sys.executable, "-c", code2], capture_output=True, timeout=60, env=env)
    assert r.returncode == 7


def test_oracle_parity_check_on_cpu(oracle_mod):
    """The N = 1 bench line's parity_vs_oracle: sampled rows (random + the longest) of a hop checked
    bit for bit against the oracle fed with the previous hop; a flipped bit is caught."""
    import torch
    from srgnn import synth
    b = _bench()
    n = 4000
    u, v = synth.rmat_undirected_t(n, 30000, seed=6)
    ip, ix = synth.symmetric_csr_t(n, u, v)
    vals = torch.from_numpy(synth.uniform_features_np(1, int(ix.numel()), seed=7)[0])
    x = torch.from_numpy(synth.uniform_features_np(n, 32, seed=8))
    y = torch.from_numpy(oracle_mod.spmm(ip.numpy(), ix.numpy(), vals.numpy(), x.numpy()))
    s = b.oracle_sample(ip, ix, vals, n, 300)
    assert s["rows"].numel() >= 300 and int((ip[1:] - ip[:-1]).argmax()) in s["rows"].tolist()
    res = b.parity_vs_oracle(s, [(1, x, y)])
    assert res["bit_exact"] and res["hops_checked"] == [1]
    r0 = int(s["rows"][0])
    y2 = y.clone()
    y2[r0, 3] = torch.nextafter(y2[r0, 3], torch.tensor(float("inf")))
    assert not b.parity_vs_oracle(s, [(1, x, y2)])["bit_exact"]
