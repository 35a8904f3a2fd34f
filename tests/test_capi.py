"""The C-ABI library: loads without a GPU, exports every symbol include/srgnn_hip.h declares, and
rejects bad arguments with a status + message before touching the device."""
import ctypes
import os
import re
import subprocess

import pytest

from srgnn import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "srgnn_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(", text, flags=re.M))


def test_header_and_python_binding_agree():
    assert declared_symbols() == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_symbols() - exported
    assert not missing, f"not exported: {missing}"


def test_library_loads_and_reports_version():
    assert "gfx950" in _lib.version()


def test_gfx950_code_object_present():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob, "no gfx950 code object in the fat binary"


def test_invalid_arguments_fail_before_launch():
    L = _lib.lib()
    rc = L.srg_spmm_csr_f32(None, None, None, -1, None, 0, 0, None, 8, None, 8, 8, 0, None)
    assert rc == _lib.SRG_ERR_INVALID
    assert "n_rows" in _lib.last_error()
    rc = L.srg_spmm_csr_f32(None, None, None, 4, None, 0, 0, None, 2, None, 8, 8, 0, None)
    assert rc == _lib.SRG_ERR_INVALID and "leading" in _lib.last_error()
    rc = L.srg_spmm_csr_f32(None, None, None, 4, None, 0, 2, ctypes.c_void_p(16), 8, ctypes.c_void_p(16), 8, 8, 0, None)
    assert rc == _lib.SRG_ERR_INVALID
    rc = L.srg_propagate_khop_f32(None, None, None, 4, None, 0, 0, None, 8, 8, -1, 0, None)
    assert rc == _lib.SRG_ERR_INVALID and "K" in _lib.last_error()
    rc = L.srg_cheby_step_f64(None, None, None, 4, None, None, None, None, 8, 8, 7, 1.0, 1.0,
                              None, None, 1, None, 32, None)
    assert rc == _lib.SRG_ERR_INVALID and "mode" in _lib.last_error()
    rc = L.srg_cheby_step_f64(None, None, None, 4, None, None, None, None, 8, 8,
                              _lib.SRG_CHEBY_STEP | _lib.SRG_CHEBY_HUB_NOJOIN, 1.0, 1.0, None, None, 1, None, 32, None)
    assert rc == _lib.SRG_ERR_INVALID and "HUB_NOJOIN" in _lib.last_error()
    L.srg_clear_error()
    assert L.srg_last_error_code() == 0


def test_empty_problem_is_a_noop_without_device():
    L = _lib.lib()
    assert L.srg_spmm_csr_f32(None, None, None, 0, None, 0, 0, None, 8, None, 8, 8, 0, None) == 0
    # the drop-in entry: zero rows -> returns without touching the device
    f = ctypes.c_void_p
    L.FloatCSRMulDenseOMP.argtypes = [f, f, f, f, f, ctypes.c_int, ctypes.c_int]
    L.FloatCSRMulDenseOMP.restype = None
    L.FloatCSRMulDenseOMP(None, None, None, None, None, 0, 5)
    assert L.srg_last_error_code() == 0
    L.FloatCSRMulDenseOMP(None, None, None, None, None, -3, 5)
    assert L.srg_last_error_code() == _lib.SRG_ERR_INVALID


def test_every_device_entry_runs_under_its_device():
    """Python callers reach the device entry points only through _lib.call(device, ...), which makes
    the operands' device current: the library resolves the null stream and its hub side streams
    from the current device."""
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scalable-roubust-gnn_amd")
    offenders = []
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py") and f != "_lib.py":
                text = open(os.path.join(root, f)).read()
                if re.search(r"lib\(\)\.srg_\w+\(", text):
                    offenders.append(f)
    assert not offenders, f"direct C-ABI calls bypassing _lib.call: {offenders}"


@pytest.mark.gpu
def test_plain_c_host_runs_the_halo_path():
    """examples/halo_loopback.c: a plain C program (gcc, no Python / torch) includes srgnn_hip.h,
    builds the halo plans of 4 ranks from a host CSR, runs K hops through the loopback communicator
    and compares every rank's rows of every hop with srg_propagate_khop_f32 on one GPU: bitwise."""
    import subprocess
    exe = os.path.join(REPO, "examples", "halo_loopback")
    assert os.path.exists(exe), "build it with `make -C examples` (__graft_entry__.build() does)"
    for args in (["4", "20000", "64", "4"], ["8", "30000", "128", "3"], ["3", "5000", "32", "5"]):
        r = subprocess.run([exe] + args, capture_output=True, timeout=120)
        out = r.stdout.decode() + r.stderr.decode()
        assert r.returncode == 0 and out.startswith("ok:"), out


def test_planner_rejects_bad_arguments_before_the_device():
    """srg_plan_build / _describe / _propagate_f32 argument checks (csrc/srg_plan.hip): every one fails
    with SRG_ERR_INVALID and a message before any HIP call, so they run without a GPU."""
    L = _lib.lib()
    out = ctypes.c_void_p()
    ip = (ctypes.c_int64 * 3)(0, 1, 2)
    A, N = _lib.SRG_PLAN_AUTO, _lib.SRG_PLAN_NONE
    cases = [
        ((ip, None, None, 2, 8, 4, 0, A, A, 0, None, None), "null plan"),
        ((None, None, None, 2, 8, 4, 0, A, A, 0, None, ctypes.byref(out)), "indptr"),
        ((ip, None, None, -1, 8, 4, 0, A, A, 0, None, ctypes.byref(out)), "n_rows"),
        ((ip, None, None, 2, 0, 4, 0, A, A, 0, None, ctypes.byref(out)), "d=0"),
        ((ip, None, None, 2, 8, -1, 0, A, A, 0, None, ctypes.byref(out)), "hops=-1"),
        ((ip, None, None, 2, 8, 4, 65, A, A, 0, None, ctypes.byref(out)), "col_blocks=65"),
        ((ip, None, None, 2, 8, 4, 0, N - 1, A, 0, None, ctypes.byref(out)), "hub_threshold=-3"),
        ((ip, None, None, 2, 8, 4, 0, A, -7, 0, None, ctypes.byref(out)), "heavy_threshold=-7"),
        ((ip, None, None, 2, 8, 4, 0, A, A, _lib.SRG_PLAN_COMPACT | _lib.SRG_PLAN_SPANS, None, ctypes.byref(out)),
         "opts"),
        ((ip, None, None, 2, 8, 4, 0, A, A, 0x100, None, ctypes.byref(out)), "opts"),
    ]
    for args, msg in cases:
        assert L.srg_plan_build(*args) == _lib.SRG_ERR_INVALID, msg
        assert msg in _lib.last_error(), (msg, _lib.last_error())
    assert L.srg_plan_describe(None, None) == _lib.SRG_ERR_INVALID
    assert L.srg_plan_propagate_f32(None, None, 8, 8, 1, 0, None) == _lib.SRG_ERR_INVALID
    assert L.srg_plan_launch(None, 0, 8, None, None, None) == _lib.SRG_ERR_INVALID
    assert L.srg_plan_hop_f32(None, None, 8, None, 8, 8, 0, None, 0, 0.0, 0, None) == _lib.SRG_ERR_INVALID
    assert L.srg_plan_destroy(None, None) == 0


@pytest.mark.gpu
def test_plain_c_host_runs_the_fp64_steps(tmp_path):
    """examples/cheby64_plan.c: a plain C program plans an operator for the fp64 Chebyshev steps (no fp32
    values, whole hub rows) and runs an order-3 two-scale filter through srg_plan_cheby_step_f64 (lean
    epilogue) and through srg_cheby_step_f64 (one launch per order): bit for bit the same, blocked (4 blocks)
    and automatic (one launch on this small panel)."""
    import json
    import subprocess

    import numpy as np
    exe = os.path.join(REPO, "examples", "cheby64_plan")
    assert os.path.exists(exe), "build it with `make -C examples` (__graft_entry__.build() does)"
    rng = np.random.default_rng(9)
    n = 30000
    deg = np.minimum(rng.zipf(1.8, n), 3000).astype(np.int64)
    deg[7] = 20000
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) for k in deg]).astype(np.int32)
    v = (rng.standard_normal(ix.size) * 0.1).astype(np.float32)
    path = tmp_path / "g.csr"
    with open(path, "wb") as f:
        f.write(b"SRGCSR1\0")
        f.write(np.array([n, ix.size], dtype=np.int64).tobytes())
        f.write(ip.tobytes())
        f.write(ix.tobytes())
        f.write(v.tobytes())
    for d, blocks, want_blocks in (("64", "4", 4), ("100", "0", 1), ("128", "7", 7)):
        r = subprocess.run([exe, str(path), d, blocks, "2"], capture_output=True, timeout=120)
        assert r.returncode == 0, r.stdout.decode() + r.stderr.decode()
        res = json.loads(r.stdout.decode())
        assert res["bitwise_vs_one_launch"] is True and res["n"] == n and res["col_blocks"] == want_blocks
        hubs = int((deg > max(2048, int(ix.size) // 4096)).sum())
        assert hubs >= 1 and res["hub_rows_whole"] == (hubs if want_blocks > 1 else 0)


@pytest.mark.gpu
def test_plain_c_host_runs_the_planner(tmp_path):
    """examples/plan_propagate.c: a plain C program reads a CSR file, plans its hops on the device
    (srg_plan_build), checks the plans' launches on the host, times the one-shot and long-lived runs
    and compares hops 1, 2 and K bit for bit with the unscheduled one-launch hops."""
    import json
    import subprocess

    import numpy as np
    exe = os.path.join(REPO, "examples", "plan_propagate")
    assert os.path.exists(exe), "build it with `make -C examples` (__graft_entry__.build() does)"
    rng = np.random.default_rng(4)
    n = 30000
    deg = np.minimum(rng.zipf(1.8, n), 3000).astype(np.int64)
    deg[7] = 20000
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.choice(n, k, replace=False)) for k in deg]).astype(np.int32)
    v = rng.standard_normal(ix.size).astype(np.float32)
    path = tmp_path / "g.csr"
    with open(path, "wb") as f:
        f.write(b"SRGCSR1\0")
        f.write(np.array([n, ix.size], dtype=np.int64).tobytes())
        f.write(ip.tobytes())
        f.write(ix.tobytes())
        f.write(v.tobytes())
    for d, K in (("64", "7"), ("128", "3")):
        r = subprocess.run([exe, str(path), d, K, "2"], capture_output=True, timeout=120)
        assert r.returncode == 0, r.stdout.decode() + r.stderr.decode()
        res = json.loads(r.stdout.decode())
        assert res["bitwise_vs_one_launch"] is True and res["n"] == n
