"""Test configuration.

Markers: `gpu` = needs a HIP device (run on the MI355X box with `-m gpu`); everything else runs on
the CPU.  Import roots: the product package directory (`operators`, `srgnn`) and the repo root
(`oracle` -- test infrastructure only).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "scalable-roubust-gnn_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def progress(msg: str) -> None:
    """A progress line for long GPU tests, appended to gpurun_out/test_progress.log on the GPU box
    (pytest captures stdout / stderr; a run that writes nothing for minutes is taken to be hung)."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if not root:
        return
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "test_progress.log"), "a") as f:
        f.write(msg + "\n")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle.oracle as o
    o.build()
    return o
