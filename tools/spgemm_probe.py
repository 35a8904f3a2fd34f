#!/usr/bin/env python3
"""Timing of the wavelet model's sparse products on the GPU (srg_spgemm_f32, srg_spmm_muladd_f32).

Operands: phi and phi^-1 of the Cora fixture (tests/golden/wav_cora.npz, the reference's own
SpectralModel output), and random CSRs of growing size.  Prints one JSON line per case with the
count + fill time, the output nnz and the product's flops (2 per multiply-add)."""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from srgnn.sparse import spgemm, spmm_scatter  # noqa: E402


def dev_csr(A):
    A = sp.csr_matrix(A, dtype=np.float32)
    return (torch.from_numpy(A.indptr.astype(np.int64)).cuda(), torch.from_numpy(A.indices.astype(np.int32)).cuda(),
            torch.from_numpy(A.data).cuda())


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        out = fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps, out


def case(name, A, B, d=16):
    a, b = dev_csr(A), dev_csr(B)
    ms, (cip, cix, cv) = timed(lambda: spgemm(*a, *b, B.shape[1]))
    madds = int(np.diff(B.indptr)[A.indices].sum())
    X = torch.rand((B.shape[1], d), device="cuda")
    ms2, _ = timed(lambda: spmm_scatter(cip, cix, cv, X))
    print(json.dumps({"case": name, "m": A.shape[0], "k": A.shape[1], "n": B.shape[1], "nnz_a": A.nnz, "nnz_b": B.nnz,
                      "nnz_c": int(cix.numel()), "multiply_adds": madds, "spgemm_ms": ms,
                      "spgemm_gflops": 2 * madds / ms / 1e6, "spmm_d": d, "spmm_ms": ms2}), flush=True)


def main():
    z = np.load(os.path.join(HERE, "..", "tests", "golden", "wav_cora.npz"), allow_pickle=False)
    n = z["adj_indptr"].size - 1
    phi = [sp.csr_matrix((z[f"phi{k}_data"], z[f"phi{k}_indices"], z[f"phi{k}_indptr"]), shape=(n, n)) for k in range(2)]
    case("cora phi @ phi^-1", phi[0], phi[1])
    case("cora phi^-1 @ phi^-1", phi[1], phi[1])
    rng = np.random.default_rng(1)
    for n, dens in ((20000, 5e-4), (100000, 1e-4), (200000, 2e-5)):
        A = sp.random(n, n, density=dens, format="csr", random_state=rng, dtype=np.float32)
        case(f"random n={n} density={dens}", A, A)


if __name__ == "__main__":
    main()
