"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own Python operators.

Run in the development container (the reference tree is mounted at /root/reference):

    make -C oracle            # builds oracle/_ref/libmatmul_ref.so from the reference's matmul.c
    python tests/golden/make_golden.py

What runs: `operators.graph_operator.symmetrical_simgraph_laplacian_operator.SymLaplacianGraphOp`,
`...symmetrical_simgraph_ppr_operator.PprGraphOp` and `operators.utils.csr_sparse_dense_matmul`
from "/root/reference/Scalable Spectral Robust GNN", unmodified.  Two substitutions, both outside
the reference's files:
  * stub modules for torch_sparse / torch_scatter / torch_geometric.utils, which operators/utils.py
    imports at module top (utils.py:10,12,14) but never calls on this path (absent from the image);
  * numpy.ctypeslib.load_library is redirected from the reference's shipped prebuilt
    csrc/libmatmul.so (never loaded) to oracle/_ref/libmatmul_ref.so, compiled here from the
    reference's own csrc/matmul.c.
Only data leaves this script: inputs, the reference's Â, and hop outputs (in full when small,
otherwise SHA-256 of the exact bytes plus sampled rows).  Exact mode is bit-exact, so hashes pin it.
"""
from __future__ import annotations

import ctypes
import hashlib
import importlib.util
import json
import os
import sys
import tempfile

import numpy as np
import scipy.sparse as sp
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_SSRG = "/root/reference/Scalable Spectral Robust GNN"
DATA = os.path.join(REF_SSRG, "sparsity_datasets", "simhomo", "Planetoid")
OUT = os.path.dirname(os.path.abspath(__file__))
REF_LIB = os.path.join(REPO, "oracle", "_ref", "libmatmul_ref.so")
FULL_LIMIT = 400_000        # store hop panels in full up to this many elements

_STUBS = {
    "torch_sparse.py": "def _absent(*a, **k):\n    raise ImportError('torch_sparse stub')\n"
                       "coalesce = spspmm = spmm = _absent\nclass SparseTensor:\n    pass\n",
    "torch_scatter.py": "def scatter_add(*a, **k):\n    raise ImportError('torch_scatter stub')\n",
    "torch_geometric/__init__.py": "",
    "torch_geometric/utils.py": "def _absent(*a, **k):\n    raise ImportError('torch_geometric stub')\n"
                                "add_self_loops = to_scipy_sparse_matrix = _absent\n",
}


def _load_synth():
    path = os.path.join(REPO, "scalable-roubust-gnn_amd", "srgnn", "synth.py")
    spec = importlib.util.spec_from_file_location("_golden_synth", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _load_golden_cases():
    path = os.path.join(REPO, "tests", "golden_cases.py")
    spec = importlib.util.spec_from_file_location("_golden_cases", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def import_reference():
    if not os.path.exists(REF_LIB):
        raise SystemExit(f"{REF_LIB} missing: run `make -C oracle` first")
    stub_dir = tempfile.mkdtemp(prefix="srg_stubs_")
    for name, text in _STUBS.items():
        path = os.path.join(stub_dir, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(text)
    sys.dont_write_bytecode = True
    sys.path[:0] = [stub_dir, REF_SSRG]
    import numpy.ctypeslib as ctl
    real_load = ctl.load_library

    def redirected(libname, loader_path):
        if os.path.basename(libname) == "libmatmul.so":
            return ctypes.cdll.LoadLibrary(REF_LIB)
        raise RuntimeError(f"unexpected native library request {libname!r}")

    ctl.load_library = redirected
    from operators.graph_operator.symmetrical_simgraph_laplacian_operator import SymLaplacianGraphOp
    from operators.graph_operator.symmetrical_simgraph_ppr_operator import PprGraphOp
    from operators.utils import csr_sparse_dense_matmul
    return SymLaplacianGraphOp, PprGraphOp, csr_sparse_dense_matmul, real_load


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def sample_rows(n, k=24, seed=11):
    rng = np.random.default_rng(seed)
    rows = np.unique(np.r_[0, n - 1, rng.choice(n, size=min(k, n), replace=False)])
    return rows.astype(np.int64)


def planetoid_adj(name, symmetric):
    torch.serialization.add_safe_globals([range])
    e = torch.load(os.path.join(DATA, name, "raw", "edge_index.pt"), weights_only=True).numpy()
    n = int(torch.load(os.path.join(DATA, name, "raw", "label.pt"), weights_only=True).shape[0])
    row, col = e[0].astype(np.int64), e[1].astype(np.int64)
    if symmetric:
        row, col = np.r_[row, col], np.r_[col, row]
    adj = sp.csr_matrix((np.ones(row.size), (row, col)), shape=(n, n))
    return adj, e


def random_adj(n, density, seed, hub=True, empty_rows=True, unsorted=False, dup=False):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < density
    if hub:
        mask[n // 3, :] = True                      # a hub row ...
        mask[:, n // 5] = True                      # ... and a hub column
    if empty_rows:
        mask[[1, n // 2, n - 2], :] = False         # rows with no stored entry
    np.fill_diagonal(mask, rng.random(n) < 0.2)     # some self-loops
    w = rng.integers(1, 33, size=(n, n)) / 8.0      # dyadic weights: exact fp64 sums in any order
    dense = np.where(mask, w, 0.0)
    adj = sp.csr_matrix(dense)
    if unsorted or dup:
        r = np.repeat(np.arange(n), np.diff(adj.indptr))
        c, v = adj.indices.copy(), adj.data.copy()
        if dup:   # duplicate a few entries (stored twice; FloatCSRMulDenseOMP folds both in order)
            pick = rng.choice(c.size, size=max(1, c.size // 20), replace=False)
            r, c, v = np.r_[r, r[pick]], np.r_[c, c[pick]], np.r_[v, v[pick] / 2]
        order = np.lexsort((rng.random(r.size), r)) if unsorted else np.argsort(r, kind="stable")
        r, c, v = r[order], c[order], v[order]
        ptr = np.zeros(n + 1, dtype=np.int32)
        np.add.at(ptr, r + 1, 1)
        adj = sp.csr_matrix((v, c.astype(np.int32), np.cumsum(ptr).astype(np.int32)), shape=(n, n))
        adj.has_sorted_indices = False
    return adj


def store_case(name, adj, X, hops, ahat=None, meta=None, x_stored=True):
    rec = {"n": adj.shape[0], "d": X.shape[1], "k": len(hops) - 1}
    rec.update(meta or {})
    arrs = {
        "adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int32),
        "adj_data": adj.data.astype(np.float64),
        "x_sha256": np.array(sha(X)),
    }
    if x_stored:
        arrs["x"] = X
    if ahat is not None:
        arrs.update({"ahat_indptr": ahat.indptr.astype(np.int64), "ahat_indices": ahat.indices.astype(np.int32),
                     "ahat_data64": ahat.data.astype(np.float64), "ahat_data": ahat.data.astype(np.float32)})
    rows = sample_rows(adj.shape[0])
    arrs["sample_rows"] = rows
    for k, h in enumerate(hops[1:], start=1):
        h = np.ascontiguousarray(h, dtype=np.float32)
        arrs[f"hop{k}_sha256"] = np.array(sha(h))
        arrs[f"hop{k}_rows"] = h[rows]
        if h.size <= FULL_LIMIT:
            arrs[f"hop{k}"] = h
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrs)
    return rec


def family_ops(TwoOrder, Com, TwoDir, norm):
    synth = _load_synth()
    gc = _load_golden_cases()
    family_adj, family_construct = gc.family_adj, gc.family_construct
    adj = family_adj()
    n = adj.shape[0]
    X = synth.uniform_features_np(n, 24, seed=70)
    K = 3
    out = {}
    for name, base in (("two_order", TwoOrder), ("complex", Com), ("two_dir", TwoDir)):
        cons = family_construct(name, norm)
        cls = type(f"Golden_{name}", (base,), {"construct_adj": lambda self, a, c=cons: c(a)})
        lists = cls(K).propagate(adj, X)
        arrs = {"adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int32),
                "adj_data": adj.data.astype(np.float64), "x": X}
        for li, lst in enumerate(lists):
            for k, t in enumerate(lst):
                h = np.ascontiguousarray(t.numpy(), dtype=np.float32)
                arrs[f"list{li}_hop{k}_sha256"] = np.array(sha(h))
                arrs[f"list{li}_hop{k}"] = h
        np.savez_compressed(os.path.join(OUT, f"fam_{name}.npz"), **arrs)
        out[f"fam_{name}"] = {"n": n, "d": 24, "k": K, "op": "family", "family": name, "lists": len(lists)}
    return out


def main():
    SymLap, Ppr, csr_mm, _ = import_reference()
    synth = _load_synth()
    manifest = {}

    # 1-2. Cora (cora_0_0) symmetrised and as stored (upper triangle), K = 3, r = 0.5, d = 1433
    Xc = synth.binary_rownorm_features_np(2708, 1433, 18, seed=7)
    for sym in (True, False):
        adj, _ = planetoid_adj("cora_0_0", sym)
        op = SymLap(3, r=0.5)
        hops = [h.numpy() for h in op.propagate(adj, Xc)]
        name = "cora_sym_k3" if sym else "cora_asstored_k3"
        manifest[name] = store_case(name, adj, Xc, hops, op.adj,
                                    {"op": "sym_laplacian", "r": 0.5, "features": "binary_rownorm(18, seed=7)"})

    # 3-4. Citeseer 0.5 / Pubmed 0.6 symmetrised, d = 500 uniform features, K = 3
    for ds, n_expect in (("citeseer_0.5_0.5", 3327), ("pubmed_0.6_0.6", 19717)):
        adj, _ = planetoid_adj(ds, True)
        assert adj.shape[0] == n_expect
        X = synth.uniform_features_np(adj.shape[0], 500, seed=7)
        op = SymLap(3, r=0.5)
        hops = [h.numpy() for h in op.propagate(adj, X)]
        name = ds.split("_")[0] + "_sym_k3"
        manifest[name] = store_case(name, adj, X, hops, op.adj,
                                    {"op": "sym_laplacian", "r": 0.5, "features": "uniform(seed=7)"},
                                    x_stored=False)

    # 5. random graphs: hubs, empty rows, self-loops, weights; d and r sweeps; PPR
    cases = [
        ("rand_d1_r05", 60, 0.08, 1, 0.5, "sym"), ("rand_d7_r03", 60, 0.08, 7, 0.3, "sym"),
        ("rand_d64_r0", 120, 0.05, 64, 0.0, "sym"), ("rand_d128_r05", 200, 0.04, 128, 0.5, "sym"),
        ("rand_d130_r1", 90, 0.06, 130, 1.0, "sym"), ("rand_d256_r05", 150, 0.05, 256, 0.5, "sym"),
        ("rand_d1433_r05", 24, 0.2, 1433, 0.5, "sym"), ("rand_d36_ppr", 100, 0.05, 36, 0.5, "ppr"),
    ]
    for i, (name, n, dens, d, r, kind) in enumerate(cases):
        adj = random_adj(n, dens, seed=100 + i)
        X = synth.uniform_features_np(n, d, seed=20 + i)
        op = SymLap(3, r=r) if kind == "sym" else Ppr(3, r=r, alpha=0.15)
        hops = [h.numpy() for h in op.propagate(adj, X)]
        manifest[name] = store_case(name, adj, X, hops, op.adj,
                                    {"op": "sym_laplacian" if kind == "sym" else "ppr", "r": r,
                                     "alpha": 0.15 if kind == "ppr" else None,
                                     "features": f"uniform(seed={20 + i})"})

    # 6. raw one-hop products through csr_sparse_dense_matmul: unsorted rows, duplicates, F-order X
    for i, (name, n, d, unsorted, dup, forder) in enumerate([
            ("raw_unsorted_d33", 80, 33, True, False, False),
            ("raw_dups_d128", 96, 128, True, True, False),
            ("raw_forder_d128", 70, 128, False, False, True)]):
        adj = random_adj(n, 0.07, seed=300 + i, unsorted=unsorted, dup=dup)
        X = synth.uniform_features_np(n, d, seed=40 + i)
        if forder:
            X = np.asfortranarray(X)
        y = csr_mm(adj, X)
        manifest[name] = store_case(name, adj, np.ascontiguousarray(X), [X, y], None,
                                    {"op": "raw_spmm", "f_order_input": forder})

    # 7b. hop aggregation: the reference's own message operators on reference hop lists
    from operators.message_operator.last_message_op import LastMessageOp
    from operators.message_operator.mean_message_op import MeanMessageOp
    from operators.message_operator.simple_weighted_message_op import SimpleWeightedMessageOp
    from operators.message_operator.sum_message_op import SumMessageOp

    def agg_ops(K):
        return {"last": LastMessageOp(), "sum_all": SumMessageOp(0, K + 1), "mean_1_end": MeanMessageOp(1, K + 1),
                "gbp_alpha015": SimpleWeightedMessageOp(0, K + 1, "alpha", 0.15),
                "gbp_alpha03_2_k": SimpleWeightedMessageOp(2, K, "alpha", 0.3),
                "hand_1_3": SimpleWeightedMessageOp(1, 3, "hand_crafted", [0.7, -0.3])}

    def store_agg(name, adj, X, K, r, meta):
        op = SymLap(K, r=r)
        feats = op.propagate(adj, X)
        arrs = {"adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int32),
                "adj_data": adj.data.astype(np.float64), "x_sha256": np.array(sha(X))}
        if X.size <= FULL_LIMIT:
            arrs["x"] = X
        rows = sample_rows(adj.shape[0])
        arrs["sample_rows"] = rows
        ops = agg_ops(K)
        for key, mop in ops.items():
            out = np.ascontiguousarray(mop.aggregate(feats).numpy(), dtype=np.float32)
            arrs[f"{key}_sha256"] = np.array(sha(out))
            arrs[f"{key}_rows"] = out[rows]
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrs)
        rec = {"n": adj.shape[0], "d": X.shape[1], "k": K, "op": "aggregate", "r": r, "msg_ops": sorted(ops),
               "torch": torch.__version__}
        rec.update(meta)
        return rec

    adj, _ = planetoid_adj("cora_0_0", True)
    manifest["agg_cora_k3"] = store_agg("agg_cora_k3", adj, Xc, 3, 0.5, {"features": "binary_rownorm(18, seed=7)"})
    adj = random_adj(200, 0.05, seed=400)
    X = synth.uniform_features_np(200, 37, seed=60)
    manifest["agg_rand_k20"] = store_agg("agg_rand_k20", adj, X, 20, 0.5, {"features": "uniform(seed=60)"})

    # 7c. the other operator families (base_operator.py:60-307) with scipy-only construct_adj
    #     subclasses defined here (the reference's own subclasses need torch_scatter / PyG)
    from operators.base_operator import ComGraphOp, TwoDirGraphOp, TwoOrderPprApproxGraphOp
    from operators.utils import adj_to_symmetric_norm
    for k, v in family_ops(TwoOrderPprApproxGraphOp, ComGraphOp, TwoDirGraphOp, adj_to_symmetric_norm).items():
        manifest[k] = v

    # 7. error behaviour of GraphOp.propagate (base_operator.py:20-30, utils.py:23-45)
    errs = {}
    adj = random_adj(30, 0.1, seed=7)
    X = synth.uniform_features_np(30, 8, seed=1)

    def outcome(fn):
        try:
            fn()
            return "ok"
        except Exception as e:  # noqa: BLE001 -- recording the class is the point
            return type(e).__name__

    errs["coo_adj"] = outcome(lambda: SymLap(2).propagate(adj.tocoo(), X))
    errs["float64_feature"] = outcome(lambda: SymLap(2).propagate(adj, X.astype(np.float64)))
    errs["dim_mismatch"] = outcome(lambda: SymLap(2).propagate(adj, X[:-1]))
    errs["list_feature"] = outcome(lambda: SymLap(2).propagate(adj, X.tolist()))
    errs["tensor_feature"] = outcome(lambda: SymLap(2).propagate(adj, torch.from_numpy(X)))
    errs["ppr_dense_adj"] = outcome(lambda: Ppr(2).propagate(adj.toarray(), X))
    errs["k0"] = outcome(lambda: SymLap(0).propagate(adj, X))
    manifest["_errors"] = errs

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(errs))
    print("wrote", len(manifest) - 1, "cases to", OUT)


if __name__ == "__main__":
    main()
