"""Golden fixtures for the directed operator families: the REFERENCE's own construct_adj and propagate.

    make -C oracle && python tests/golden/make_golden_directed.py      (development container only)

Runs, unmodified, from "/root/reference/Scalable Spectral Robust GNN":
  operators/graph_operator/symmetrical_directed_magnetic_laplacian_operator.py  SymDirMagLaplacianGraphOp
  operators/graph_operator/symmetrical_directed_magnetic_comppr_operator.py     SymDirMagComPprGraphOp
  operators/graph_operator/symmetrical_directed_fast_ppr_approximate_operator.py SymDirFastPprApproxGraphOp
  operators/graph_operator/in_out_directed_laplacian_operator.py                TwoDirLaplacianGraphOp
  operators/graph_operator/symmetrical_directed_two_order_ppr_approximate_operator.py
                                                                                SymDirTwoOrderPprApproxGraphOp
and operators/utils.py's PyGSD_adj_to_directed_symmetric_mag_norm.

Those need three third-party functions that are absent from this image (the reference pins no
versions).  The stubs below restate their published algorithms (test infrastructure, never shipped):
  * torch_scatter 2.x  scatter_add = scatter_sum: out = zeros(dim_size).scatter_add_(0, index, src)
                        (torch_scatter/scatter.py: the CPU path IS torch's scatter_add_);
  * torch_sparse 0.6.x coalesce(index, value, m, n, op="add"): SparseStorage(is_sorted=False)
                        sorts by row * n + col, then segment_csr sums each run of equal keys
                        (torch_sparse/coalesce.py, storage.py).  The stub sorts stably; the runs
                        here hold at most two entries (an edge and its reverse), so their sum does
                        not depend on the order;
  * torch_geometric 2.x add_self_loops(edge_index, edge_attr, fill_value, num_nodes): appends
                        arange(N) loops after the edges and full((N,), fill_value) after the
                        attributes (torch_geometric/utils/loop.py).
One shim: scipy 1.15 no longer exports scipy.newaxis (an alias of numpy.newaxis = None), which
utils.py:283 uses; it is set back before the reference is imported.
numpy.ctypeslib.load_library is redirected to oracle/_ref/libmatmul_ref.so (the reference's own
csrc/matmul.c compiled here), as in make_golden.py.  Only data is written.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import tempfile

import numpy as np
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

_STUBS = {
    "torch_scatter.py": (
        "import torch\n"
        "def scatter_add(src, index, dim=-1, out=None, dim_size=None):\n"
        "    assert src.dim() == 1 and dim in (0, -1) and out is None\n"
        "    size = dim_size if dim_size is not None else (int(index.max()) + 1 if index.numel() else 0)\n"
        "    return torch.zeros(size, dtype=src.dtype, device=src.device).scatter_add_(0, index, src)\n"),
    "torch_sparse.py": (
        "import torch\n"
        "def coalesce(index, value, m, n, op='add'):\n"
        "    assert op == 'add'\n"
        "    if index.shape[1] == 0:\n"
        "        return index, value\n"
        "    row, col = index[0], index[1]\n"
        "    key = n * row + col\n"
        "    key, perm = key.sort(stable=True)\n"
        "    row, col, value = row[perm], col[perm], value[perm]\n"
        "    mask = torch.ones(key.numel(), dtype=torch.bool)\n"
        "    mask[1:] = key[1:] > key[:-1]\n"
        "    ptr = torch.cat([mask.nonzero().flatten(), torch.tensor([key.numel()])])\n"
        "    out = torch.stack([value[ptr[i]:ptr[i + 1]].sum(0) if ptr[i + 1] - ptr[i] > 1 else value[ptr[i]]\n"
        "                       for i in range(ptr.numel() - 1)])\n"
        "    return torch.stack([row[mask], col[mask]], dim=0), out\n"
        "def spspmm(*a, **k):\n    raise ImportError('torch_sparse stub')\n"
        "spmm = spspmm\nclass SparseTensor:\n    pass\n"),
    "torch_geometric/__init__.py": "",
    "torch_geometric/utils.py": (
        "import torch\n"
        "def add_self_loops(edge_index, edge_attr=None, fill_value=None, num_nodes=None):\n"
        "    N = int(num_nodes) if num_nodes is not None else int(edge_index.max()) + 1\n"
        "    loop = torch.arange(0, N, dtype=torch.long, device=edge_index.device).unsqueeze(0).repeat(2, 1)\n"
        "    if edge_attr is not None:\n"
        "        fill = 1. if fill_value is None else fill_value\n"
        "        edge_attr = torch.cat([edge_attr, edge_attr.new_full((N,) + edge_attr.size()[1:], fill)], dim=0)\n"
        "    return torch.cat([edge_index, loop], dim=1), edge_attr\n"
        "def to_scipy_sparse_matrix(*a, **k):\n    raise ImportError('torch_geometric stub')\n"),
}

OPS = {
    # name: (module, class, kwargs)
    "mag_lap": ("symmetrical_directed_magnetic_laplacian_operator", "SymDirMagLaplacianGraphOp", {"r": 0.5, "q": 0.25}),
    "mag_lap_q01_r03": ("symmetrical_directed_magnetic_laplacian_operator", "SymDirMagLaplacianGraphOp",
                        {"r": 0.3, "q": 0.1}),
    "mag_comppr": ("symmetrical_directed_magnetic_comppr_operator", "SymDirMagComPprGraphOp",
                   {"r": 0.5, "q": 0.25, "ppr_alpha": 0.15}),
    "fast_ppr": ("symmetrical_directed_fast_ppr_approximate_operator", "SymDirFastPprApproxGraphOp",
                 {"r": 0.5, "ppr_alpha": 0.1}),
    "two_dir": ("in_out_directed_laplacian_operator", "TwoDirLaplacianGraphOp", {"r": 0.5}),
    "two_order": ("symmetrical_directed_two_order_ppr_approximate_operator", "SymDirTwoOrderPprApproxGraphOp",
                  {"r": 0.5, "ppr_alpha": 0.1}),
}


def import_reference():
    if not os.path.exists(MG.REF_LIB):
        raise SystemExit(f"{MG.REF_LIB} missing: run `make -C oracle` first")
    stub_dir = tempfile.mkdtemp(prefix="srg_dir_stubs_")
    for name, text in _STUBS.items():
        path = os.path.join(stub_dir, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(text)
    sys.dont_write_bytecode = True
    sys.path[:0] = [stub_dir, MG.REF_SSRG]
    import scipy
    scipy.newaxis = np.newaxis
    import numpy.ctypeslib as ctl

    def redirected(libname, loader_path):
        if os.path.basename(libname) == "libmatmul.so":
            return ctypes.cdll.LoadLibrary(MG.REF_LIB)
        raise RuntimeError(f"unexpected native library request {libname!r}")

    ctl.load_library = redirected
    import importlib
    classes = {}
    for key, (mod, cls, _) in OPS.items():
        classes[key] = getattr(importlib.import_module(f"operators.graph_operator.{mod}"), cls)
    from operators.utils import PyGSD_adj_to_directed_symmetric_mag_norm
    return classes, PyGSD_adj_to_directed_symmetric_mag_norm


def directed_random(n, density, seed):
    """A directed weighted graph: dyadic weights, reciprocal pairs with different weights, self-loops,
    a hub row and column, rows and columns with no entry."""
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < density
    mask[n // 3, :] = rng.random(n) < 0.5
    mask[:, n // 4] = rng.random(n) < 0.5
    mask[[2, n // 2], :] = False
    mask[:, [3, n - 3]] = False
    np.fill_diagonal(mask, rng.random(n) < 0.15)
    w = rng.integers(1, 17, size=(n, n)) / 4.0
    return sp.csr_matrix(np.where(mask, w, 0.0))


def csr_arrays(prefix, m):
    m = m.tocsr()
    return {f"{prefix}_indptr": m.indptr.astype(np.int64), f"{prefix}_indices": m.indices.astype(np.int32),
            f"{prefix}_data": np.asarray(m.data)}


def main():
    classes, pygsd = import_reference()
    synth = MG._load_synth()
    manifest = {}
    graphs = {}
    adj, _ = MG.planetoid_adj("cora_0_0", False)          # as stored: a directed (upper-triangular) graph
    graphs["cora"] = (adj, synth.uniform_features_np(adj.shape[0], 24, seed=80), 3)
    adj = directed_random(90, 0.06, seed=500)
    graphs["rand"] = (adj, synth.uniform_features_np(90, 16, seed=81), 3)
    # edge cases: a single node with a self-loop; one directed edge plus an isolated node; no edges
    graphs["tiny1"] = (sp.csr_matrix(np.array([[2.0]])), synth.uniform_features_np(1, 4, seed=82), 2)
    graphs["tiny3"] = (sp.csr_matrix(np.array([[0.0, 1.5, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]])),
                       synth.uniform_features_np(3, 4, seed=83), 2)
    graphs["empty4"] = (sp.csr_matrix((4, 4)), synth.uniform_features_np(4, 4, seed=84), 2)
    for gname, (adj, X, K) in graphs.items():
        for key, (_, _, kw) in OPS.items():
            if gname != "rand" and key == "mag_lap_q01_r03":
                continue
            op = classes[key](K, **kw)
            try:
                lists = op.propagate(adj, X)
            except Exception as e:  # noqa: BLE001 -- the reference's own failure is the fixture
                name = f"dir_{gname}_{key}"
                manifest[name] = {"n": adj.shape[0], "d": X.shape[1], "k": K, "op": "directed_error",
                                  "operator": key, "class": OPS[key][1], "kwargs": kw, "error": type(e).__name__,
                                  "message": str(e)[:200]}
                np.savez_compressed(os.path.join(MG.OUT, f"{name}.npz"),
                                    adj_indptr=adj.indptr.astype(np.int64), adj_indices=adj.indices.astype(np.int32),
                                    adj_data=adj.data.astype(np.float64), x=X)
                print(name, "raises", type(e).__name__, str(e)[:80], flush=True)
                continue
            if key in ("mag_lap", "mag_lap_q01_r03", "mag_comppr"):
                mats = {"real": op.real_adj, "imag": op.imag_adj}
            elif key == "two_dir":
                mats = {"un": op.un_adj, "in": op.in_adj, "out": op.out_adj}
            elif key == "two_order":
                mats = {"one": op.one_adj, "two": op.two_adj}
            else:
                mats = {"adj": op.adj}
                lists = (lists,)
            arrs = {"adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int32),
                    "adj_data": adj.data.astype(np.float64), "x": X}
            for mname, m in mats.items():
                arrs.update(csr_arrays(f"m_{mname}", m))
            for li, lst in enumerate(lists):
                for k, t in enumerate(lst):
                    arrs[f"list{li}_hop{k}"] = np.ascontiguousarray(t.numpy(), dtype=np.float32)
            name = f"dir_{gname}_{key}"
            np.savez_compressed(os.path.join(MG.OUT, f"{name}.npz"), **arrs)
            manifest[name] = {"n": adj.shape[0], "d": X.shape[1], "k": K, "op": "directed", "operator": key,
                              "class": OPS[key][1], "kwargs": kw, "matrices": list(mats),
                              "dtypes": {k: str(np.asarray(m.data).dtype) for k, m in mats.items()},
                              "lists": len(lists)}
            print(name, {k: (m.nnz, str(m.dtype)) for k, m in mats.items()}, flush=True)
        # utils.py's PyGSD variant (not used by an operator; part of the module's API)
        re, im = pygsd(adj.tocoo(), 0.5, 0.25)
        arrs = {"adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int32),
                "adj_data": adj.data.astype(np.float64)}
        arrs.update(csr_arrays("m_real", re))
        arrs.update(csr_arrays("m_imag", im))
        name = f"dir_{gname}_pygsd_mag"
        np.savez_compressed(os.path.join(MG.OUT, f"{name}.npz"), **arrs)
        manifest[name] = {"n": adj.shape[0], "op": "directed_norm", "operator": "pygsd_mag",
                          "kwargs": {"r": 0.5, "q": 0.25}, "matrices": ["real", "imag"]}
    path = os.path.join(MG.OUT, "manifest.json")
    with open(path) as f:
        full = json.load(f)
    full = {k: v for k, v in full.items() if not k.startswith("dir_")}
    full.update(manifest)
    with open(path, "w") as f:
        json.dump(full, f, indent=1, sort_keys=True)
    print("wrote", len(manifest), "directed cases")


if __name__ == "__main__":
    main()
