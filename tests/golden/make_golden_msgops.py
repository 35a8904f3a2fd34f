"""Golden fixtures for the learnable / consumer message operators (GAMLP, NAFS and their relatives):
the REFERENCE's own modules, seeded, on fixed hop lists (development container only).

    python tests/golden/make_golden_msgops.py

Imports, unmodified, from "/root/reference/Scalable Spectral Robust GNN/operators/message_operator":
learnable_weighted_messahe_op.LearnableWeightedMessageOp (simple / simple_allow_neg / gate / ori_ref / jk),
iterate_learnable_weighted_message_op.IterateLearnableWeightedMessageOp (recursive) and
over_smooth_distance_op.OverSmoothDistanceWeightedOp, with make_golden.py's import stubs (operators/utils.py
imports torch_sparse / torch_scatter / PyG at module top; these modules never call them).  For each case:
torch.manual_seed(seed), build the op, run combine on the stored hop list; the parameters (state_dict)
and the output are written.  Only data leaves this script.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

CASES = [
    # name, module, class, ctor args (start, end, type, *extra) or (), hops, n, d, seed
    ("lw_simple", "learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (0, 4, "simple", 3), 4, 50, 12, 1),
    ("lw_simple_allow_neg", "learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (1, 4, "simple_allow_neg", 3), 4, 50, 12, 2),
    ("lw_gate", "learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (0, 5, "gate", 12), 5, 40, 12, 3),
    ("lw_ori_ref", "learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (1, 5, "ori_ref", 12), 5, 40, 12, 4),
    ("lw_jk", "learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (0, 4, "jk", 3, 12), 4, 30, 12, 5),
    ("ilw_recursive", "iterate_learnable_weighted_message_op", "IterateLearnableWeightedMessageOp", (0, 5, "recursive", 10), 6, 30, 10, 6),
    ("osd", "over_smooth_distance_op", "OverSmoothDistanceWeightedOp", (), 5, 60, 9, 7),
]


def main():
    MG.import_reference()
    import importlib
    rng = np.random.default_rng(90)
    arrs = {}
    for name, mod, cls, args, hops, n, d, seed in CASES:
        feats = [torch.from_numpy(rng.standard_normal((n, d)).astype(np.float32)) for _ in range(hops)]
        klass = getattr(importlib.import_module(f"operators.message_operator.{mod}"), cls)
        torch.manual_seed(seed)
        op = klass(*args)
        with torch.no_grad():
            out = op.aggregate(feats)
        for k, v in op.state_dict().items():
            arrs[f"{name}__param__{k}"] = v.numpy()
        for h, f in enumerate(feats):
            arrs[f"{name}__hop{h}"] = f.numpy()
        arrs[f"{name}__out"] = out.numpy()
    np.savez_compressed(os.path.join(HERE, "msgops.npz"), **arrs)
    print("wrote", len(CASES), "message-operator cases")


if __name__ == "__main__":
    main()
