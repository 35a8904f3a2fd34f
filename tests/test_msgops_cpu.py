"""The learnable / consumer message operators (GAMLP, NAFS, SIGN and relatives) against the REFERENCE's
own modules (tests/golden/msgops.npz, tests/golden/make_golden_msgops.py): seeded construction gives
the same parameters, and combine the same output, bit for bit, on the CPU."""
import importlib
import sys
import types

import numpy as np
import pytest
import torch

import golden_cases as G

CASES = {
    "lw_simple": ("learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (0, 4, "simple", 3), 4, 1),
    "lw_simple_allow_neg": ("learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (1, 4, "simple_allow_neg", 3), 4, 2),
    "lw_gate": ("learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (0, 5, "gate", 12), 5, 3),
    "lw_ori_ref": ("learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (1, 5, "ori_ref", 12), 5, 4),
    "lw_jk": ("learnable_weighted_messahe_op", "LearnableWeightedMessageOp", (0, 4, "jk", 3, 12), 4, 5),
    "ilw_recursive": ("iterate_learnable_weighted_message_op", "IterateLearnableWeightedMessageOp", (0, 5, "recursive", 10), 6, 6),
    "osd": ("over_smooth_distance_op", "OverSmoothDistanceWeightedOp", (), 5, 7),
}


@pytest.fixture(scope="module")
def golden():
    return np.load(f"{G.GOLDEN}/msgops.npz", allow_pickle=False)


@pytest.mark.parametrize("name", sorted(CASES))
def test_message_op_equals_reference(golden, name):
    mod, cls, args, hops, seed = CASES[name]
    klass = getattr(importlib.import_module(f"operators.message_operator.{mod}"), cls)
    torch.manual_seed(seed)
    op = klass(*args)
    params = {k[len(name) + 9:]: golden[k] for k in golden.files if k.startswith(f"{name}__param__")}
    mine = op.state_dict()
    assert sorted(mine) == sorted(params)
    for k, v in params.items():
        assert np.array_equal(mine[k].numpy(), v), f"{name}: parameter {k} differs"
    feats = [torch.from_numpy(golden[f"{name}__hop{h}"]) for h in range(hops)]
    with torch.no_grad():
        out = op.aggregate(feats)
    assert np.array_equal(out.numpy(), golden[f"{name}__out"])


def test_message_op_errors_match_reference():
    from operators.message_operator.iterate_learnable_weighted_message_op import IterateLearnableWeightedMessageOp
    from operators.message_operator.learnable_weighted_messahe_op import LearnableWeightedMessageOp
    with pytest.raises(ValueError, match="Type must be 'simple'"):
        LearnableWeightedMessageOp(0, 2, "mean", 3)
    with pytest.raises(ValueError, match="for the simple learnable"):
        LearnableWeightedMessageOp(0, 2, "simple_allow_neg")
    with pytest.raises(ValueError, match="for the jk learnable"):
        LearnableWeightedMessageOp(0, 2, "jk", 3)
    with pytest.raises(ValueError, match="'recursive'"):
        IterateLearnableWeightedMessageOp(0, 2, "gate", 3)
    # the reference indexes the weights by absolute hop, so start > 0 fails on its second hop
    op = IterateLearnableWeightedMessageOp(1, 3, "recursive", 4)
    with pytest.raises(IndexError):
        op.aggregate([torch.ones(5, 4) for _ in range(3)])


def test_projected_concat_structure():
    """SIGN's op with a stand-in for the reference's MultiLayerPerceptron (models/ stays the
    reference's): hop `start` through MLP 0, later hops through their MLP and a ReLU, concatenated."""
    fake = types.ModuleType("models.base_scalable.simple_models")

    class MultiLayerPerceptron(torch.nn.Module):
        def __init__(self, nfeat, hidden, num_layers, nclass, dropout):
            super().__init__()
            self.lin = torch.nn.Linear(nfeat, nclass)

        def forward(self, x):
            return self.lin(x)
    fake.MultiLayerPerceptron = MultiLayerPerceptron
    saved = {k: sys.modules.get(k) for k in ("models", "models.base_scalable", "models.base_scalable.simple_models")}
    sys.modules["models"] = types.ModuleType("models")
    sys.modules["models.base_scalable"] = types.ModuleType("models.base_scalable")
    sys.modules["models.base_scalable.simple_models"] = fake
    try:
        from operators.message_operator.projected_concat_message_op import ProjectedConcatMessageOp
        torch.manual_seed(0)
        op = ProjectedConcatMessageOp(1, 4, 6, 5, 2, 0.0)
        feats = [torch.randn(7, 6) for _ in range(5)]
        out = op.aggregate(feats)
        want = torch.hstack([op.learnable_weight[0](feats[1])] +
                            [torch.relu(op.learnable_weight[i](feats[1 + i])) for i in (1, 2)])
        assert out.shape == (7, 15) and torch.equal(out, want)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
