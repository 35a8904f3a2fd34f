"""IterateLearnableWeightedMessageOp (SSRG/operators/message_operator/iterate_learnable_weighted_message_op.py:
8-51): 'recursive' combination -- hop i's per-node weight comes from Linear(2 feat_dim, 1) on
[hop i | the running combination], the weights so far are re-softmaxed, and the combination is
rebuilt from hop `start` with them.  Same parameters and arithmetic order as the reference."""
import torch
import torch.nn.functional as F
from torch.nn import Linear

from operators.base_operator import MessageOp


class IterateLearnableWeightedMessageOp(MessageOp):
    def __init__(self, start, end, combination_type, *args):
        super(IterateLearnableWeightedMessageOp, self).__init__(start, end)
        self.aggr_type = "iterate_learnable_weighted"
        if combination_type != "recursive":
            raise ValueError("Invalid weighted combination type! Type must be 'recursive'.")
        self.combination_type = combination_type
        if len(args) != 1:
            raise ValueError("Invalid parameter numbers for the recursive iterate weighted aggregator!")
        self.learnable_weight = Linear(2 * args[0], 1)

    def combine(self, feat_list):
        base = feat_list[self.start]
        combined = base
        weights = None
        for i in range(self.start, self.end):
            w_i = torch.sigmoid(self.learnable_weight(torch.hstack((feat_list[i], combined))))
            weights = w_i if weights is None else torch.hstack((weights, w_i))
            weights = F.softmax(weights, dim=1)
            combined = torch.mul(base, weights[:, 0].view(-1, 1))
            for j in range(1, i + 1):
                combined = combined + torch.mul(feat_list[self.start + j], weights[:, j].view(-1, 1))
        return combined
