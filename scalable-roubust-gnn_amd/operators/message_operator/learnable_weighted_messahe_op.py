"""LearnableWeightedMessageOp (SSRG/operators/message_operator/learnable_weighted_messahe_op.py:10-103,
the file name's spelling kept): GAMLP's learnable hop combination.  Consumes the hop list on whatever
device the model keeps it; same parameters (created in the reference's order, so a seeded run draws
the same initial values), same forward arithmetic.

    simple / simple_allow_neg  (prop_steps)           one weight per hop, softmax(sigmoid(w)) or w itself
    gate                       (feat_dim)             per-node weights from Linear(feat_dim, 1) on each hop
    ori_ref                    (feat_dim)             ... on [hop 0 | hop]
    jk                         (prop_steps, feat_dim) ... on [all hops | hop]
"""
import torch
import torch.nn.functional as F
from torch import nn

from operators.base_operator import MessageOp
from operators.utils import one_dim_weighted_add, squeeze_first_dimension, two_dim_weighted_add

_ARITY = {"simple": 1, "simple_allow_neg": 1, "gate": 1, "ori_ref": 1, "jk": 2}


class LearnableWeightedMessageOp(MessageOp):
    def __init__(self, start, end, combination_type, *args):
        super(LearnableWeightedMessageOp, self).__init__(start, end)
        self.aggr_type = "learnable_weighted"
        if combination_type not in _ARITY:
            raise ValueError(
                "Invalid weighted combination type! Type must be 'simple', 'simple_allow_neg', 'gate', 'ori_ref' or 'jk'.")
        self.combination_type = combination_type
        self.learnable_weight = None
        if len(args) != _ARITY[combination_type]:
            kind = "simple" if combination_type == "simple_allow_neg" else combination_type
            raise ValueError(f"Invalid parameter numbers for the {kind} learnable weighted aggregator!")
        if combination_type in ("simple", "simple_allow_neg"):
            # xavier_normal_ needs a 2-d tensor: draw [1, K+1], keep it flat
            w = torch.FloatTensor(1, args[0] + 1)
            nn.init.xavier_normal_(w)
            self.learnable_weight = nn.Parameter(w.view(-1))
        else:
            in_dim = {"gate": args[0], "ori_ref": 2 * args[0]}.get(combination_type)
            if combination_type == "jk":
                in_dim = args[1] + (args[0] + 1) * args[1]
            self.learnable_weight = nn.Linear(in_dim, 1)

    def _hop_weights(self, feat_list):
        hops = self.end - self.start
        kind = self.combination_type
        if kind == "simple":
            return F.softmax(torch.sigmoid(self.learnable_weight[self.start:self.end]), dim=0)
        if kind == "simple_allow_neg":
            return self.learnable_weight[self.start:self.end]
        stacked = torch.vstack(feat_list[self.start:self.end])
        if kind == "gate":
            scores = self.learnable_weight(stacked).view(hops, -1).T
        else:
            ref = feat_list[0] if kind == "ori_ref" else torch.hstack(feat_list)
            scores = self.learnable_weight(torch.hstack((ref.repeat(hops, 1), stacked))).view(-1, hops)
        return F.softmax(torch.sigmoid(scores), dim=1)

    def combine(self, feat_list):
        feat_list = squeeze_first_dimension(feat_list)
        weights = self._hop_weights(feat_list)
        add = one_dim_weighted_add if self.combination_type in ("simple", "simple_allow_neg") else two_dim_weighted_add
        return add(feat_list[self.start:self.end], weight_list=weights)
