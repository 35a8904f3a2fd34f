"""OverSmoothDistanceWeightedOp (SSRG/operators/message_operator/over_smooth_distance_op.py:6-33), NAFS's
combination: per node, hop j weighted by softmax_j of the cosine similarity between hop 0 and hop j
(norms + 1e-10).  The reference accumulates node by node in Python (`fea = 0.; fea += w[i][j] *
hop_j[i]` for j in order); here the same per-element products and left-to-right additions from 0
run as whole-panel operations, one per hop -- the same bits, without N * hops Python steps."""
import torch
import torch.nn.functional as F

from operators.base_operator import MessageOp


class OverSmoothDistanceWeightedOp(MessageOp):
    def __init__(self):
        super(OverSmoothDistanceWeightedOp, self).__init__()
        self.aggr_type = "over_smooth_dis_weighted"

    def combine(self, feat_list):
        first = feat_list[0]
        n0 = torch.norm(first, 2, 1).add(1e-10)
        sims = []
        for hop in feat_list:
            nh = torch.norm(hop, 2, 1).add(1e-10)
            sims.append(torch.div(torch.div((first * hop).sum(1), nh), n0).unsqueeze(-1))
        weight = F.softmax(torch.cat(sims, dim=1), dim=1)
        out = torch.zeros_like(first, dtype=torch.result_type(weight, first))
        for j, hop in enumerate(feat_list):
            out = out + weight[:, j:j + 1] * hop
        return out
