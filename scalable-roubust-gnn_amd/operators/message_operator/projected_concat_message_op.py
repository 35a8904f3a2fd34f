"""ProjectedConcatMessageOp (SSRG/operators/message_operator/projected_concat_message_op.py:9-30), SIGN's
combination: hop `start` through its own MLP, every later hop through its own MLP and a ReLU, all
concatenated.  The MLP is the reference's models.base_scalable.simple_models.MultiLayerPerceptron
(the models package stays the reference's own), imported when the op is built."""
import torch
import torch.nn.functional as F
from torch.nn import ModuleList

from operators.base_operator import MessageOp
from operators.utils import squeeze_first_dimension


class ProjectedConcatMessageOp(MessageOp):
    def __init__(self, start, end, feat_dim, hidden_dim, num_layers, dropout):
        super(ProjectedConcatMessageOp, self).__init__(start, end)
        self.aggr_type = "proj_concat"
        from models.base_scalable.simple_models import MultiLayerPerceptron
        self.learnable_weight = ModuleList(
            MultiLayerPerceptron(feat_dim, hidden_dim, num_layers, hidden_dim, dropout) for _ in range(end - start))

    def combine(self, feat_list):
        hops = squeeze_first_dimension(feat_list)[self.start:self.end]
        out = self.learnable_weight[0](hops[0])
        for mlp, hop in zip(self.learnable_weight[1:], hops[1:]):
            out = torch.hstack((out, F.relu(mlp(hop))))
        return out
