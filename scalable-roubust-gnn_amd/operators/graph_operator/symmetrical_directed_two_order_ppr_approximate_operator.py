"""SymDirTwoOrderPprApproxGraphOp (SSRG/operators/graph_operator/symmetrical_directed_two_order_ppr_
approximate_operator.py:7-17): first- and second-order PPR-approximated operators of
utils.py:324-424 (built on the GPU) propagated by the two-order family (TwoOrderPprApproxGraphOp)."""
from operators.base_operator import TwoOrderPprApproxGraphOp
from operators.utils import adj_to_slow_first_second_ppr_approx_symmetric_norm


class SymDirTwoOrderPprApproxGraphOp(TwoOrderPprApproxGraphOp):
    def __init__(self, prop_steps, r=0.5, ppr_alpha=0.1):
        super(SymDirTwoOrderPprApproxGraphOp, self).__init__(prop_steps)
        self.r = r
        self.ppr_alpha = ppr_alpha

    def construct_adj(self, adj):
        return adj_to_slow_first_second_ppr_approx_symmetric_norm(adj.tocoo(), self.r, self.ppr_alpha)
