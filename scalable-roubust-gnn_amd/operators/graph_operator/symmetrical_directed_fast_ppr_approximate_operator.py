"""SymDirFastPprApproxGraphOp (SSRG/operators/graph_operator/symmetrical_directed_fast_ppr_
approximate_operator.py:7-17): GraphOp over the fast PPR-approximated symmetric operator
(utils.py:262-322).  construct_adj_device builds it on the GPU and the hops run there with the
reference's fp32 product (the operator's values: a few ulps from the reference's, see utils)."""
from operators.base_operator import GraphOp
from operators.utils import adj_to_fast_ppr_approx_symmetric_norm


class SymDirFastPprApproxGraphOp(GraphOp):
    def __init__(self, prop_steps, r=0.5, ppr_alpha=0.1):
        super(SymDirFastPprApproxGraphOp, self).__init__(prop_steps)
        self.r = r
        self.ppr_alpha = ppr_alpha

    def construct_adj(self, adj):
        return adj_to_fast_ppr_approx_symmetric_norm(adj.tocoo(), self.r, self.ppr_alpha)

    def construct_adj_device(self, adj, device):
        from srgnn.directed import fast_ppr_norm
        coo = adj.tocoo()
        return fast_ppr_norm(coo.row, coo.col, adj.shape[0], self.r, self.ppr_alpha, device=device)
