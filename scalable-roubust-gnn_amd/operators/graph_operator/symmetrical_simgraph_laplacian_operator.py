"""SymLaplacianGraphOp: Â = D^(r-1) (A+I)^T D^(-r), the operator every precompute model uses
(SSRG/operators/graph_operator/symmetrical_simgraph_laplacian_operator.py:7-15)."""
import scipy.sparse as sp  # noqa: F401

from operators.base_operator import GraphOp
from operators.utils import adj_to_symmetric_norm


class SymLaplacianGraphOp(GraphOp):
    def __init__(self, prop_steps, r=0.5):
        super(SymLaplacianGraphOp, self).__init__(prop_steps)
        self.r = r

    def construct_adj(self, adj):
        return adj_to_symmetric_norm(adj.tocoo(), self.r).tocsr()

    def construct_adj_device(self, adj, device):
        """construct_adj on the GPU (srgnn.construct.sym_norm), bit-identical to the host scipy."""
        from srgnn.construct import sym_norm
        return sym_norm(adj.indptr, adj.indices, adj.data, adj.shape[0], self.r, device=device)
