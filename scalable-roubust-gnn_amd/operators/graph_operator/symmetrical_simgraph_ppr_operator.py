"""PprGraphOp: (1 - alpha) Â + alpha I (SSRG/operators/graph_operator/
symmetrical_simgraph_ppr_operator.py:7-21).  Same GraphOp path, different operator values."""
import scipy.sparse as sp

from operators.base_operator import GraphOp
from operators.utils import adj_to_symmetric_norm


class PprGraphOp(GraphOp):
    def __init__(self, prop_steps, r=0.5, alpha=0.15):
        super(PprGraphOp, self).__init__(prop_steps)
        self.r = r
        self.alpha = alpha

    def construct_adj(self, adj):
        if isinstance(adj, sp.csr_matrix):
            adj = adj.tocoo()
        elif not isinstance(adj, sp.coo_matrix):
            raise TypeError("The adjacency matrix must be a scipy.sparse.coo_matrix/csr_matrix!")
        norm = adj_to_symmetric_norm(adj, self.r)
        return ((1 - self.alpha) * norm + self.alpha * sp.eye(adj.shape[0])).tocsr()

    def construct_adj_device(self, adj, device):
        """construct_adj on the GPU (srgnn.construct.ppr_norm), bit-identical to the host scipy."""
        from srgnn.construct import ppr_norm
        return ppr_norm(adj.indptr, adj.indices, adj.data, adj.shape[0], self.r, self.alpha, device=device)
