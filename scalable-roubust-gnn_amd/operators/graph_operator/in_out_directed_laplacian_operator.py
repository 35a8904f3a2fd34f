"""TwoDirLaplacianGraphOp (SSRG/operators/graph_operator/in_out_directed_laplacian_operator.py:7-16):
the undirected, in- and out-direction operators of utils.py:195-260 (built on the GPU) propagated by
the two-direction family (TwoDirGraphOp)."""
from operators.base_operator import TwoDirGraphOp
from operators.utils import adj_to_un_in_out_dir_symmetric_norm


class TwoDirLaplacianGraphOp(TwoDirGraphOp):
    def __init__(self, prop_steps, r=0.5):
        super(TwoDirLaplacianGraphOp, self).__init__(prop_steps)
        self.r = r

    def construct_adj(self, adj):
        un, i, o = adj_to_un_in_out_dir_symmetric_norm(adj.tocoo(), self.r)
        return un.tocsr(), i.tocsr(), o.tocsr()
