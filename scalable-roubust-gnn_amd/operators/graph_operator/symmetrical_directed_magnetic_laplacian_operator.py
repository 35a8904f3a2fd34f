"""SymDirMagLaplacianGraphOp (SSRG/operators/graph_operator/symmetrical_directed_magnetic_laplacian_
operator.py:7-16): the magnetic Laplacian's real and imaginary operators (utils.py:95-138, built on
the GPU) propagated by the complex family (ComGraphOp), every product on the GPU."""
from operators.base_operator import ComGraphOp
from operators.utils import adj_to_directed_symmetric_mag_norm, PyGSD_adj_to_directed_symmetric_mag_norm  # noqa: F401


class SymDirMagLaplacianGraphOp(ComGraphOp):
    def __init__(self, prop_steps, r=0.5, q=0.25):
        super(SymDirMagLaplacianGraphOp, self).__init__(prop_steps)
        self.r = r
        self.q = q

    def construct_adj(self, adj):
        return adj_to_directed_symmetric_mag_norm(adj.tocoo(), self.r, self.q)
