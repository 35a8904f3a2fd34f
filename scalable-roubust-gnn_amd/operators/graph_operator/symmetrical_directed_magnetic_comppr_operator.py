"""SymDirMagComPprGraphOp (SSRG/operators/graph_operator/symmetrical_directed_magnetic_comppr_
operator.py:26-37): complex personalised PageRank on the magnetic Laplacian,
real' = (1 - alpha) real + alpha I, imag' = (1 - alpha) imag, built on the GPU (srgnn.directed.
magnetic_com_ppr, bit-identical to the reference's scipy arithmetic: the canonical sum drops zero
results, the scalar product keeps the structure)."""
from operators.base_operator import ComGraphOp
from operators.utils import _coo_of, _scipy


class SymDirMagComPprGraphOp(ComGraphOp):
    def __init__(self, prop_steps, r=0.5, q=0.25, ppr_alpha=0.15):
        super(SymDirMagComPprGraphOp, self).__init__(prop_steps)
        self.r = r
        self.q = q
        self.ppr_alpha = ppr_alpha

    def construct_adj(self, adj):
        from srgnn.directed import magnetic_com_ppr
        row, col, data, n = _coo_of(adj.tocoo())
        re, im = magnetic_com_ppr(row, col, data, n, self.r, self.q, self.ppr_alpha)
        return _scipy(re, n), _scipy(im, n)
