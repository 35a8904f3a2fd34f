"""The other operator families (SSRG/operators/base_operator.py:60-307: two-order PPR
approximation, complex/magnetic, un/in/out directed) vs the reference's own base classes
(tests/golden/fam_*.npz, made by make_golden.py with scipy-only construct_adj subclasses)."""
import numpy as np
import pytest

import golden_cases as G

FAMILIES = {"two_order": "TwoOrderPprApproxGraphOp", "complex": "ComGraphOp", "two_dir": "TwoDirGraphOp"}


def _check(c, lists):
    for li, lst in enumerate(lists):
        assert len(lst) == c.k + 1
        for k, h in enumerate(lst):
            h = np.ascontiguousarray(np.asarray(h), dtype=np.float32)
            np.testing.assert_array_equal(h, c[f"list{li}_hop{k}"], err_msg=f"{c.name} list {li} hop {k}")
            assert G.sha(h) == str(c[f"list{li}_hop{k}_sha256"])


@pytest.mark.parametrize("name", G.names("family"))
def test_family_restatement_with_oracle(oracle_mod, name):
    """The families' algorithms (this build's host mirrors: calculator, calculate_real_imag_feat)
    with the oracle's fp32 product equal the reference's outputs."""
    from operators.base_operator import calculate_real_imag_feat, calculator
    from operators.utils import adj_to_symmetric_norm
    c = G.Case(name)
    fam = c.meta["family"]
    adjs = G.family_construct(fam, adj_to_symmetric_norm)(c.adj())
    x = c["x"]

    def mm(a, v):
        return oracle_mod.spmm(a.indptr, a.indices, a.data.astype(np.float32), v)

    if fam != "complex":
        lists = [[x] + [h for h in oracle_mod.propagate(a.indptr, a.indices, a.data.astype(np.float32), x, c.k)[1:]]
                 for a in adjs]
    else:
        ar, ai = adjs
        r0, i0 = calculator(x), calculator(x)
        real, imag = [r0.value], [i0.value]
        tin, tout = [], []
        for step in range(c.k):
            if step == 0:
                r0.set_variable(mm(ar, real[-1]), r=True); tin.append(r0); real.append(r0.value)
                i0.set_variable(mm(ai, imag[-1]), i=True); tin.append(i0); imag.append(i0.value)
            else:
                for t in tin:
                    nc = calculator(t.value, t.r_step, t.i_step); nc.set_variable(mm(ar, t.value), r=True); tout.append(nc)
                for t in tin:
                    nc = calculator(t.value, t.r_step, t.i_step); nc.set_variable(mm(ai, t.value), i=True)
                    nc.reversal(); tout.append(nc)
                rf, imf = calculate_real_imag_feat(tout)
                real.append(rf); imag.append(imf)
                tin, tout = tout, []
        lists = [real, imag]
    _check(c, lists)


@pytest.mark.gpu
@pytest.mark.parametrize("name", G.names("family"))
def test_family_gpu_equals_reference(name):
    import operators.base_operator as B
    from operators.utils import adj_to_symmetric_norm
    c = G.Case(name)
    fam = c.meta["family"]
    cons = G.family_construct(fam, adj_to_symmetric_norm)
    cls = type(f"T_{fam}", (getattr(B, FAMILIES[fam]),), {"construct_adj": lambda self, a: cons(a)})
    lists = cls(c.k).propagate(c.adj(), c["x"])
    _check(c, [[t.numpy() for t in lst] for lst in lists])
    with pytest.raises(TypeError):                       # construct_adj accepts coo; the check then refuses it
        cls(c.k).propagate(c.adj().tocoo(), c["x"])
    with pytest.raises(ValueError):
        cls(c.k).propagate(c.adj(), c["x"][:-1])


def test_family_message_ops():
    import torch
    from operators.message_operator.twodir_message_operator.twodir_last_message_op import TwoDirLastMessageOp
    from operators.message_operator.twoorder_message_operator.twoorder_last_message_op import TwoOrderLastMessageOp
    a = [torch.zeros(2), torch.ones(2)]
    b = [torch.ones(2), torch.full((2,), 2.0)]
    assert TwoOrderLastMessageOp().aggregate(a, b)[1].tolist() == [2.0, 2.0]
    assert TwoDirLastMessageOp().aggregate(a, b, a)[2].tolist() == [1.0, 1.0]
    with pytest.raises(TypeError):
        TwoOrderLastMessageOp().aggregate([np.zeros(2)], b)
