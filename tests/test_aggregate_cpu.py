"""Host logic of the fused hop aggregation (srgnn.aggregate): the planned order of element-wise
steps, executed here with numpy fp32 arithmetic, reproduces the reference's MessageOp.combine
(oracle.combine = the reference's torch CPU operations) bit for bit.  No GPU."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scalable-roubust-gnn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from oracle import oracle as O  # noqa: E402
from srgnn import aggregate as G  # noqa: E402

f32 = np.float32


def run_steps_np(steps, hops, n, d):
    """numpy model of aggregate._DeviceSteps (INIT / ADD / fold / DIV / tail record / row_sum)."""
    slots, hist = {}, {}
    ts, tl = G.tail_range(n, d)
    for s in steps:
        if s[0] == "acc":
            _, slot, k, w = s
            p = (f32(w) * hops[k]).astype(f32)
            slots[slot] = (slots.get(slot, np.zeros((n, d), f32)) + p).astype(f32)
        elif s[0] == "fold":
            _, dst, src = s
            if src in slots:
                slots[dst] = slots.pop(src) if dst not in slots else (slots[dst] + slots.pop(src)).astype(f32)
        elif s[0] == "div":
            slots[0] = (slots.get(0, np.zeros((n, d), f32)) / f32(s[1])).astype(f32)
        elif s[0] == "tail":
            _, k, w, t = s
            hist[t] = (f32(w) * hops[k].reshape(-1)[ts:ts + tl]).astype(f32)
        elif s[0] == "rowsum":
            T = s[1]
            if tl == 0 or T == 0:
                continue

            def mrs(rows):
                size = len(rows)
                clog2 = 1 if size <= 2 else (size - 1).bit_length()
                lp = max(4, clog2 // 4)
                step, mask = 1 << lp, (1 << lp) - 1
                acc = [np.zeros(tl, f32) for _ in range(4)]
                i = 0
                while i + step <= size:
                    for _ in range(step):
                        acc[0] = (acc[0] + rows[i]).astype(f32)
                        i += 1
                    for j in range(1, 4):
                        acc[j] = (acc[j] + acc[j - 1]).astype(f32)
                        acc[j - 1] = np.zeros(tl, f32)
                        if i & (mask << (j * lp)):
                            break
                while i < size:
                    acc[0] = (acc[0] + rows[i]).astype(f32)
                    i += 1
                for j in range(1, 4):
                    acc[0] = (acc[0] + acc[j]).astype(f32)
                return acc[0]
            rows = [hist[t] for t in range(T)]
            n4 = T // 4
            p = [mrs(rows[c::4][:n4]) for c in range(4)]
            for i in range(4 * n4, T):
                p[0] = (p[0] + rows[i]).astype(f32)
            for c in range(1, 4):
                p[0] = (p[0] + p[c]).astype(f32)
            flat = slots.setdefault(0, np.zeros((n, d), f32)).reshape(-1)
            flat[ts:] = (f32(0) + p[0]).astype(f32)
    return slots.get(0, np.zeros((n, d), f32))


class _Msg:
    def __init__(self, aggr, start=None, end=None, combination_type=None, alpha=None, weight_list=None):
        self.aggr_type, self.start, self.end = aggr, start, end
        self.combination_type, self.alpha, self.weight_list = combination_type, alpha, weight_list


def _hops(n, d, K, seed):
    rng = np.random.default_rng(seed)
    hs = [rng.standard_normal((n, d)).astype(f32) * f32(2.0 ** -k) for k in range(K + 1)]
    hs[1][0, :] = -0.0                           # signed zeros in a hop
    return hs


def _ref(msg, hops):
    feats = [torch.from_numpy(h.copy()) for h in hops]
    if msg.aggr_type == "simple_weighted":
        return O.combine(msg.aggr_type, feats, msg.start, msg.end, alpha=msg.alpha, weight_list=msg.weight_list).numpy()
    return O.combine(msg.aggr_type, feats, msg.start, msg.end).numpy()


def _fused_np(msg, hops):
    """Plan -> hop schedule (as propagate_aggregate consumes it) -> numpy execution."""
    mode, terms, div = G.combine_plan(msg, len(hops))
    if mode == "last":
        return hops[-1]
    n, d = hops[0].shape
    steps = G.combine_steps(mode, terms, div)
    groups, trailing = G.schedule(steps)
    assert len(groups) <= len(hops)
    flat = [s for g in groups for s in g] + trailing
    assert sorted(map(id, flat)) == sorted(map(id, steps))
    for k, g in enumerate(groups):
        assert all(G.step_hop(s) in (k, None) for s in g)
    return run_steps_np(flat, hops, n, d)


SHAPES = [(7, 1), (3, 3), (5, 7), (40, 33), (101, 13), (256, 128), (37, 500)]


@pytest.mark.parametrize("n,d", SHAPES)
@pytest.mark.parametrize("K", [1, 2, 3, 5, 10, 15, 16, 17, 20, 33, 70])
def test_weighted_alpha_bit_exact(n, d, K):
    hops = _hops(n, d, K, seed=n * 1000 + K)
    for start, end in [(None, None), (1, None), (0, K + 1), (2, K)]:
        if len(range(K + 1)[slice(start, end)]) == 0:
            continue
        msg = _Msg("simple_weighted", start, end, "alpha", alpha=0.15)
        np.testing.assert_array_equal(_fused_np(msg, hops), _ref(msg, hops), err_msg=f"{n}x{d} K={K} {start}:{end}")


@pytest.mark.parametrize("n,d", SHAPES)
@pytest.mark.parametrize("K", [1, 3, 10, 20])
def test_sum_mean_last_bit_exact(n, d, K):
    hops = _hops(n, d, K, seed=K)
    for msg in [_Msg("last"), _Msg("sum", 0, K + 1), _Msg("sum", 1, K), _Msg("mean", 0, K + 1),
                _Msg("mean", 2, K + 1), _Msg("mean", 0, K + 3)]:
        if msg.aggr_type != "last" and not range(K + 1)[slice(msg.start, msg.end)]:
            continue
        np.testing.assert_array_equal(_fused_np(msg, hops), _ref(msg, hops),
                                      err_msg=f"{msg.aggr_type} {msg.start}:{msg.end}")


def test_hand_crafted_weights():
    hops = _hops(50, 21, 4, seed=3)
    w = [0.5, -0.25, 1.0 / 3.0]
    msg = _Msg("simple_weighted", 1, 4, "hand_crafted", weight_list=torch.FloatTensor(w))
    np.testing.assert_array_equal(_fused_np(msg, hops), _ref(msg, hops))
    bad = _Msg("simple_weighted", 0, 4, "hand_crafted", weight_list=torch.FloatTensor(w))
    with pytest.raises(ValueError):
        G.combine_plan(bad, 5)
    with pytest.raises(ValueError):
        G.combine_plan(_Msg("simple_weighted", 1, 4, "hand_crafted",
                            weight_list=torch.tensor(w, dtype=torch.float64)), 5)
    with pytest.raises(ValueError):
        G.combine_plan(_Msg("learnable_weighted"), 5)
    with pytest.raises(ValueError):
        G.combine_plan(_Msg("sum", 4, 2), 5)


def test_plan_shape():
    # <= 15 terms: one sequential chain; 16..31: a 16-term block folded into level 1
    steps = G.combine_steps("weighted", [(k, 1.0) for k in range(20)])
    kinds = [s[0] for s in steps]
    assert kinds.count("acc") == 20 and kinds.count("tail") == 20 and kinds[-1] == "rowsum"
    assert ("fold", 1, 0) in steps
    assert G.tail_range(2708, 1433) == (2708 * 1433 // 32 * 32, 2708 * 1433 % 32)
    assert G.tail_range(1, 7) == (4, 3) and G.tail_range(2449029, 128)[1] == 0


def test_operators_utils_helpers():
    """operators.utils weighted adds / squeeze (host helpers the reference's message operators call,
    utils.py:426-460): same values and error classes as the reference's definitions."""
    from operators.utils import one_dim_weighted_add, squeeze_first_dimension, two_dim_weighted_add
    g = torch.Generator().manual_seed(0)
    feats = [torch.randn(5, 3, generator=g) for _ in range(4)]
    w = torch.tensor([0.5, -1.0, 0.25, 2.0])
    want = sum(wi * f for wi, f in zip(w, feats))
    torch.testing.assert_close(one_dim_weighted_add(feats, w), want)
    w2 = torch.randn(5, 4, generator=g)
    want2 = sum(w2[:, i:i + 1] * f for i, f in enumerate(feats))
    torch.testing.assert_close(two_dim_weighted_add(feats, w2), want2)
    with pytest.raises(TypeError):
        one_dim_weighted_add(feats, w.tolist())
    with pytest.raises(ValueError):
        one_dim_weighted_add(feats, w[:3])
    with pytest.raises(IndexError):                # the reference indexes shape[1] before its 2-d check
        two_dim_weighted_add(feats, w)
    with pytest.raises(ValueError):
        two_dim_weighted_add(feats, w2[:, :3])
    batched = [f.unsqueeze(0) for f in feats]
    out = squeeze_first_dimension(batched)
    assert out is batched and all(torch.equal(a, b) for a, b in zip(out, feats))
    assert torch.equal(squeeze_first_dimension(feats[0].unsqueeze(0)), feats[0])
    assert squeeze_first_dimension(feats[0]) is feats[0]
