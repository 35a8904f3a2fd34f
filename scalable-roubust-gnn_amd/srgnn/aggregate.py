"""Fused hop aggregation: the precompute of SGC / SSGC / GBP-style models without the K+1 panels.

The reference builds the whole hop list [X, ÂX, …, Â^K X] (GraphOp.propagate, SSRG/operators/
base_operator.py:19-36) and then combines it on the host (BaseSGModel.preprocess, SSRG/models/
base_scalable/base_model.py:34-44, via the MessageOp of the model):

    last            feat_list[-1]                                   (last_message_op.py:9-10)
    sum             sum(feat_list[start:end])                       (sum_message_op.py:9-10)
    mean            sum(feat_list[start:end]) / (end - start)       (mean_message_op.py:9-10)
    simple_weighted one_dim_weighted_add(feat_list[start:end], w)   (simple_weighted_message_op.py:36-53,
                    w = [alpha, alpha(1-alpha), ...][start:end] or a hand-crafted list;  utils.py:426-437)

Here the hops run on the GPU with two ping-pong panels and one or two accumulators: memory is
4-5 panels instead of K+1 (papers100M-sized features fit one MI355X), nothing goes to the host.

Exactness.  Python's sum() is ((0 + f0) + f1) + ...; one_dim_weighted_add is torch's CPU dim-0
sum of the rounded products f_k * w_k over the flattened [T, n*d] stack, whose order is ATen's
cascade_sum (SumKernel.cpp): 16-term blocks folded into up to 4 level accumulators, and for the
last (n*d mod 32) flat elements the scalar row_sum order (4 interleaved partials).  `combine_steps`
plans exactly that order as element-wise steps (INIT / ADD / DIV / fold / tail), which the HIP
kernels execute with separate multiply / add / divide -- bit-identical to the reference on the
same hops.  (For n*d == 1 torch uses its whole-tensor reduction: exact only below 8 terms.)
"""
from __future__ import annotations

import torch

from . import _lib
from .csr import DeviceCSR
from .spmm import hop, spmm, spmm_agg  # noqa: F401


def _slice_indices(n: int, start, end):
    return list(range(n))[slice(start, end)]


def combine_plan(msg_op, n_hops: int):
    """(mode, [(hop, fp32 weight)], divisor) reproducing `msg_op.combine(feat_list)` for a list of
    n_hops = K + 1 panels.  Raises ValueError for learnable / non-linear message operators."""
    aggr = getattr(msg_op, "aggr_type", None)
    start, end = getattr(msg_op, "start", None), getattr(msg_op, "end", None)
    if aggr == "last":
        return "last", [(n_hops - 1, 1.0)], None
    if aggr in ("sum", "mean"):
        hops = _slice_indices(n_hops, start, end)
        if not hops:
            raise ValueError("empty hop slice: the reference's sum() of it is the int 0, not a panel")
        div = float(end - start) if aggr == "mean" else None
        return aggr, [(k, 1.0) for k in hops], div
    if aggr == "simple_weighted":
        hops = _slice_indices(n_hops, start, end)
        if msg_op.combination_type == "alpha":
            w = [msg_op.alpha]
            for _ in range(n_hops - 1):
                w.append((1 - msg_op.alpha) * w[-1])
            w32 = torch.FloatTensor(w[start:end]).tolist()
        else:
            wl = msg_op.weight_list
            if isinstance(wl, torch.Tensor) and wl.dtype != torch.float32:
                raise ValueError("fused aggregation takes float32 weights (the reference promotes "
                                 f"the result to {wl.dtype} for {wl.dtype} weights)")
            w32 = torch.as_tensor(wl, dtype=torch.float32).reshape(-1).tolist()
        if len(w32) != len(hops):
            raise ValueError("The feature list and the weight list have different lengths!")
        return "weighted", list(zip(hops, w32)), None
    raise ValueError(f"message operator {aggr!r} has no fused form (learnable or non-linear)")


def tail_range(n: int, d: int):
    """(flat_start, length) of the elements torch's dim-0 sum of [T, n*d] reduces in row_sum order."""
    m = n * d
    ts = (m // 32) * 32 if m >= 8 else (m // 4) * 4
    return ts, m - ts


def combine_steps(mode: str, terms, divisor=None):
    """The reference's accumulation order for `terms` = [(hop, fp32 weight)] as a list of steps:
      ("acc", slot, hop, w)   slot = slot + w * hop   (slot starts as +0: first use is INIT)
      ("fold", dst, src)      slot dst = dst + src; src = +0
      ("div", w)              slot 0 = slot 0 / w
      ("tail", hop, w, t)     record w * hop's tail elements as term t      (weighted mode only)
      ("rowsum", T)           tail elements of slot 0 = 0 + row_sum(terms)  (weighted mode only)
    Result: slot 0 (+0 everywhere if it was never written)."""
    steps = []
    if mode in ("sum", "mean"):
        steps += [("acc", 0, k, w) for k, w in terms]
        if mode == "mean":
            steps.append(("div", divisor))
        return steps
    if mode != "weighted":
        raise ValueError(f"no accumulation plan for mode {mode!r}")
    T = len(terms)
    clog2 = 1 if T <= 2 else (T - 1).bit_length()
    lp = max(4, clog2 // 4)
    step, mask = 1 << lp, (1 << lp) - 1
    i = 0
    while i + step <= T:
        for _ in range(step):
            steps.append(("acc", 0, terms[i][0], terms[i][1]))
            i += 1
        for j in range(1, 4):
            steps.append(("fold", j, j - 1))
            if i & (mask << (j * lp)):
                break
    while i < T:
        steps.append(("acc", 0, terms[i][0], terms[i][1]))
        i += 1
    for j in range(1, 4):
        steps.append(("fold", 0, j))
    # tail terms are recorded in term order, right after their main-path accumulation
    out, t = [], 0
    for s in steps:
        out.append(s)
        if s[0] == "acc":
            out.append(("tail", s[2], s[3], t))
            t += 1
    out.append(("rowsum", T))
    return out


class _DeviceSteps:
    """Executes combine_steps on the device through the C-ABI (one stream, torch's current)."""

    def __init__(self, n, d, device):
        self.n, self.d, self.device = n, d, device
        self.slots = {}
        self.pool = []
        self.stream = _lib.stream(device)
        self.ts, self.tl = tail_range(n, d)
        self.hist = None

    def _buf(self):
        return self.pool.pop() if self.pool else torch.empty((self.n, self.d), dtype=torch.float32,
                                                             device=self.device)

    def _acc(self, agg, y, w, mode):
        _lib.call(self.device, "srg_hop_accumulate_f32", agg.data_ptr(), agg.stride(0),
                  y.data_ptr() if y is not None else None, y.stride(0) if y is not None else agg.stride(0),
                  self.n, self.d, float(w), mode, self.stream)

    def run(self, s, hop_panel=None):
        kind = s[0]
        if kind == "acc":
            slot, w = s[1], s[3]
            if slot not in self.slots:
                self.slots[slot] = self._buf()
                self._acc(self.slots[slot], hop_panel, w, _lib.SRG_ACC_INIT)
            else:
                self._acc(self.slots[slot], hop_panel, w, _lib.SRG_ACC_ADD)
        elif kind == "fold":
            dst, src = s[1], s[2]
            if src not in self.slots:
                return
            if dst not in self.slots:               # 0 + x == x: accumulators are never -0
                self.slots[dst] = self.slots.pop(src)
            else:
                self._acc(self.slots[dst], self.slots[src], 1.0, _lib.SRG_ACC_ADD)
                self.pool.append(self.slots.pop(src))
        elif kind == "div":
            self._acc(self.result(), None, s[1], _lib.SRG_ACC_DIV)
        elif kind == "tail":
            if self.tl == 0:
                return
            t = s[3]
            if self.hist is None or self.hist.shape[0] <= t:
                grown = torch.empty((max(2 * t, 16), _lib.SRG_TAIL_MAX), dtype=torch.float32, device=self.device)
                if self.hist is not None:
                    grown[: self.hist.shape[0]].copy_(self.hist)
                self.hist = grown
            _lib.call(self.device, "srg_tail_record_f32", self.hist[t].data_ptr(), hop_panel.data_ptr(),
                      hop_panel.stride(0), self.d, self.ts, self.tl, float(s[2]), self.stream)
        elif kind == "rowsum":
            if self.tl == 0 or s[1] == 0:
                return
            agg = self.result()
            _lib.call(self.device, "srg_tail_rowsum_f32", agg.data_ptr(), agg.stride(0), self.d, self.ts, self.tl,
                      self.hist.data_ptr(), s[1], self.stream)
        else:
            raise ValueError(f"unknown step {s!r}")

    def fused_target(self, s):
        """(panel, init) that an ("acc", 0, k, w) step folds into when fused into hop k's SpMM."""
        if 0 not in self.slots:
            self.slots[0] = self._buf()
            return self.slots[0], True
        return self.slots[0], False

    def result(self):
        if 0 not in self.slots:
            self.slots[0] = self._buf()
            self.slots[0].zero_()
        return self.slots[0]


def step_hop(s):
    """The hop a step reads (None for folds / div / rowsum)."""
    if s[0] == "acc":
        return s[2]
    if s[0] == "tail":
        return s[1]
    return None


def schedule(steps):
    """Groups steps by the hop they wait for: ([steps run when hop k appears] for k = 0..last,
    [steps run after the last hop]).  Steps that read no hop run with the preceding ones."""
    groups, trailing, cur = [], [], -1
    for s in steps:
        k = step_hop(s)
        if k is None:
            (groups[cur] if cur >= 0 else trailing).append(s)
            continue
        if k < cur:
            raise ValueError("steps must visit hops in increasing order")
        while cur < k:
            groups.append([])
            cur += 1
        groups[k].append(s)
    if groups:                                   # folds after the last hop's terms go last
        last = groups[-1]
        i = len(last)
        while i > 0 and step_hop(last[i - 1]) is None:
            i -= 1
        trailing = last[i:] + trailing
        del last[i:]
    return groups, trailing


def propagate_aggregate(A: DeviceCSR, X: torch.Tensor, K: int, steps=None, last_only: bool = False,
                        fuse: bool = True, col_blocks=None):
    """Runs hops 1..K of Â on the device panel X ([n, d], row-major) with two ping-pong panels and
    executes `steps` (combine_steps) as each hop appears; returns the aggregated panel, or Â^K X
    when last_only.  Hops beyond the last one a step needs are not computed.  With `fuse`, a hop's
    first accumulation step runs in the SpMM's epilogue (srg_spmm_agg_f32: same arithmetic, one
    panel pass less).  col_blocks: column blocks per hop (spmm.hop; None = auto_col_blocks)."""
    n, d = X.shape
    if A.n_rows != n or A.n_cols != n:
        raise ValueError("propagate_aggregate needs a square operator matching X")
    if X.dim() != 2 or X.dtype != torch.float32 or X.stride(1) != 1 or X.stride(0) < d:
        raise ValueError("X must be a row-major float32 [n, d] device panel")
    from .spmm import prepare
    # the layout for the K hops (the native plan, srgnn.plan: its single hops take the epilogue)
    col_blocks = prepare(A, d, K, col_blocks) if K > 0 else 1
    groups, trailing = schedule(steps or [])
    if len(groups) > K + 1:
        raise ValueError("hop index out of range")
    last = K if last_only else len(groups) - 1
    ex = None if last_only else _DeviceSteps(n, d, X.device)

    def consume(k, panel):
        if ex is not None and k < len(groups):
            for s in groups[k]:
                ex.run(s, panel if step_hop(s) is not None else None)

    consume(0, X)
    cur = X
    if last >= 1:
        bufs = [torch.empty((n, d), dtype=torch.float32, device=X.device) for _ in range(min(2, last))]
        for k in range(1, last + 1):
            nxt = bufs[(k - 1) % len(bufs)]
            g = groups[k] if ex is not None and k < len(groups) else []
            if fuse and g and g[0][0] == "acc" and g[0][1] == 0:
                agg, init = ex.fused_target(g[0])
                hop(A, cur, nxt, col_blocks=col_blocks, agg=(agg, g[0][3], init))
                cur = nxt
                for s_ in g[1:]:
                    ex.run(s_, cur if step_hop(s_) is not None else None)
            else:
                hop(A, cur, nxt, col_blocks=col_blocks)
                cur = nxt
                consume(k, cur)
    if last_only:
        return cur.clone() if cur is X else cur
    for s in trailing:
        ex.run(s)
    return ex.result()


def fused_combine(A: DeviceCSR, X: torch.Tensor, K: int, msg_op) -> torch.Tensor:
    """msg_op.combine([X, ÂX, …, Â^K X]) computed on the device without the hop list."""
    mode, terms, div = combine_plan(msg_op, K + 1)
    if mode == "last":
        return propagate_aggregate(A, X, K, last_only=True)
    return propagate_aggregate(A, X, K, combine_steps(mode, terms, div))
