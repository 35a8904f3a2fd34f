"""P = 8 per-rank hop compute with the row chunks cut into owner-aligned column blocks (A/B probe).

Block bounds at the rank's own rows in GLOBAL column order -- [0, r0) the halo owned by lower ranks,
[r0, r1) the rank's own rows, [r1, n) the halo of higher ranks -- so each launch gathers from one
segment of the local panel (the own rows: ~157 MB on products, each halo side ~215 MB), every chain
continued across the blocks in CSR order (bitwise the unblocked chunk, checked here).  Rows of
<= csr.BLOCK_WHOLE_MAX entries stay whole in block 0 as in HaloPartitionedOperator.chunk_blocks.

    python tools/probes/owner_blocks_probe.py [--chunks 3,6] [--worlds 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn import dist as D  # noqa: E402


def owner_bounds(op, B):
    """_block_bounds replacement: B == 3 -> owner-aligned bounds (lower halo | own | upper halo)."""
    key = ("bounds", B)
    if key in op._cb:
        return op._cb[key]
    from srgnn.csr import BLOCK_WHOLE_MAX
    lip = op._lip
    nloc = op.rows + op.halo
    g = op._lix_glob.to(torch.int64)
    cuts = []
    for t in (op.r0, op.r1):
        below = (g < t).to(torch.int64)
        cs = torch.zeros(g.numel() + 1, dtype=torch.int64, device=g.device)
        torch.cumsum(below, 0, out=cs[1:])
        cuts.append(lip[:-1] + (cs[lip[1:]] - cs[lip[:-1]]))
    deg = lip[1:] - lip[:-1]
    whole = (deg <= BLOCK_WHOLE_MAX) if BLOCK_WHOLE_MAX > 0 else torch.zeros_like(deg, dtype=torch.bool)
    cuts = [torch.where(whole, lip[1:], c) for c in cuts]
    assert nloc == deg.numel()
    op._cb[key] = ([lip[:-1]] + cuts + [lip[1:]], whole)
    return op._cb[key]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--worlds", default="8")
    ap.add_argument("--chunks", default="3,6")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev)
    x = synth.uniform_features_t(n, d, device=dev)
    out = []
    for P in [int(w) for w in a.worlds.split(",")]:
        for C in [int(c) for c in a.chunks.split(",")]:
            for mode in ("plain", "owner3"):
                worst = 0.0
                for q in range(P):
                    op = D.HaloPartitionedOperator(ip, ix, vals, n, chunks=C, device=dev, rank=q, world=P,
                                                   col_blocks=3 if mode == "owner3" else 1)
                    if mode == "owner3":
                        op._block_bounds = lambda B, op=op: owner_bounds(op, B)
                    src = op.new_panel(d)
                    src[: op.rows].copy_(x[op.r0:op.r1])
                    src[op.rows:].uniform_(-1, 1)
                    dst = op.new_panel(d)
                    for _ in range(a.warmup):
                        op.compute(src, dst)
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
                    for r in range(a.reps):
                        ev[2 * r].record()
                        op.compute(src, dst)
                        ev[2 * r + 1].record()
                    torch.cuda.synchronize()
                    ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))[a.reps // 2]
                    if mode == "owner3" and q == 0:
                        ref = op.new_panel(d)
                        op2 = D.HaloPartitionedOperator(ip, ix, vals, n, chunks=C, device=dev, rank=q, world=P, col_blocks=1)
                        op2.compute(src, ref)
                        torch.cuda.synchronize()
                        same = bool(torch.equal(ref[: op.rows].view(torch.int32), dst[: op.rows].view(torch.int32)))
                        print(f"  rank 0 owner-blocked == unblocked: {same}", file=sys.stderr, flush=True)
                        assert same
                        del op2, ref
                    worst = max(worst, ms)
                    del op, src, dst
                    torch.cuda.empty_cache()
                print(f"P={P} chunks {C} {mode}: hop compute {worst:.3f} ms (max over ranks)", file=sys.stderr, flush=True)
                out.append({"P": P, "chunks": C, "mode": mode, "max_hop_compute_ms": worst})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
