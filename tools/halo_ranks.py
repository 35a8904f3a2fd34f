#!/usr/bin/env python3
"""Per-rank compute of the halo-exchange partition, measured on ONE GPU with virtual ranks.

For P in --worlds, builds every rank's HaloPartitionedOperator share of the products-shaped graph
and times, with HIP events, one hop of its local kernels (each group's launch, the hub group
separately) on halo-filled panels.  The max over ranks is the compute floor of one hop at P GPUs;
together with each rank's inbound halo bytes it bounds what the driver's N-GPU run can reach.

    python tools/halo_ranks.py [--config products] [--worlds 2,4,8] [--reps 5]   -> JSON
"""
from __future__ import annotations

import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scalable-roubust-gnn_amd"))

import torch  # noqa: E402

from srgnn import graphs, synth  # noqa: E402
from srgnn.dist import HaloPartitionedOperator  # noqa: E402
from srgnn.spmm import gather_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="products")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=20,
                    help="untimed op.compute calls before the timed ones (--quick): the GPU's clocks ramp up "
                         "after the host-side plan build left it idle")
    ap.add_argument("--d", type=int, default=None, help="feature width (default: the config's)")
    ap.add_argument("--fast", action="store_true", help="the hub group in tolerance mode (SRG_SPMM_FAST)")
    ap.add_argument("--hub-threshold", default="auto",
                    help="hub row length(s): 'auto' (nnz_rank / (1024 chunks), floor 2048) or a comma list")
    ap.add_argument("--heavy-threshold", type=int, default=None, help="chunk slice-wave row length (default: auto)")
    ap.add_argument("--col-blocks", default=None,
                    help="column blocks of the row chunks' launches: one value or a comma list (default: auto)")
    ap.add_argument("--quick", action="store_true",
                    help="time only each rank's hop compute (op.compute), no breakdowns: for A/B sweeps")
    ap.add_argument("--ghost", default="auto",
                    help="ghost row degree cap(s): 'auto' (the operator's cost model) or a comma list")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix, vals, n, d, K = graphs.build(a.config, dev, d=a.d)
    x = synth.uniform_features_t(n, d, device=dev)
    print(f"{a.config}: n={n} nnz={int(ix.numel())} d={d} built", file=sys.stderr, flush=True)
    out = {"config": a.config, "n": n, "nnz": int(ix.numel()), "d": d, "worlds": {}}
    ghosts = [None] if a.ghost == "auto" else [int(c) for c in a.ghost.split(",")]
    cbs = [None] if a.col_blocks is None else [int(c) for c in a.col_blocks.split(",")]
    hcb = None
    hubs = [None] if a.hub_threshold == "auto" else [int(h) for h in a.hub_threshold.split(",")]
    for P, ghost, cb, hub in [(int(w), gc, cb, h) for w in a.worlds.split(",") for gc in ghosts for cb in cbs
                              for h in hubs]:
        ranks = []
        for q in range(P):
            import time
            t_plan = time.perf_counter()
            op = HaloPartitionedOperator(ip, ix, vals, n, chunks=a.chunks, device=dev, rank=q, world=P,
                                         ghost_max_degree=ghost, fast=a.fast, col_blocks=cb, hub_threshold=hub,
                                         heavy_threshold=a.heavy_threshold)
            torch.cuda.synchronize()
            t_plan = time.perf_counter() - t_plan
            src = op.new_panel(d)
            src[: op.rows].copy_(x[op.r0:op.r1])
            src[op.rows:].uniform_(-1, 1)
            dst = op.new_panel(d)
            times = {}
            G = op.n_groups            # op._A[G] is the ghost rows' launch (into dst's halo)
            if a.quick:
                for _ in range(a.warmup):
                    op.compute(src, dst)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
                for r in range(a.reps):
                    ev[2 * r].record()
                    op.compute(src, dst)
                    ev[2 * r + 1].record()
                torch.cuda.synchronize()
                ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
                ranks.append({"rank": q, "rows": op.rows, "nnz": op.nnz_local, "hub_rows": op.views[op.C][1],
                              "ghost_max_degree": op.ghost_max_degree, "s_operator_build": round(t_plan, 3),
                              "ms_compute": ms[len(ms) // 2]})
                print(f"  P={P} rank {q}: compute {ms[len(ms) // 2]:.3f} ms", file=sys.stderr, flush=True)
                del op, src, dst
                torch.cuda.empty_cache()
                continue
            for name, groups in (("all", range(G + 1)), ("hub", [op.C]), ("chunks", list(range(op.C)) + [G]),
                                 ("ghosts", [G])):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
                for r in range(a.reps):
                    ev[2 * r].record()
                    for g in groups:
                        if g == G:
                            if op.n_ghost:
                                op._spmm(op._A[G], src, dst)
                        elif op.views[g][1]:
                            op._spmm(op._A[g], src, dst[: op.rows])
                    ev[2 * r + 1].record()
                torch.cuda.synchronize()
                ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
                times[name] = ms[len(ms) // 2]
            # the hop's own launch as it issues it: hub group on its side stream beside the chunks,
            # then the ghost rows (the per-rank compute of one hop)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
            for r in range(a.reps):
                ev[2 * r].record()
                op.compute(src, dst)
                ev[2 * r + 1].record()
            torch.cuda.synchronize()
            ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
            times["compute"] = ms[len(ms) // 2]
            # the hub group as the hop issues it (its column blocks chained on the side stream)
            if op.views[op.C][1] and op.views[op.C][3]:
                from srgnn import _lib
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
                for r in range(a.reps):
                    ev[2 * r].record()
                    op._hub_launch(src, dst[: op.rows])
                    _lib.call(dev, "srg_hub_join", _lib.stream(dev))
                    ev[2 * r + 1].record()
                torch.cuda.synchronize()
                ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
                times["hub_launch"] = ms[len(ms) // 2]
            # the send-side pack (index_select of the rows peers need, per group) alone, and the
            # chunks with each group's pack on a second stream as the real hop issues it
            for name, fn in (("pack_index_select", lambda t, i: t.index_select(0, i)), ("pack", gather_rows)):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
                for r in range(a.reps):
                    ev[2 * r].record()
                    for g in range(op.n_groups):
                        if op.send_cat[g].numel():
                            fn(src[: op.rows], op.send_cat[g])
                    ev[2 * r + 1].record()
                torch.cuda.synchronize()
                ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
                times[name] = ms[len(ms) // 2]
            side = torch.cuda.Stream(dev)
            main = torch.cuda.current_stream(dev)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
            for r in range(a.reps):
                ev[2 * r].record()
                for g in range(op.C):
                    if op.views[g][1]:
                        op._spmm(op._A[g], src, dst[: op.rows])
                    if g == op.C - 1 and op.n_ghost:
                        op._spmm(op._A[G], src, dst)
                    e = torch.cuda.Event()
                    e.record(main)
                    side.wait_event(e)
                    if op.send_cat[g].numel():
                        with torch.cuda.stream(side):
                            gather_rows(dst[: op.rows], op.send_cat[g])
                main.wait_stream(side)
                ev[2 * r + 1].record()
            torch.cuda.synchronize()
            ms = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(a.reps))
            times["chunks_pack"] = ms[len(ms) // 2]
            rec = {"rank": q, "ms_pack": times["pack"], "ms_pack_index_select": times["pack_index_select"], "ms_chunks_with_pack": times["chunks_pack"],
                   "rows": op.rows, "nnz": op.nnz_local, "halo_rows": op.halo, "recv_rows": op.n_recv,
                   "ghost_rows": op.n_ghost, "ghost_nnz": int(op._ghost_pos.numel()),
                   "ghost_max_degree": op.ghost_max_degree, "ms_ghosts": times["ghosts"],
                   "max_link_rows": max(sum(op.recv_counts[g][s] for g in range(G)) for s in range(P)),
                   "halo_bytes": op.n_recv * d * 4, "send_rows": int(sum(t.numel() for t in op.send_cat)),
                   "hub_rows": op.views[op.C][1],
                   "ms_all_serial": times["all"], "ms_hub": times["hub"], "ms_chunks": times["chunks"],
                   "ms_compute": times["compute"], "ms_hub_launch": times.get("hub_launch")}
            ranks.append(rec)
            print(f"  P={P} rank {q}: rows={op.rows} halo={op.halo} (received {op.n_recv}, ghosts {op.n_ghost} "
                  f"<= degree {op.ghost_max_degree}) chunks {times['chunks']:.3f} ms (ghosts {times['ghosts']:.3f}), "
                  f"hub {times['hub']:.3f} ms (as launched {times.get('hub_launch', 0.0):.3f}), "
                  f"compute {times['compute']:.3f} ms", file=sys.stderr, flush=True)
            del op, src, dst
            torch.cuda.empty_cache()
        if a.quick:
            key = f"{P}" + ("" if cb is None else f"/cb{cb}") + ("" if hub is None else f"/hub{hub}")
            out["worlds"][key] = {"ranks": ranks, "max_hop_compute_ms": max(r["ms_compute"] for r in ranks)}
            print(f"P={P} col blocks {cb} hub threshold {hub or 'auto'}: hop compute "
                  f"{out['worlds'][key]['max_hop_compute_ms']:.3f} ms (max over ranks)", file=sys.stderr, flush=True)
            continue
        worst = max(ranks, key=lambda r: max(r["ms_hub"], r["ms_chunks"]))
        key = (f"{P}" if a.ghost == "auto" else f"{P}/ghost{ghost}") + ("" if cb is None else f"/cb{cb}") + \
            ("" if hcb is None else f"/hcb{hcb}")
        out["worlds"][key] = {"ranks": ranks, "col_blocks": cb, "hub_col_blocks": hcb,
                            "max_hop_compute_ms": max(r["ms_compute"] for r in ranks),
                            "max_compute_ms": max(max(r["ms_hub"], r["ms_chunks"]) for r in ranks),
                            "mean_chunks_ms": sum(r["ms_chunks"] for r in ranks) / P,
                            "worst_rank": worst["rank"],
                            "max_halo_GB": max(r["halo_bytes"] for r in ranks) / 1e9}
        W = out["worlds"][key]
        print(f"P={P} col blocks {cb} hub blocks {hcb} ghost cap {ranks[0]['ghost_max_degree']}: hop compute {W['max_hop_compute_ms']:.3f} ms, "
              f"max compute {W['max_compute_ms']:.3f} ms "
              f"(rank {worst['rank']}: chunks {worst['ms_chunks']:.3f}, hub {worst['ms_hub']:.3f}), "
              f"mean chunks {W['mean_chunks_ms']:.3f} ms, max received halo "
              f"{W['max_halo_GB']:.2f} GB, busiest link {max(r['max_link_rows'] for r in ranks) * d * 4 / 1e9:.3f} GB; pack {worst['ms_pack']:.3f} ms alone (index_select {worst['ms_pack_index_select']:.3f}), chunks+pack "
              f"{worst['ms_chunks_with_pack']:.3f} ms", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
