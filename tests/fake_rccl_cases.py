"""Run in a child process by tests/test_fake_rccl_gpu.py with SRGNN_RCCL_LIB pointing at the test-only
tests/_build/libfake_rccl.so: the library's RCCL code paths -- srg_dist_propagate_khop_f32 (the
owner-chunked all-gather overlapped with the column-block SpMM) and the RCCL branch of
srg_halo_propagate_f32's exchange (halo_transport, srg_comm.hip) -- with P = 2, 3 and 8 ranks of one
process on one GPU (real RCCL refuses a repeated device).  Every rank's rows of every hop are compared
bitwise with the one-GPU hops.  Prints one JSON line {"cases": [...], "ok": bool}."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))

import torch  # noqa: E402


def graph(n, e, d, seed):
    from srgnn import synth
    from srgnn.normalize import sym_norm_binary
    u, v = synth.rmat_undirected_t(n, e, seed=seed, device="cuda")
    ip, ix = synth.symmetric_csr_t(n, u, v)
    ip, ix, vals = sym_norm_binary(ip, ix, n, 0.5)
    return ip, ix, vals, synth.uniform_features_t(n, d, device="cuda")


def main():
    assert os.environ.get("SRGNN_RCCL_LIB", "").endswith("libfake_rccl.so"), "run with the fake RCCL"
    from srgnn import _lib
    from srgnn.comm import Comm, HaloPlan, HaloShare, halo_propagate
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import propagate
    cases = []
    ip, ix, vals, X = graph(20000, 200000, 64, 5)
    n, d, K = X.shape[0], X.shape[1], 4
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device="cuda")
    want = propagate(A, X, K, col_blocks=1)
    ipn, ixn, vn = ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy()
    for P in (2, 3, 8):
        # srg_dist_propagate_khop_f32: uneven contiguous row blocks (one empty at P = 8)
        starts = [0] + [min(n, (i * n) // P + (37 * i if i < P - 1 else 0)) for i in range(1, P)] + [n]
        if P == 8:
            starts[3] = starts[2]
        comm = Comm.init_all([0] * P)
        try:
            blocks = [A.rows(starts[i], starts[i + 1]) for i in range(P)]
            out = comm.propagate(blocks, starts, [X[starts[i]:starts[i + 1]].clone() for i in range(P)], K)
            ok = all(torch.equal(torch.cat([out[i][k] for i in range(P)]), want[k]) for k in range(K + 1))
            cases.append({"path": "srg_dist_propagate_khop_f32", "P": P, "bitwise_equal_one_gpu": ok})
        finally:
            comm.destroy()
        # srg_halo_propagate_f32 through RCCL grouped send / receive (not the loopback copies)
        for chunks, ghost, x_filled in ((3, 0, False), (6, 2, True)):
            plans = [HaloPlan(ipn, ixn, n, P, r, chunks=chunks, ghost_max_degree=ghost, hub_threshold=256)
                     for r in range(P)]
            shares = [HaloShare(p, vn, 0, d) for p in plans]
            panels = [[s.new_panel(d) for _ in range(K + 1)] for s in shares]
            for s, ps in zip(shares, panels):
                if x_filled:
                    s.fill_x_halo(X, ps[0])
                else:
                    ps[0][: s.rows].copy_(X[s.plan.info["row0"]:s.plan.info["row0"] + s.rows])
            streams = [torch.cuda.Stream() for _ in range(P)]
            for st in streams:
                st.wait_stream(torch.cuda.current_stream())
            comm = Comm.init_all([0] * P)
            try:
                halo_propagate(comm, shares, panels, K, x_halo_filled=x_filled, streams=[st.cuda_stream for st in streams])
                torch.cuda.synchronize()
                ok = all(torch.equal(torch.cat([ps[k][: s.rows] for s, ps in zip(shares, panels)]), want[k])
                         for k in range(K + 1))
                halo_ok = True
                for s, ps in zip(shares, panels):
                    ids = torch.from_numpy(s.plan.array(_lib.SRG_HALO_HALO_IDS)).cuda()
                    if ids.numel():
                        halo_ok &= bool(torch.equal(ps[K - 1][s.rows:s.rows + s.halo], want[K - 1][ids]))
                cases.append({"path": "srg_halo_propagate_f32 (RCCL branch)", "P": P, "chunks": chunks, "ghost": ghost,
                              "x_halo_filled": x_filled, "bitwise_equal_one_gpu": ok, "halo_rows_equal_owners": halo_ok})
            finally:
                comm.destroy()
                for s in shares:
                    s.destroy()
    # plans that disagree across ranks: the exchange must fail with the library's own check, not hang.
    #  * ghost caps (same chunk count): the per-group counts differ -> verify_counts' second exchange;
    #  * graphs (rank 1 planned another graph, same n and chunks): n / nnz differ -> the fixed-size header
    #    verify_counts exchanges FIRST (its length never depends on the plan, so ranks whose
    #    plans have different chunk counts -- count messages of different lengths, which real RCCL would
    #    block on -- still exchange matching messages and fail);
    #  * chunk counts: in ONE process the shares are side by side and srg_halo_propagate_f32's host check
    #    sees them first; across processes (one share each) it is the header above that catches them.
    ip2, ix2, vals2, _ = graph(20000, 199000, 64, 6)
    ip2n, ix2n, v2n = ip2.cpu().numpy(), ix2.cpu().numpy(), vals2.cpu().numpy()
    assert ix2n.size != ixn.size
    mismatches = []
    for what, chunk_of, ghost_of, graph_of, want in (
            ("ghost caps", lambda r: 3, lambda r: 4 if r == 1 else 0, lambda r: 0, "plans disagree"),
            ("graphs", lambda r: 3, lambda r: 0, lambda r: 1 if r == 1 else 0, "plan is of a graph"),
            ("chunk counts", lambda r: 4 if r == 1 else 3, lambda r: 0, lambda r: 0, "different chunk counts")):
        P = 3
        g_of = [(ipn, ixn, vn), (ip2n, ix2n, v2n)]
        plans = [HaloPlan(g_of[graph_of(r)][0], g_of[graph_of(r)][1], n, P, r, chunks=chunk_of(r),
                          ghost_max_degree=ghost_of(r), hub_threshold=256) for r in range(P)]
        shares = [HaloShare(p, g_of[graph_of(r)][2], 0, d) for r, p in enumerate(plans)]
        panels = [[s.new_panel(d) for _ in range(3)] for s in shares]
        comm = Comm.init_all([0] * P)
        try:
            halo_propagate(comm, shares, panels, 2)
            torch.cuda.synchronize()
            msg = "not detected"
        except _lib.SrgError as e:
            msg = str(e)
        finally:
            comm.destroy()
            for s in shares:
                s.destroy()
        cases.append({"path": f"mismatched plans ({what})", "error": msg, "detected_by_library_check": want in msg})
        mismatches.append(want in msg)
    ok = all(c.get("bitwise_equal_one_gpu", True) and c.get("halo_rows_equal_owners", True) for c in cases) and \
        all(mismatches)
    print(json.dumps({"cases": cases, "ok": ok}))


if __name__ == "__main__":
    main()
