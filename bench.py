#!/usr/bin/env python3
"""Benchmark of the K-hop propagation precompute (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config products]

One "step" = one full K-hop propagate ([X, ÂX, …, Â^K X]) of the configuration's synthetic
power-law graph with inputs already resident in HBM: K = 10 hops of the
products-shaped graph (N = 2,449,029, 61.9 M undirected edges, d = 128) by default.
value = propagated edges/s = steps * K * nnz(Â) / time (nnz counts the self-loops), whole job.

N > 1: one process per GPU (torchrun), 1-D row partition balanced by nonzeros (strong scaling of
the same graph).  --exchange halo (default): each rank receives only the remote rows its rows
reference, in nnz-balanced groups exchanged with RCCL all_to_all_single as soon as each group's
kernel finishes (overlapping the later groups); --exchange allgather: one padded
all_gather_into_tensor of the whole panel per hop.  Both are bitwise equal to 1 GPU.

--gpus N without torchrun (WORLD_SIZE unset): this process spawns the N ranks itself (one worker
process per GPU, 127.0.0.1 rendezvous) before touching any GPU, and forwards rank 0's line.

Extra objects on the JSON line:
  roofline         the SpMM hop (one hop = `launches_per_hop` column-block launches): HBM bytes
                   per hop from rocprofv3 PMC counters (2 * FETCH_SIZE + WRITE_SIZE, the gfx950
                   correction of MI355X_MICROARCH.md), measured by this run in separate --pmc
                   passes of tools/spmm_probe.py before the GPU is touched (--pmc), else the
                   committed profiles/pmc_<config>.json, / the hop's duration (HIP events on the
                   launch stream) -> achieved, frac.  frac_no_reuse (SURVEY §8(d)'s no-reuse byte
                   model, > 1 where caches serve re-read rows) and frac_compulsory beside it.
  cpu_baseline     rank 0, N = 1 only: the reference's FloatCSRMulDenseOMP compiled from its own
                   matmul.c (oracle/_ref/libmatmul_ref.so), kernel-only hops on pre-converted
                   buffers of the same graph, bounded to ~--cpu-seconds of work
  parity_vs_oracle N = 1: after the timed steps, outside the timed region, sampled rows (random +
                   the longest) of hop 1 and hop K of the timed operator checked bit for bit
                   against the CPU oracle (test infrastructure, the checker only) fed with the
                   GPU's previous hop
  parity_vs_1gpu   N > 1: every rank's rows of hop 1 and hop K against the one-GPU kernels
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import shutil
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "scalable-roubust-gnn_amd"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from srgnn import graphs, roofline, synth  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="products", choices=sorted(synth.CONFIGS))
    ap.add_argument("--k", type=int, default=None, help="hops (default: the config's K)")
    ap.add_argument("--d", type=int, default=None)
    ap.add_argument("--heavy-threshold", type=int, default=None)
    ap.add_argument("--roofline-reps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--nt-store", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="one GPU, K-hop panels mode: capture one step (its K hops, hub forks and joins) in a "
                         "HIP graph after the warm-up and replay it for the timed steps")
    ap.add_argument("--col-blocks", type=int, default=None,
                    help="column blocks per hop on one GPU (default: srgnn.spmm.auto_col_blocks; 1 = one launch)")
    ap.add_argument("--exchange", default="halo", choices=["halo", "allgather"])
    ap.add_argument("--chunks", type=int, default=None,
                    help="halo exchange groups per hop (row chunks; default 4 at 2 GPUs, 6 above: the "
                         "hop compute is within 3 %% over 2-8 chunks, more chunks shorten the last "
                         "group's exposed exchange)")
    ap.add_argument("--exchange-x", action="store_true",
                    help="halo exchange: receive hop 0's halo (X) from its owners instead of gathering "
                         "it from the whole X every rank holds")
    ap.add_argument("--ghost-max-degree", type=int, default=None,
                    help="halo exchange: compute halo rows of at most this degree locally instead of "
                         "receiving them (default: the operator's cost model; 0 = off)")
    ap.add_argument("--op", default="khop", choices=["khop", "wavelet"],
                    help="khop: the K-hop propagate (GraphOp.propagate); wavelet: the heat-wavelet "
                         "Chebyshev filter bank (order 3, scales -0.5/+0.5) applied to the feature panel")
    ap.add_argument("--col-block", type=int, default=None, help="wavelet: column block width")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"],
                    help="wavelet: f64 = the reference's precision (pygsp cheby_op in fp64, base_model.py:236-265): "
                         "each order the fp64 Chebyshev step (column-blocked with hub workgroups where the panel "
                         "outgrows the caches), bit-exact vs the oracle; f32 = the reduced-"
                         "precision variant (load-balanced SpMM + epilogue)")
    ap.add_argument("--fused-epilogue", action="store_true",
                    help="wavelet: one srg_spmm_cheby_f32 launch per order (two work panels) instead of the "
                         "SpMM + epilogue launches (three work panels); same bits, measured slower")
    ap.add_argument("--aggregate", default=None, choices=["sum", "mean", "weighted"],
                    help="one GPU: fused hop aggregation (SGC/SSGC/GBP precompute) instead of the K+1 "
                         "panels: sum / mean over hops 0..K, or GBP weights alpha(1-alpha)^k, alpha 0.15")
    ap.add_argument("--fast", action="store_true",
                    help="tolerance mode (SRG_SPMM_FAST): hub rows as 64 exact segment chains plus their "
                         "ordered sum; other rows bit-exact; parity then checked within tolerance")
    ap.add_argument("--pmc", default="auto", choices=["auto", "on", "off"],
                    help="measure the hop's HBM traffic with rocprofv3 --pmc passes of tools/spmm_probe.py "
                         "before this process touches the GPU (auto: one GPU, K-hop, not under a profiler)")
    ap.add_argument("--dist-parity", default="auto", choices=["auto", "sampled"],
                    help="N > 1: auto = bitwise against the whole-graph one-GPU hops when they fit beside a "
                         "rank's share, else sampled rows against the oracle; sampled = always the latter")
    ap.add_argument("--parity-rows", type=int, default=2000,
                    help="one GPU: random rows (plus the 20 longest) checked against the oracle after timing")
    ap.add_argument("--mode", default="auto", choices=["auto", "panels", "last"],
                    help="panels: all K+1 hop panels kept (GraphOp.propagate); last: two ping-pong "
                         "panels, only A^K X kept (SGC-style, fused aggregation); auto: panels if "
                         "they fit in HBM")
    return ap.parse_args()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def granted_threads():
    """(threads, note): the host threads this job may use -- the CPUs of its affinity mask, capped by
    the cgroup's CPU quota and by OMP_NUM_THREADS where those are set (a box may show the whole
    machine in the mask and grant a share through either)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    # every limit that is set: the affinity mask, the cgroup quota, and OMP_NUM_THREADS, which the
    # GPU box sets to the CPU share it grants one job (its mask may show the whole machine)
    threads = min([aff] + ([quota] if quota else []) + ([omp] if omp > 0 else []))
    note = (f"threads used = {threads}, the minimum of the limits set: affinity mask {aff} CPUs"
            + (f", cgroup CPU quota {quota}" if quota else ", no cgroup CPU quota")
            + (f", OMP_NUM_THREADS={omp} (the CPU share the box grants one job)" if omp else "")
            + f"; the host shows {os.cpu_count()} logical CPUs")
    return max(1, threads), note


def _omp_set_threads(k):
    """Sets the OpenMP team size of the system libgomp (the one matmul.c / the oracle link)."""
    import ctypes
    try:
        ctypes.CDLL("libgomp.so.1").omp_set_num_threads(int(k))
        return True
    except OSError:
        return False


def cpu_baseline(ip, ix, vals, x_host, n, d, budget_s):
    """The reference's FloatCSRMulDenseOMP (built from SSRG/operators/csrc/matmul.c) on the host:
    whole hops, all threads, for ~budget_s; plus a 1-thread rate on a row block.  When the graph
    overflows the reference's int32 offsets (nnz >= 2^31 or N*d >= 2^31, matmul.c:29,33) the
    oracle's int64 restatement of the same fma chains runs instead, on row blocks ("port")."""
    from oracle import oracle as O
    nnz = int(ip[-1])
    threads, threads_note = granted_threads()
    use_ref = nnz < 2 ** 31 and n * d < 2 ** 31 and O.ref_lib() is not None
    cur = np.ascontiguousarray(x_host)
    ix32 = np.ascontiguousarray(ix, dtype=np.int32)
    v32 = np.ascontiguousarray(vals, dtype=np.float32)
    if use_ref:
        L = O.ref_lib()
        ip32 = np.ascontiguousarray(ip, dtype=np.int32)

        def rows(r0, r1, src, dst):      # dst rows [r0, r1) of one hop, zeroed first
            dst[r0:r1].fill(0.0)
            L.FloatCSRMulDenseOMP(O._ptr(dst[r0:]), O._ptr(v32), O._ptr(ix32), O._ptr(ip32[r0:]),
                                  O._ptr(src), r1 - r0, d)
    else:
        ip64 = np.ascontiguousarray(ip, dtype=np.int64)

        def rows(r0, r1, src, dst):
            O.spmm(ip64[r0:r1 + 1], ix32, v32, src, out=dst[r0:r1])
    nxt = np.empty_like(cur)
    _omp_set_threads(threads)
    edges, hops, t0 = 0, 0, time.perf_counter()
    block = n if use_ref else max(1, int(n * min(1.0, 2e8 / max(nnz, 1))))
    r0 = 0
    while True:
        r1 = min(n, r0 + block)
        rows(r0, r1, cur, nxt)
        edges += int(ip[r1] - ip[r0])
        r0 = r1
        if r0 == n:
            hops += 1
            r0 = 0
            cur, nxt = nxt, cur
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    # 1 thread, a row block of ~1/8 of the budget
    one = None
    if _omp_set_threads(1):
        r1 = max(1, int(n * min(1.0, (budget_s / 8) * edges / dt / threads / max(nnz, 1))))
        t1 = time.perf_counter()
        rows(0, r1, cur, nxt)
        one = int(ip[r1] - ip[0]) / (time.perf_counter() - t1)
        _omp_set_threads(threads)
    scipy_rate = _scipy_rate(ip, ix32, v32, cur, n, budget_s / 8)
    what = "the reference's FloatCSRMulDenseOMP (oracle/_ref, built from matmul.c)" if use_ref else \
        "the oracle's int64 C restatement (the reference's int32 matmul.c cannot address this graph)"
    return {"value": edges / dt, "unit": "propagated edges/s", "cores": threads,
            "cores_note": threads_note,
            "kind": "reference" if use_ref else "port",
            "value_1thread": one, "cpu_model": _cpu_model(),
            "scipy_value_1thread": scipy_rate,
            "scipy_threads": 1,
            "scipy_sample": ("the reference's non-Linux branch (base_operator.py:309-314: adj.dot(x), an fp64 csr "
                             "times the fp32 panel, fp64 result) on a row block.  scipy's csr_matvecs is "
                             f"single-threaded by design, so it runs on 1 of the {threads} threads whatever the "
                             "thread count; no parallel variant is invented for it"),
            "sample": f"{what}: {edges} propagated edges ({hops} full hop(s) + row blocks) of the "
                      f"{n}-node graph (nnz {nnz}, d {d}), kernel-only on pre-converted int32/fp32 "
                      f"buffers, {threads} OpenMP threads, {dt:.1f} s; value_1thread on a row block"}


def _scipy_rate(ip, ix32, v32, x, n, budget_s):
    """Propagated edges/s of scipy's csr @ dense (fp64 Â values, fp32 X: scipy upcasts, as the
    reference's adj.dot(x) does) on a row block sized to ~budget_s; None if scipy is unusable."""
    try:
        import scipy.sparse as sps
        nnz = int(ip[-1])
        r1 = max(1, int(n * min(1.0, 2e7 / max(nnz, 1))))
        e1 = int(ip[r1])
        A = sps.csr_matrix((v32[:e1].astype(np.float64), ix32[:e1], np.asarray(ip[:r1 + 1], dtype=np.int64)),
                           shape=(r1, n))
        t0 = time.perf_counter()
        reps = 0
        while True:
            A.dot(x)
            reps += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        return e1 * reps / (time.perf_counter() - t0)
    except Exception as e:  # noqa: BLE001
        log(f"scipy baseline skipped: {e!r}")
        return None


def pmc_traffic(config, launches_per_hop=1, measured=None):
    """(fabric bytes per hop, source, read bytes per hop): from this run's PMC passes (`measured`),
    else from the committed profiles/pmc_<config>.json (tools/pmc_traffic.py) when it was taken with
    the same hop layout.  The bytes are L2 -> fabric bytes (2 * FETCH_SIZE + WRITE_SIZE), Infinity-
    Cache hits included: an upper bound on DRAM bytes."""
    if measured is not None and int(measured.get("launches_per_hop", 1)) == int(launches_per_hop):
        return (float(measured["hbm_bytes_per_hop"]), measured["source"],
                2.0 * float(measured["fetch_kib_per_hop"]) * 1024)
    path = os.path.join(HERE, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None, None, None
    try:
        with open(path) as f:
            rec = json.load(f)
        if int(rec.get("launches_per_hop", 1)) != int(launches_per_hop):
            return None, None, None       # measured with another hop layout
        b = rec["hbm_bytes_per_hop"] if "hbm_bytes_per_hop" in rec else rec["hbm_bytes_per_launch"]   # pre-round-5 key
        rd = rec.get("hbm_read_bytes_per_hop", rec.get("hbm_read_bytes_per_launch"))
        return float(b), f"committed profiles/pmc_{config}.json (tools/pmc_traffic.py)", \
            (float(rd) if rd is not None else None)
    except Exception:  # noqa: BLE001
        return None, None, None


def _under_profiler() -> bool:
    pre = os.environ.get("LD_PRELOAD", "")
    return "rocprof" in pre or any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def measure_pmc(a):
    """HBM traffic of one hop of the bench's operator, from two rocprofv3 --pmc passes (FETCH_SIZE,
    then WRITE_SIZE: they do not fit one pass) of tools/spmm_probe.py, each in a child process
    with its own time limit.  Must run before this process initialises the GPU (a process that has
    must not exec another program).  traffic = 2 * FETCH_SIZE + WRITE_SIZE per hop (gfx950:
    FETCH_SIZE counts half the bytes of wide reads, MI355X_MICROARCH.md).  None on any failure."""
    import csv
    import glob
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    out = tempfile.mkdtemp(prefix="srg_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    probe = None
    sums = {}
    # the kernel whose traffic is the roofline's: the hop's k_spmm launches, or the fp64 Chebyshev step
    # (fp64 step: the block launches k_cheby_blk64, the hub workgroups k_cheby_hub64, or one k_cheby<double>)
    kern = "k_cheby" if (a.op == "wavelet" and a.dtype == "f64") else "k_spmm<"
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(out, counter)
            cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", counter, "-d", d, "-o", "p",
                   "--output-format", "csv", "--", sys.executable, os.path.join(HERE, "tools", "spmm_probe.py"),
                   "--config", a.config, "--reps", "3"]
            k = a.k if a.k is not None else synth.CONFIGS[a.config].get("k", 3)
            if a.op == "wavelet":       # order 3, every column block of the panel
                d_cfg = a.d or synth.CONFIGS[a.config]["d"]
                k = 3 * max(1, d_cfg // (a.col_block or 64))
            cmd += ["--hops", str(k * (a.steps + a.warmup))]
            if a.d is not None:
                cmd += ["--d", str(a.d)]
            if a.op == "wavelet":
                cmd += ["--op", "wavelet64" if a.dtype == "f64" else "wavelet"] + \
                    (["--col-block", str(a.col_block)] if a.col_block else [])
            elif a.col_blocks is not None:
                cmd += ["--col-blocks", str(a.col_blocks)]
            if a.heavy_threshold is not None:
                cmd += ["--heavy-threshold", str(a.heavy_threshold)]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               timeout=150)
            if r.returncode != 0:
                log(f"pmc pass {counter} failed ({r.returncode}): {r.stderr.decode(errors='replace')[-400:]}")
                return None
            probe = json.loads(r.stdout.decode().strip().splitlines()[-1])
            total, launches = 0.0, 0
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        name = row.get("Kernel_Name", "")
                        if kern in name and "k_spmm_hub" not in name and row.get("Counter_Name") == counter:
                            total += float(row["Counter_Value"])
                            launches += 1
            if not launches:
                log(f"pmc pass {counter}: no {kern} rows")
                return None
            sums[counter] = total / probe["reps"]           # KiB per hop (all of a hop's launches)
    except Exception as e:  # noqa: BLE001
        log(f"pmc passes failed: {e!r}")
        return None
    finally:
        shutil.rmtree(out, ignore_errors=True)
    hop_bytes = 2.0 * sums["FETCH_SIZE"] * 1024 + sums["WRITE_SIZE"] * 1024
    log(f"pmc: {hop_bytes / 1e9:.2f} GB per hop ({probe['launches_per_hop']} launches)")
    return {"hbm_bytes_per_hop": hop_bytes, "launches_per_hop": probe["launches_per_hop"],
            "fetch_kib_per_hop": sums["FETCH_SIZE"], "write_kib_per_hop": sums["WRITE_SIZE"],
            "source": "measured by this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/spmm_probe.py "
                      "(the same operator and hop layout), 2 * FETCH_SIZE + WRITE_SIZE"}


def oracle_sample(ip, ix, vals, n, n_random, n_top=20, seed=11):
    """Rows checked against the oracle after the timed steps (random rows plus the longest ones) and
    their sub-problem, extracted on the device: the rows' own entries in CSR order with the column
    ids renumbered over the X rows they gather (so the oracle needs only those rows)."""
    deg = ip[1:] - ip[:-1]
    g = torch.Generator(device="cpu").manual_seed(seed)
    pick = [torch.randint(0, n, (n_random,), generator=g).to(ip.device)] if n_random else []
    pick.append(torch.sort(deg, descending=True).indices[:n_top])
    rows = torch.unique(torch.cat(pick))
    beg, cnt = ip[rows], deg[rows]
    tot = int(cnt.sum())
    pos = torch.repeat_interleave(beg - torch.cumsum(cnt, 0) + cnt, cnt, output_size=tot) + \
        torch.arange(tot, device=ip.device)
    ucols, inv = torch.unique(ix[pos].long(), return_inverse=True)
    return {"rows": rows, "ucols": ucols, "ip": np.r_[0, np.cumsum(cnt.cpu().numpy())].astype(np.int64),
            "ix": inv.to(torch.int32).cpu().numpy(), "v": vals[pos].cpu().numpy()}


def parity_vs_oracle(sample, checks, tolerance=False):
    """Bit-for-bit check of sampled rows of GPU hops against the C oracle (oracle/srg_oracle.c:
    one fp32 fma chain per element in CSR order, matmul.c:23-40) fed with the GPU's previous hop.
    checks: [(k, prev_panel, panel)].  tolerance (FAST mode): also whether every element is within
    the fp32 forward-error bound gamma_{len+65} * sum |a| |x| of the exact value (the oracle's fp64
    product).  Test infrastructure used as the checker, outside the timed region; nothing measured
    runs through it."""
    from oracle import oracle as O
    done, ok, within = [], True, True
    lens = np.diff(sample["ip"]).astype(np.float64)[:, None]
    for k, prev, got in checks:
        x = prev[sample["ucols"]].cpu().numpy()
        want = O.spmm(sample["ip"], sample["ix"], sample["v"], x)
        have = got[sample["rows"]].cpu().numpy()
        ok = ok and np.array_equal(have.view(np.uint32), want.view(np.uint32))
        if tolerance:
            exact = O.spmm64(sample["ip"], sample["ix"], sample["v"].astype(np.float64), x.astype(np.float64))
            mag = O.spmm64(sample["ip"], sample["ix"], np.abs(sample["v"]).astype(np.float64), np.abs(x).astype(np.float64))
            n_ops = lens + 65
            gamma = n_ops * 2.0 ** -24 / (1 - n_ops * 2.0 ** -24)
            within = within and bool((np.abs(have.astype(np.float64) - exact) <= gamma * mag).all())
        done.append(k)
    res = {"hops_checked": done, "rows_checked": int(sample["rows"].numel()),
           "rows": "random rows + the 20 longest", "bit_exact": bool(ok),
           "checker": "oracle/srg_oracle.c fp32 fma chains fed with the GPU's previous hop (outside the timed region)"}
    if tolerance:
        res["within_fp32_bound_of_exact"] = within
    return res


def one_shot(ip, ix, vals, n, X, K, dev, heavy_threshold=None):
    """The reference's own call pattern: NodeClassification.execute runs preprocess once per run
    (SSRG/tasks/node_classification.py:62), i.e. ONE propagate(K) on a freshly built operator.  Here:
    a fresh DeviceCSR from the device arrays (validated; its row schedule is left to first use),
    srgnn.spmm.propagate laying it out for a K-hop run with the native planner (srg_plan_build: column
    blocks, compact launch-ordered copies from SRG_PLAN_MIN_HOPS_TO_COMPACT hops) and the K output panels
    allocated inside the bracket; HIP events on the launch stream plus the host wall clock around it.
    Â and X already resident (GraphOp.propagate's construct_adj and H2D / D2H are tools/e2e_api.py's)."""
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import col_blocks_of, prepare, propagate
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    d = X.shape[1]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(stream)
    A1 = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=heavy_threshold, device=dev)
    ev[1].record(stream)
    # what propagate(A1, X, K) does, in its three parts: the layout for K hops, the K output panels
    # (a fresh allocation: the caching allocator was emptied), the hops
    prepare(A1, d, K)
    ev[2].record(stream)
    buf = torch.empty((K, n, d), dtype=torch.float32, device=dev)
    ev[3].record(stream)
    out = propagate(A1, X, K, panels=[X] + [buf[k] for k in range(K)])
    ev[4].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    B = col_blocks_of(A1, d)
    nnz = int(ix.numel())
    res = {"what": ("one GraphOp.propagate(K) hop loop as the reference calls it (once per run, "
                    "node_classification.py:62): fresh operator + column cut + K hops + output panels, "
                    "inside the bracket"),
           "ms_total": wall * 1e3, "ms_operator_build": ev[0].elapsed_time(ev[1]),
           "ms_propagate": ev[1].elapsed_time(ev[4]),
           "ms_per_hop": ev[1].elapsed_time(ev[4]) / max(1, K),
           "ms_plan_build": ev[1].elapsed_time(ev[2]), "ms_panel_alloc": ev[2].elapsed_time(ev[3]),
           "ms_hops": ev[3].elapsed_time(ev[4]), "column_blocks": B,
           "value": K * nnz / wall, "unit": "propagated edges/s"}
    del out, buf, A1
    torch.cuda.empty_cache()
    return res


def rank_devices(dev, backend, world, group=None):
    """Every rank's device (all-gathered): index, name, PCI domain:bus:device, host -- so a
    multi-GPU record shows that the ranks ran on N distinct GPUs."""
    me = {"rank": dist.get_rank(group), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "host": socket.gethostname()}
    if dev.type == "cuda":
        pr = torch.cuda.get_device_properties(dev)
        me.update({"device": dev.index, "name": pr.name,
                   "pci": "%04x:%02x:%02x" % (getattr(pr, "pci_domain_id", 0), getattr(pr, "pci_bus_id", 0),
                                              getattr(pr, "pci_device_id", 0))})
    allr = [None] * world
    dist.all_gather_object(allr, me, group=group)
    pcis = {(r.get("host"), r.get("pci")) for r in allr}
    return {"backend": backend, "world_size": world, "ranks": allr,
            "distinct_gpus": len(pcis), "one_gpu_per_rank": len(pcis) == world}


def dist_sampled_parity(op, panels, K, n_random=1500, n_top=10, seed=13, n_halo=256, group=None):
    """The N-GPU check where the whole graph's panels do not fit beside a rank's share
    (papers100M, RMAT-26): after the timed steps, outside the timed region,
      * sampled own rows of hop 1 and hop K (random + the longest) against the CPU oracle
        (oracle/srg_oracle.c, one fp32 fma chain per element in CSR order, matmul.c:23-40) fed with
        the rank's own previous panel -- the local operator's rows keep their CSR order, their
        columns remapped into [own | halo], so the oracle runs the one-GPU chain;
      * the halo those hops read: sampled halo rows (received and ghost) of panels 0 and K-1 sent
        to their owners, which compare them with their own rows bit for bit.
    Returns {"bit_exact": ...} (the minimum over ranks).  Test infrastructure used as the checker
    only; nothing measured runs through it."""
    from oracle import oracle as O
    P = op.world
    dev = panels[0].device
    rows = op.rows
    ok = True
    ip = op._lip[: rows + 1]
    deg = ip[1:] - ip[:-1]
    g = torch.Generator(device="cpu").manual_seed(seed + op.rank)
    pick = [torch.randint(0, max(rows, 1), (min(n_random, rows),), generator=g).to(ip.device),
            torch.sort(deg, descending=True).indices[:n_top]] if rows else []
    checked = 0
    if rows:
        r = torch.unique(torch.cat(pick))
        beg, cnt = ip[r], deg[r]
        tot = int(cnt.sum())
        pos = torch.repeat_interleave(beg - torch.cumsum(cnt, 0) + cnt, cnt, output_size=tot) + \
            torch.arange(tot, device=ip.device)
        ucols, inv = torch.unique(op._lix[pos].long(), return_inverse=True)
        sub = (np.r_[0, np.cumsum(cnt.cpu().numpy())].astype(np.int64), inv.to(torch.int32).cpu().numpy(),
               op._lvv[pos].cpu().numpy())
        ks = [1] + ([K] if K > 1 else [])
        for k in ks:
            want = O.spmm(*sub, panels[k - 1][ucols.to(dev)].cpu().numpy())
            have = panels[k][r.to(dev)].cpu().numpy()
            ok = ok and np.array_equal(have.view(np.uint32), want.view(np.uint32))
        checked = int(r.numel())
    # the halo of the panels those hops read, checked by the rows' owners
    halo_ok = True
    ids = op.halo_ids()
    owners = torch.bucketize(ids, torch.tensor(op.starts[1:], device=ids.device), right=True) if ids.numel() else ids
    sel = torch.randperm(ids.numel(), generator=g)[:n_halo].to(ids.device) if ids.numel() else ids
    mine = {}
    for k in sorted({0, K - 1}):
        vals = panels[k][rows + sel.to(dev)].cpu() if sel.numel() else torch.zeros((0, panels[k].shape[1]))
        mine[k] = (ids[sel].cpu(), owners[sel].cpu(), vals)
    allm = [None] * P
    dist.all_gather_object(allm, mine, group=group)
    for other in allm:
        for k, (gid, own, vals) in other.items():
            m = own == op.rank
            if bool(m.any()):
                loc = (gid[m] - op.r0).to(dev)
                halo_ok = halo_ok and torch.equal(panels[k][loc].cpu(), vals[m])
    flags = torch.tensor([int(ok), int(halo_ok)], dtype=torch.int64,
                         device=dev if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(flags, op=dist.ReduceOp.MIN, group=group)
    return {"hops_checked": [1] + ([K] if K > 1 else []), "rows_checked_rank0": checked,
            "rows": f"{n_random} random + the {n_top} longest own rows per rank",
            "halo_rows_checked_per_rank": int(min(n_halo, ids.numel())), "halo_panels_checked": sorted({0, K - 1}),
            "bit_exact": bool(flags[0].item()), "halo_equal_to_owners": bool(flags[1].item()),
            "checker": "oracle/srg_oracle.c fp32 fma chains fed with the rank's previous panel (outside the timed region)"}


def launch_ranks(n_ranks, args, script=None):
    """--gpus N without torchrun: spawn the N ranks as worker processes of this script (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as torchrun sets them), before this process
    touches any GPU, forward rank 0's JSON line and return the first failing exit code."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n_ranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_ranks),
                   LOCAL_WORLD_SIZE=str(n_ranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script or __file__)] + list(args), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    import threading

    def forward():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode())
            sys.stdout.flush()
    t = threading.Thread(target=forward, daemon=True)
    t.start()
    first_bad = 0
    while True:           # a rank that fails leaves the others waiting in a collective: end them
        rcs = [p.poll() for p in procs]
        failed = [rc for rc in rcs if rc not in (None, 0)]
        if failed:
            first_bad = failed[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            break
        if all(rc is not None for rc in rcs):
            break
        time.sleep(0.2)
    rcs = [p.wait() for p in procs]
    t.join(timeout=10)
    if first_bad:
        log(f"worker exit codes {rcs}")
    return first_bad


def reference_hops(ip, ix, vals, n, X, K, dev):
    """Hop 1 and hop K of the whole graph computed by this rank alone with the one-GPU kernels
    (bitwise the 1-GPU bench, and so the reference's product): an N-GPU run checks its own rows
    against them after the timed steps, so the first run over RCCL on a node also proves the
    exchange bitwise.  None when three whole panels do not fit in half of the free memory."""
    from srgnn.csr import DeviceCSR
    from srgnn.spmm import spmm
    free, _ = torch.cuda.mem_get_info(dev)
    if K < 1 or 3 * n * X.shape[1] * 4 > 0.5 * free:
        return None
    A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, device=dev, validate=False)
    bufs = [torch.empty_like(X), torch.empty_like(X)]
    out, cur = {}, X
    for k in range(1, K + 1):
        nxt = bufs[(k - 1) % 2] if k > 1 or K == 1 else torch.empty_like(X)
        spmm(A, cur, out=nxt)
        if k == 1:
            out[1] = nxt
        cur = nxt
    out[K] = cur
    torch.cuda.synchronize()
    return out


def run_wavelet(a, dev, world=1, rank=0, pmc=None):
    """SpectralModel's wavelet operator (SSRG/models/base_scalable/base_model.py:180-265) on the
    config's graph: R_s = sum_k c_{s,k} T_k(L~) X for tau = -0.5, +0.5, Chebyshev order 3, fp32.
    value = order * nnz(L) * steps / time: every order is one SpMM pass over the whole panel (in
    column blocks when the panels do not fit one GPU).  N > 1: srgnn.dist.HaloWaveletFilter (row
    partition, one halo exchange per order, bitwise equal to one GPU)."""
    if world > 1:
        return run_wavelet_dist(a, dev, world, rank)
    if a.dtype == "f64":
        return run_wavelet_f64(a, dev, pmc)
    from srgnn import wavelet as W
    from srgnn.csr import DeviceCSR
    from srgnn import _lib
    from srgnn.spmm import col_blocks_of, hop, launches_per_hop, spmm_cheby
    t_build = time.perf_counter()
    ip, ix, lv, n, d, lmax = graphs.build_laplacian(a.config, dev, d=a.d)
    nnz = int(ix.numel())
    order = 3
    filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=order, lmax=lmax,
                                           dtype=torch.float32, heavy_threshold=a.heavy_threshold)
    X = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device=dev)
    R = torch.empty((2, n, d), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()          # the builders' temporaries
    free, _ = torch.cuda.mem_get_info(dev)
    cb = a.col_block or d
    fused = a.fused_epilogue
    n_work = filt.work_panels(fused)
    # widest block whose work panels fit beside what is resident (1 GiB kept free): wide blocks
    # gather more bytes per nonzero (RMAT-26: 64 columns 1.37 s per step, 32 columns 1.87 s)
    while not a.col_block and cb > 8 and n_work * n * cb * 4 > free - 2 ** 30:
        cb //= 2
    from srgnn.plan import _torch_free
    while True:
        # the native plans of L and F for cb-column panels; their memory comes from torch's cache (which
        # the graph build left fragmented), so what must still fit is the work panels: narrower blocks
        # until they do
        filt.prepare_column_blocks(cb, hops=order * (d // cb) * (a.steps + a.warmup))
        torch.cuda.synchronize()
        if a.col_block or cb <= 8 or n_work * n * cb * 4 <= _torch_free(dev) - 2 ** 30:
            break
        filt.drop_layouts()
        torch.cuda.synchronize()
        cb //= 2
    layout = "native plan (in torch's caching allocator)"
    log(f"wavelet {a.config}: n={n} nnz(L)={nnz} d={d} lmax={lmax} col_block={cb} layout={layout} "
        f"hub={filt.n_hub} heavy={filt.n_heavy} built in {time.perf_counter() - t_build:.1f}s")

    def step():
        filt.apply(X, col_block=cb, out=R, fused_epilogue=fused)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # roofline: one order's launch at the block width (HIP events on the launch stream): a
    # Chebyshev step (srg_spmm_cheby_f32, T_{k+1} over T_{k-1}) with the fused epilogue, else the
    # SpMM launch of the split path
    stream = torch.cuda.current_stream(dev)
    Fm = filt._csr(filt.fvals)
    B = 1 if fused else col_blocks_of(Fm, cb)
    LB = launches_per_hop(Fm, B, cb)
    tb = torch.zeros((n, cb), dtype=torch.float32, device=dev)
    ns = len(filt.taus)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.roofline_reps)]
    for r in range(a.roofline_reps):
        ev[2 * r].record(stream)
        if fused:
            spmm_cheby(Fm, X[:, :cb], tb, _lib.SRG_CHEBY_STEP, filt.a1, filt.a2, tb, None, filt.coeffs[:, 2],
                       R[:, :, :cb])
        else:
            hop(Fm, X[:, :cb], tb)
        ev[2 * r + 1].record(stream)
    torch.cuda.synchronize()
    kern_s = float(np.mean([ev[2 * r].elapsed_time(ev[2 * r + 1]) * 1e-3 for r in range(a.roofline_reps)]))
    del tb
    # the fused step also reads T_{k-1} and reads + writes every scale's output once
    extra = n * cb * 4 * (1 + 2 * ns) if fused else 0
    b_alg = roofline.bytes_no_reuse(n, nnz, cb) + extra
    b_comp = roofline.bytes_compulsory(n, nnz, cb, n_cols=n) + extra
    peak = roofline.MI355X_HBM_PEAK_GBS
    traffic = float(pmc["hbm_bytes_per_hop"]) if pmc is not None and int(pmc["launches_per_hop"]) == LB else None
    achieved = (traffic if traffic else b_comp) / kern_s / 1e9
    res = {
        "metric": "propagated edges/sec (wavelet-basis Chebyshev propagation)",
        "value": a.steps * order * nnz / dt,
        "unit": "propagated edges/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic (R-MAT power-law graph with the {a.config} node/edge counts, U[-1,1) features)",
        "config": {"workload": f"{a.config}-shaped heat-wavelet filter bank", "n_nodes": n, "nnz_L": nnz,
                   "d": d, "chebyshev_order": order, "scales": [-0.5, 0.5], "lmax": lmax,
                   "col_block": cb, "parallelism": "x1",
                   "mode": ("fp32, one load-balanced launch per order with the Chebyshev epilogue fused"
                            if fused else "fp32, split path (SpMM + epilogue launches)")
                           + " (bit-identical to the fused Chebyshev kernel)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "achieved_basis": ("L2 -> fabric bytes per order's SpMM (Infinity-Cache hits included; PMC "
                                        "2 * FETCH_SIZE + WRITE_SIZE = traffic) / its time" if traffic
                                        else "compulsory bytes / the SpMM's time (no counter run: a lower bound)"),
                     "traffic_source": pmc["source"] if traffic else None,
                     "unit_of_work": f"one Chebyshev order's SpMM over a {cb}-column block ({B} column blocks, {LB} launches)",
                     "kernel": (f"k_spmm with the Chebyshev epilogue: one order over a {cb}-column block" if fused
                                else f"k_spmm: one Chebyshev order's SpMM over a {cb}-column block"),
                     "kernel_ms": kern_s * 1e3, "launches_per_hop": LB, "kernel_ms_per_launch": kern_s * 1e3 / LB,
                     "frac_no_reuse": b_alg / kern_s / 1e9 / peak, "frac_compulsory": b_comp / kern_s / 1e9 / peak,
                     "algorithmic_bytes_per_hop": b_alg, "compulsory_bytes_per_hop": b_comp,
                     "traffic_over_compulsory": (traffic / b_comp) if traffic else None},
        "cpu_baseline": None,
    }
    if not a.no_cpu_baseline:
        log("cpu baseline ...")
        host = (ip.cpu().numpy(), ix.cpu().numpy(), filt.fvals.cpu().numpy(), X.cpu().numpy())
        cb_res = cpu_baseline(*host, n, d, a.cpu_seconds)
        cb_res["sample"] = "the SpMM part of each Chebyshev order: " + cb_res["sample"]
        res["cpu_baseline"] = cb_res
    print(json.dumps(res), flush=True)


def run_wavelet_f64(a, dev, pmc=None):
    """The filter bank at the reference's precision: pygsp cheby_op is fp64 (SSRG/models/base_scalable/
    base_model.py:236-265, :243), R_s = sum_k c_{s,k} T_k(L~) S for tau = -0.5, +0.5, order 3.  Each order
    is HeatWaveletFilter.order_step: the row-wave gather with the recurrence and every scale's output fused,
    scipy's operation order (bit-exact vs the oracle's restatement of cheby_op) -- over the filter's
    column-blocked plan (srg_plan_cheby_step_f64: one launch per column block, the whole hub rows as hub
    workgroups on the side stream) where the fp64 panel outgrows the caches, else one srg_cheby_step_hub_f64
    launch.  The panel is the
    config's d columns, or -- where five fp64 panels of that width (S, two T work panels, the two scales'
    R) do not fit -- the widest power-of-two column block that does (RMAT-26): a step then filters that
    block, and `config.col_block` says so.  value = order * nnz(L) * steps / time.  Parity after the
    timed steps: every row of two columns of R against oracle.cheby_op (fp64, whole graph) bit for bit.
    cpu_baseline: the reference's CPU path for one order, scipy's fp64 csr @ dense (pygsp's L.dot), on
    a row block."""
    from srgnn import wavelet as W
    t_build = time.perf_counter()
    ip, ix, lv, n, d, lmax = graphs.build_laplacian(a.config, dev, d=a.d)
    nnz = int(ix.numel())
    order, taus = 3, [-0.5, 0.5]
    ns = len(taus)
    filt = W.HeatWaveletFilter.from_device(ip, ix, lv, n, taus, order=order, lmax=lmax, dtype=torch.float64,
                                           heavy_threshold=a.heavy_threshold)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    cb = a.col_block or d
    while not a.col_block and cb > 1 and (3 + ns) * n * cb * 8 > free - 4 * 2 ** 30:
        cb //= 2
    S = synth.uniform_features_t(n, cb, seed=synth.FEATURE_SEED, device=dev).to(torch.float64)
    R = torch.empty((ns, n, cb), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    log(f"wavelet f64 {a.config}: n={n} nnz(L)={nnz} d={d} col_block={cb} lmax={lmax} hub={filt.n_hub} "
        f"heavy={filt.n_heavy} built in {time.perf_counter() - t_build:.1f}s")

    def step():
        filt.apply(S, split=False, out=R)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # roofline: one Chebyshev STEP order (F T_k - T_{k-1}, both scales' R updated: every block launch and the
    # hub workgroups, joined back), HIP events on the launch stream, over work panels of the block's width
    P64 = filt._plan64(cb)
    step_launches = P64.n_launch if P64 is not None else 1
    from srgnn import _lib
    stream = torch.cuda.current_stream(dev)
    t_cur, t_old = torch.empty_like(S), torch.empty_like(S)
    t_cur.copy_(S)
    t_old.zero_()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.roofline_reps)]
    for r in range(a.roofline_reps):
        ev[2 * r].record(stream)
        filt.order_step(filt.fvals, S, t_old, t_cur, _lib.SRG_CHEBY_STEP, None, filt.coeffs[:, 2], R)
        ev[2 * r + 1].record(stream)
    torch.cuda.synchronize()
    kern_s = float(np.mean([ev[2 * r].elapsed_time(ev[2 * r + 1]) * 1e-3 for r in range(a.roofline_reps)]))
    del t_cur, t_old
    b_alg = roofline.cheby_step_bytes_no_reuse_f64(n, nnz, cb, ns)
    b_comp = roofline.cheby_step_bytes_compulsory_f64(n, nnz, cb, ns)
    peak = roofline.MI355X_HBM_PEAK_GBS
    traffic = float(pmc["hbm_bytes_per_hop"]) if pmc is not None else None
    achieved = (traffic if traffic else b_comp) / kern_s / 1e9
    # parity: the whole recurrence on two columns, every row, against the oracle's fp64 cheby_op
    filt.apply(S, split=False, out=R)
    torch.cuda.synchronize()
    from oracle import oracle as O
    cols = [0, cb - 1] if cb > 1 else [0]
    host = (ip.cpu().numpy(), ix.cpu().numpy(), lv.to(torch.float64).cpu().numpy())
    want = O.cheby_op(host, filt.coeffs, S[:, cols].cpu().numpy(), lmax)
    got = R[:, :, cols].cpu().numpy()
    parity = {"checked": f"every row of R (both scales) in columns {cols}, after the timed steps",
              "bit_exact": bool(np.array_equal(got.view(np.uint64), want.view(np.uint64))),
              "checker": "oracle.cheby_op: oracle/srg_oracle.c's fp64 restatement of pygsp cheby_op (scipy's "
                         "csr_matvecs order), the whole graph"}
    log(f"parity vs oracle fp64: {parity['bit_exact']}")
    res = {
        "metric": "propagated edges/sec (wavelet-basis Chebyshev propagation)",
        "value": a.steps * order * nnz / dt,
        "unit": "propagated edges/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64",
        "data": f"synthetic (R-MAT power-law graph with the {a.config} node/edge counts, U[-1,1) features)",
        "config": {"workload": f"{a.config}-shaped heat-wavelet filter bank, fp64 (the reference's precision)",
                   "n_nodes": n, "nnz_L": nnz, "d": d, "col_block": cb,
                   "columns_per_step": cb, "chebyshev_order": order, "scales": taus, "lmax": lmax,
                   "parallelism": "x1",
                   "mode": ("fp64, per order %d column-block launches of srg_plan_cheby_step_f64 + %d whole hub rows "
                            "as hub workgroups beside them (SpMM + recurrence + both scales fused)"
                            % (P64.col_blocks, P64.hub_rows_whole) if P64 is not None else
                            "fp64, one srg_cheby_step_hub_f64 launch per order (SpMM + recurrence + both scales fused)")
                           + ("" if cb == d else f"; a step filters one {cb}-column block of the {d}-column "
                                                 "panel (the widest whose five fp64 panels fit)")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "achieved_basis": ("L2 -> fabric bytes of one Chebyshev STEP launch (PMC 2 * FETCH_SIZE + "
                                        "WRITE_SIZE = traffic) / its time" if traffic
                                        else "compulsory bytes / the launch's time (no counter run: a lower bound)"),
                     "traffic_source": pmc["source"] if traffic else None,
                     "unit_of_work": f"one Chebyshev STEP order over a {cb}-column fp64 panel",
                     "kernel": ("k_cheby_blk64 (+ k_cheby_hub64 beside it): one STEP order = %d launches "
                                "(srg_plan_cheby_step_f64)" % step_launches if P64 is not None
                                else "k_cheby<double> (+ k_cheby_hub64 beside it; srg_cheby_step_hub_f64, SRG_CHEBY_STEP)"),
                     "kernel_ms": kern_s * 1e3, "launches_per_step": step_launches,
                     "frac_no_reuse": b_alg / kern_s / 1e9 / peak, "frac_compulsory": b_comp / kern_s / 1e9 / peak,
                     "algorithmic_bytes_per_launch": b_alg, "compulsory_bytes_per_launch": b_comp,
                     "traffic_over_compulsory": (traffic / b_comp) if traffic else None},
        "parity_vs_oracle": parity,
        "cpu_baseline": None,
    }
    if not a.no_cpu_baseline:
        log("cpu baseline ...")
        res["cpu_baseline"] = cpu_baseline_cheby64(host[0], host[1], filt.fvals.cpu().numpy(),
                                                   S.cpu().numpy(), n, cb, a.cpu_seconds)
    print(json.dumps(res), flush=True)


def cpu_baseline_cheby64(ip, ix, fv, S, n, d, budget_s):
    """The reference's CPU path for one Chebyshev order at its precision: pygsp cheby_op's
    `L.dot(T)` is scipy's fp64 csr @ dense (one thread: scipy's csr_matvecs), timed on row blocks of
    F = (2/a1)(L - a2 I) for ~budget_s."""
    import scipy.sparse as sp
    nnz = int(ip[-1])
    block = max(1, int(n * min(1.0, 5e7 / max(nnz, 1))))
    edges, t0, r0 = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < budget_s:
        r1 = min(n, r0 + block)
        e0, e1 = int(ip[r0]), int(ip[r1])
        A = sp.csr_matrix((fv[e0:e1], ix[e0:e1], ip[r0:r1 + 1] - e0), shape=(r1 - r0, n))
        _ = A @ S
        edges += e1 - e0
        r0 = 0 if r1 == n else r1
    dt = time.perf_counter() - t0
    return {"value": edges / dt, "unit": "propagated edges/s", "cores": 1, "kind": "reference",
            "cpu_model": _cpu_model(),
            "sample": f"scipy {sp.__name__} fp64 csr @ dense [n, {d}] (pygsp cheby_op's L.dot, base_model.py:243) on "
                      f"row blocks of ~{block} rows of F for {dt:.1f} s, one thread"}


def run_wavelet_dist(a, dev, world, rank):
    from srgnn.dist import HaloWaveletFilter
    devices = rank_devices(dev, os.environ.get("SRGNN_DIST_BACKEND", "nccl"), world)
    t_build = time.perf_counter()
    ip, ix, lv, n, d, lmax = graphs.build_laplacian(a.config, dev, d=a.d)
    nnz = int(ix.numel())
    order = 3
    f64 = a.dtype == "f64"
    tdt, esz = (torch.float64, 8) if f64 else (torch.float32, 4)
    f = HaloWaveletFilter(ip, ix, lv, n, [-0.5, 0.5], order=order, lmax=lmax, chunks=(a.chunks or (4 if world <= 2 else 6)),
                          heavy_threshold=a.heavy_threshold, device=dev, dtype=tdt)
    # fp64: the widest power-of-two column block whose five [rows + halo] panels fit (as one GPU's fp64 line)
    cb = a.col_block or d
    if f64 and not a.col_block:
        torch.cuda.synchronize()
        free, _ = torch.cuda.mem_get_info(dev)
        while cb > 1 and 5 * (f.rows + f.opL.halo) * cb * esz > free - 8 * 2 ** 30:
            cb //= 2
    X = synth.uniform_features_t(n, cb, seed=synth.FEATURE_SEED, device=dev).to(tdt)
    S_local = X[f.r0:f.r1].contiguous()
    # this rank's rows of the one-GPU filter bank on the whole graph, checked after the timed steps
    ref = None
    free, _ = torch.cuda.mem_get_info(dev)
    if 6 * n * cb * esz < 0.5 * free:
        from srgnn import wavelet as W
        one = W.HeatWaveletFilter.from_device(ip, ix, lv, n, [-0.5, 0.5], order=order, lmax=lmax,
                                              dtype=tdt, heavy_threshold=a.heavy_threshold)
        ref = one.apply(X)[:, f.r0:f.r1].clone()
        one.drop_layouts()
        del one
    del X, ip, ix, lv
    torch.cuda.empty_cache()
    log(f"rank {rank}: wavelet rows={f.rows} halo={f.opL.halo} built in {time.perf_counter() - t_build:.1f}s")
    R = None
    for _ in range(a.warmup):
        f.apply(S_local)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        R = f.apply(S_local)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ok = ref is not None and R is not None and torch.equal(R, ref)
    flags = torch.tensor([int(ref is not None), int(ok)], dtype=torch.int32, device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    parity = ({"outputs_checked": "every scale, this rank's rows", "bitwise_equal_to_1gpu": bool(flags[1].item()),
               "ranks": world} if flags[0].item() else {"skipped": "the whole graph's panels do not fit beside a rank's share"})
    res = {"metric": "propagated edges/sec (wavelet-basis Chebyshev propagation)",
           "value": a.steps * order * nnz / dt, "unit": "propagated edges/s", "n_gpus": world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f64" if f64 else "f32",
           "data": f"synthetic (R-MAT power-law graph with the {a.config} node/edge counts, U[-1,1) features)",
           "config": {"workload": f"{a.config}-shaped heat-wavelet filter bank" + (", fp64 (the reference's precision)"
                                                                                   if f64 else ""),
                      "n_nodes": n, "nnz_L": nnz, "d": d, "col_block": cb,
                      "chebyshev_order": order, "scales": [-0.5, 0.5], "lmax": lmax,
                      "parallelism": f"row-partition x{world} (halo exchange per order)",
                      "mode": ("fp64: per order one fused srg_cheby_step_hub_f64 launch per row chunk of each rank, "
                               "each chunk's fp64 halo rows sent while the next chunks compute" if f64
                               else "fp32 split path per rank")
                      + ("" if cb == d else f"; a step filters one {cb}-column block of the {d}-column panel")},
           "roofline": None, "cpu_baseline": None, "parity_vs_1gpu": parity,
           "devices": devices}
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # the PMC passes are child processes: they must run before this process touches the GPU
    pmc = None
    if world == 1 and not a.aggregate and not a.fused_epilogue and \
            (a.pmc == "on" or (a.pmc == "auto" and not _under_profiler())):
        pmc = measure_pmc(a)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # one rank per GPU.  SRGNN_DIST_BACKEND=gloo rehearses the N-rank path on fewer GPUs (ranks share
    # devices round-robin; gloo moves the halo through the host, so its numbers are not a benchmark)
    backend = os.environ.get("SRGNN_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    def init_pg():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if a.op == "wavelet":
        if world > 1:
            init_pg()
        return run_wavelet(a, dev, world, rank, pmc)
    devices = None
    if world > 1:
        init_pg()
        devices = rank_devices(dev, backend, world)
        log(f"rank {rank}: backend {backend}, {devices['distinct_gpus']} distinct GPUs over {world} ranks")

    from srgnn.csr import DeviceCSR
    from srgnn.spmm import hop, launches_per_hop, prepare, propagate, spmm

    t_build = time.perf_counter()
    ip, ix, vals, n, d, K = graphs.build(a.config, dev, d=a.d)
    K = a.k if a.k is not None else K
    nnz = int(ix.numel())
    X = synth.uniform_features_t(n, d, seed=synth.FEATURE_SEED, device=dev)
    torch.cuda.synchronize()
    log(f"graph {a.config}: n={n} nnz={nnz} d={d} K={K} built in {time.perf_counter() - t_build:.1f}s")

    stream = torch.cuda.current_stream(dev)
    mode = a.mode
    ref_full = reference_hops(ip, ix, vals, n, X, K, dev) if world > 1 and a.dist_parity == "auto" else None
    if world == 1:
        A = DeviceCSR.from_tensors(ip, ix, vals, n_cols=n, heavy_threshold=a.heavy_threshold, device=dev)
        if mode == "auto":
            free, _ = torch.cuda.mem_get_info(dev)
            mode = "panels" if K * n * d * 4 < 0.9 * free else "last"
            log(f"mode {mode}: {K} panels need {K * n * d * 4 / 1e9:.1f} GB, {free / 1e9:.1f} GB free")
        # the operator serves every warm-up and timed step: cut it once here when that amortises
        col_blocks = prepare(A, d, K * (a.steps + a.warmup), a.col_blocks)
        launches = launches_per_hop(A, col_blocks, d, agg=bool(a.aggregate))
        log(f"schedule: n_hub={A.n_hub} n_heavy={A.n_heavy} column blocks per hop={col_blocks} ({launches} launches)")
        if a.aggregate:
            from srgnn.aggregate import combine_plan, combine_steps, propagate_aggregate

            class _Msg:
                aggr_type = {"weighted": "simple_weighted"}.get(a.aggregate, a.aggregate)
                start, end, combination_type, alpha, weight_list = 0, K + 1, "alpha", 0.15, None
            plan_mode, terms, div = combine_plan(_Msg(), K + 1)
            steps_plan = combine_steps(plan_mode, terms, div)
            mode = f"aggregate-{a.aggregate}"
            panels = [X, None]

            def step():
                panels[1] = None
                panels[1] = propagate_aggregate(A, X, K, steps_plan, col_blocks=col_blocks)
        elif mode == "panels":
            buf = torch.empty((K, n, d), dtype=torch.float32, device=dev)
            panels = [X] + [buf[k] for k in range(K)]

            def step():
                propagate(A, X, K, panels=panels, nt_store=a.nt_store, col_blocks=col_blocks, fast=a.fast)
        else:
            from srgnn.aggregate import propagate_aggregate
            panels = [X, None]

            def step():
                panels[1] = None
                panels[1] = propagate_aggregate(A, X, K, last_only=True, col_blocks=col_blocks)
        local_rows, local_nnz = n, nnz
    else:
        col_blocks = launches = 1
    if world > 1 and a.exchange == "allgather":
        from srgnn.dist import RowPartitionedOperator
        op = RowPartitionedOperator(ip, ix, vals, n, heavy_threshold=a.heavy_threshold, device=dev)
        A = op.A
        x_loc = op.new_panel(d)
        x_loc[: op.rows].copy_(X[op.r0:op.r1])
        panels = [x_loc] + [op.new_panel(d) for _ in range(K)]
        del X

        def step():
            op.propagate(x_loc, K, panels=panels)
        local_rows, local_nnz = op.rows, op.nnz_local
    elif world > 1:
        from srgnn.dist import HaloPartitionedOperator
        op = HaloPartitionedOperator(ip, ix, vals, n, chunks=(a.chunks or (4 if world <= 2 else 6)), heavy_threshold=a.heavy_threshold,
                                     device=dev, ghost_max_degree=a.ghost_max_degree, fast=a.fast)
        log(f"rank {rank}: rows={op.rows} nnz={op.nnz_local} halo={op.halo} (received {op.n_recv}, "
            f"ghosts {op.n_ghost} <= degree {op.ghost_max_degree}, {op._ghost_pos.numel()} ghost nnz; "
            f"link {op.link_bps / 1e9:.1f} GB/s) "
            f"hub_rows={op.views[-1][1]} groups={op.n_groups}")
        panels = [op.new_panel(d) for _ in range(K + 1)]
        panels[0][: op.rows].copy_(X[op.r0:op.r1])
        x_loc = panels[0]
        # GraphOp.propagate takes the whole feature matrix; every rank holds it, so hop 0's halo
        # is gathered locally (--exchange-x: from its owners, as when a rank holds only its rows)
        x_full = None if a.exchange_x else X
        del X

        def step():
            op.propagate(x_loc, K, panels=panels, x_full=x_full)
        # one hop's kernels also compute the ghost rows (the roofline counts that work)
        local_rows, local_nnz = op.rows + op.n_ghost, op.nnz_local + int(op._ghost_pos.numel())

    one_shot_res = None
    if world == 1 and mode == "panels" and K > 0 and not a.fast and \
            torch.cuda.mem_get_info(dev)[0] > 1.3 * K * n * d * 4:
        one_shot(ip, ix, vals, n, X, K, dev, a.heavy_threshold)        # warm (allocator, code objects)
        one_shot_res = one_shot(ip, ix, vals, n, X, K, dev, a.heavy_threshold)
        log(f"one-shot propagate(K={K}): {one_shot_res['ms_total']:.1f} ms "
            f"({one_shot_res['ms_per_hop']:.2f} ms per hop)")
    sample = oracle_sample(ip, ix, vals, n, a.parity_rows) if world == 1 and K > 0 else None
    refs = None
    if ref_full is not None:     # this rank's rows of the 1-GPU hops, checked after the timed steps
        refs = {k: v[op.r0:op.r1].clone() for k, v in ref_full.items()}
    del ref_full
    torch.cuda.empty_cache()
    host_copy = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        host_copy = (ip.cpu().numpy(), ix.cpu().numpy(), vals.cpu().numpy(), X.cpu().numpy())
    del ip, ix, vals

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    graphed = False
    if a.graph and world == 1 and mode == "panels" and not a.fast:
        # the step's launches (hub forks / joins included: the side stream joins the capture through
        # the library's events) as one HIP graph on a capture stream warmed up first (the library's
        # side stream for it is created outside the capture); replayed on the launch stream
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        with torch.cuda.stream(cap):
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            step()
        torch.cuda.synchronize()
        plain_step, step = step, g.replay
        g.replay()
        torch.cuda.synchronize()
        graphed = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_run = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev_run[0].record(stream)
    for _ in range(a.steps):
        step()
    ev_run[1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    run_s = ev_run[0].elapsed_time(ev_run[1]) * 1e-3        # the timed steps, HIP events on the launch stream
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    parity = None
    oracle_checks = None
    if sample is not None and mode == "panels":
        # hop 1 from X and hop K from hop K-1, as the timed steps left them
        oracle_checks = parity_vs_oracle(sample, [(1, panels[0], panels[1])] +
                                         ([(K, panels[K - 1], panels[K])] if K > 1 else []), tolerance=a.fast)
    if world > 1:
        # the N-GPU hops of this rank's rows against the 1-GPU kernels on the whole graph, bit for bit
        if a.fast:      # hub rows re-associated: normwise relative difference per row vs the exact hops
            ok = refs is not None and all(
                bool(((panels[k][: op.rows] - v).norm(dim=1) <= 1e-5 * v.norm(dim=1) + 1e-30).all())
                for k, v in refs.items())
        else:
            ok = refs is not None and all(torch.equal(panels[k][: op.rows], v) for k, v in refs.items())
        flags = torch.tensor([int(refs is not None), int(ok)], dtype=torch.int32, device=dev)
        dist.all_reduce(flags, op=dist.ReduceOp.MIN)
        if flags[0].item():
            parity = {"hops_checked": sorted(refs), ("within_1e-5_of_1gpu" if a.fast else "bitwise_equal_to_1gpu"):
                      bool(flags[1].item()), "ranks": world}
        elif a.exchange == "halo" and not a.fast:
            # the whole graph's panels do not fit beside a rank's share: sampled own rows of hop 1
            # and hop K against the oracle, and sampled halo rows against their owners
            parity = {"whole_graph_reference": ("not computed (--dist-parity sampled)" if a.dist_parity == "sampled"
                                                else "does not fit beside a rank's share"),
                      "sampled_vs_oracle": dist_sampled_parity(op, panels, K)}
        else:
            parity = {"skipped": "the whole graph's panels do not fit beside a rank's share"}
        del refs

    # roofline: average duration of one hop's SpMM launches on this rank (HIP events on the
    # launch stream; the hub side stream is joined back into it by the library)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.roofline_reps)]
    if world == 1:
        def one_hop():
            hop(A, panels[0], panels[1], nt_store=a.nt_store, col_blocks=col_blocks, fast=a.fast)
        if panels[1] is None:
            panels[1] = torch.empty_like(X)
    elif a.exchange == "allgather":
        src = op._gather(panels[0])

        def one_hop():
            spmm(A, src, out=panels[1][: op.rows])
    else:
        def one_hop():
            op.compute(panels[0], panels[1])
    for r in range(a.roofline_reps):
        ev[2 * r].record(stream)
        one_hop()
        ev[2 * r + 1].record(stream)
    torch.cuda.synchronize()
    durs = [ev[2 * r].elapsed_time(ev[2 * r + 1]) * 1e-3 for r in range(a.roofline_reps)]
    kern_isolated_s = float(np.mean(durs))
    if sample is not None and oracle_checks is None:
        # last-hop / aggregate modes keep no hop K-1: the isolated launches above left hop 1 of X
        # (the timed operator, the same launches) in panels[1]
        oracle_checks = parity_vs_oracle(sample, [(1, panels[0], panels[1])], tolerance=a.fast)
    # one hop's launch duration: over the timed region itself on one GPU (K hop launches per step,
    # back to back on the launch stream, so the events bracket exactly the kernels plus their
    # few-microsecond gaps); on N GPUs the timed region also waits on the exchange, so the
    # isolated launches above are the kernel's duration there
    in_run = world == 1 and not a.aggregate and K > 0
    kern_s = run_s / (a.steps * K) if in_run else kern_isolated_s
    b_alg = roofline.bytes_no_reuse(local_rows, local_nnz, d)
    b_comp = roofline.bytes_compulsory(local_rows, local_nnz, d, n_cols=n)
    peak = roofline.MI355X_HBM_PEAK_GBS
    traffic, traffic_src, traffic_rd = pmc_traffic(a.config, launches_per_hop=launches, measured=pmc) if world == 1 \
        else (None, None, None)
    # the same bytes with the gather read calibration applied (reads / PMC_READ_CALIBRATION: the
    # counters read 3.8 % above the bytes a random-row gather asks for, profiles/r04_pmc_gather_calibration.txt)
    traffic_cal = (traffic_rd / roofline.PMC_READ_CALIBRATION + (traffic - traffic_rd)) \
        if traffic and traffic_rd is not None else None
    # achieved: HBM bytes the counters saw per hop / hop time (a lower bound -- the compulsory
    # bytes -- where no counter run exists for this layout)
    achieved = (traffic if traffic else b_comp) / kern_s / 1e9

    exchange_stats = {}
    if world > 1 and a.exchange == "halo":
        # per-hop exchange volume: max over ranks of the rows received and of the busiest peer link
        link = max(sum(op.recv_counts[g][q] for g in range(op.n_groups)) for q in range(world))
        st = torch.tensor([op.n_recv, link, op.n_ghost], dtype=torch.float64, device=dev)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        exchange_stats = {"halo_rows_received_max": int(st[0]), "busiest_link_GB_per_hop": float(st[1]) * d * 4 / 1e9,
                          "ghost_rows_max": int(st[2]), "halo_groups": op.n_groups,
                          "link_GBps_measured_for_ghost_plan": op.link_bps / 1e9}
    value = a.steps * K * nnz / dt
    res = {
        "metric": "propagated edges/sec (K-hop SpMM precompute)",
        "value": value,
        "unit": "propagated edges/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (R-MAT power-law graph with the {a.config} node/edge counts, U[-1,1) features)",
        "config": {"workload": f"{a.config}-shaped K-hop propagate", "n_nodes": n, "nnz_ahat": nnz,
                   "d": d, "K": K, "normalization": "sym r=0.5",
                   **({"column_blocks_per_hop": col_blocks} if world == 1 else {}),
                   "parallelism": f"row-partition x{world}" + (f" ({a.exchange} exchange)" if world > 1 else "")
                   + (f", ghost rows <= degree {op.ghost_max_degree}" if world > 1 and a.exchange == "halo" else "")
                   + (", X whole on every rank (hop 0's halo gathered locally)" if world > 1 and a.exchange == "halo"
                      and not a.exchange_x else ""),
                   "mode": "exact (bit-identical to reference)",
                   **({"launch": "HIP graph of one step, replayed"} if graphed else {}),
                   "outputs": ("all K+1 hop panels" if mode in ("panels", "auto") else
                               f"fused {a.aggregate} of hops 0..K (srgnn.aggregate, bit-exact vs the reference combine)"
                               if a.aggregate else "last hop only (2 ping-pong panels)")
                   if world == 1 else "all K+1 hop panels (row slices)",
                   **exchange_stats},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "achieved_basis": ("L2 -> fabric bytes per hop (Infinity-Cache hits included; PMC "
                                        "2 * FETCH_SIZE + WRITE_SIZE = traffic) / hop time" if traffic else
                                        "compulsory bytes per hop / hop time (no counter run for this layout: a lower bound)"),
                     "frac_calibrated": (traffic_cal / kern_s / 1e9 / peak) if traffic_cal else None,
                     "traffic_calibrated": traffic_cal,
                     "calibration": (f"reads / {roofline.PMC_READ_CALIBRATION} (profiles/r04_pmc_gather_calibration.txt)"
                                     if traffic_cal else None),
                     "traffic_source": traffic_src,
                     "unit_of_work": "one hop" + (f" = {col_blocks} column blocks in {launches} launches" if col_blocks > 1
                                                  else " (one launch)")
                                     + " + the hub workgroups beside them",
                     "kernel": "k_spmm (+ k_spmm_hub beside it): one hop" + (" of rank 0's rows" if world > 1 else "")
                     + (f" = {col_blocks} column blocks in {launches} launches (bitwise the one-launch hop)"
                        if col_blocks > 1 else ""),
                     "kernel_ms": kern_s * 1e3,
                     "launches_per_hop": launches,
                     "kernel_ms_per_launch": kern_s * 1e3 / launches,
                     "kernel_ms_source": ("HIP events over the timed steps / (steps x K)" if in_run
                                          else f"HIP events around {a.roofline_reps} isolated hop launches"),
                     "kernel_ms_isolated": kern_isolated_s * 1e3,
                     # SURVEY §8(d)'s no-reuse model counts every gathered X row as an HBM read, so
                     # cache hits push it past 1; the compulsory model counts every byte once
                     "frac_no_reuse": b_alg / kern_s / 1e9 / peak,
                     "frac_compulsory": b_comp / kern_s / 1e9 / peak,
                     "algorithmic_bytes_per_hop": b_alg,
                     "compulsory_bytes_per_hop": b_comp,
                     "traffic_over_compulsory": (traffic / b_comp) if traffic else None},
        "cpu_baseline": None,
    }
    if devices is not None:
        res["devices"] = devices
    if one_shot_res is not None:
        res["one_shot"] = one_shot_res
    if parity is not None:
        res["parity_vs_1gpu"] = parity
    if oracle_checks is not None:
        res["parity_vs_oracle"] = oracle_checks
        if a.fast:
            res["config"]["mode"] = ("fast (SRG_SPMM_FAST: hub rows re-associated in 64 segments; sampled rows within "
                                     "the fp32 error bound of the exact product)"
                                     if oracle_checks["within_fp32_bound_of_exact"] else "fast mode, OUT OF TOLERANCE")
        else:
            res["config"]["mode"] = ("exact: sampled rows bit-identical to the oracle (reference arithmetic)"
                                     if oracle_checks["bit_exact"] else "exact mode, ORACLE MISMATCH")
    if host_copy is not None:
        log("cpu baseline ...")
        ipn, ixn, vn, xn = host_copy
        res["cpu_baseline"] = cpu_baseline(ipn, ixn, vn, xn, n, d, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
