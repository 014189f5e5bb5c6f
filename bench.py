#!/usr/bin/env python3
"""bench.py — node2vec walk-steps/s on MI355X (+ TopSim pair-updates/s).

Headline (BASELINE.json configs[1]): node2vec p=0.25 q=4 on a synthetic
Graph500 R-MAT scale-20 graph (a,b,c = 0.57,0.19,0.19, edge factor 16, seed
42, symmetrised, deduplicated, no self loops), walk_length 80, 10 walks per
node.  One "step" = one pass of the hot path over one batch: 10 walks from
every vertex (6.47M walks, ~5.1e8 walk-steps) written to HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]

N>1: launched by torch.distributed.run, one rank per GPU.  The graph is
replicated; each rank walks its own block of global walk indices (walks are
a pure function of (seed, global walk index), so shards never overlap and
need no collective).  `value` = walk-steps of all ranks / max-over-ranks
time ("scaling": "weak").  `--allgather` adds the RCCL all-gather of the
emitted walks (north_star option) inside the timed step.

Also reported (same JSON line):
  roofline      36 algorithmic bytes per walk-step / kernel time,
                kernel time from HIP events on the launch stream; traffic from
                the committed rocprofv3 PMC pass (profiles/), or null.
  cpu_baseline  the oracle's C restatement of the same sampling (OpenMP),
                timed on a bounded sample of the same workload (rank 0, N=1).
  secondary     .topsim: TopSim_singleSample on lshrank blog (STEP=5,
                SAMPLE=10000, C=0.6, top-20, all 10,313 sources): pair-updates/s
                (--topsim-graphs adds arxiv / moreno / p10m under .topsim.more);
                .walk_10m / .walk_10m_p1q1: the north_star's 10M-node/100M-edge
                graph (R-MAT scale 24, ef 6), 1 walk per node, at the bench's
                p/q and at p=q=1, each with its CPU sample;
                .simrank_naive: SimRank.java (STEP=3, C=0.6) on blog, dense
                10,313^2 fp64 result: rounds/s, LDS-gather roofline.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
sys.path.insert(0, ROOT)

BYTES_PER_STEP = 36       # row bounds 16 + alias q/J 12 + nbr 4 + walk write 4
TOPSIM_B_EXT = 52         # per path-extension
TOPSIM_B_UPD = 24         # per pair-update
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
RANDOM_LINE_PEAK = 4.9e10 # measured: random 64 B sectors, one load instruction each, 8-32 GB tables (tools/calib/calib_sweep.hip)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--p", type=float, default=0.25)
    ap.add_argument("--q", type=float, default=4.0)
    ap.add_argument("--walk-length", type=int, default=80)
    ap.add_argument("--num-walks", type=int, default=10)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--allgather", action="store_true")
    ap.add_argument("--mode", choices=["auto", "bitset", "rejection"], default="auto",
                    help="second-order sampler (auto: bitset when it fits in HBM)")
    ap.add_argument("--no-topsim", action="store_true")
    ap.add_argument("--no-simrank", action="store_true")
    ap.add_argument("--no-walk10m", action="store_true",
                    help="skip the north_star 10M-node/100M-edge walk measurement")
    ap.add_argument("--walk10m-scale", type=int, default=24)
    ap.add_argument("--walk10m-edge-factor", type=int, default=6)
    ap.add_argument("--simrank-graph", default="blog", help="naive SimRank graph (blog or moreno)")
    ap.add_argument("--simrank-rounds", type=int, default=3, help="SimRank.java STEP")
    ap.add_argument("--no-rmat24", action="store_true",
                    help="skip config 4 (R-MAT-24 ef 16, p=1 q=0.5) on this GPU")
    ap.add_argument("--secondary", choices=["auto", "all", "none"], default="auto",
                    help="secondary workloads: auto = all at 1 GPU, none when ranks > 1 (scaling runs time "
                         "the headline only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--topsim-sample", type=int, default=10000)
    ap.add_argument("--topsim-step", type=int, default=5)
    ap.add_argument("--topsim-graphs", default="blog", help="comma list of blog,arxiv,moreno,p10m")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(csr, args, sample_walk0):
    """Oracle (C restatement, OpenMP) on a bounded sample of the same walks."""
    import oracle
    import numpy as np
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    c = dict(offsets=csr["offsets"], nbrs=csr["nbrs"], weights=None, node_order=csr["node_order"])
    L = args.walk_length
    nw = 20000
    t0 = time.perf_counter()
    _, lens, _ = oracle.walks_scale(c, args.p, args.q, args.seed, L, sample_walk0, nw, nthreads=cores)
    dt = time.perf_counter() - t0
    nw2 = int(min(3_000_000, max(nw, nw * args.cpu_seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    _, lens, _ = oracle.walks_scale(c, args.p, args.q, args.seed, L, sample_walk0, nw2, nthreads=cores)
    dt = time.perf_counter() - t0
    steps = int((lens.astype(np.int64) - 1).sum())
    return {"value": steps / dt, "unit": "walk-steps/s", "cores": cores, "kind": "port",
            "sample": f"{nw2} walks ({steps} walk-steps) of the same R-MAT-{args.scale} p={args.p} q={args.q} "
                      f"L={L} workload, oracle/oracle.c or_walks_scale, {dt:.1f} s",
            "reference_python_context": "reference node2vec.py measured 41,266 walk-steps/s/core on "
                                        "RMAT-12 in the build container (SURVEY §6); it cannot run at scale 20 "
                                        "(per-edge alias tables need 7.0e10 entries)"}


def topsim_cpu_baseline(tg, sample, step, args):
    """Oracle restatement of TopSim_singleSample (Java-literal queue, OpenMP
    over sources) on a bounded prefix of the same sources."""
    import oracle
    import numpy as np
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    n = tg.getVCount()
    ns = min(n, 256)
    t0 = time.perf_counter()
    _, st = oracle.topsim(tg._offs, tg._nbrs, 0, sample, step, C=0.6, seed=args.seed,
                          sources=np.arange(ns, dtype=np.int32), nthreads=cores)
    dt = time.perf_counter() - t0
    ns2 = int(min(n, max(ns, ns * args.cpu_seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    _, st = oracle.topsim(tg._offs, tg._nbrs, 0, sample, step, C=0.6, seed=args.seed,
                          sources=np.arange(ns2, dtype=np.int32), nthreads=cores)
    dt = time.perf_counter() - t0
    return {"value": st["pair_updates"] / dt, "unit": "pair-updates/s", "cores": cores, "kind": "port",
            "sample": f"sources 0..{ns2 - 1} ({st['pair_updates']} pair-updates), oracle/oracle.c or_topsim "
                      f"(TopSim_singleSample.java queue restated), {dt:.1f} s; the Java reference cannot run "
                      "here (no JDK)"}


def lib_digest():
    import hashlib
    from gwamd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_traffic(tag, launch_steps):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, only
    when it was measured on this exact library build and workload."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(tag)
        if e and e.get("walk_steps_per_launch") == launch_steps and e.get("lib_sha256") == lib_digest():
            return e
    except Exception:
        pass
    return None


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.secondary == "none" or (args.secondary == "auto" and world > 1):
        args.no_topsim = args.no_walk10m = args.no_simrank = args.no_rmat24 = True
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = local % max(1, torch.cuda.device_count())  # (ranks > GPUs only in rehearsals)
        torch.cuda.set_device(local)
        backend = os.environ.get("GW_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import gwamd
    from gwamd import _lib as C
    from gwamd import dist as gdist
    L = args.walk_length

    # ---- graph (host build, replicated on every rank) ----
    t0 = time.perf_counter()
    G = gwamd.GWGraph.rmat(args.scale, args.edge_factor, 0.57, 0.19, 0.19, args.seed)
    inf = G.info()
    n, nnz = inf.n, inf.nnz
    log(f"[rank {rank}] rmat-{args.scale}: n={n} nnz={nnz} maxdeg={inf.max_degree} "
        f"built in {time.perf_counter() - t0:.1f}s")
    G.to_device(dev.index)
    # sampler: per-edge 64 B entries + common-neighbour regions when they fit
    # in HBM (exact 3-way mixture, ~1.5 lines per step), else rejection sampling
    t0 = time.perf_counter()
    mode = "bitset" if args.mode in ("auto", "bitset") else "rejection"
    if mode == "bitset":
        try:
            C.check(C.lib().gw_n2v_prepare(G.handle, args.p, args.q, C.N2V_BITSET), G.handle)
        except C.CapacityError as e:
            if args.mode == "bitset":
                raise
            log(f"[rank {rank}] bitset tables do not fit ({e}); using rejection sampling")
            mode = "rejection"
    if mode == "rejection":
        C.check(C.lib().gw_n2v_prepare(G.handle, args.p, args.q, C.N2V_REJECTION), G.handle)
    torch.cuda.synchronize()
    prep_s = time.perf_counter() - t0
    sampler_gb = G.info().sampler_bytes / 1e9
    log(f"[rank {rank}] prepare ({mode}) {prep_s:.2f}s, sampler tables {sampler_gb:.2f} GB")

    B = args.num_walks * n                      # walks per rank per step
    out = torch.empty((B, L), dtype=torch.int32, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    gather = None
    if args.allgather and world > 1:
        gather = torch.empty((world * B, L), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = C.ctypes.c_void_p(stream.cuda_stream)

    def step(i, events=None):
        # global walk index block of (rank, step i): iterations
        # num_walks*(i*world+rank) ... +num_walks-1 of the reference loop
        w0 = gdist.weak_block(i, world, rank, B)
        if events is not None:
            events[0].record(stream)
        C.check(C.lib().gw_n2v_walks(G.handle, L, args.seed, w0, B, 1, C.ptr(out), None, C.ptr(cnt), sh),
                G.handle)
        if events is not None:
            events[1].record(stream)
        if gather is not None:
            dist.all_gather_into_tensor(gather, out)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    cnt.zero_()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    steps_local = int(cnt[0].item())
    trials_local = int(cnt[1].item())
    kms = [a.elapsed_time(b) for a, b in evs]
    k_avg_ms = sum(kms) / len(kms)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        s = torch.tensor([steps_local, trials_local], dtype=torch.int64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        steps_total, trials_total = int(s[0].item()), int(s[1].item())
    else:
        steps_total, trials_total = steps_local, trials_local
    value = steps_total / el
    launch_steps = steps_local // args.steps
    achieved = BYTES_PER_STEP * launch_steps / (k_avg_ms * 1e-3) / 1e9
    tag = f"n2v_rmat{args.scale}_p{args.p}_q{args.q}_L{L}_r{args.num_walks}_{mode}"
    prof = load_traffic(tag, launch_steps)
    traffic = prof["hbm_bytes_per_launch"] if prof else None
    # random-line roofline: the kernel's 64 B fabric read requests per second
    # against the calibrated random-gather rate (tools/calib: 4.8e10 lines/s)
    line_rate = None
    if prof and prof.get("fabric_read_requests_per_launch"):
        lr = prof["fabric_read_requests_per_launch"] / (k_avg_ms * 1e-3)
        line_rate = {"achieved_lines_per_s": lr, "calibrated_peak_lines_per_s": RANDOM_LINE_PEAK,
                     "frac": lr / RANDOM_LINE_PEAK,
                     "lines_per_step": prof["fabric_read_requests_per_launch"] / max(launch_steps, 1)}

    # ---- parity spot check (cheap): every step follows an edge ----
    if rank == 0 and not (os.environ.get("GW_DIAG_BS") or os.environ.get("GW_DIAG_NO_STORE")):  # (diag knobs: wrong walks)
        csr = G.export_csr()
        smp = out[:2000].cpu().numpy()
        offs, nbrs = csr["offsets"], csr["nbrs"]
        a, b = smp[:, :-1].ravel(), smp[:, 1:].ravel()
        pos = np.array([np.searchsorted(nbrs[offs[x]:offs[x + 1]], y) for x, y in zip(a, b)])
        ok = all(nbrs[offs[x] + p] == y for x, y, p in zip(a, b, pos))
        if not ok:
            log("PARITY SPOT CHECK FAILED: a step does not follow an edge")
            sys.exit(3)

    # ---- TopSim secondary metric (config 3: lshrank graphs) ----
    TOPSIM_GRAPHS = {"blog": ("blog.txt", 10313, ",", "lshrank blog, V=10313, 333,983 edges"),
                     "arxiv": ("arxiv_author_pub.txt", 38741, "\t", "lshrank arxiv, V=38741, 58,595 edges"),
                     "moreno": ("moreno_crime_crime.txt", 1380, "\t", "lshrank moreno, V=1380, 1,476 edges")}

    def run_topsim(name):
        from gwamd import topsim
        K = 20
        sample, step = args.topsim_sample, args.topsim_step
        if name == "p10m":
            # config 5: 10M-vertex Java-semantics R-MAT (reference quadrant
            # recursion), 1e8 generated lines, all non-isolated sources, top-100
            t0 = time.perf_counter()
            pg = gwamd.GWGraph.rmat_java(10_000_000, 100_000_000, 0.57, 0.19, 0.19, args.seed)
            deg = np.diff(pg.export_csr()["offsets"])
            log(f"[rank {rank}] p10m built in {time.perf_counter() - t0:.1f}s")
            pg.to_device(dev.index)
            h = pg.handle
            srcs = np.nonzero(deg > 0)[0].astype(np.int32)
            V = len(srcs)
            desc = f"10M vertices, 1e8 R-MAT lines, {V} non-isolated sources"
            K, sample, step = 100, 1000, 3
            src = torch.as_tensor(srcs, device=dev)
        else:
            fname, V, sep, desc = TOPSIM_GRAPHS[name]
            tg = topsim.Graph(os.path.join(ROOT, "tests", "golden", "data", fname), V, separator=sep,
                              device=dev.index)
            tg._ensure_device()
            h = tg._g.handle
            src = torch.arange(V, dtype=torch.int32, device=dev)
        ids = torch.empty((V, K), dtype=torch.int32, device=dev)
        sc = torch.empty((V, K), dtype=torch.float64, device=dev)
        st = torch.zeros(4, dtype=torch.int64, device=dev)

        def ts_run(stats_ptr):
            C.check(C.lib().gw_topsim(h, C.TOPSIM_SINGLE_SAMPLE, sample, step, 0.6,
                                      args.seed, C.ptr(src), V, K, C.ptr(ids), C.ptr(sc), stats_ptr, sh), h)

        ts_run(None)  # warm-up (also sizes the workspace)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        e0.record(stream)
        ts_run(C.ptr(st))
        e1.record(stream)
        torch.cuda.synchronize()
        tel = time.perf_counter() - t1
        kt = e0.elapsed_time(e1) * 1e-3
        if world > 1:
            t = torch.tensor([tel], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tel = float(t.item())
            dist.all_reduce(st, op=dist.ReduceOp.SUM)
        ext, upd = int(st[0].item()), int(st[1].item())
        alg = (TOPSIM_B_EXT * ext + TOPSIM_B_UPD * upd) / max(world, 1)
        cpu_ts = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline and name != "p10m":
            cpu_ts = topsim_cpu_baseline(tg, sample, step, args)
        return {
            "metric": "SimRank pair-updates/sec (TopSim_singleSample)", "value": upd / tel,
            "unit": "pair-updates/s", "path_extensions_per_s": ext / tel,
            "config": {"workload": f"TopSim_singleSample on {name} ({desc}, Java multigraph), "
                                   "all sources, replicated per rank",
                       "step": step, "sample": sample, "C": 0.6, "topk": K},
            "pair_updates": upd, "path_extensions": ext, "seconds": tel, "cpu_baseline": cpu_ts,
            "roofline": {"bound": "hbm", "achieved": alg / kt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / kt / 1e9 / HBM_PEAK_GBS, "traffic": None,
                         "kernel": f"k_topsim<{step},*>", "kernel_ms": kt * 1e3},
        }

    secondary = {}
    if not args.no_topsim:
        names = args.topsim_graphs.split(",")
        res = [run_topsim(nm) for nm in names]
        secondary["topsim"] = res[0]
        if len(res) > 1:
            secondary["topsim"]["more"] = res[1:]

    # ---- naive SimRank (SimRank.java) on the GPU: the TopSim ground truth ----
    def run_simrank(name):
        from gwamd import topsim
        fname, V, sep, desc = TOPSIM_GRAPHS[name]
        tg = topsim.Graph(os.path.join(ROOT, "tests", "golden", "data", fname), V, separator=sep,
                          device=dev.index)
        tg._ensure_device()
        h = tg._g.handle
        rounds = args.simrank_rounds
        S = torch.empty((V, V), dtype=torch.float64, device=dev)
        C.check(C.lib().gw_simrank_naive(h, 0.6, rounds, C.ptr(S), sh), h)  # warm-up, workspace
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        C.check(C.lib().gw_simrank_naive(h, 0.6, rounds, C.ptr(S), sh), h)
        e1.record(stream)
        torch.cuda.synchronize()
        sec = e0.elapsed_time(e1) * 1e-3
        deg = np.diff(tg._offs)
        nnz = int(deg.sum())
        m = int((deg > 0).sum())
        # entry gathers of the two passes (pass 1: m*nnz, pass 2: rows j > i only)
        tail = np.cumsum(deg[::-1])[::-1]  # entries of rows >= v
        p2 = int(tail[1:][deg[:-1] > 0].sum())
        gathers = rounds * (m * nnz + p2)
        lds_peak = 128.0 / 8 * 256 * 2.4e9  # 8 B gathers at 128 B/clk/CU
        java_pairs = (nnz * nnz - int((deg.astype(np.int64) ** 2).sum())) // 2
        cpu_sr = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            import oracle
            nth = min(16, os.cpu_count() or 1)
            budget, acc, re_ = 1.2e11, 0, 1
            suffix = nnz - np.cumsum(deg)
            while re_ < V and acc < budget:
                acc += int(deg[re_]) * int(suffix[re_])
                re_ += 1
            Sh = np.eye(V)
            t0 = time.perf_counter()
            _, pairs = oracle.simrank_round_rows(tg._offs, tg._nbrs, 0.6, Sh, 1, re_, nthreads=nth)
            dt = time.perf_counter() - t0
            cpu_sr = {"value": pairs / dt / java_pairs, "unit": "rounds/s", "cores": nth, "kind": "port",
                      "sample": f"rows 1..{re_ - 1} of one round ({pairs} neighbour pairs, {dt:.1f} s), "
                                f"oracle/oracle.c or_simrank_round_rows (SimRank.java loop order), "
                                f"scaled by the round's {java_pairs} pairs"}
        return {
            "metric": "naive SimRank rounds/sec (SimRank.java)", "value": rounds / sec, "unit": "rounds/s",
            "config": {"workload": f"SimRank(g).compute() on {name} ({desc}, Java multigraph)",
                       "rounds": rounds, "C": 0.6, "dense_result": f"{V}x{V} fp64"},
            "seconds": sec, "entry_gathers": gathers, "java_neighbour_pairs_per_round": java_pairs,
            "roofline": {"bound": "lds", "achieved": gathers / sec, "peak": lds_peak, "unit": "gathers/s",
                         "frac": gathers / sec / lds_peak, "traffic": None, "kernel": "k_sr_gather<true,*>"},
            "cpu_baseline": cpu_sr,
        }

    # ---- north_star: walks on a ~10M-node / ~100M-edge power-law graph ----
    def run_walk10m(BG, build_s, wp, wq, scale, ef, what="north_star 10M/100M graph", force_rejection=False):
        bi = BG.info()
        t0 = time.perf_counter()
        bmode = "bitset"
        try:
            if force_rejection:
                raise C.CapacityError(C.GW_ERR_CAPACITY, "rejection requested")
            C.check(C.lib().gw_n2v_prepare(BG.handle, wp, wq, C.N2V_BITSET), BG.handle)
        except C.CapacityError:
            bmode = "rejection"
            C.check(C.lib().gw_n2v_prepare(BG.handle, wp, wq, C.N2V_REJECTION), BG.handle)
        torch.cuda.synchronize()
        if wp == 1.0 and wq == 1.0:
            bmode = "first-order"  # k_walk_scale<true,...>: no per-edge tables
        bprep = time.perf_counter() - t0
        bsampler_gb = BG.info().sampler_bytes / 1e9
        nb = int(bi.n)
        bout = torch.empty((nb, L), dtype=torch.int32, device=dev)
        bcnt = torch.zeros(2, dtype=torch.int64, device=dev)

        def bstep(i):
            w0 = gdist.weak_block(i, world, rank, nb)
            C.check(C.lib().gw_n2v_walks(BG.handle, L, args.seed, w0, nb, 1, C.ptr(bout), None, C.ptr(bcnt), sh),
                    BG.handle)
        bstep(0)
        torch.cuda.synchronize()
        bcnt.zero_()
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        e0.record(stream)
        bstep(1)
        e1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        sec = time.perf_counter() - t1
        bsteps = int(bcnt[0].item())
        if world > 1:
            tt = torch.tensor([sec], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            sec = float(tt.item())
            ss = torch.tensor([bsteps], dtype=torch.int64, device=dev)
            dist.all_reduce(ss, op=dist.ReduceOp.SUM)
            bsteps = int(ss.item())
        kms = e0.elapsed_time(e1)
        cpu_b = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            import oracle
            csr_b = BG.export_csr()
            nth = min(16, os.cpu_count() or 1)
            # the CPU restatement of the rejection sampler (same walk distribution): the oracle's
            # bitset restatement rebuilds each bitset per step and is no fair CPU baseline
            fn = lambda c, *a, **k: oracle.walks_scale(dict(c, weights=None), *a, **k)  # noqa: E731
            nw = 2000
            t2 = time.perf_counter()
            fn(csr_b, wp, wq, args.seed, L, 0, nw, nthreads=nth)
            dt = time.perf_counter() - t2
            if dt < 5.0:  # grow the sample to ~10 s of CPU work (first-order walks are cheap: cap it)
                nw = int(nw * min(1000.0, 10.0 / max(dt, 1e-3)))
                t2 = time.perf_counter()
                fn(csr_b, wp, wq, args.seed, L, 0, nw, nthreads=nth)
                dt = time.perf_counter() - t2
            cpu_b = {"value": nw * (L - 1) / dt, "unit": "walk-steps/s", "cores": nth, "kind": "port",
                     "sample": f"{nw} walks of the same graph, p and q, oracle/oracle.c or_walks_scale "
                               f"(rejection sampler), {dt:.1f} s",
                     "reference_python_context": "the reference node2vec.py cannot build per-edge alias tables "
                                                 "for this graph (sum(deg^2) entries); SURVEY §6 measured "
                                                 "4.1e4-3.7e5 walk-steps/s/core on small graphs"}
        del bout
        return {"metric": f"walk-steps/sec (node2vec, {what})", "value": bsteps / sec,
                "unit": "walk-steps/s",
                "config": {"workload": f"node2vec p={wp} q={wq} on Graph500 R-MAT scale-{scale} "
                                       f"ef {ef} (n={bi.n}, adjacency entries={bi.nnz}), "
                                       f"walk_length={L}, 1 walk/node per rank",
                           "sampler": bmode},
                "kernel_ms": kms, "host_build_s": build_s, "prepare_s": bprep, "sampler_tables_gb": bsampler_gb,
                "cpu_baseline": cpu_b}

    if not args.no_walk10m:
        t0 = time.perf_counter()
        BG = gwamd.GWGraph.rmat(args.walk10m_scale, args.walk10m_edge_factor, 0.57, 0.19, 0.19, args.seed + 1)
        build_s = time.perf_counter() - t0
        BG.to_device(dev.index)
        # the bench's p/q, then p=q=1 (the north_star graph walked first-order)
        sc, ef = args.walk10m_scale, args.walk10m_edge_factor
        secondary["walk_10m"] = run_walk10m(BG, build_s, args.p, args.q, sc, ef)
        secondary["walk_10m_p1q1"] = run_walk10m(BG, build_s, 1.0, 1.0, sc, ef)
        BG.free()

    if not args.no_rmat24:
        # config 4 on one GPU: R-MAT-24 ef 16, p=1 q=0.5 (bitset tables would need ~390 GB:
        # rejection sampler with slot entries and per-row neighbour hash sets)
        t0 = time.perf_counter()
        BG = gwamd.GWGraph.rmat(24, 16, 0.57, 0.19, 0.19, args.seed)
        build_s = time.perf_counter() - t0
        BG.to_device(dev.index)
        secondary["walk_rmat24_p1q05"] = run_walk10m(BG, build_s, 1.0, 0.5, 24, 16, "config 4 R-MAT-24 ef 16",
                                                     force_rejection=True)
        BG.free()

    if not args.no_simrank:
        sr = run_simrank(args.simrank_graph)
        secondary["simrank_naive"] = sr

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(G.export_csr(), args, 0)

    if rank == 0:
        res = {
            "metric": "walk-steps/sec (node2vec)",
            "value": value,
            "unit": "walk-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32 ids / f64 accept tests",
            "data": "synthetic",
            "config": {"workload": f"node2vec p={args.p} q={args.q} on synthetic Graph500 R-MAT scale-{args.scale} "
                                   f"(ef {args.edge_factor}, a,b,c=0.57,0.19,0.19, seed {args.seed}; n={n}, "
                                   f"adjacency entries={nnz}), walk_length={L}, {args.num_walks} walks/node per "
                                   f"rank per step",
                       "walks_per_step": B * world, "walk_length": L, "parallelism": f"replicated graph, walks sharded over {world} rank(s)",
                       "allgather": bool(gather is not None)},
            "walk_steps": steps_total,
            "sampler": mode, "prepare_seconds": prep_s, "sampler_tables_gb": sampler_gb,
            "rejection_trials_per_step": trials_total / max(steps_total, 1),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_walk_bitset" if mode == "bitset" else "k_walk_scale<false,false,false>",
                         "kernel_ms": k_avg_ms,
                         "bytes_per_unit": BYTES_PER_STEP, "units_per_launch": launch_steps,
                         "lib_sha256": lib_digest(), "random_line_roofline": line_rate},
            "cpu_baseline": cpu,
            "secondary": secondary or None,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
