#!/usr/bin/env python3
"""bench.py — node2vec walk-steps/s on MI355X (+ TopSim pair-updates/s).

Headline (BASELINE.json configs[1], `--config 2`, the default): node2vec
p=0.25 q=4 on a synthetic Graph500 R-MAT scale-20 graph (a,b,c = 0.57,0.19,
0.19, edge factor 16, seed 42, symmetrised, deduplicated, no self loops),
walk_length 80, 10 walks per node.  One "step" = one pass of the hot path over
one batch: 10 walks from every vertex (6.47M walks, ~5.1e8 walk-steps) written
to HBM, per rank.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config {2,4,5}]

Ranks.  `--gpus N > 1` without WORLD_SIZE in the environment: bench.py starts
`python -m torch.distributed.run --nproc-per-node N` as a CHILD process (before
anything touches the GPU) and exits with its status; with WORLD_SIZE set (the
driver's own torch.distributed.run launch) it must equal N.  One rank per GPU,
backend "nccl" (= RCCL over xGMI); GW_DIST_BACKEND=gloo overrides it (CPU
rehearsals).  The graph is replicated; rank r walks the global walk-index block
(step*world + r)*B: walks are a pure function of (seed, global walk index), so
shards never overlap and need no collective ("scaling": "weak").  `value` =
walk-steps of all ranks / max-over-ranks time.  At world > 1 the RCCL
all-gather of the emitted walks (north_star) is timed as a second measurement
(`allgather` in the same JSON line: walk + all-gather per step), and rank 0
checks the gathered block of the last rank byte-for-byte against its own
recomputation of that block.

Configs (BASELINE.json):
  2  headline above; secondaries (1 GPU): TopSim on lshrank blog (config 3),
     the north_star 10M/100M graph at the bench's p/q and at p=q=1, config 4 and
     config 5 on one GPU, naive SimRank on blog.  At world > 1 the secondaries
     are configs 4 and 5, sharded.
  4  node2vec p=1 q=0.5 on R-MAT-24 ef 16 (rejection sampler), 1 walk/node per
     rank per step as the headline.
  5  TopSim_singleSample on the 10M-vertex power-law graph (top-100, STEP 3,
     SAMPLE 1000): all non-isolated sources split over the ranks (strong
     scaling); value = pair-updates/s.

Also in the JSON line:
  roofline      36 algorithmic bytes per walk-step / kernel time
                (HIP events on the launch stream); traffic = HBM bytes per launch
                from the committed rocprofv3 PMC summary of this exact library
                build (profiles/pmc_summary.json), or null; random_line_roofline
                = fabric read requests/s vs the calibrated random-block rate for
                the sampler tables' size (profiles/calib_r02.json).
  cpu_baseline  the oracle's C restatement of the same sampling (OpenMP), timed
                on a bounded sample of the same workload (rank 0, N=1).
`--plumbing-check` runs the launcher, rank and collective path with synthetic
rows and no GPU work (CPU gloo test of this file); it reports no throughput.
"""
import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
sys.path.insert(0, ROOT)

BYTES_PER_STEP = 36       # row bounds 16 + alias q/J 12 + nbr 4 + walk write 4
TOPSIM_B_EXT = 52         # per path-extension
TOPSIM_B_UPD = 24         # per pair-update
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
L2_PEAK_GBS = 34500.0     # MI355X_MICROARCH.md §L2: 32 MiB aggregate, ~34.5 TB/s
CALIB_FILE = os.path.join(ROOT, "profiles", "calib_r02.json")
GATHER_FULL_LIMIT = int(os.environ.get("GW_BENCH_GATHER_LIMIT", 48 << 30))  # gathered walks kept whole per rank; above: chunked ring


def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, choices=[2, 4, 5], default=2,
                    help="BASELINE.json config timed as the headline")
    ap.add_argument("--scale", type=int, default=None)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--rmat-params", choices=["graph500", "reference"], default="graph500",
                    help="R-MAT (a,b,c): Graph500 0.57/0.19/0.19 (SURVEY §8d) or the reference "
                         "generator's 0.45/0.15/0.15 (RMATGraphGenerator.java:179-182)")
    ap.add_argument("--p", type=float, default=None)
    ap.add_argument("--q", type=float, default=None)
    ap.add_argument("--walk-length", type=int, default=80)
    ap.add_argument("--num-walks", type=int, default=None,
                    help="walks per node per step: per rank (config 2, weak) or in total (config 4, strong)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--allgather", choices=["auto", "on", "off"], default="auto",
                    help="time the RCCL all-gather of the walks (auto: when ranks > 1)")
    ap.add_argument("--host-shard", choices=["auto", "on", "off"], default="auto",
                    help="time each rank writing its own shard to pinned host memory instead of exchanging "
                         "(SURVEY §8e's fallback; auto: when ranks > 1, and for the 1-GPU config-4 / config-5 lines)")
    ap.add_argument("--mode", choices=["auto", "bitset", "rejection"], default=None,
                    help="second-order sampler (auto: bitset when it fits in HBM)")
    ap.add_argument("--no-topsim", action="store_true")
    ap.add_argument("--no-simrank", action="store_true")
    ap.add_argument("--no-walk10m", action="store_true",
                    help="skip the north_star 10M-node/100M-edge walk measurement")
    ap.add_argument("--walk10m-scale", type=int, default=24)
    ap.add_argument("--walk10m-edge-factor", type=int, default=6)
    ap.add_argument("--simrank-graph", default="blog", help="naive SimRank graph (blog or moreno)")
    ap.add_argument("--simrank-rounds", type=int, default=3, help="SimRank.java STEP")
    ap.add_argument("--no-rmat24", action="store_true", help="skip config 4 as a secondary")
    ap.add_argument("--no-p10m", action="store_true", help="skip config 5 as a secondary")
    ap.add_argument("--no-p10m-stretch", action="store_true",
                    help="skip config 5's stretch (SAMPLE 10000, STEP 5) as a secondary")
    ap.add_argument("--stretch-stride", type=int, default=16,
                    help="the stretch runs every stride-th P10M source (1 = all 4.8M)")
    ap.add_argument("--no-arxiv", action="store_true",
                    help="skip the arxiv line (same graph as the reference CPU fixture)")
    ap.add_argument("--secondary", choices=["auto", "all", "none"], default="auto",
                    help="secondary workloads: auto = all at 1 GPU, configs 4 and 5 (sharded) at ranks > 1")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--topsim-sample", type=int, default=10000)
    ap.add_argument("--topsim-step", type=int, default=5)
    ap.add_argument("--topsim-graphs", default="blog", help="comma list of blog,arxiv,moreno")
    ap.add_argument("--no-config3", action="store_true",
                    help="skip the config-3 sweep (the reference driver's loop: blog, moreno, arxiv x SAMPLE)")
    ap.add_argument("--config3-graphs", default="blog,moreno,arxiv")
    ap.add_argument("--config3-samples", default="1000,2500,5000,10000,20000,40000",
                    help="Test_u_u_TopSim_singleSample.java:36 samples (STEP 5, top-20)")
    ap.add_argument("--config3-cpu-samples", default="1000,10000,40000",
                    help="sweep points that also time the CPU oracle")
    ap.add_argument("--config3-cpu-seconds", type=float, default=3.0)
    ap.add_argument("--p10m-vertices", type=int, default=10_000_000,
                    help="config 5 graph size (BASELINE: 10M vertices, 10 R-MAT lines per vertex); smaller for tests")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="ranks + collectives with synthetic rows, no GPU work, no throughput")
    a = ap.parse_args(argv)
    cfg = {2: dict(scale=20, p=0.25, q=4.0, num_walks=10, mode="auto"),
           4: dict(scale=24, p=1.0, q=0.5, num_walks=10, mode="rejection"),
           5: dict(scale=20, p=0.25, q=4.0, num_walks=10, mode="auto")}[a.config]
    for k, v in cfg.items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def rmat_abc(args):
    return (0.57, 0.19, 0.19) if args.rmat_params == "graph500" else (0.45, 0.15, 0.15)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv):
    """--gpus N > 1 outside torch.distributed.run: run it as a child (no exec,
    nothing has touched the GPU in this process) and return its exit status;
    rank 0's JSON line reaches our stdout through the inherited descriptor."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=env)


# ---- calibrations / committed profiles ---------------------------------------
def calib_rate(table_bytes, block=64):
    """Random-block read rate (blocks/s) measured by tools/calib/calib_sweep.hip
    (profiles/calib_r02.json: dependent reads, 5 waves/SIMD) for the table size
    nearest (log scale) to `table_bytes`."""
    import math
    with open(CALIB_FILE) as f:
        d = json.load(f)["dep_w5_blocks_per_s"][str(block)]
    mb = max(1.0, table_bytes / 2**20)
    key = min(d, key=lambda k: abs(math.log(float(k)) - math.log(mb)))
    return float(d[key]), int(key)


def lib_digest():
    import hashlib
    from gwamd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_prof(tag, units=None):
    """PMC summary entry (tools/pmc_summary.py) measured on this exact library
    build and workload size, else None."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            e = json.load(f).get(tag)
        if e and e.get("lib_sha256") == lib_digest() and (units is None or e.get("units_per_launch") == units):
            return e
    except Exception:
        pass
    return None


def grid_threads(count, block=256):
    return (count + block - 1) // block * block


def line_roofline(prof, kernel_s, table_bytes, block=64):
    """Fabric read requests per second of the profiled launch against the
    calibrated random-block rate for a table of that size (one request per
    random 32-128 B block, profiles/calib_r02.json)."""
    peak, table_mb = calib_rate(table_bytes, block)
    r = {"calibrated_peak_lines_per_s": peak, "calib_table_mb": table_mb, "calib_file": os.path.relpath(CALIB_FILE, ROOT)}
    if prof and prof.get("fabric_read_requests_per_launch"):
        lr = prof["fabric_read_requests_per_launch"] / kernel_s
        r.update({"achieved_lines_per_s": lr, "frac": lr / peak,
                  "lines_per_unit": prof["fabric_read_requests_per_launch"] / max(prof["units_per_launch"], 1)})
    return r


def cores_used():
    try:
        c = len(os.sched_getaffinity(0))
    except Exception:
        c = os.cpu_count() or 1
    return max(1, min(c, 16))


# ---- CPU baselines (oracle: rank 0, N=1 only) --------------------------------
def cpu_baseline_walks(csr, p, q, seed, L, walk0, seconds, max_walks=3_000_000):
    """Oracle (C restatement of the rejection sampler, OpenMP) on a bounded sample."""
    import numpy as np
    import oracle
    cores = cores_used()
    c = dict(offsets=csr["offsets"], nbrs=csr["nbrs"], weights=None, node_order=csr["node_order"])
    nw = 2000
    t0 = time.perf_counter()
    oracle.walks_scale(c, p, q, seed, L, walk0, nw, nthreads=cores)
    dt = time.perf_counter() - t0
    nw = int(min(max_walks, max(nw, nw * seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    _, lens, _ = oracle.walks_scale(c, p, q, seed, L, walk0, nw, nthreads=cores)
    dt = time.perf_counter() - t0
    steps = int((lens.astype(np.int64) - 1).sum())
    return {"value": steps / dt, "unit": "walk-steps/s", "cores": cores, "kind": "port",
            "sample": f"{nw} walks ({steps} walk-steps) of the same graph, p={p} q={q} L={L}, "
                      f"oracle/oracle.c or_walks_scale (rejection sampler, same walk law), {dt:.1f} s"}


def cpu_baseline_topsim(offs, nbrs, n, sample, step, seed, seconds, sources=None, topk=20):
    """Oracle restatement of TopSim_singleSample (Java-literal queue, OpenMP
    over sources) plus the per-source top-k the GPU line also produces
    (oracle.topsim_topk: one reused row per thread, no n-wide rows), on an
    evenly strided sample of the same sources (R-MAT puts its hubs at low ids,
    so a prefix would over-weight them)."""
    import numpy as np
    import oracle
    cores = cores_used()
    srcs = np.arange(n, dtype=np.int32) if sources is None else np.asarray(sources, np.int32)

    def strided(k):
        k = max(1, min(len(srcs), k))
        return srcs[np.linspace(0, len(srcs) - 1, k).astype(np.int64)]
    # grow the sample until it takes about `seconds` (the first calls also pay the
    # per-thread row allocation, so one extrapolation undershoots on large graphs)
    ns2 = min(len(srcs), 256)
    for _ in range(4):
        t0 = time.perf_counter()
        _, _, st = oracle.topsim_topk(offs, nbrs, 0, sample, step, topk, C=0.6, seed=seed, sources=strided(ns2),
                                      nthreads=cores)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * seconds or ns2 >= len(srcs):
            break
        ns2 = int(min(len(srcs), max(2 * ns2, ns2 * seconds / max(dt, 1e-3))))
    return {"value": st["pair_updates"] / dt, "unit": "pair-updates/s", "cores": cores, "kind": "port",
            "sample": f"{ns2} of the {len(srcs)} sources, evenly strided ({st['pair_updates']} pair-updates), "
                      f"oracle/oracle.c or_topsim_topk (TopSim_singleSample.java queue restated + top-{topk} per "
                      f"row), {dt:.1f} s; the Java reference cannot run here (no JDK)"}


def reference_cpu_fixture():
    """profiles/cpu_reference_node2vec.json: the reference node2vec.py walk
    loop timed in the build container (tools/ref_cpu_node2vec.py)."""
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_reference_node2vec.json")) as f:
            return json.load(f)
    except Exception:
        return None


# ---- ranks and collectives -----------------------------------------------------
class Ranks:
    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = None
        self.plumbing = args.plumbing_check
        import torch
        self.torch = torch
        if self.world > 1:
            import torch.distributed as dist
            self.dist = dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            self.backend = "gloo" if self.plumbing else os.environ.get("GW_DIST_BACKEND", "nccl")
        if self.plumbing:
            self.dev = torch.device("cpu")
            self.ngpu = 0
        else:
            ndev = torch.cuda.device_count()
            if ndev < 1:
                raise SystemExit("bench.py: no GPU visible (use --plumbing-check for the CPU rehearsal)")
            self.ngpu = min(self.world, ndev)
            torch.cuda.set_device(self.local % ndev)  # ranks > GPUs only in gloo rehearsals
            self.dev = torch.device("cuda", torch.cuda.current_device())
        if self.world > 1:
            if self.backend == "nccl":
                self.dist.init_process_group("nccl", device_id=self.dev)  # RCCL
            else:
                self.dist.init_process_group(self.backend)
            got = self.dist.get_world_size()
            if got != self.world:
                raise SystemExit(f"bench.py: process group has {got} ranks, WORLD_SIZE={self.world}")
        self.cdev = self.dev if self.backend == "nccl" else torch.device("cpu")

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def sync(self):
        if self.dev.type == "cuda":
            self.torch.cuda.synchronize()

    def allreduce(self, vals, op="sum", dtype=None):
        """Reduce a list of numbers over ranks (op: sum | max)."""
        if self.world == 1:
            return list(vals)
        torch = self.torch
        t = torch.tensor(list(vals), dtype=dtype or torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return t.tolist()

    def allgather_into(self, out, src):
        """out[world * rows] = every rank's src[rows] (rank order)."""
        if self.backend == "gloo" and src.device.type == "cuda":
            tmp = self.torch.empty(out.shape, dtype=out.dtype)
            self.dist.all_gather_into_tensor(tmp, src.cpu())
            out.copy_(tmp)
        else:
            self.dist.all_gather_into_tensor(out, src)

    def allgather_list(self, vals):
        """[rank][i] = every rank's list of int64 numbers."""
        if self.world == 1:
            return [list(vals)]
        torch = self.torch
        t = torch.tensor(list(vals), dtype=torch.int64, device=self.cdev)
        out = torch.empty((self.world, len(vals)), dtype=torch.int64, device=self.cdev)
        self.dist.all_gather_into_tensor(out, t) if self.backend == "nccl" else \
            self.dist.all_gather(list(out.unbind(0)), t)
        return out.tolist()

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def time_steps(R, step, steps, warmup, stream=None, events=True):
    """Warm-up, then K steps bracketed by barrier + synchronize on both sides;
    returns (max-over-ranks seconds, mean kernel ms from HIP events or None)."""
    torch = R.torch
    for i in range(warmup):
        step(i, None)
    R.sync()
    evs = None
    if events and R.dev.type == "cuda":
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    R.barrier()
    R.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i, evs[i] if evs else None)
    R.sync()
    R.barrier()
    el = time.perf_counter() - t0
    el = R.allreduce([el], "max")[0]
    kms = None
    if evs:
        kms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    return el, kms


def gather_timing(R, args, step, out, L, B, begin_of=None, count_of=None):
    """walk + RCCL all-gather of the emitted walks per step (north_star's
    exchange), timed like the headline; rank 0 then checks the last rank's
    gathered block against its own recomputation of that block.  `out` holds
    B rows per rank (strong shards: padded to the largest shard); rank r's
    block of step i starts at global walk begin_of(i, r) and has count_of(r)
    valid rows (default: weak blocks of B)."""
    torch = R.torch
    from gwamd import dist as gdist
    row_bytes = L * 4
    world = R.world
    if begin_of is None:
        begin_of = lambda i, r: gdist.weak_block(i, world, r, B)  # noqa: E731
    if count_of is None:
        count_of = lambda r: B  # noqa: E731
    full = world * B * row_bytes <= GATHER_FULL_LIMIT
    if full:
        rows_c = B
    else:  # chunked ring: 256 MB per rank per call into a reused buffer
        rows_c = max(1, min(B, (256 << 20) // row_bytes, GATHER_FULL_LIMIT // (world * row_bytes)))
    gbuf = torch.empty((world * rows_c, L), dtype=torch.int32, device=R.dev)

    def gstep(i, ev):
        step(i, ev)
        for r0 in range(0, B, rows_c):
            n = min(B, r0 + rows_c) - r0
            R.allgather_into(gbuf[:world * n], out[r0:r0 + n])  # rank-major [rank][n rows]
    el, _ = time_steps(R, gstep, args.steps, 0, events=False)
    # check: the last timed step's gathered block of rank world-1 (full mode) or
    # the last chunk (ring mode) equals what this rank computes for that block
    check = None
    last = args.steps - 1
    rl = world - 1
    if R.rank == 0:
        if full:
            lo, n = 0, B
        else:
            lo = ((B - 1) // rows_c) * rows_c
            n = B - lo
        got = gbuf[rl * n:(rl + 1) * n].clone()
        nv = max(0, min(n, count_of(rl) - lo))  # valid (non-padding) rows of that block
        mine = step.recompute(begin_of(last, rl) + lo, nv)
        check = bool(torch.equal(got[:nv].cpu(), mine.cpu()))
    ok = R.allreduce([1.0 if (check is None or check) else 0.0], "max")
    return {"seconds": el, "ms_per_step": el / args.steps * 1e3,
            "gathered_bytes_per_step_per_rank": (world - 1) * B * row_bytes,
            "mode": "whole" if full else f"ring of {rows_c}-row chunks",
            "check_last_rank_block_identical": check}, ok


HOST_PIN_LIMIT = 16 << 30  # a rank's host shard is pinned up to this size, else pageable


def host_buffer(R, shape, dtype):
    """Host memory for a rank's shard: pinned (page-locked, DMA target) up to
    HOST_PIN_LIMIT bytes, pageable above it and in CPU rehearsals."""
    torch = R.torch
    nbytes = dtype.itemsize if hasattr(dtype, "itemsize") else torch.empty((), dtype=dtype).element_size()
    for d in shape:
        nbytes *= d
    pin = R.dev.type == "cuda" and nbytes <= HOST_PIN_LIMIT
    return torch.empty(shape, dtype=dtype, pin_memory=pin), pin


def walk_host_shard_timing(R, args, steps, write, recompute, host, first, cnt, pinned, units):
    """SURVEY §8e's alternative to the all-gather: every rank writes its own
    walk shard straight to host memory (the reference's multi-worker split
    writes per-worker files, SingleRandomWalkApproxMultiThreads.java:59, 174)
    — no collective.  `write(i)` walks step i's shard into `host`
    (gw_n2v_walks_host: chunks walked on one stream while the previous chunk is
    copied out on another).  Timed like the headline (barrier + max over
    ranks); each rank then checks three row windows of its host shard of the
    last step against a device recomputation of the same walks."""
    torch = R.torch
    el, _ = time_steps(R, lambda i, ev: write(i), steps, 0, events=False)
    last = steps - 1
    ok = True
    for lo in sorted({0, max(0, cnt // 2 - 500), max(0, cnt - 1000)}):
        n = min(1000, cnt - lo)
        if n <= 0:
            continue
        mine = recompute(first(last) + lo, n).cpu()
        ok = ok and bool(torch.equal(host[lo:lo + n], mine))
    allok = R.allreduce([0.0 if ok else 1.0], "max")[0] == 0.0
    nbytes = cnt * host.shape[1] * 4
    return {"seconds": el, "ms_per_step": el / steps * 1e3, "value": units / el,
            "unit": "walk-steps/s (each rank's walks written to its host memory)",
            "bytes_per_step_per_rank": nbytes, "host_GBps_per_rank": nbytes * steps / el / 1e9,
            "host_memory": "pinned" if pinned else "pageable",
            "mode": "gw_n2v_walks_host: walk chunk k+1 while chunk k is copied D2H (no collective)",
            "check_host_rows_equal_device_rows": bool(allok)}


def topk_host_shard_timing(R, args, run, ids, sc, nloc, upd):
    """TopSim + each rank's own top-k rows copied to host memory (no
    exchange), beside the all-gather; also the copy alone."""
    torch = R.torch
    K = ids.shape[1]
    hid, pinned = host_buffer(R, (max(nloc, 1), K), torch.int32)
    hsc, _ = host_buffer(R, (max(nloc, 1), K), torch.float64)

    def copy():
        hid[:nloc].copy_(ids[:nloc], non_blocking=True)
        hsc[:nloc].copy_(sc[:nloc], non_blocking=True)

    def both(i, ev):
        run(None)
        copy()
    el, _ = time_steps(R, both, 1, 0, events=False)
    cel, _ = time_steps(R, lambda i, ev: copy(), 1, 0, events=False)
    ok = bool(torch.equal(hid[:nloc], ids[:nloc].cpu()) and torch.equal(hsc[:nloc], sc[:nloc].cpu()))
    allok = R.allreduce([0.0 if ok else 1.0], "max")[0] == 0.0
    nbytes = nloc * K * 12
    return {"seconds": el, "value": upd / el if upd else None,
            "unit": "pair-updates/s (each rank's top-k rows copied to its host memory)",
            "d2h_only_s": cel, "bytes_per_rank": nbytes, "host_GBps_per_rank": nbytes / max(cel, 1e-9) / 1e9,
            "host_memory": "pinned" if pinned else "pageable", "mode": "TopSim, then its rows D2H (no collective)",
            "check_host_rows_equal_device_rows": bool(allok)}


def checksum(t):
    """Position-weighted checksum of a tensor's bytes (int64, device-side)."""
    import torch
    v = t.contiguous().view(torch.int32).reshape(-1).to(torch.int64)
    w = torch.arange(v.numel(), dtype=torch.int64, device=v.device) % 65521 + 1
    return int((v * w).sum().item())


def gather_rows_timing(R, args, tensors, run=None):
    """All-gather of per-rank row blocks (same row count on every rank:
    strong shards padded), timed over args.steps, each step optionally
    preceded by `run()`; every rank's received blocks are checked against
    the senders' checksums (all-gathered beforehand)."""
    torch = R.torch
    world = R.world
    bufs = [torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=R.dev) for t in tensors]

    def gstep(i, ev):
        if run is not None:
            run()
        for t, g in zip(tensors, bufs):
            R.allgather_into(g, t)
    el, _ = time_steps(R, gstep, args.steps, 0, events=False)
    mine = [checksum(t) for t in tensors]
    sums = R.allgather_list(mine)  # [rank][tensor]
    ok = all(checksum(g[r * t.shape[0]:(r + 1) * t.shape[0]]) == sums[r][k]
             for k, (t, g) in enumerate(zip(tensors, bufs)) for r in range(world))
    allok = R.allreduce([0.0 if ok else 1.0], "max")[0] == 0.0
    nbytes = sum(t.numel() * t.element_size() for t in tensors)
    return {"seconds": el, "ms_per_step": el / args.steps * 1e3,
            "gathered_bytes_per_step_per_rank": (world - 1) * nbytes,
            "xgmi_GBps_per_rank": (world - 1) * nbytes * args.steps / el / 1e9,
            "check_blocks_match_sender_checksums": bool(allok)}


# ---- workloads -----------------------------------------------------------------
def stream_copy_gbps(R, nbytes=4 << 30, reps=5):
    """Achievable HBM bandwidth on this box: a device-to-device copy of
    `nbytes` (read + write counted), best of `reps` (SURVEY §8d asks for the
    streaming copy beside the 8 TB/s spec)."""
    torch = R.torch
    a = torch.empty(nbytes // 4, dtype=torch.int32, device=R.dev)
    b = torch.empty_like(a)
    a.fill_(1)
    best = 0.0
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        best = max(best, 2 * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del a, b
    return best


def walk_headline(R, args):
    """Headline node2vec measurement (configs 2 and 4)."""
    import numpy as np
    torch = R.torch
    from gwamd import dist as gdist
    L = args.walk_length
    world, rank = R.world, R.rank

    strong = args.config == 4  # BASELINE config 4: the r=10 workload split over the ranks

    def shape(n):
        """(rows per rank buffer, this rank's first walk of step i, valid rows per rank)."""
        if strong:
            total = args.num_walks * n
            b0, cnt = gdist.shard_range(total, world, rank)
            rows = -(-total // world)
            return rows, (lambda i: b0), cnt, total, \
                (lambda i, r: gdist.shard_range(total, world, r)[0]), (lambda r: gdist.shard_range(total, world, r)[1])
        B = args.num_walks * n
        return B, (lambda i: gdist.weak_block(i, world, rank, B)), B, B * world, None, None

    if R.plumbing:
        n = 1 << args.scale
        B, first, cnt_w, total, begin_of, count_of = shape(n)
        out = torch.full((B, L), -1, dtype=torch.int32)

        def synth(w0, cnt):  # NOT walks: row w = (w*L + t) mod 2^31, for the rank/collective plumbing only
            w = torch.arange(w0, w0 + cnt, dtype=torch.int64).unsqueeze(1)
            return ((w * L + torch.arange(L, dtype=torch.int64)) % (2**31 - 1)).to(torch.int32)
        def step(i, ev):
            out[:cnt_w].copy_(synth(first(i), cnt_w))
        step.recompute = synth
        el, _ = time_steps(R, step, args.steps, args.warmup, events=False)
        steps_total = int(R.allreduce([args.steps * cnt_w * (L - 1)], "sum", torch.int64)[0])
        res = {"value": None, "walk_steps": steps_total, "seconds": el, "n": n, "nnz": None, "mode": "plumbing",
               "B": B, "walks_per_step": total}
        if world > 1 and args.allgather != "off":
            g, ok = gather_timing(R, args, step, out, L, B, begin_of, count_of)
            res["allgather"] = g
            res["allgather_all_ranks_ok"] = bool(ok[0] >= 1.0)
        if args.host_shard == "on" or (args.host_shard == "auto" and world > 1):
            host, pinned = host_buffer(R, (cnt_w, L), torch.int32)

            def write(i):
                step(i, None)
                host.copy_(out[:cnt_w])
            res["host_shard"] = walk_host_shard_timing(R, args, args.steps, write, synth, host, first, cnt_w, pinned,
                                                       steps_total)
        return res

    import gwamd
    from gwamd import _lib as C
    a, b, c = rmat_abc(args)
    t0 = time.perf_counter()
    G = gwamd.GWGraph.rmat(args.scale, args.edge_factor, a, b, c, args.seed)
    inf = G.info()
    n, nnz = inf.n, inf.nnz
    log(f"[rank {rank}] rmat-{args.scale} ef {args.edge_factor}: n={n} nnz={nnz} maxdeg={inf.max_degree} "
        f"built in {time.perf_counter() - t0:.1f}s")
    G.to_device(R.dev.index)
    # the sampler tables are chosen for this rank's share of one BASELINE
    # workload pass (r walks from every vertex)
    G.options(expected_steps=shape(n)[2] * (L - 1))
    t0 = time.perf_counter()
    mode = "bitset" if args.mode in ("auto", "bitset") else "rejection"
    if args.p == 1.0 and args.q == 1.0:
        mode = "rejection"
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
    sampler_bytes = G.info().sampler_bytes
    if args.p == 1.0 and args.q == 1.0:
        mode = "first-order"
    log(f"[rank {rank}] prepare ({mode}) {prep_s:.2f}s, sampler tables {sampler_bytes / 1e9:.2f} GB")

    B, first, cnt_w, total, begin_of, count_of = shape(n)  # buffer rows per rank, shard start, valid rows
    out = torch.empty((B, L), dtype=torch.int32, device=R.dev)
    if cnt_w < B:
        out[cnt_w:].fill_(-1)  # padding row of a short strong shard (gathered, never walked)
    cnt = torch.zeros(2, dtype=torch.int64, device=R.dev)
    stream = torch.cuda.current_stream(R.dev)
    sh = C.ctypes.c_void_p(stream.cuda_stream)

    def launch(w0, count, dst, counters):
        C.check(C.lib().gw_n2v_walks(G.handle, L, args.seed, w0, count, 1, C.ptr(dst), None,
                                     C.ptr(counters) if counters is not None else None, sh), G.handle)

    def step(i, ev):
        # global walk-index block of (rank, step i): weak, iterations
        # num_walks*(i*world+rank) ...; strong, this rank's shard of the r=10 workload
        w0 = first(i)
        if ev is not None:
            ev[0].record(stream)
        launch(w0, cnt_w, out, cnt)
        if ev is not None:
            ev[1].record(stream)

    def recompute(w0, count):
        dst = torch.empty((count, L), dtype=torch.int32, device=R.dev)
        launch(w0, count, dst, None)
        torch.cuda.synchronize()
        return dst
    step.recompute = recompute

    for i in range(args.warmup):
        step(i, None)
    torch.cuda.synchronize()
    cnt.zero_()
    el, k_avg_ms = time_steps(R, step, args.steps, 0)
    steps_local, trials_local = int(cnt[0].item()), int(cnt[1].item())
    steps_total, trials_total = (int(x) for x in R.allreduce([steps_local, trials_local], "sum", torch.int64))
    value = steps_total / el
    launch_steps = steps_local // args.steps  # this rank's launch
    achieved = BYTES_PER_STEP * launch_steps / (k_avg_ms * 1e-3) / 1e9
    kname = walk_kernel_name(mode, G)
    tag = f"n2v_rmat{args.scale}_ef{args.edge_factor}_p{args.p}_q{args.q}_L{L}_r{args.num_walks}_{mode}"
    prof = load_prof(tag, launch_steps)
    traffic = prof["hbm_bytes_per_launch"] if prof else None
    table = sampler_bytes if mode == "bitset" else max(sampler_bytes, 16 * nnz)
    line_rate = line_roofline(prof, k_avg_ms * 1e-3, table)
    # structural ceiling of the 36 B/step metric: every step reads at least one
    # random block (one fabric request), so at the calibrated request rate
    line_rate["ceiling_frac_at_one_request_per_step"] = \
        BYTES_PER_STEP * line_rate["calibrated_peak_lines_per_s"] / (HBM_PEAK_GBS * 1e9)

    # ---- parity spot check (cheap): every step of a sample follows an edge ----
    if rank == 0:
        csr = G.export_csr()
        smp = out[:2000].cpu().numpy()
        offs, nbrs = csr["offsets"], csr["nbrs"]
        ok = True
        for row in smp:
            ln = int((row >= 0).sum())
            for x, y in zip(row[:ln - 1], row[1:ln]):
                s = nbrs[offs[x]:offs[x + 1]]
                k = np.searchsorted(s, y)
                if k >= len(s) or s[k] != y:
                    ok = False
        if not ok:
            log("PARITY SPOT CHECK FAILED: a step does not follow an edge")
            sys.exit(3)

    res = {"value": value, "walk_steps": steps_total, "seconds": el, "n": n, "nnz": nnz, "mode": mode,
           "B": B, "walks_per_step": total, "prep_s": prep_s, "sampler_gb": sampler_bytes / 1e9,
           "end_to_end": end_to_end(prep_s, el / args.steps, steps_total // args.steps, 1.0,
                                    "prepare + one step (the BASELINE workload: every vertex starts "
                                    f"{args.num_walks} walks of length {L})"),
           "trials_per_step": trials_total / max(steps_total, 1),
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "traffic_note": (prof or {}).get("note"),
                        "pmc_tag": tag, "pmc_match": {"kernel": kname, "grid": grid_threads(B)},
                        "kernel": kname, "kernel_ms": k_avg_ms,
                        "bytes_per_unit": BYTES_PER_STEP, "units_per_launch": launch_steps,
                        "lib_sha256": lib_digest(), "random_line_roofline": line_rate}}
    if world > 1 and args.allgather != "off":
        g, ok = gather_timing(R, args, step, out, L, B, begin_of, count_of)
        g["value"] = steps_total / g["seconds"]
        g["unit"] = "walk-steps/s (walks all-gathered to every rank)"
        g["xgmi_GBps_per_rank"] = g["gathered_bytes_per_step_per_rank"] * args.steps / g["seconds"] / 1e9
        res["allgather"] = g
        res["allgather_all_ranks_ok"] = bool(ok[0] >= 1.0)
    if args.host_shard == "on" or (args.host_shard == "auto" and world > 1):
        res["host_shard"] = walks_to_host(R, args, G, L, first, cnt_w, args.steps, recompute, steps_total)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_walks(G.export_csr(), args.p, args.q, args.seed, L, 0, args.cpu_seconds)
    if rank == 0:
        res["copy_gbps"] = stream_copy_gbps(R)
    if mode == "bitset" and world == 1:
        # the same BASELINE pass end to end with the plain rejection sampler
        # (16 B slot entries + neighbour hash, no per-edge tables): the
        # sampler a one-shot run should pick is the faster end to end
        G.options(listed=0)
        t0 = time.perf_counter()
        C.check(C.lib().gw_n2v_prepare(G.handle, args.p, args.q, C.N2V_REJECTION), G.handle)
        torch.cuda.synchronize()
        rprep = time.perf_counter() - t0
        launch(first(0), cnt_w, out, None)
        cnt.zero_()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch(first(0), cnt_w, out, cnt)
        e1.record(stream)
        torch.cuda.synchronize()
        rw = e0.elapsed_time(e1) * 1e-3
        alt = end_to_end(rprep, rw, launch_steps, 1.0, "prepare + one step, rejection sampler (mixture proposal "
                                                       "at q > 1, no per-edge tables)")
        alt["walk_steps_per_s"] = launch_steps / rw
        alt["trials_per_step"] = int(cnt[1].item()) / max(int(cnt[0].item()), 1)
        rname = walk_kernel_name("rejection", G)
        alt["roofline"] = walk_roofline(
            rname, f"n2v_rmat{args.scale}_ef{args.edge_factor}_p{args.p}_q{args.q}_L{L}_r{args.num_walks}_rejection",
            int(cnt[0].item()), rw, max(G.info().sampler_bytes, 16 * nnz), grid_threads(cnt_w))
        res["end_to_end_rejection"] = alt
        res["end_to_end_best"] = "bitset" if res["end_to_end"]["total_s"] <= alt["total_s"] else "rejection"
    del out
    G.free()
    return res


def walks_to_host(R, args, G, L, first, cnt, steps, recompute, units):
    """This rank's walks of `steps` steps written to host memory by
    gw_n2v_walks_host (see walk_host_shard_timing)."""
    torch = R.torch
    from gwamd import _lib as C
    host, pinned = host_buffer(R, (cnt, L), torch.int32)

    def write(i):
        C.check(C.lib().gw_n2v_walks_host(G.handle, L, args.seed, first(i), cnt, 1, C.ptr(host), None, None),
                G.handle)
    write(0)  # first touch of the host pages, device staging buffers
    return walk_host_shard_timing(R, args, steps, write, recompute, host, first, cnt, pinned, units)


def walk_roofline(kname, tag, steps, kernel_s, table_bytes, grid):
    """36 B per walk-step over one launch's event time, with the
    PMC traffic / fabric requests of this library build when
    profiles/pmc_summary.json holds an entry keyed to it (pmc_tag +
    lib_sha256 + steps per launch)."""
    prof = load_prof(tag, steps)
    achieved = BYTES_PER_STEP * steps / kernel_s / 1e9
    line = line_roofline(prof, kernel_s, table_bytes)
    line["ceiling_frac_at_one_request_per_step"] = \
        BYTES_PER_STEP * line["calibrated_peak_lines_per_s"] / (HBM_PEAK_GBS * 1e9)
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": prof["hbm_bytes_per_launch"] if prof else None,
            "traffic_note": (prof or {}).get("note"), "kernel": kname, "kernel_ms": kernel_s * 1e3,
            "bytes_per_unit": BYTES_PER_STEP, "units_per_launch": steps, "pmc_tag": tag,
            "pmc_match": {"kernel": kname, "grid": grid}, "lib_sha256": lib_digest(),
            "random_line_roofline": line}


def end_to_end(prep_s, launch_s, launch_steps, launches, what):
    """Prepare (preprocess_transition_probs' replacement) plus every walk of
    the BASELINE workload: `launches` launches of `launch_s` seconds
    (measured; scaled when the timed launch is a fraction of the workload)."""
    walk_s = launch_s * launches
    return {"prepare_s": prep_s, "walk_s": walk_s, "total_s": prep_s + walk_s,
            "walk_steps": int(launch_steps * launches), "value": launch_steps * launches / (prep_s + walk_s),
            "unit": "walk-steps/s", "prepare_share": prep_s / (prep_s + walk_s), "workload": what}


def walk_kernel_name(mode, G):
    """The kernel a prepared graph's walks launch: the bitset sampler, the
    listed rejection sampler (64 B slot entries, built for unweighted
    undirected graphs when they fit) or k_walk_scale (16 B entries)."""
    if mode == "bitset":
        return "k_walk_bitset"
    inf = G.info()
    if mode == "rejection" and inf.sampler_bytes >= 64 * inf.nnz:
        return "k_walk_listed"
    # the template's first argument tells first-order launches from second-order
    # ones of the same grid (a secondary also times the rejection sampler on its graph)
    return "k_walk_scale<true" if mode == "first-order" else "k_walk_scale<false"


def walk_secondary(R, args, BG, build_s, wp, wq, scale, ef, what, force_rejection=False, walks_per_node=1,
                   strong_walks=None, baseline_r=10):
    """One launch on graph BG: `walks_per_node` walks per node per rank (weak),
    or, with strong_walks = r, the fixed workload of r walks per node split
    over the ranks (BASELINE config 4: strong scaling) followed at ranks > 1 by
    the timed RCCL all-gather of every walk into every rank.  end_to_end =
    prepare + all walks of the BASELINE workload (r = baseline_r walks per
    node; a 1-walk launch is scaled by r)."""
    torch = R.torch
    import gwamd  # noqa: F401
    from gwamd import _lib as C
    from gwamd import dist as gdist
    L = args.walk_length
    world, rank = R.world, R.rank
    bi = BG.info()
    t0 = time.perf_counter()
    bmode = "bitset"
    try:
        if force_rejection or (wp == 1.0 and wq == 1.0):
            raise C.CapacityError(C.GW_ERR_CAPACITY, "rejection requested")
        C.check(C.lib().gw_n2v_prepare(BG.handle, wp, wq, C.N2V_BITSET), BG.handle)
    except C.CapacityError:
        bmode = "rejection"
        C.check(C.lib().gw_n2v_prepare(BG.handle, wp, wq, C.N2V_REJECTION), BG.handle)
    torch.cuda.synchronize()
    if wp == 1.0 and wq == 1.0:
        bmode = "first-order"  # k_walk_scale<true,...>: no per-edge tables
    bprep = time.perf_counter() - t0
    if strong_walks:
        total = int(bi.n) * strong_walks
        b0, nb = gdist.shard_range(total, world, rank)
        rows = -(-total // world)
        first = lambda i: b0  # noqa: E731
        begin_of = lambda i, r: gdist.shard_range(total, world, r)[0]  # noqa: E731
        count_of = lambda r: gdist.shard_range(total, world, r)[1]  # noqa: E731
    else:
        nb = rows = int(bi.n) * walks_per_node
        total = nb * world
        first = lambda i: gdist.weak_block(i, world, rank, nb)  # noqa: E731
        begin_of = count_of = None
    bout = torch.empty((rows, L), dtype=torch.int32, device=R.dev)
    if nb < rows:
        bout[nb:].fill_(-1)
    bcnt = torch.zeros(2, dtype=torch.int64, device=R.dev)
    stream = torch.cuda.current_stream(R.dev)
    sh = C.ctypes.c_void_p(stream.cuda_stream)

    def launch(w0, count, dst, counters):
        C.check(C.lib().gw_n2v_walks(BG.handle, L, args.seed, w0, count, 1, C.ptr(dst), None,
                                     C.ptr(counters) if counters is not None else None, sh), BG.handle)

    def bstep(i, ev):
        if ev is not None:
            ev[0].record(stream)
        launch(first(i), nb, bout, bcnt)
        if ev is not None:
            ev[1].record(stream)

    def recompute(w0, count):
        dst = torch.empty((count, L), dtype=torch.int32, device=R.dev)
        launch(w0, count, dst, None)
        torch.cuda.synchronize()
        return dst
    bstep.recompute = recompute

    bstep(0, None)
    torch.cuda.synchronize()
    bcnt.zero_()
    sec, kms = time_steps(R, lambda i, ev: bstep(1 + i, ev), 1, 0)
    bsteps = int(R.allreduce([int(bcnt[0].item())], "sum", torch.int64)[0])
    local_steps = int(bcnt[0].item())
    gather = None
    if world > 1 and strong_walks and args.allgather != "off":
        ga = argparse.Namespace(**vars(args))
        ga.steps = 1
        g, ok = gather_timing(R, ga, lambda i, ev: bstep(1 + i, ev), bout, L, rows,
                              lambda i, r: begin_of(i, r), count_of)
        g["value"] = bsteps / g["seconds"]
        g["unit"] = "walk-steps/s (walks all-gathered to every rank)"
        g["xgmi_GBps_per_rank"] = g["gathered_bytes_per_step_per_rank"] / g["seconds"] / 1e9
        g["all_ranks_ok"] = bool(ok[0] >= 1.0)
        gather = g
    host = None
    if strong_walks and (args.host_shard == "on" or (args.host_shard == "auto")):
        host = walks_to_host(R, args, BG, L, lambda i: first(1 + i), nb, 1, recompute, bsteps)
    cpu_b = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_b = cpu_baseline_walks(BG.export_csr(), wp, wq, args.seed, L, 0, 10.0, max_walks=2_000_000)
    del bout
    kname = walk_kernel_name(bmode, BG)
    rtag = strong_walks if strong_walks else walks_per_node
    tag = f"n2v_rmat{scale}_ef{ef}_p{wp}_q{wq}_L{L}_r{rtag}_{bmode}" + (f"_of{world}" if strong_walks and world > 1
                                                                         else "")
    prof = load_prof(tag, local_steps)
    sbytes = BG.info().sampler_bytes
    line = line_roofline(prof, kms * 1e-3, sbytes if bmode == "bitset" else max(sbytes, 16 * bi.nnz))
    r_run = strong_walks if strong_walks else walks_per_node * world
    e2e = end_to_end(bprep, sec, bsteps, baseline_r / r_run,
                     f"prepare + {baseline_r} walks from every vertex (BASELINE workload)" +
                     ("" if r_run == baseline_r else f"; the timed launch ran {r_run}, scaled"))
    e2e_rej = e2e_best = None
    if bmode == "bitset" and world == 1:
        # the same BASELINE pass end to end with the rejection sampler (mixture
        # proposal at q > 1; milliseconds to prepare): a one-shot caller's pick
        sbytes_b = BG.info().sampler_bytes
        BG.options(listed=0)
        t0 = time.perf_counter()
        C.check(C.lib().gw_n2v_prepare(BG.handle, wp, wq, C.N2V_REJECTION), BG.handle)
        torch.cuda.synchronize()
        rprep = time.perf_counter() - t0
        rout = torch.empty((nb, L), dtype=torch.int32, device=R.dev)
        rcnt = torch.zeros(2, dtype=torch.int64, device=R.dev)
        launch(first(1), nb, rout, None)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch(first(1), nb, rout, rcnt)
        e1.record(stream)
        torch.cuda.synchronize()
        rw = e0.elapsed_time(e1) * 1e-3
        rsteps = int(rcnt[0].item())
        e2e_rej = end_to_end(rprep, rw, rsteps, baseline_r / r_run,
                             f"prepare + {baseline_r} walks from every vertex, rejection sampler")
        e2e_rej["walk_steps_per_s"] = rsteps / rw
        e2e_rej["trials_per_step"] = int(rcnt[1].item()) / max(rsteps, 1)
        rname = walk_kernel_name("rejection", BG)
        e2e_rej["roofline"] = walk_roofline(
            rname, f"n2v_rmat{scale}_ef{ef}_p{wp}_q{wq}_L{L}_r{walks_per_node}_rejection", rsteps, rw,
            max(BG.info().sampler_bytes, 16 * bi.nnz), grid_threads(nb))
        e2e_best = "bitset" if e2e["total_s"] <= e2e_rej["total_s"] else "rejection"
        del rout
        BG.options(listed=-1)
        sbytes = sbytes_b
    return {"metric": f"walk-steps/sec (node2vec, {what})", "value": bsteps / sec, "unit": "walk-steps/s",
            "n_ranks": world, "scaling": "strong" if strong_walks else "weak",
            "config": {"workload": f"node2vec p={wp} q={wq} on Graph500 R-MAT scale-{scale} ef {ef} "
                                   f"(n={bi.n}, adjacency entries={bi.nnz}), walk_length={L}, " +
                                   (f"{strong_walks} walks/node in total split over {world} rank(s)" if strong_walks
                                    else f"{walks_per_node} walk(s)/node per rank"),
                       "sampler": bmode, "walks": total},
            "kernel_ms": kms, "walk_steps": bsteps,
            "roofline": {"bound": "hbm", "achieved": BYTES_PER_STEP * local_steps / (kms * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": BYTES_PER_STEP * local_steps / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "traffic": prof["hbm_bytes_per_launch"] if prof else None, "kernel": kname,
                         "units_per_launch": local_steps, "pmc_tag": tag,
                         "pmc_match": {"kernel": kname, "grid": grid_threads(nb)},
                         "random_line_roofline": line},
            "host_build_s": build_s, "prepare_s": bprep, "sampler_tables_gb": sbytes / 1e9,
            "end_to_end": e2e, "end_to_end_rejection": e2e_rej, "end_to_end_best": e2e_best,
            "allgather": gather, "host_shard": host, "cpu_baseline": cpu_b}


TOPSIM_GRAPHS = {"blog": ("blog.txt", 10313, ",", "lshrank blog, V=10313, 333,983 edges"),
                 "arxiv": ("arxiv_author_pub.txt", 38741, "\t", "lshrank arxiv, V=38741, 58,595 edges"),
                 "moreno": ("moreno_crime_crime.txt", 1380, "\t", "lshrank moreno, V=1380, 1,476 edges")}


_TS_DISPATCH = {}  # kernel name -> gw_topsim* dispatches of it so far in this process


def ts_dispatch(h, call):
    """Run one gw_topsim* call; return (the kernel it dispatched, the ordinal
    of that dispatch among this process's dispatches of the same kernel).  The
    PMC passes run the same bench command, so tools/pmc_summary.py picks the
    timed dispatch of a line by that ordinal (lines that share a kernel — the
    config-3 sweep — are told apart by it, not by name or grid)."""
    from gwamd import _lib as C
    call()
    name = C.lib().gw_topsim_kernel(h).decode()
    k = _TS_DISPATCH.get(name, 0)
    _TS_DISPATCH[name] = k + 1
    return name, k


def ts_kernel_attrs(h):
    """VGPRs and scratch per lane, LDS per workgroup of the handle's TopSim kernel."""
    from gwamd import _lib as C
    v, sc, lds = C.ctypes.c_int32(), C.ctypes.c_int32(), C.ctypes.c_int32()
    C.check(C.lib().gw_topsim_kernel_attrs(h, C.ctypes.byref(v), C.ctypes.byref(sc), C.ctypes.byref(lds)), h)
    return {"vgprs": v.value, "scratch_bytes_per_lane": sc.value, "lds_bytes_per_workgroup": lds.value}


def topsim_roofline(ext, upd, kt, tag, nsrc, nnz, step, n=None, kernel=None, nth=None):
    """52 B per path extension + 24 B per pair-update / kernel time.
    The denominator follows where the data lives: the slot table (16 B per
    adjacency entry) and the level records of lshrank graphs stay in the 256 MB
    Infinity Cache (MI355X_MICROARCH.md §Infinity Cache), so their bound is the
    calibrated random-block rate of a cache-resident table x 128 B, not 8 TB/s;
    P10M's 3.2 GB slot table is HBM.  traffic = HBM-side bytes from the PMC
    passes of this library build (2 x FETCH_SIZE + WRITE_SIZE, as
    tools/pmc_summary.py documents), or null."""
    alg = TOPSIM_B_EXT * ext + TOPSIM_B_UPD * upd
    prof = load_prof(tag, nsrc)
    achieved = alg / kt / 1e9
    table = 16 * nnz
    rate, table_mb = calib_rate(table, 128)
    if table <= 200 << 20:
        bound, peak = "infinity-cache (random 128 B blocks)", rate * 128 / 1e9
    else:
        bound, peak = "hbm", HBM_PEAK_GBS
    return {"bound": bound, "achieved": achieved, "peak": peak, "unit": "GB/s", "frac": achieved / peak,
            "traffic": prof["hbm_bytes_per_launch"] if prof else None,
            "traffic_GBps": prof["hbm_bytes_per_launch"] / kt / 1e9 if prof else None,
            "algorithmic_bytes": alg, "slot_table_bytes": table, "kernel": kernel or "k_topsim",
            "kernel_ms": kt * 1e3, "units_per_launch": nsrc, "pmc_tag": tag,
            # the timed dispatch: the exact kernel and its ordinal among this process's dispatches of it
            "pmc_match": ({"kernel": "^" + re.escape(kernel) + "$", "grid": None, "nth": [nth]} if kernel else
                          {"kernel": (f"k_topsim(_pipe_row)?<{step}[,>]" if n is not None and n * 8 <= 96 * 1024
                                      else f"k_topsim(_2wg|_pipe)<{step}[,>]"), "grid": None}),
            "scratch_bytes_per_lane": prof.get("scratch_bytes") if prof else None,
            "random_line_roofline": line_roofline(prof, kt, table, 128)}


_P10M_GRAPH = {}  # the P10M graph built once per run (config 5 and its SAMPLE 10000 / STEP 5 stretch)


def p10m_graph(R, args):
    import numpy as np
    import gwamd
    key = (args.p10m_vertices, args.seed, args.rmat_params)
    if key not in _P10M_GRAPH:
        t0 = time.perf_counter()
        a, b, c = rmat_abc(args)
        pg = gwamd.GWGraph.rmat_java(args.p10m_vertices, 10 * args.p10m_vertices, a, b, c, args.seed)
        csr = pg.export_csr()
        log(f"[rank {R.rank}] p10m built in {time.perf_counter() - t0:.1f}s")
        pg.to_device(R.dev.index)
        _P10M_GRAPH.clear()
        _P10M_GRAPH[key] = (pg, csr["offsets"], csr["nbrs"], np.diff(csr["offsets"]))
    return _P10M_GRAPH[key]


def run_topsim(R, args, name, sample=None, step=None, stride=1, cpu_seconds=None, cpu=True):
    """TopSim_singleSample: lshrank graphs (config 3; every rank all sources;
    default SAMPLE / STEP from --topsim-sample / --topsim-step) or P10M
    (config 5 at SAMPLE 1000 / STEP 3, or the SURVEY §8d stretch SAMPLE 10000
    / STEP 5; sources split over ranks, strong scaling).  At ranks > 1 the P10M
    rows are all-gathered (RCCL) and, beside it, every rank's own rows are
    copied to pinned host memory (SURVEY §8e's per-rank output, the reference's
    per-worker files: SingleRandomWalkApproxMultiThreads.java:59, 174)."""
    import numpy as np
    torch = R.torch
    import gwamd
    from gwamd import _lib as C
    from gwamd import dist as gdist
    from gwamd import topsim
    world, rank = R.world, R.rank
    K = 20
    if name != "p10m":
        sample, step = sample or args.topsim_sample, step or args.topsim_step
    offs = nbrs = None
    if R.plumbing:  # config 5's rank / collective path with synthetic rows (no GPU)
        K, nsrc_all = 100, 1 << args.scale
        srcs = np.arange(nsrc_all, dtype=np.int32)[rank::world]
        rows = -(-nsrc_all // world)
        ids = torch.full((rows, K), -1, dtype=torch.int32)
        sc = torch.zeros((rows, K), dtype=torch.float64)

        def synth():
            s_ = torch.as_tensor(srcs, dtype=torch.int64).unsqueeze(1)
            ids[:len(srcs)] = ((s_ * K + torch.arange(K)) % nsrc_all).to(torch.int32)
            sc[:len(srcs)] = s_.to(torch.float64) + torch.arange(K, dtype=torch.float64) / K
        synth()
        g = gather_rows_timing(R, args, [ids, sc], run=synth) if world > 1 else None
        host = None
        if args.host_shard == "on" or (args.host_shard == "auto" and world > 1):
            host = topk_host_shard_timing(R, args, lambda _: synth(), ids, sc, len(srcs), 0)
        return {"metric": "SimRank pair-updates/sec (TopSim_singleSample)", "value": None, "unit": "pair-updates/s",
                "n_ranks": world, "scaling": "strong", "seconds": g["seconds"] if g else 0.0,
                "config": {"workload": f"plumbing: {nsrc_all} synthetic top-{K} rows split round-robin",
                           "topk": K}, "pair_updates": 0, "cpu_baseline": None, "roofline": None, "allgather": g,
                "host_shard": host}
    if name == "p10m":
        # config 5: 10M-vertex Java-semantics R-MAT (reference quadrant recursion),
        # 1e8 generated lines, all non-isolated sources, top-100
        pg, offs, nbrs, deg = p10m_graph(R, args)
        h = pg.handle
        srcs_all = np.nonzero(deg > 0)[0].astype(np.int32)
        # round-robin split: R-MAT puts the hubs (the expensive sources) at low
        # ids, so contiguous ranges would load rank 0 with most of the work;
        # rows are keyed by source, so any split gives the same rows
        if stride > 1:  # every stride-th source (the stretch is ~18x config 5's work per source)
            srcs_all = srcs_all[::stride].copy()
        srcs = srcs_all[rank::world]
        desc = (f"{args.p10m_vertices} vertices, {10 * args.p10m_vertices} R-MAT lines, {len(srcs_all)} non-isolated "
                f"sources" + (f" (every {stride}th)" if stride > 1 else "") + f" split round-robin over {world} rank(s)")
        K, sample, step = 100, sample or 1000, step or 3
        scaling = "strong"
        keep = pg
    else:
        fname, V, sep, desc = TOPSIM_GRAPHS[name]
        tg = topsim.Graph(os.path.join(ROOT, "tests", "golden", "data", fname), V, separator=sep,
                          device=R.dev.index)
        tg._ensure_device()
        h = tg._g.handle
        offs, nbrs = tg._offs, tg._nbrs
        srcs = np.arange(V, dtype=np.int32)
        scaling = "weak"
        keep = tg
    nloc = len(srcs)
    src = torch.as_tensor(srcs, device=R.dev)
    ids = torch.empty((max(nloc, 1), K), dtype=torch.int32, device=R.dev)
    sc = torch.empty((max(nloc, 1), K), dtype=torch.float64, device=R.dev)
    st = torch.zeros(4, dtype=torch.int64, device=R.dev)
    stream = torch.cuda.current_stream(R.dev)
    sh = C.ctypes.c_void_p(stream.cuda_stream)

    last = {}

    def ts_run(stats_ptr):
        if nloc == 0:
            return
        last["kernel"], last["nth"] = ts_dispatch(h, lambda: C.check(
            C.lib().gw_topsim(h, C.TOPSIM_SINGLE_SAMPLE, sample, step, 0.6, args.seed, C.ptr(src), nloc, K,
                              C.ptr(ids), C.ptr(sc), stats_ptr, sh), h))

    ts_run(None)  # warm-up (also sizes the workspace)
    torch.cuda.synchronize()

    def tstep(i, ev):
        if ev is not None:
            ev[0].record(stream)
        ts_run(C.ptr(st))
        if ev is not None:
            ev[1].record(stream)
    tel, kms = time_steps(R, tstep, 1, 0)
    timed = dict(last)
    kattrs = ts_kernel_attrs(h) if nloc else None
    ext_l, upd_l = int(st[0].item()), int(st[1].item())
    ext, upd = (int(x) for x in R.allreduce([ext_l, upd_l], "sum", torch.int64))
    gather = None
    if name == "p10m" and world > 1 and args.allgather != "off":
        # every rank receives all top-k rows (k x (int32 + fp64)
        # per source; round-robin shards padded to the longest)
        rows = -(-len(srcs_all) // world)
        gid = torch.full((rows, K), -1, dtype=torch.int32, device=R.dev)
        gsc = torch.zeros((rows, K), dtype=torch.float64, device=R.dev)
        gid[:nloc].copy_(ids[:nloc])
        gsc[:nloc].copy_(sc[:nloc])
        ga = argparse.Namespace(**vars(args))
        ga.steps = 1
        gonly = gather_rows_timing(R, ga, [gid, gsc])

        def both():
            ts_run(None)
            gid[:nloc].copy_(ids[:nloc])
            gsc[:nloc].copy_(sc[:nloc])
        gboth = gather_rows_timing(R, ga, [gid, gsc], run=both)
        gather = dict(gboth, allgather_only_s=gonly["seconds"], rows_per_rank=rows,
                      value=upd / gboth["seconds"], unit="pair-updates/s (top-k rows all-gathered to every rank)",
                      check_blocks_match_sender_checksums=gonly["check_blocks_match_sender_checksums"] and
                      gboth["check_blocks_match_sender_checksums"])
    host = None
    if name == "p10m" and stride == 1 and args.host_shard != "off":
        host = topk_host_shard_timing(R, args, ts_run, ids, sc, nloc, upd)
    tag = f"topsim_{name}_s{sample}_t{step}_k{K}" + (f"_stride{stride}" if stride > 1 else "")
    cpu_ts = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu:
        cpu_ts = cpu_baseline_topsim(offs, nbrs, len(offs) - 1, sample, step, args.seed,
                                     cpu_seconds or (args.cpu_seconds if name != "p10m" else 15.0), sources=srcs,
                                     topk=K)
    if name == "p10m":
        desc += f", SAMPLE {sample}, STEP {step}" + (" (SURVEY §8d stretch)" if (sample, step) != (1000, 3) else "")
    del keep
    return {
        "metric": "SimRank pair-updates/sec (TopSim_singleSample)", "value": upd / tel,
        "unit": "pair-updates/s", "path_extensions_per_s": ext / tel, "n_ranks": world, "scaling": scaling,
        "config": {"workload": f"TopSim_singleSample on {name} ({desc}, Java multigraph)",
                   "step": step, "sample": sample, "C": 0.6, "topk": K},
        "pair_updates": upd, "path_extensions": ext, "seconds": tel, "cpu_baseline": cpu_ts, "allgather": gather,
        "host_shard": host, "kernel": timed.get("kernel"), "kernel_attrs": kattrs,
        "roofline": topsim_roofline(ext_l, upd_l, kms * 1e-3, tag, nloc, int(offs[-1]), step, len(offs) - 1,
                                    timed.get("kernel"), timed.get("nth")),
    }


def run_config3_sweep(R, args):
    """BASELINE config 3 as the reference driver runs it
    (Test_u_u_TopSim_singleSample.java:28-42, MyConfiguration.java:27-32):
    TopSim_singleSample on lshrank blog, moreno and arxiv (the driver's files
    0-2; file 3, power_biGraph_10000_5, is not in the reference) at STEP 5 for
    every SAMPLE of its loop, all sources, top-20 rows (testTopK = {20}).
    Each point: the kernel dispatched and its registers / scratch, the roofline
    with the keyed PMC traffic of that dispatch, and (at --config3-cpu-samples)
    the CPU oracle on a bounded strided sample."""
    cpu_at = {int(x) for x in args.config3_cpu_samples.split(",") if x}
    pts = []
    for name in args.config3_graphs.split(","):
        for sample in (int(x) for x in args.config3_samples.split(",")):
            pts.append(run_topsim(R, args, name, sample, 5, cpu_seconds=args.config3_cpu_seconds,
                                  cpu=sample in cpu_at))
            p = pts[-1]
            log(f"[config 3] {name} SAMPLE {sample}: {p['value']:.3e} pair-updates/s, {p['seconds'] * 1e3:.2f} ms, "
                f"{p['kernel']} {p['kernel_attrs']}")
    return {"metric": "SimRank pair-updates/sec (TopSim_singleSample, the reference driver's sweep)",
            "unit": "pair-updates/s",
            "config": {"workload": "Test_u_u_TopSim_singleSample loop: lshrank blog / moreno / arxiv, STEP 5, "
                                   f"SAMPLE in {args.config3_samples}, every source, top-20"},
            "points": [{"graph": p["config"]["workload"].split(" ")[2], "sample": p["config"]["sample"], **p}
                       for p in pts]}


LDS_CALIB_FILE = os.path.join(ROOT, "profiles", "r03", "calib_lds.jsonl")


def lds_gather_calib(achieved):
    """The measured ceiling of the gather loop itself (tools/calib/calib_lds.hip:
    one 1024-thread workgroup per CU, fp64 row in LDS, 4 B offsets streamed 16
    per lane, random 8 B gathers summed): random-address LDS gathers conflict,
    so 128 B/clk/CU is not reachable by this access."""
    try:
        rows = [json.loads(ln) for ln in open(LDS_CALIB_FILE) if ln.startswith("{")]
        peak = max(r["gathers_per_s"] for r in rows)
    except Exception:
        return None
    return {"calibrated_peak_gathers_per_s": peak, "frac": achieved / peak,
            "calib_file": os.path.relpath(LDS_CALIB_FILE, ROOT)}


def run_simrank(R, args, name):
    """naive SimRank (SimRank.java) on the GPU: the TopSim ground truth."""
    import numpy as np
    torch = R.torch
    from gwamd import _lib as C
    from gwamd import topsim
    fname, V, sep, desc = TOPSIM_GRAPHS[name]
    tg = topsim.Graph(os.path.join(ROOT, "tests", "golden", "data", fname), V, separator=sep, device=R.dev.index)
    tg._ensure_device()
    h = tg._g.handle
    rounds = args.simrank_rounds
    S = torch.empty((V, V), dtype=torch.float64, device=R.dev)
    stream = torch.cuda.current_stream(R.dev)
    sh = C.ctypes.c_void_p(stream.cuda_stream)
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
    tail = np.cumsum(deg[::-1])[::-1]  # entries of rows >= v
    p2 = int(tail[1:][deg[:-1] > 0].sum())
    gathers = rounds * (m * nnz + p2)  # entry gathers of the two passes (pass 2: rows j > i only)
    lds_peak = 128.0 / 8 * 256 * 2.4e9  # 8 B gathers at 128 B/clk/CU
    java_pairs = (nnz * nnz - int((deg.astype(np.int64) ** 2).sum())) // 2
    cpu_sr = None
    if R.rank == 0 and R.world == 1 and not args.no_cpu_baseline:
        import oracle
        nth = cores_used()
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
                     "frac": gathers / sec / lds_peak, "traffic": None, "kernel": "k_sr_gather<true,*>",
                     "random_gather_roofline": lds_gather_calib(gathers / sec)},
        "cpu_baseline": cpu_sr,
    }


def run_arxiv(R, args):
    """node2vec on lshrank arxiv (p=0.25, q=4, L=80, 10 walks/node): the graph on
    which the reference node2vec.py itself was timed (profiles/
    cpu_reference_node2vec.json), so GPU and reference share a workload."""
    torch = R.torch
    import gwamd
    from gwamd import _lib as C
    G = gwamd.GWGraph.from_edgelist(os.path.join(ROOT, "tests", "golden", "data", "arxiv_author_pub.txt"),
                                    "\t", "nx").to_device(R.dev.index)
    p, q, L, r = 0.25, 4.0, args.walk_length, 10
    C.check(C.lib().gw_n2v_prepare(G.handle, p, q, C.N2V_BITSET), G.handle)
    n = G.info().n
    B = r * n
    out = torch.empty((B, L), dtype=torch.int32, device=R.dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=R.dev)
    stream = torch.cuda.current_stream(R.dev)
    sh = C.ctypes.c_void_p(stream.cuda_stream)

    def st(i, ev):
        if ev is not None:
            ev[0].record(stream)
        C.check(C.lib().gw_n2v_walks(G.handle, L, args.seed, i * B, B, 1, C.ptr(out), None, C.ptr(cnt), sh),
                G.handle)
        if ev is not None:
            ev[1].record(stream)
    st(0, None)
    torch.cuda.synchronize()
    cnt.zero_()
    sec, kms = time_steps(R, lambda i, ev: st(1 + i, ev), 3, 0)
    steps = int(cnt[0].item())
    ref = reference_cpu_fixture()
    refline = None
    if ref:
        for e in ref.get("graphs", []):
            if e.get("graph") == "arxiv" and e.get("p") == p and e.get("q") == q:
                refline = {"value": e["walk_steps_per_s_1proc"], "unit": "walk-steps/s", "cores": 1,
                           "kind": "reference", "sample": e.get("sample"), "cpu_model": ref.get("cpu_model"),
                           "value_8proc": e.get("walk_steps_per_s_8proc"),
                           "source": "profiles/cpu_reference_node2vec.json (reference node2vec.py timed in the "
                                     "build container: it cannot travel to the GPU box)"}
    G.free()
    return {"metric": "walk-steps/sec (node2vec, lshrank arxiv)", "value": steps / sec, "unit": "walk-steps/s",
            "config": {"workload": f"node2vec p={p} q={q} on lshrank arxiv_author_pub (nx semantics, n={n}), "
                                   f"walk_length={L}, {r} walks/node", "sampler": "bitset"},
            "kernel_ms": kms, "cpu_baseline": refline}


def main(argv):
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        return launch_ranks(args, argv)
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        return 2
    R = Ranks(args)
    secondary = {}
    cpu = None
    if args.config == 5:
        h = run_topsim(R, args, "p10m")
        value, metric, unit = h["value"], h["metric"], h["unit"]
        head = h
    else:
        head = walk_headline(R, args)
        value, metric, unit = head["value"], "walk-steps/sec (node2vec)", "walk-steps/s"
        cpu = head.get("cpu_baseline")
    sec_mode = args.secondary
    if not R.plumbing and sec_mode != "none" and args.config == 2:
        if R.world == 1 or sec_mode == "all":
            if not args.no_config3:
                secondary["topsim_config3"] = run_config3_sweep(R, args)
            if not args.no_topsim:
                done = {(p["graph"], p["sample"], p["config"]["step"]): p
                        for p in (secondary.get("topsim_config3") or {}).get("points", [])}
                res = [done.get((nm, args.topsim_sample, args.topsim_step)) or run_topsim(R, args, nm)
                       for nm in args.topsim_graphs.split(",")]
                secondary["topsim"] = res[0]
                if len(res) > 1:
                    secondary["topsim"]["more"] = res[1:]
            if not args.no_arxiv:
                secondary["walk_arxiv"] = run_arxiv(R, args)
            if not args.no_walk10m:
                t0 = time.perf_counter()
                a, b, c = rmat_abc(args)
                BG = gwamd_graph_rmat(args.walk10m_scale, args.walk10m_edge_factor, a, b, c, args.seed + 1)
                build_s = time.perf_counter() - t0
                BG.to_device(R.dev.index)
                sc, ef = args.walk10m_scale, args.walk10m_edge_factor
                secondary["walk_10m"] = walk_secondary(R, args, BG, build_s, args.p, args.q, sc, ef,
                                                       "north_star 10M/100M graph")
                secondary["walk_10m_p1q1"] = walk_secondary(R, args, BG, build_s, 1.0, 1.0, sc, ef,
                                                            "north_star 10M/100M graph")
                BG.free()
            if not args.no_simrank:
                secondary["simrank_naive"] = run_simrank(R, args, args.simrank_graph)
        if not args.no_rmat24:
            # config 4: R-MAT-24 ef 16, p=1 q=0.5 (bitset tables would need ~390 GB: rejection
            # sampler with slot entries and per-row neighbour hash sets); 1 walk/node per rank
            t0 = time.perf_counter()
            a, b, c = rmat_abc(args)
            BG = gwamd_graph_rmat(24, 16, a, b, c, args.seed)
            build_s = time.perf_counter() - t0
            BG.to_device(R.dev.index)
            BG.options(expected_steps=10 * BG.n * (args.walk_length - 1))  # the sampler is chosen for r=10
            secondary["walk_rmat24_p1q05"] = walk_secondary(R, args, BG, build_s, 1.0, 0.5, 24, 16,
                                                            "config 4 R-MAT-24 ef 16", force_rejection=True,
                                                            strong_walks=10)
            BG.free()
        if not args.no_p10m:
            secondary["topsim_p10m"] = run_topsim(R, args, "p10m")
        if not args.no_p10m_stretch:
            secondary["topsim_p10m_stretch"] = run_topsim(R, args, "p10m", 10000, 5, args.stretch_stride)
    if R.rank == 0:
        ngpu = R.ngpu
        res = {
            "metric": metric,
            "value": value,
            "unit": unit,
            "n_gpus": ngpu,
            "ranks": R.world,
            "steps": args.steps if args.config != 5 else 1,
            "warmup": args.warmup if args.config != 5 else 1,
            "ms_per_step": head["seconds"] / (args.steps if args.config != 5 else 1) * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.config == 2 else "strong",
            "vs_baseline": None,
            "dtype": "int32 ids / f64 accept tests" if args.config != 5 else "f64 scores / int32 ids",
            "data": "synthetic" if not R.plumbing else "plumbing-check: synthetic rows, no GPU work",
            "backend": R.backend,
        }
        if R.world > 1 and R.ngpu < R.world:
            res["rehearsal"] = f"{R.world} ranks share {R.ngpu} GPU(s): not a scaling measurement"
        if args.config == 5:
            res["config"] = dict(head["config"], parallelism=f"replicated graph, sources split over {R.world} rank(s)")
            res["roofline"] = head["roofline"]
            res["cpu_baseline"] = head["cpu_baseline"]
            res["pair_updates"] = head["pair_updates"]
            if head.get("allgather"):
                res["allgather"] = head["allgather"]
            if head.get("host_shard"):
                res["host_shard"] = head["host_shard"]
        else:
            a, b, c = rmat_abc(args)
            res["config"] = {
                "workload": f"node2vec p={args.p} q={args.q} on synthetic R-MAT scale-{args.scale} (ef "
                            f"{args.edge_factor}, a,b,c={a},{b},{c}, seed {args.seed}; n={head['n']}, "
                            f"adjacency entries={head['nnz']}), walk_length={args.walk_length}, "
                            f"{args.num_walks} walks/node " + ("per step in total (split over the ranks)"
                                                               if args.config == 4 else "per rank per step"),
                "baseline_config": args.config,
                "walks_per_step": head["walks_per_step"], "walk_length": args.walk_length,
                "parallelism": f"replicated graph, walks sharded over {R.world} rank(s)" +
                               (" (the fixed r-walk workload split: strong scaling)" if args.config == 4 else "")}
            res["walk_steps"] = head["walk_steps"]
            for k in ("mode", "prep_s", "sampler_gb", "trials_per_step", "end_to_end", "end_to_end_rejection",
                      "end_to_end_best"):
                if k in head:
                    res[{"mode": "sampler", "prep_s": "prepare_seconds", "sampler_gb": "sampler_tables_gb",
                         "trials_per_step": "rejection_trials_per_step"}.get(k, k)] = head[k]
            res["roofline"] = head.get("roofline")
            res["cpu_baseline"] = cpu
            if res["roofline"] is not None and R.rank == 0:
                res["roofline"]["stream_copy_GBps"] = head.get("copy_gbps")
            if "allgather" in head:
                res["allgather"] = head["allgather"]
                res["allgather_all_ranks_ok"] = head["allgather_all_ranks_ok"]
            if "host_shard" in head:
                res["host_shard"] = head["host_shard"]
        ref = reference_cpu_fixture()
        if ref and not R.plumbing:
            res["reference_cpu_context"] = {"file": "profiles/cpu_reference_node2vec.json",
                                            "summary": ref.get("summary")}
        res["secondary"] = secondary or None
        res["summary"] = tail_summary(res)
        print(json.dumps(res), flush=True)
    R.close()
    return 0


def tail_summary(res):
    """A compact digest of the secondary lines, printed LAST in the JSON line:
    a driver that keeps only the line's tail (the last ~2000 characters) still
    records every config-3 point and the config-5 lines.  Lists, no key names:
    config3 rows are [graph, SAMPLE, kernel ms, pair-updates/s, roofline frac,
    counter traffic GB (null: no keyed PMC entry), kernel, scratch B/lane]."""
    sec = res.get("secondary") or {}

    def r3(x):
        return None if x is None else float(f"{x:.3g}")

    def e3(x):  # large rates as short strings ("3.59e+10")
        return None if x is None else f"{x:.3g}"
    out = {}
    pts = (sec.get("topsim_config3") or {}).get("points") or []
    if pts:
        out["config3_cols"] = "graph,SAMPLE,ms,pair-updates/s,frac,traffic_GB,kernel,scratch_B"
        out["config3"] = [[p["graph"], p["sample"], round(p["seconds"] * 1e3, 2), e3(p["value"]),
                           round(p["roofline"]["frac"], 3),
                           None if p["roofline"].get("traffic") is None else round(p["roofline"]["traffic"] / 1e9, 1),
                           (p.get("kernel") or "").replace("k_topsim_", "").replace(" ", "").replace("<", "")
                           .replace(">", ""),
                           (p.get("kernel_attrs") or {}).get("scratch_bytes_per_lane")] for p in pts]
    for k in ("topsim_p10m", "topsim_p10m_stretch", "walk_rmat24_p1q05"):
        v = sec.get(k)
        if not v or not v.get("roofline"):
            continue
        r = v["roofline"]
        out[k] = {"s": r3(v.get("seconds") or (v.get("kernel_ms") or 0) * 1e-3), "value": e3(v.get("value")),
                  "frac": r3(r.get("frac")), "traffic_GB": None if r.get("traffic") is None else round(r["traffic"] / 1e9, 1),
                  "rate": r3((r.get("random_line_roofline") or {}).get("frac")),
                  "host_shard_s": r3((v.get("host_shard") or {}).get("seconds"))}
    return out or None


def gwamd_graph_rmat(scale, ef, a, b, c, seed):
    import gwamd
    return gwamd.GWGraph.rmat(scale, ef, a, b, c, seed)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
