"""In-process A/B of TopSim library variants (config 5 P10M and the lshrank graphs).

Every library (ctypes, RTLD_LOCAL) builds its own graph; launches are
interleaved A B B A ... with HIP events on one stream, so each variant sees
the same box state.  Also reports the counters and the top-k agreement of
every variant with the first (fp64 atomics make the last bits order-dependent).

    python tools/ts_lib_ab.py main abl/ts_flat.so [--graphs p10m,blog,arxiv] [--reps 4]
("main" = the in-tree gwamd/libgraphwalk.so, "diag" = gwamd/libgraphwalk_diag.so;
"LIB:VAR=value" sets that environment variable around the variant's launches,
e.g. diag:GW_DIAG_TS=1024 — entries naming the same library share ONE library
instance and ONE graph handle, so a knob A/B sees the same allocations
("diag#2:VAR=value" gets a handle of its own);
--sample / --step / --stride override the P10M workload, e.g. the config-5
stretch SAMPLE 10000 / STEP 5 on every 16th source)

Two library instances in one process can differ by up to ~5% on P10M by the
placement of their tables alone (profiles/r04/ts_lib_ab_three_way.jsonl), so
--procs N instead runs every library alone in a child process, N rounds in
alternating order (A B, B A, ...), and reports the median over rounds of
each process's median launch time.  The parent never touches the GPU.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))

GRAPHS = {"blog": ("blog.txt", 10313, ",", 10000, 5, 20),
          "arxiv": ("arxiv_author_pub.txt", 38741, "\t", 10000, 5, 20),
          "moreno": ("moreno_crime_crime.txt", 1380, "\t", 10000, 5, 20)}


def load(path, C):
    L = ctypes.CDLL(path)
    for name, (res, args) in C.SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--graphs", default="p10m,blog,arxiv")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--procs", type=int, default=0, help="rounds of one child process per library")
    ap.add_argument("--sample", type=int, default=1000, help="P10M SAMPLE")
    ap.add_argument("--step", type=int, default=3, help="P10M STEP")
    ap.add_argument("--stride", type=int, default=1, help="P10M: every stride-th non-isolated source")
    ap.add_argument("--ls-sample", type=int, default=0, help="lshrank graphs: SAMPLE (default 10000)")
    a = ap.parse_args()
    if a.procs > 0:
        import subprocess
        med = {(g, x): [] for g in a.graphs.split(",") for x in a.libs}
        for rnd in range(a.procs):
            order = a.libs if rnd % 2 == 0 else list(reversed(a.libs))
            for x in order:
                out = subprocess.run([sys.executable, os.path.abspath(__file__), x, "--graphs", a.graphs,
                                      "--reps", str(a.reps), "--sample", str(a.sample), "--step", str(a.step),
                                      "--stride", str(a.stride), "--ls-sample", str(a.ls_sample)],
                                     check=True, stdout=subprocess.PIPE, text=True).stdout
                for line in out.splitlines():
                    d = json.loads(line)
                    med[(d["graph"], x)].append(d["median_ms"])
                    print(f"[round {rnd}] {x} {d['graph']}: {d['median_ms']:.3f} ms", file=sys.stderr, flush=True)
        for g in a.graphs.split(","):
            base = statistics.median(med[(g, a.libs[0])])
            for x in a.libs:
                m = statistics.median(med[(g, x)])
                print(json.dumps({"graph": g, "lib": x, "median_ms": round(m, 3), "process_medians_ms": med[(g, x)],
                                  "vs_first": round(m / base, 4), "mode": "separate processes"}), flush=True)
        return
    import numpy as np
    import torch
    from gwamd import _lib as C
    def path_of(x):
        x = x.split(":")[0].split("#")[0]
        if x in ("main", "diag"):
            return os.path.join(ROOT, "graph-embedding_amd", "gwamd",
                                "libgraphwalk.so" if x == "main" else "libgraphwalk_diag.so")
        return os.path.join(ROOT, x)
    envs = [dict([x.split(":", 1)[1].split("=", 1)]) if ":" in x else {} for x in a.libs]
    paths = [path_of(x) for x in a.libs]
    loaded = {}
    for pth in paths:
        if pth not in loaded:
            loaded[pth] = load(pth, C)
    libs = [loaded[pth] for pth in paths]
    # entries of one library share its graph handle (a "#tag" after the path
    # gives an entry its own handle: knobs read when the workspace is sized,
    # e.g. GW_DIAG_TS_PIPE_MAX, must not re-prepare inside the timed launches)
    hkey = [x.split(":")[0] for x in a.libs]
    first_of = [hkey.index(k) for k in hkey]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    for gname in a.graphs.split(","):
        hs = []
        for k, L in enumerate(libs):
            if first_of[k] != k:
                hs.append(hs[first_of[k]])
                continue
            h = ctypes.c_void_p()
            t0 = time.perf_counter()
            if gname == "p10m":
                rc = L.gw_graph_rmat_java(10_000_000, 100_000_000, 0.57, 0.19, 0.19, 42, ctypes.byref(h))
                K, sample, step = 100, a.sample, a.step
            else:
                f, V, sep, sample, step, K = GRAPHS[gname]
                sample = a.ls_sample or sample
                rc = L.gw_graph_load_edgelist(os.path.join(ROOT, "tests", "golden", "data", f).encode(),
                                              sep.encode(), C.SEM_JAVA_MULTI, 0, 0, V, ctypes.byref(h))
            if rc != 0 or L.gw_graph_to_device(h, 0) != 0:
                raise SystemExit(f"graph {gname}: rc {rc}")
            hs.append(h)
            print(f"[{gname}] graph built in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        inf = C.GraphInfo()
        libs[0].gw_graph_info(hs[0], ctypes.byref(inf))
        n = int(inf.n)
        offs = np.empty(n + 1, np.int64)
        # sources: every vertex with an edge (degree from the exported CSR)
        nnz = int(inf.nnz)
        nb = np.empty(max(nnz, 1), np.int32)
        libs[0].gw_graph_export_csr(hs[0], offs.ctypes.data, nb.ctypes.data, None, None, None)
        srcs = np.nonzero(np.diff(offs) > 0)[0].astype(np.int32)
        if gname == "p10m" and a.stride > 1:
            srcs = srcs[::a.stride].copy()
        del nb
        src = torch.as_tensor(srcs, device=dev)
        ns = len(srcs)
        outs = [(torch.empty((ns, K), dtype=torch.int32, device=dev),
                 torch.empty((ns, K), dtype=torch.float64, device=dev)) for _ in libs]
        st = torch.zeros(4, dtype=torch.int64, device=dev)
        times = [[] for _ in libs]
        stats = [None] * len(libs)

        def run(k):
            st.zero_()
            os.environ.update(envs[k])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            rc = libs[k].gw_topsim(hs[k], C.TOPSIM_SINGLE_SAMPLE, sample, step, 0.6, 42, C.ptr(src), ns, K,
                                   C.ptr(outs[k][0]), C.ptr(outs[k][1]), C.ptr(st), sh)
            e1.record(stream)
            torch.cuda.synchronize()
            for v in envs[k]:
                os.environ.pop(v, None)
            if rc != 0:
                raise SystemExit(libs[k].gw_last_error(hs[k]).decode())
            return e0.elapsed_time(e1)
        for k in range(len(libs)):
            run(k)  # warm-up, workspace
        for r in range(a.reps):
            order = list(range(len(libs))) if r % 2 == 0 else list(reversed(range(len(libs))))
            for k in order:
                times[k].append(run(k))
                stats[k] = [int(x) for x in st.cpu().tolist()]
            print(f"[{gname}] rep {r}: " + " ".join(f"{t[-1]:.2f}" for t in times), file=sys.stderr, flush=True)
        base = statistics.median(times[0])
        for k, name in enumerate(a.libs):
            ids_eq = float((outs[k][0] == outs[0][0]).float().mean().item())
            rel = float(((outs[k][1] - outs[0][1]).abs() / outs[0][1].abs().clamp_min(1e-300)).max().item())
            med = statistics.median(times[k])
            print(json.dumps({"graph": gname, "lib": name, "median_ms": round(med, 3),
                              "ms": [round(x, 3) for x in times[k]], "vs_first": round(med / base, 4),
                              "stats": stats[k], "ids_equal_frac_vs_first": ids_eq,
                              "max_rel_score_diff_vs_first": rel}), flush=True)
        for k, (L, h) in enumerate(zip(libs, hs)):
            if first_of[k] == k:
                L.gw_graph_free(h)
        del outs
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
