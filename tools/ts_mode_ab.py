"""In-process A/B of TopSim accumulator modes (GW_DIAG_TS_HASH, diag library).

Loads gwamd/libgraphwalk_diag.so (build: python graph-embedding_amd/build.py --diag),
builds P10M (config 5) and/or lshrank arxiv once, then alternates the modes
(each: gw_topsim_prepare under the env knob, one warm launch, one timed launch)
so every mode sees the same box state.  Prints one JSON line per (graph, mode)
with the launch times, the device counters and the top-k agreement with the
first mode (fp64 atomics make the last bits order-dependent).

    python tools/ts_mode_ab.py [--modes 2,3] [--graphs p10m,arxiv] [--reps 3]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GW_LIB", os.path.join(ROOT, "graph-embedding_amd", "gwamd", "libgraphwalk_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="2,3")
    ap.add_argument("--graphs", default="p10m,arxiv")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--env", default="GW_DIAG_TS_HASH", help="diag knob the modes are values of")
    a = ap.parse_args()
    import numpy as np
    import torch
    import gwamd
    from gwamd import _lib as C
    from gwamd import topsim
    modes = a.modes.split(",")
    for name in a.graphs.split(","):
        t0 = time.perf_counter()
        if name == "p10m":
            g = gwamd.GWGraph.rmat_java(10_000_000, 100_000_000, 0.57, 0.19, 0.19, 42)
            csr = g.export_csr()
            deg = np.diff(csr["offsets"])
            g.to_device(0)
            h = g.handle
            srcs = np.nonzero(deg > 0)[0].astype(np.int32)
            K, sample, step = 100, 1000, 3
        else:
            f, V, sep = {"arxiv": ("arxiv_author_pub.txt", 38741, "\t"), "blog": ("blog.txt", 10313, ","),
                         "moreno": ("moreno_crime_crime.txt", 1380, "\t")}[name]
            g = topsim.Graph(os.path.join(ROOT, "tests", "golden", "data", f), V, separator=sep, device=0)
            g._ensure_device()
            h = g._g.handle
            srcs = np.arange(V, dtype=np.int32)
            K, sample, step = 20, 10000, 5
        print(f"[{name}] built in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        dev = torch.device("cuda:0")
        src = torch.as_tensor(srcs, device=dev)
        n = len(srcs)
        res = {}
        for m in modes:
            res[m] = {"ms": [], "ids": torch.empty((n, K), dtype=torch.int32, device=dev),
                      "sc": torch.empty((n, K), dtype=torch.float64, device=dev)}
        st = torch.zeros(4, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream(dev)
        sh = C.ctypes.c_void_p(stream.cuda_stream)
        for rep in range(a.reps):
            for m in modes:
                os.environ[a.env] = m
                C.check(C.lib().gw_topsim_prepare(h, C.TOPSIM_SINGLE_SAMPLE, sample, step, K), h)
                r = res[m]
                for timed in (False, True):
                    st.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    C.check(C.lib().gw_topsim(h, C.TOPSIM_SINGLE_SAMPLE, sample, step, 0.6, 42, C.ptr(src), n, K,
                                              C.ptr(r["ids"]), C.ptr(r["sc"]), C.ptr(st), sh), h)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    if timed:
                        r["ms"].append(e0.elapsed_time(e1))
                        r["stats"] = [int(x) for x in st.cpu().tolist()]
                print(f"[{name}] rep {rep} mode {m}: {r['ms'][-1]:.2f} ms", file=sys.stderr, flush=True)
        base = res[modes[0]]
        for m in modes:
            r = res[m]
            same_ids = float((r["ids"] == base["ids"]).float().mean().item())
            rel = float(((r["sc"] - base["sc"]).abs() / base["sc"].abs().clamp_min(1e-300)).max().item())
            print(json.dumps({"graph": name, "mode": m, "ms": [round(x, 3) for x in r["ms"]],
                              "median_ms": round(statistics.median(r["ms"]), 3), "stats": r["stats"],
                              "ids_equal_frac_vs_first": same_ids, "max_rel_score_diff_vs_first": rel}), flush=True)
        del g


if __name__ == "__main__":
    main()
