"""Time naive SimRank (SimRank.java) on the GPU: blog / moreno / g333.

    python tools/sr_time.py [blog moreno ...]
    python tools/sr_time.py --knob GW_DIAG_<KNOB> --modes 0,1 --reps 5 blog
        (diag library: the knob's values alternate in one process, 3 rounds each,
        and every mode's result is compared with the first mode's)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("graphs", nargs="*", default=["blog"])
ap.add_argument("--knob", default="")
ap.add_argument("--modes", default="0,1")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
if a.knob:
    os.environ.setdefault("GW_LIB", os.path.join(ROOT, "graph-embedding_amd", "gwamd", "libgraphwalk_diag.so"))
import ctypes  # noqa: E402

import torch  # noqa: E402

from gwamd import _lib as C  # noqa: E402
from gwamd import topsim  # noqa: E402

DATA = os.path.join(ROOT, "tests", "golden", "data")
G = {"blog": ("blog.txt", 10313, ","), "moreno": ("moreno_crime_crime.txt", 1380, "\t"),
     "g333": ("0_333_5038.txt", 333, " ")}


def launch(h, sim, sp, iters):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    C.check(C.lib().gw_simrank_naive(h, 0.6, iters, C.ptr(sim), sp), h)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


for name in a.graphs:
    f, V, sep = G[name]
    g = topsim.Graph(os.path.join(DATA, f), V, separator=sep)
    g._ensure_device()
    sim = torch.empty((V, V), dtype=torch.float64, device="cuda")
    h = g._g.handle
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nnz = len(g._nbrs)
    if not a.knob:
        launch(h, sim, sp, 3)  # warm (workspace)
        for iters in (1, 3):
            ms = launch(h, sim, sp, iters)
            print(json.dumps({"graph": name, "V": V, "nnz": nnz, "iters": iters, "ms": round(ms, 3),
                              "gathers_per_s": 1.5 * V * nnz * iters / (ms / 1e3)}), flush=True)
        continue
    modes = a.modes.split(",")
    times = {m: [] for m in modes}
    res = {}
    for m in modes:  # warm every variant
        os.environ[a.knob] = m
        launch(h, sim, sp, 3)
    for r in range(a.reps):
        for m in (modes if r % 2 == 0 else modes[::-1]):
            os.environ[a.knob] = m
            times[m].append(launch(h, sim, sp, 3))
            res[m] = sim.clone()
    for m in modes:
        med = statistics.median(times[m])
        d = (res[m] - res[modes[0]]).abs().max().item()
        print(json.dumps({"graph": name, "knob": a.knob, "mode": m, "iters": 3, "median_ms": round(med, 3),
                          "ms": [round(x, 3) for x in times[m]],
                          "gathers_per_s": 1.5 * V * nnz * 3 / (med / 1e3),
                          "max_abs_diff_vs_first": d, "bitwise_equal_vs_first": bool(torch.equal(res[m], res[modes[0]]))}),
              flush=True)
