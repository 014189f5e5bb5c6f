"""Time naive SimRank (SimRank.java) on the GPU: blog / moreno / g333."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
import ctypes  # noqa: E402

import torch  # noqa: E402

from gwamd import _lib as C  # noqa: E402
from gwamd import topsim  # noqa: E402

DATA = os.path.join(ROOT, "tests", "golden", "data")
G = {"blog": ("blog.txt", 10313, ","), "moreno": ("moreno_crime_crime.txt", 1380, "\t"),
     "g333": ("0_333_5038.txt", 333, " ")}
for name in sys.argv[1:] or ["blog"]:
    f, V, sep = G[name]
    g = topsim.Graph(os.path.join(DATA, f), V, separator=sep)
    g._ensure_device()
    sim = torch.empty((V, V), dtype=torch.float64, device="cuda")
    h = g._g.handle
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    C.check(C.lib().gw_simrank_naive(h, 0.6, 3, C.ptr(sim), sp), h)  # warm (workspace)
    torch.cuda.synchronize()
    for iters in (1, 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        C.check(C.lib().gw_simrank_naive(h, 0.6, iters, C.ptr(sim), sp), h)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        nnz = len(g._nbrs)
        print(json.dumps({"graph": name, "V": V, "nnz": nnz, "iters": iters, "ms": round(ms, 3),
                          "gathers_per_s": 1.5 * V * nnz * iters / (ms / 1e3)}), flush=True)
