"""PCIe-inclusive and text-output rates of the host-buffer boundary
(gw_n2v_walks_host, gw_write_walks_text) on the bench workload.

    python tools/host_rate.py [--scale 20] [--text-walks 1000000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--p", type=float, default=0.25)
    ap.add_argument("--q", type=float, default=4.0)
    ap.add_argument("--text-walks", type=int, default=1_000_000)
    a = ap.parse_args()
    import numpy as np
    import gwamd
    from gwamd import _lib as C
    G = gwamd.GWGraph.rmat(a.scale, 16, 0.57, 0.19, 0.19, 42).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, a.p, a.q, C.N2V_BITSET), G.handle)
    n, L = G.n, 80
    nw = 10 * n
    out = np.empty((nw, L), dtype=np.int32)
    lens = np.empty(nw, dtype=np.int32)
    cnt = np.zeros(2, dtype=np.uint64)
    res = {}
    for rep in range(2):  # first call: workspace + page faults on the fresh host buffer
        t0 = time.perf_counter()
        C.check(C.lib().gw_n2v_walks_host(G.handle, L, 42, 0, nw, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt)), G.handle)
        dt = time.perf_counter() - t0
        res[f"walks_host_s_rep{rep}"] = dt
    steps = int(cnt[0])  # counters of the last call (the host form overwrites them)
    res["walk_steps"] = steps
    res["walks_host_walk_steps_per_s"] = steps / res["walks_host_s_rep1"]
    res["walks_host_GB_per_s"] = out.nbytes / res["walks_host_s_rep1"] / 1e9
    path = "/tmp/gw_walks.txt"
    k = min(a.text_walks, nw)
    t0 = time.perf_counter()
    C.check(C.lib().gw_write_walks_text(G.handle, path.encode(), C.ptr(out), C.ptr(lens), k, L), G.handle)
    dt = time.perf_counter() - t0
    sz = os.path.getsize(path)
    os.unlink(path)
    res["text_walks"] = k
    res["text_s"] = dt
    res["text_MB_per_s"] = sz / dt / 1e6
    res["text_walk_steps_per_s"] = k * (L - 1) / dt
    print(json.dumps(res))


if __name__ == "__main__":
    main()
