"""Lane utilisation of the headline walk kernel (k_walk_bitset): the fraction
of a wave's loop iterations in which a lane still has steps to take.  Lanes
of one wave run the wave-uniform loop until the slowest one's walk ends (the
trial and region-select iterations differ per walk).  Diag library only
(GW_DIAG_BS=64 fills counters[2..3]).

    python tools/bs_lane_util.py [LIB] [--scale 20] [--walks 10]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default="abv/diag.so")
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--walks", type=int, default=10)
    ap.add_argument("--p", type=float, default=0.25)
    ap.add_argument("--q", type=float, default=4.0)
    a = ap.parse_args()
    os.environ["GW_LIB"] = os.path.join(ROOT, a.lib)
    import torch
    from gwamd import _lib as C
    import gwamd
    G = gwamd.GWGraph.rmat(a.scale, 16, 0.57, 0.19, 0.19, 42).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, a.p, a.q, C.N2V_BITSET), G.handle)
    n, L = G.n, 80
    B = a.walks * n
    out = torch.empty((B, L), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
    os.environ["GW_DIAG_BS"] = "64"
    C.check(C.lib().gw_n2v_walks(G.handle, L, 42, 0, B, 1, C.ptr(out), None, C.ptr(cnt), None), G.handle)
    torch.cuda.synchronize()
    c = [int(x) for x in cnt.cpu().tolist()]
    print(json.dumps({"graph": f"R-MAT-{a.scale}", "p": a.p, "q": a.q, "walks": B, "steps": c[0], "trials": c[1],
                      "lane_iterations": c[2], "active_lane_iterations": c[3],
                      "lane_utilisation": c[3] / max(c[2], 1), "iterations_per_step": c[3] / max(c[0], 1)}))


if __name__ == "__main__":
    main()
