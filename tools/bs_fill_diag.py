#!/usr/bin/env python3
"""Timing-only split of the bitset build's FILL pass (diag library, GW_DIAG_BS_FILL).

    rocprofv3 --kernel-trace --output-format csv -d DIR -- python tools/bs_fill_diag.py [--graph r20]

Prepares the bitset sampler once per knob value (0 = full, 1 = no payload
emission, 2 = no region-bit stores, 4 = no payload flush, 7 = all three off),
each twice, in that order; the kernel trace's k_bs_tri<true> rows follow the
same order.  Tables built with a knob set are wrong on purpose.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GW_LIB", os.path.join(ROOT, "graph-embedding_amd", "gwamd", "libgraphwalk_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
GRAPHS = {"r20": (20, 16, 0.25, 4.0), "r24e6": (24, 6, 0.25, 4.0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="r20")
    ap.add_argument("--knobs", default="0,1,2,4,7")
    a = ap.parse_args()
    import torch
    import gwamd
    from gwamd import _lib as C
    sc, ef, p, q = GRAPHS[a.graph]
    G = gwamd.GWGraph.rmat(sc, ef, 0.57, 0.19, 0.19, 42)
    G.to_device(0)
    for k in a.knobs.split(","):
        os.environ["GW_DIAG_BS_FILL"] = k
        for _ in range(2):
            C.check(C.lib().gw_n2v_prepare(G.handle, p, q, C.N2V_BITSET), G.handle)
            torch.cuda.synchronize()
        print(f"[fill-diag] knob {k} done", file=sys.stderr, flush=True)
    G.free()


if __name__ == "__main__":
    main()
