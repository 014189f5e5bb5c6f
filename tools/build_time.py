#!/usr/bin/env python3
"""Wall time of gw_n2v_prepare (the per-edge table builds) on the bench graphs.

    python tools/build_time.py [--graphs r20,r24e6,r22] [--reps 2]

For each graph: BITSET prepare (full per-edge bitsets: k_bs_tri count + fill
passes, region layout) and REJECTION prepare with listed entries forced on
(lists-only build) and off (16 B slot entries + neighbour hash only).  The
first repetition warms the allocator; later ones are reported.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))

GRAPHS = {"r20": (20, 16, 0.25, 4.0), "r24e6": (24, 6, 0.25, 4.0), "r22": (22, 16, 1.0, 0.5),
          "r24": (24, 16, 1.0, 0.5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default="r20,r24e6,r22")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--modes", default="bitset,listed,plain")
    ap.add_argument("--walks", type=int, default=0, help="also time one launch of this many walks per vertex")
    a = ap.parse_args()
    import torch
    import gwamd
    from gwamd import _lib as C
    out = {}
    for name in a.graphs.split(","):
        sc, ef, p, q = GRAPHS[name]
        t0 = time.perf_counter()
        G = gwamd.GWGraph.rmat(sc, ef, 0.57, 0.19, 0.19, 42)
        inf = G.info()
        G.to_device(0)
        res = {"n": inf.n, "nnz": inf.nnz, "max_degree": inf.max_degree, "host_build_s": time.perf_counter() - t0}
        for mode in a.modes.split(","):
            if mode == "bitset":
                G.options(listed=-1)
                m = C.N2V_BITSET
            else:
                G.options(listed=1 if mode == "listed" else 0)
                m = C.N2V_REJECTION
            ts = []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                try:
                    C.check(C.lib().gw_n2v_prepare(G.handle, p, q, m), G.handle)
                except C.CapacityError as e:
                    ts.append(None)
                    res[mode + "_error"] = str(e)
                    break
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            res[mode + "_prepare_s"] = ts[-1]
            res[mode + "_sampler_gb"] = G.info().sampler_bytes / 1e9
            if a.walks and ts[-1] is not None:
                # one BASELINE pass: `walks` walks from every vertex, L = 80 (launched twice, second timed)
                nw, L = a.walks * inf.n, 80
                wbuf = torch.empty((nw, L), dtype=torch.int32, device="cuda")
                cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
                for rep in range(2):
                    cnt.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    C.check(C.lib().gw_n2v_walks(G.handle, L, 42, 0, nw, 1, C.ptr(wbuf), None, C.ptr(cnt), None),
                            G.handle)
                    e1.record()
                    torch.cuda.synchronize()
                ws = e0.elapsed_time(e1) * 1e-3
                steps = int(cnt[0])
                res[mode + "_walk_s"] = ws
                res[mode + "_walk_steps_per_s"] = steps / ws
                res[mode + "_end_to_end_s"] = ts[-1] + ws
                del wbuf
                print(f"[walk] {name} {mode}: {ws * 1e3:.1f} ms, {steps / ws:.3e} steps/s, "
                      f"e2e {ts[-1] + ws:.3f} s", file=sys.stderr, flush=True)
            print(f"[build] {name} {mode}: {ts}", file=sys.stderr, flush=True)
        G.free()
        out[name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
