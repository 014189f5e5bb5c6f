"""In-process A/B timing of library variants on the headline walk launch.

Process-to-process spread of the bench (a few discrete levels, +-3%) hides
changes of a few percent; here every variant is loaded into ONE process
(ctypes, RTLD_LOCAL), builds its own graph and tables, and the launches are
interleaved A B A B ... with HIP events, so each variant sees the same clock
and memory state.  Tables are rebuilt `--rebuild` times to average over
placement.

    python tools/ab_inproc.py LIB_A LIB_B [...] [--scale 20] [--reps 6] [--rebuild 2]
(LIB "main" = the in-tree build, "diag" = gwamd/libgraphwalk_diag.so; a
variant "LIB:VAR=value" sets that environment variable around its launches,
e.g. diag:GW_DIAG_BS=4 — the diag library's knobs are read per launch.)
Prints one JSON line per variant.
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


def load(path, C):
    L = ctypes.CDLL(path)
    for name, (res, args) in C.SIGNATURES.items():
        f = getattr(L, name, None)  # older builds (tools/build_rev_lib.sh) lack newer entry points
        if f is None:
            continue
        f.restype = res
        f.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--ef", type=int, default=16)
    ap.add_argument("--p", type=float, default=0.25)
    ap.add_argument("--q", type=float, default=4.0)
    ap.add_argument("--L", type=int, default=80)
    ap.add_argument("--walks", type=int, default=10, help="walks per vertex per launch")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--rebuild", type=int, default=2)
    ap.add_argument("--mode", default="bitset")
    ap.add_argument("--listed", type=int, default=-1,
                    help="gw_options_t.listed for the rejection sampler (0: plain 16 B entries, k_walk_scale)")
    a = ap.parse_args()
    import torch
    from gwamd import _lib as C
    def path_of(x):
        x = x.split(":")[0]
        if x in ("main", "diag"):
            return os.path.join(ROOT, "graph-embedding_amd", "gwamd",
                                "libgraphwalk.so" if x == "main" else "libgraphwalk_diag.so")
        if os.path.sep in x:
            return x
        ab = os.path.join(ROOT, "graph-embedding_amd", "gwamd", "ab", "libgraphwalk_" + x + ".so")
        return ab if os.path.exists(ab) else os.path.join(ROOT, "abl", x + ".so")
    envs = [dict([x.split(":", 1)[1].split("=", 1)]) if ":" in x else {} for x in a.libs]
    paths = [path_of(x) for x in a.libs]
    libs = [load(p, C) for p in paths]
    mode = C.N2V_BITSET if a.mode == "bitset" else C.N2V_REJECTION
    stream = torch.cuda.current_stream()
    sh = ctypes.c_void_p(stream.cuda_stream)
    times = {x: [] for x in a.libs}
    steps = {}
    same = {a.libs[0]: True}
    for rb in range(a.rebuild):
        hs = []
        for name, L in zip(a.libs, libs):
            h = ctypes.c_void_p()
            C.check(L.gw_graph_rmat(a.scale, a.ef, 0.57, 0.19, 0.19, 42, ctypes.byref(h)))
            if L.gw_graph_to_device(h, 0) != 0:
                raise SystemExit(L.gw_last_error(h).decode())
            if a.listed != -1:
                o = C.Options()
                C.check(L.gw_graph_get_options(h, ctypes.byref(o)))
                o.listed = a.listed
                C.check(L.gw_graph_set_options(h, ctypes.byref(o)))
            t0 = time.perf_counter()
            if L.gw_n2v_prepare(h, a.p, a.q, mode) != 0:
                raise SystemExit(L.gw_last_error(h).decode())
            torch.cuda.synchronize()
            inf = C.GraphInfo()
            L.gw_graph_info(h, ctypes.byref(inf))
            print(f"{name}: prepare {time.perf_counter() - t0:.2f} s, sampler tables {inf.sampler_bytes / 1e9:.2f} GB",
                  file=sys.stderr, flush=True)
            hs.append(h)
        inf = C.GraphInfo()
        libs[0].gw_graph_info(hs[0], ctypes.byref(inf))
        B = a.walks * inf.n
        out = torch.empty((B, a.L), dtype=torch.int32, device="cuda")
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        for L, h in zip(libs, hs):  # warm-up
            L.gw_n2v_walks(h, a.L, 7, 0, B, 1, C.ptr(out), None, None, sh)
        torch.cuda.synchronize()
        for r in range(a.reps):
            order = list(range(len(libs))) if r % 2 == 0 else list(reversed(range(len(libs))))
            for k in order:
                L, h, name = libs[k], hs[k], a.libs[k]
                cnt.zero_()
                os.environ.update(envs[k])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rc = L.gw_n2v_walks(h, a.L, 7, (r + 1) * B, B, 1, C.ptr(out), None, C.ptr(cnt), sh)
                e1.record(stream)
                torch.cuda.synchronize()
                for v in envs[k]:
                    os.environ.pop(v, None)
                if rc != 0:
                    raise SystemExit(L.gw_last_error(h).decode())
                times[name].append(e0.elapsed_time(e1))
                steps[name] = int(cnt[0].item())
        if rb == 0:  # the variants must emit the same walks (same launch, bitwise)
            ref = None
            for L, h, name in zip(libs, hs, a.libs):
                os.environ.update(envs[libs.index(L)])
                L.gw_n2v_walks(h, a.L, 7, 0, B, 1, C.ptr(out), None, None, sh)
                torch.cuda.synchronize()
                for v in envs[libs.index(L)]:
                    os.environ.pop(v, None)
                if ref is None:
                    ref = out.clone()
                else:
                    same[name] = bool(torch.equal(out, ref))
            del ref
        for L, h in zip(libs, hs):
            L.gw_graph_free(h)
        del out
        torch.cuda.synchronize()
    base = statistics.median(times[a.libs[0]])
    for name in a.libs:
        t = times[name]
        med = statistics.median(t)
        print(json.dumps({"lib": name, "median_ms": round(med, 3), "min_ms": round(min(t), 3),
                          "max_ms": round(max(t), 3), "n": len(t), "vs_first": round(med / base, 4),
                          "Gsteps_per_s": round(steps[name] / med / 1e6, 3),
                          "walks_equal_first": same.get(name)}), flush=True)


if __name__ == "__main__":
    main()
