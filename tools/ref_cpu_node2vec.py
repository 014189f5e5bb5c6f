"""Reference CPU baseline: the reference's own node2vec.py walk loop, timed.

BUILD-CONTAINER ONLY (the reference does not exist on the GPU box).  Imports
/root/reference/node2vec/src/node2vec.py exactly as oracle/gen_goldens.py does
(`np.int = int` harness shim for node2vec.py:125; graph built with networkx as
main.py:76-89) and times, per graph:

* `preprocess_transition_probs()` (node2vec.py:83-113) — once per process;
* the walk loop `simulate_walks(r, L)` (node2vec.py:41-59) alone;
* 1 process, and 8 shard processes that each walk a contiguous 1/8 of the
  start nodes (each shard preprocesses its own copy first, untimed), the
  aggregate = all shards' walk-steps / the slowest shard's walk time.

Writes profiles/cpu_reference_node2vec.json (CPU model, core count).  bench.py
quotes the arxiv entry beside its GPU line on the same graph and p, q.

    python tools/ref_cpu_node2vec.py [--graphs karate,moreno,arxiv,rmat10,...]
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
DATA = os.path.join(ROOT, "tests", "golden", "data")

GRAPHS = {
    "karate": ("karate.edgelist", " "),
    "moreno": ("moreno_crime_crime.txt", "\t"),
    "arxiv": ("arxiv_author_pub.txt", "\t"),
}


def build_graph(name):
    import networkx as nx
    import gen_goldens as gg
    if name in GRAPHS:
        f, delim = GRAPHS[name]
        return gg.read_graph(os.path.join(DATA, f), delim, False, False)
    scale = int(name[4:])  # rmatNN: the bench's Graph500 R-MAT at scale NN (ef 16, seed 42)
    import gwamd
    c = gwamd.GWGraph.rmat(scale, 16, 0.57, 0.19, 0.19, 42).export_csr()
    offs, nbrs = c["offsets"], c["nbrs"]
    G = nx.DiGraph()
    src = np.repeat(np.arange(len(offs) - 1), np.diff(offs))
    G.add_edges_from(zip(src.tolist(), nbrs.tolist()), weight=1)
    return G.to_undirected()


def _walk(name, p, q, r, L, shard, nshards, seed, out):
    import gen_goldens as gg
    n2v = gg._import_reference()
    G = build_graph(name)
    g = n2v.Graph(G, False, p, q)
    t0 = time.perf_counter()
    g.preprocess_transition_probs()
    prep = time.perf_counter() - t0
    nodes = list(G.nodes())
    if nshards > 1:  # contiguous 1/nshards of the start nodes, same loop body as simulate_walks
        b = len(nodes) * shard // nshards
        e = len(nodes) * (shard + 1) // nshards
        nodes = nodes[b:e]
    random.seed(seed)
    np.random.seed(seed)
    t0 = time.perf_counter()
    steps = 0
    if nshards == 1:
        walks = g.simulate_walks(r, L)  # node2vec.py:41-59, prints its progress
        steps = sum(len(w) - 1 for w in walks)
    else:
        for _ in range(r):
            random.shuffle(nodes)
            for v in nodes:
                steps += len(g.node2vec_walk(walk_length=L, start_node=v)) - 1
    dt = time.perf_counter() - t0
    out.put((shard, prep, dt, steps))


def run(name, p, q, r, L, nshards, seed=0):
    ctx = mp.get_context("fork")
    qu = ctx.Queue()
    ps = [ctx.Process(target=_walk, args=(name, p, q, r, L, s, nshards, seed, qu)) for s in range(nshards)]
    for x in ps:
        x.start()
    res = [qu.get() for _ in ps]
    for x in ps:
        x.join()
    prep = max(x[1] for x in res)
    wall = max(x[2] for x in res)
    steps = sum(x[3] for x in res)
    return prep, wall, steps


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default="karate,moreno,arxiv,rmat10,rmat11,rmat12")
    ap.add_argument("--walks", type=int, default=10)
    ap.add_argument("--length", type=int, default=80)
    ap.add_argument("--shards", type=int, default=8)
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles", "cpu_reference_node2vec.json")
    try:
        doc = json.load(open(out))
    except Exception:
        doc = {"graphs": []}
    doc.update({"tool": "tools/ref_cpu_node2vec.py", "reference": "node2vec/src/node2vec.py (imported as is; "
                "np.int shim)", "cpu_model": cpu_model(), "cores": os.cpu_count(),
                "python": platform.python_version(), "where": "build container (no GPU; the reference cannot "
                "travel to the GPU box)"})
    cases = []
    for gname in a.graphs.split(","):
        pqs = [(1.0, 1.0), (0.25, 4.0)] if gname == "karate" else [(0.25, 4.0)]
        r = a.walks if not gname.startswith("rmat") else 1
        for p, q in pqs:
            prep1, t1, s1 = run(gname, p, q, r, a.length, 1)
            prep8, t8, s8 = run(gname, p, q, r, a.length, a.shards)
            e = {"graph": gname, "p": p, "q": q, "walks_per_node": r, "walk_length": a.length,
                 "walk_steps": s1, "preprocess_s": prep1, "walk_s_1proc": t1,
                 "walk_steps_per_s_1proc": s1 / t1, "walk_s_8proc": t8, "walk_steps_8proc": s8,
                 "walk_steps_per_s_8proc": s8 / t8,
                 "sample": f"{gname}: simulate_walks({r}, {a.length}) walk loop only; preprocess "
                           f"{prep1:.1f} s untimed"}
            print(json.dumps(e), flush=True)
            cases.append(e)
    keep = [g for g in doc["graphs"] if (g["graph"], g["p"], g["q"]) not in {(c["graph"], c["p"], c["q"])
                                                                             for c in cases}]
    doc["graphs"] = keep + cases
    best = max(doc["graphs"], key=lambda x: x["walk_steps_per_s_8proc"])
    doc["summary"] = (f"reference node2vec.py walk loop on {doc['cpu_model']} ({doc['cores']} cores): "
                      + ", ".join(f"{g['graph']} p={g['p']} q={g['q']}: {g['walk_steps_per_s_1proc']:.3g} "
                                  f"(1 proc) / {g['walk_steps_per_s_8proc']:.3g} (8 procs) walk-steps/s"
                                  for g in doc["graphs"])
                      + f"; best 8-process rate {best['walk_steps_per_s_8proc']:.3g} walk-steps/s ({best['graph']})")
    json.dump(doc, open(out, "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main()
