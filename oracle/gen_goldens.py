"""Golden-vector generator for the H1 (node2vec) parity tests.

TEST INFRASTRUCTURE ONLY.  This script is run once, in the build container
(the only place `/root/reference` exists), and its outputs are committed under
`tests/golden/`.  It imports the reference's own `node2vec.py`
(/root/reference/node2vec/src/node2vec.py) and runs it exactly as the reference
driver does:

* graph construction restates `read_graph` (node2vec/src/main.py:76-89) with
  networkx calls only (main.py itself cannot be imported: gensim is absent);
* `np.int = int` is a harness-side shim for node2vec.py:125 under numpy>=1.24
  (no reference file is edited);
* seeding is `random.seed(S); np.random.seed(S)` before `simulate_walks`.

Nothing produced here is shipped or executed on the product path; the files
are data (inputs and expected outputs) read by `tests/`.

Usage:  python oracle/gen_goldens.py   (writes tests/golden/n2v_*.npz + index.json)
"""
import contextlib
import hashlib
import io
import json
import os
import random
import sys

import numpy as np

REF = "/root/reference/node2vec/src"
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")
DATA = os.path.join(GOLD, "data")


def _import_reference():
    sys.path.insert(0, REF)
    np.int = int  # shim for node2vec.py:125 (np.int removed in numpy 1.24)
    import node2vec  # noqa: E402  (the reference module)
    return node2vec


def read_graph(path, delimiter, weighted, directed):
    """Restatement of main.py:76-89 `read_graph` (networkx calls only)."""
    import networkx as nx
    if weighted:
        G = nx.read_edgelist(path, nodetype=int, data=(("weight", float),),
                             create_using=nx.DiGraph(), delimiter=delimiter)
    else:
        G = nx.read_edgelist(path, nodetype=int, create_using=nx.DiGraph(),
                             delimiter=delimiter)
        for edge in G.edges():
            G[edge[0]][edge[1]]["weight"] = 1
    if not directed:
        G = G.to_undirected()
    return G


def csr_by_label(G):
    """CSR in sorted-label node order, neighbours sorted by label (the order
    node2vec.py:25,67,94 draws over)."""
    labels = np.array(sorted(G.nodes()), dtype=np.int64)
    offs = [0]
    nbrs, wts = [], []
    for u in labels:
        ns = sorted(G.neighbors(int(u)))
        nbrs.extend(ns)
        wts.extend(float(G[int(u)][v]["weight"]) for v in ns)
        offs.append(len(nbrs))
    return labels, np.array(offs, np.int64), np.array(nbrs, np.int64), np.array(wts, np.float64)


def run_case(n2v, name, path, delimiter, weighted, directed, p, q, seed, r, L,
             full_walks=True, n_uniforms=1000):
    G = read_graph(path, delimiter, weighted, directed)
    labels, offs, nbrs, wts = csr_by_label(G)
    g = n2v.Graph(G, directed, p, q)
    g.preprocess_transition_probs()
    # alias tables in CSR order (nodes by sorted label; edges by CSR slot)
    aJ, aq, eJ, eq, eoff = [], [], [], [], [0]
    for i, u in enumerate(labels):
        J, qq = g.alias_nodes[int(u)]
        aJ.extend(int(x) for x in J)
        aq.extend(float(x) for x in qq)
        for v in nbrs[offs[i]:offs[i + 1]]:
            J, qq = g.alias_edges[(int(u), int(v))]
            eJ.extend(int(x) for x in J)
            eq.extend(float(x) for x in qq)
            eoff.append(len(eJ))
    # the reference's own walk generation, seeded as a caller would
    random.seed(seed)
    np.random.seed(seed)
    # record start orders by replaying the shuffle on a private generator that
    # mirrors the global one (random.shuffle on list(G.nodes()), cumulative)
    rs = random.Random(seed)
    nodes = list(G.nodes())
    starts = []
    for _ in range(r):
        rs.shuffle(nodes)
        starts.extend(nodes)
    with contextlib.redirect_stdout(io.StringIO()):
        walks = g.simulate_walks(r, L)
    W = np.full((len(walks), L), -1, dtype=np.int64)
    lens = np.zeros(len(walks), np.int64)
    for i, w in enumerate(walks):
        W[i, :len(w)] = w
        lens[i] = len(w)
    assert [w[0] for w in walks] == starts, "start-order replay mismatch"
    ru = np.random.RandomState(seed)
    uni = ru.random_sample(n_uniforms)
    out = dict(
        node_order=np.array(list(G.nodes()), np.int64),
        labels=labels, offsets=offs, nbrs=nbrs, weights=wts,
        alias_node_J=np.array(aJ, np.int64), alias_node_q=np.array(aq, np.float64),
        alias_edge_J=np.array(eJ, np.int64), alias_edge_q=np.array(eq, np.float64),
        alias_edge_off=np.array(eoff, np.int64),
        starts=np.array(starts, np.int64), lens=lens, uniforms=uni,
    )
    sha = hashlib.sha256(W.tobytes()).hexdigest()
    if full_walks:
        out["walks"] = W
    else:
        out["walks_head"] = W[:64]
        out["walks_tail"] = W[-64:]
        # drop the big alias-edge tables for the large case; keep a digest
        for k in ("alias_edge_J", "alias_edge_q", "alias_edge_off"):
            out[k + "_sha256"] = np.frombuffer(
                hashlib.sha256(out[k].tobytes()).digest(), np.uint8)
            del out[k]
    fn = f"n2v_{name}_p{p}_q{q}_s{seed}.npz"
    np.savez_compressed(os.path.join(GOLD, fn), **out)
    return dict(file=fn, graph=os.path.basename(path), delimiter=delimiter,
                weighted=weighted, directed=directed, p=p, q=q, seed=seed,
                num_walks=r, walk_length=L, n=int(len(labels)),
                nnz=int(len(nbrs)), walks_sha256=sha, full_walks=full_walks,
                total_steps=int((lens - 1).clip(min=0).sum()))


def write_synthetic():
    """Small synthetic edgelists for the quirk cases (seeded, committed)."""
    rng = np.random.RandomState(12345)
    # directed graph with sinks: 40 nodes, labels scattered, some sinks
    lines = []
    labels = rng.permutation(np.arange(100, 100 + 40))
    for i in range(120):
        u, v = rng.randint(0, 40, size=2)
        if u % 7 == 0:  # make every 7th node a sink (no out-edges)
            continue
        lines.append(f"{labels[u]} {labels[v]}")
    lines.append(f"{labels[3]} {labels[7]}")  # guarantee edges into sinks
    with open(os.path.join(DATA, "directed_sinks.edgelist"), "w") as f:
        f.write("\n".join(lines) + "\n")
    # weighted undirected with duplicates, reciprocal pairs (last-seen / node
    # order quirk of to_undirected), and a self loop
    lines = ["3 9 1.0", "1 3 5.0", "3 1 2.0", "9 9 0.5", "2 4 1.5", "4 2 3.5",
             "7 3 0.25", "9 1 4.0", "1 9 0.75", "2 7 1.0", "7 2 2.0", "5 6 1.0",
             "6 5 1.0", "5 1 3.0"]
    for _ in range(40):
        u, v = rng.randint(1, 12, size=2)
        lines.append(f"{u} {v} {rng.randint(1, 9) / 4.0}")
    with open(os.path.join(DATA, "weighted_quirks.edgelist"), "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    n2v = _import_reference()
    os.makedirs(GOLD, exist_ok=True)
    write_synthetic()
    D = DATA
    cases = []
    for seed in (0, 1, 7):
        for (p, q) in ((1, 1), (0.25, 4)):
            cases.append(run_case(n2v, "karate", f"{D}/karate.edgelist", " ",
                                  False, False, p, q, seed, 10, 80))
    cases.append(run_case(n2v, "directed_sinks", f"{D}/directed_sinks.edgelist",
                          " ", False, True, 0.5, 2, 3, 4, 12))
    cases.append(run_case(n2v, "weighted_quirks", f"{D}/weighted_quirks.edgelist",
                          " ", True, False, 2, 0.5, 5, 6, 15))
    cases.append(run_case(n2v, "moreno", f"{D}/moreno_crime_crime.txt", "\t",
                          False, False, 0.25, 4, 11, 2, 20))
    cases.append(run_case(n2v, "arxiv", f"{D}/arxiv_author_pub.txt", "\t",
                          False, False, 0.25, 4, 42, 1, 80, full_walks=False))
    with open(os.path.join(GOLD, "index.json"), "w") as f:
        json.dump(dict(generator="oracle/gen_goldens.py",
                       reference="node2vec/src/node2vec.py (imported)",
                       python=sys.version.split()[0], numpy=np.__version__,
                       networkx=__import__("networkx").__version__,
                       cases=cases), f, indent=1)
    print(json.dumps(cases, indent=1))


if __name__ == "__main__":
    main()
