"""GPU parity for node2vec (H1): the HIP kernels behind the C ABI against the
reference goldens (exact replay) and against the oracle (Philox scale mode)."""
import hashlib
import os
import random

import numpy as np
import pytest

from conftest import DATA, golden_index, load_golden

pytestmark = pytest.mark.gpu
CASES = golden_index()["cases"]


def _nx_graph(case):
    import networkx as nx
    path = os.path.join(DATA, case["graph"])
    if case["weighted"]:
        G = nx.read_edgelist(path, nodetype=int, data=(("weight", float),), create_using=nx.DiGraph(),
                             delimiter=case["delimiter"])
    else:
        G = nx.read_edgelist(path, nodetype=int, create_using=nx.DiGraph(), delimiter=case["delimiter"])
        for e in G.edges():
            G[e[0]][e[1]]["weight"] = 1
    if not case["directed"]:
        G = G.to_undirected()
    return G


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["file"])
def test_replay_mirror_matches_reference(case, gw):
    """gwamd.node2vec.Graph (drop-in for node2vec.Graph) reproduces the
    reference walks bit-for-bit from the same seeds, and advances the global
    RNG states exactly as the reference does."""
    from gwamd import node2vec
    g = load_golden(case["file"])
    G = _nx_graph(case)
    random.seed(case["seed"])
    np.random.seed(case["seed"])
    n2v = node2vec.Graph(G, case["directed"], case["p"], case["q"])
    n2v.preprocess_transition_probs()
    walks = n2v.simulate_walks(case["num_walks"], case["walk_length"])
    L = case["walk_length"]
    W = np.full((len(walks), L), -1, np.int64)
    for i, w in enumerate(walks):
        W[i, :len(w)] = w
    assert hashlib.sha256(W.tobytes()).hexdigest() == case["walks_sha256"]
    if case["full_walks"]:
        np.testing.assert_array_equal(W, g["walks"])
    # global stream advanced by exactly 2 uniforms per step
    ref = np.random.RandomState(case["seed"])
    ref.random_sample(2 * int((g["lens"] - 1).sum()))
    assert np.random.random_sample() == ref.random_sample()
    # alias tables exposed like the reference dicts
    lab = g["labels"]
    u = int(lab[0])
    J, q = n2v.alias_nodes[u]
    b, e = g["offsets"][0], g["offsets"][1]
    np.testing.assert_array_equal(J, g["alias_node_J"][b:e])
    assert q.tobytes() == g["alias_node_q"][b:e].tobytes()


@pytest.mark.parametrize("case", [c for c in CASES if c["full_walks"]], ids=lambda c: c["file"])
def test_gpu_alias_tables_bitwise(case, gw):
    """k_alias_nodes / k_alias_edges == reference alias tables, bitwise."""
    from gwamd import _lib as C
    g = load_golden(case["file"])
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, case["graph"]), case["delimiter"], "nx",
                                 case["directed"], case["weighted"]).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(case["p"]), float(case["q"]), C.N2V_REPLAY), G.handle)
    inf = G.info()
    nJ = np.empty(inf.nnz, np.int32)
    nq = np.empty(inf.nnz, np.float64)
    eoff = np.empty(inf.nnz + 1, np.int64)
    eJ = np.empty(inf.edge_alias_entries, np.int32)
    eq = np.empty(inf.edge_alias_entries, np.float64)
    C.check(C.lib().gw_n2v_export_alias(G.handle, C.ptr(nJ), C.ptr(nq), C.ptr(eoff), C.ptr(eJ), C.ptr(eq)),
            G.handle)
    np.testing.assert_array_equal(nJ, g["alias_node_J"])
    assert nq.tobytes() == g["alias_node_q"].tobytes()
    np.testing.assert_array_equal(eoff, g["alias_edge_off"])
    np.testing.assert_array_equal(eJ, g["alias_edge_J"])
    assert eq.tobytes() == g["alias_edge_q"].tobytes()


def test_alias_setup_standalone(gw, oracle):
    from gwamd.node2vec import alias_setup
    rng = np.random.RandomState(5)
    for K in (1, 2, 3, 7, 49, 1000):
        p = rng.rand(K)
        p /= p.sum()
        J, q = alias_setup(p)
        J2, q2 = oracle.alias_setup(p)
        np.testing.assert_array_equal(J, J2)
        assert q.tobytes() == q2.tobytes()


def _scale_case(gw, oracle, path, delim, directed, weighted, p, q, seed, L, begin, count, shuffle=True):
    import torch
    from gwamd import _lib as C
    G = gw.GWGraph.from_edgelist(path, delim, "nx", directed, weighted).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), C.N2V_REJECTION), G.handle)
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, seed, begin, count, int(shuffle), C.ptr(out), C.ptr(lens),
                                 C.ptr(cnt), None), G.handle)
    torch.cuda.synchronize()
    csr = G.export_csr()
    o2, l2, c2 = oracle.walks_scale(csr if weighted else dict(csr, weights=None), p, q, seed, L, begin,
                                    count, shuffle=shuffle, directed=directed, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), o2)
    np.testing.assert_array_equal(lens.cpu().numpy(), l2)
    assert int(cnt[0]) == int(c2[0]) and int(cnt[1]) == int(c2[1])
    return out.cpu().numpy(), csr


@pytest.mark.parametrize("p,q", [(1, 1), (0.25, 4), (1, 0.5), (4, 0.25), (2, 1)])
@pytest.mark.parametrize("graph,delim", [("karate.edgelist", " "), ("moreno_crime_crime.txt", "\t"),
                                         ("arxiv_author_pub.txt", "\t")])
def test_scale_walks_gpu_equals_oracle(gw, oracle, graph, delim, p, q):
    n = {"karate.edgelist": 34, "moreno_crime_crime.txt": 1380, "arxiv_author_pub.txt": 38741}[graph]
    count = min(3 * n, 50000)
    _scale_case(gw, oracle, os.path.join(DATA, graph), delim, False, False, p, q, 1234, 40, n // 3, count)


@pytest.mark.parametrize("directed,weighted,graph", [(True, False, "directed_sinks.edgelist"),
                                                     (False, True, "weighted_quirks.edgelist")])
def test_scale_walks_directed_weighted(gw, oracle, directed, weighted, graph):
    for (p, q) in [(1, 1), (0.5, 2), (0.25, 4)]:
        _scale_case(gw, oracle, os.path.join(DATA, graph), " ", directed, weighted, p, q, 99, 25, 0, 500)


def test_scale_walks_shard_invariance_and_properties(gw, oracle):
    """Output is a pure function of the global walk index: any shard split
    gives the same walks; every step follows an edge; each iteration starts
    every vertex exactly once (per-iteration keyed permutation)."""
    import torch
    from gwamd import _lib as C
    G = gw.GWGraph.rmat(14, 16, seed=7).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, 0.25, 4.0, C.N2V_REJECTION), G.handle)
    n = G.n
    L = 20
    tot = 2 * n
    full = torch.empty((tot, L), dtype=torch.int32, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 5, 0, tot, 1, C.ptr(full), None, None, None), G.handle)
    parts = []
    for b, e in [(0, 777), (777, n + 5), (n + 5, tot)]:
        t = torch.empty((e - b, L), dtype=torch.int32, device="cuda")
        C.check(C.lib().gw_n2v_walks(G.handle, L, 5, b, e - b, 1, C.ptr(t), None, None, None), G.handle)
        parts.append(t)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(torch.cat(parts).cpu().numpy(), full.cpu().numpy())
    W = full.cpu().numpy()
    csr = G.export_csr()
    offs, nbrs = csr["offsets"], csr["nbrs"]
    for it in range(2):
        starts = np.sort(W[it * n:(it + 1) * n, 0])
        np.testing.assert_array_equal(starts, np.arange(n))
    a, b = W[:, :-1].ravel(), W[:, 1:].ravel()
    ok = np.array([np.searchsorted(nbrs[offs[x]:offs[x + 1]], y) < offs[x + 1] - offs[x] and
                   nbrs[offs[x] + np.searchsorted(nbrs[offs[x]:offs[x + 1]], y)] == y
                   for x, y in zip(a[:20000], b[:20000])])
    assert ok.all()
    # oracle parity on a random window
    o2, _, _ = oracle.walks_scale(dict(csr, weights=None), 0.25, 4.0, 5, L, 1000, 3000, nthreads=8)
    np.testing.assert_array_equal(W[1000:4000], o2)


def test_replay_capi_from_loader(gw, oracle):
    """C-ABI replay path on the C++-parsed graph == oracle replay."""
    from gwamd import _lib as C
    case = [c for c in CASES if c["file"].startswith("n2v_moreno")][0]
    g = load_golden(case["file"])
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, case["graph"]), "\t", "nx").to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, case["p"], case["q"], C.N2V_REPLAY), G.handle)
    csr = G.export_csr()
    rank = {int(x): i for i, x in enumerate(csr["labels"])}
    starts = np.array([rank[int(x)] for x in g["starts"]], np.int32)
    L = case["walk_length"]
    U = np.random.RandomState(case["seed"]).random_sample(2 * (L - 1) * len(starts))
    out = np.empty((len(starts), L), np.int32)
    lens = np.empty(len(starts), np.int32)
    used = C.I64(0)
    C.check(C.lib().gw_n2v_walks_replay(G.handle, L, len(starts), C.ptr(starts), C.ptr(U), len(U), C.ptr(out),
                                        C.ptr(lens), C.ctypes.byref(used)), G.handle)
    np.testing.assert_array_equal(csr["labels"][out], g["walks"])
    assert used.value == 2 * int((g["lens"] - 1).sum())


def test_replay_refuses_huge_edge_tables(gw):
    from gwamd import _lib as C
    G = gw.GWGraph.rmat(18, 16, seed=1).to_device(0)
    with pytest.raises(C.CapacityError):
        C.check(C.lib().gw_n2v_prepare(G.handle, 0.25, 4.0, C.N2V_REPLAY), G.handle)


def test_cli_replay_and_scale(gw, tmp_path):
    """gwamd.cli (main.py flags): replay mode writes the reference walks in
    DeepSim's save_list format; scale mode writes walks that follow edges."""
    from gwamd import cli, io
    g = load_golden("n2v_karate_p0.25_q4_s7.npz")
    out = tmp_path / "walks.txt"
    assert cli.main(["--input", os.path.join(DATA, "karate.edgelist"), "--delimiter", " ", "--p", "0.25",
                     "--q", "4", "--seed", "7", "--walks", str(out)]) == 0
    got = io.read_list(str(out))
    assert [[int(x) for x in w] for w in got] == g["walks"].tolist()
    out2 = tmp_path / "w2.npy"
    assert cli.main(["--input", os.path.join(DATA, "karate.edgelist"), "--delimiter", " ", "--p", "0.25",
                     "--q", "4", "--seed", "7", "--mode", "scale", "--walks", str(out2)]) == 0
    W = np.load(str(out2))
    assert W.shape == (340, 80)
    adj = set()
    for line in open(os.path.join(DATA, "karate.edgelist")):
        a, b = map(int, line.split())
        adj.add((a, b))
        adj.add((b, a))
    assert all((int(a), int(b)) in adj for a, b in zip(W[:, :-1].ravel(), W[:, 1:].ravel()))


@pytest.mark.parametrize("p,q", [(0.25, 4), (1, 0.5), (4, 0.25), (2, 1), (1, 1)])
@pytest.mark.parametrize("graph", ["karate", "moreno", "arxiv", "rmat12"])
def test_bitset_walks_gpu_equals_oracle(gw, oracle, graph, p, q):
    """GW_N2V_BITSET (per-edge common-neighbour bitsets) == oracle restatement."""
    import torch
    from gwamd import _lib as C
    if graph == "rmat12":
        G = gw.GWGraph.rmat(12, 16, seed=11)
    else:
        f, dl = {"karate": ("karate.edgelist", " "), "moreno": ("moreno_crime_crime.txt", "\t"),
                 "arxiv": ("arxiv_author_pub.txt", "\t")}[graph]
        G = gw.GWGraph.from_edgelist(os.path.join(DATA, f), dl, "nx")
    G.to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), C.N2V_BITSET), G.handle)
    n = G.n
    L = 30
    begin, count = n // 2, min(3 * n, 40000)
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 77, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    csr = G.export_csr()
    if p == 1 and q == 1:
        ref, rl, rc = oracle.walks_scale(dict(csr, weights=None), p, q, 77, L, begin, count, nthreads=8)
    else:
        ref, rl, rc = oracle.walks_bitset(csr, p, q, 77, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])


def test_bitset_refused_for_weighted_or_directed(gw):
    from gwamd import _lib as C
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "weighted_quirks.edgelist"), " ", "nx", False, True).to_device(0)
    with pytest.raises(C.UnsupportedError):
        C.check(C.lib().gw_n2v_prepare(G.handle, 0.5, 2.0, C.N2V_BITSET), G.handle)


def _mixed_mode_edgelist(path):
    """Unweighted graph whose slots exercise every bitset payload and build
    path: superhubs (deg ~2000) and a dense core (deg ~300-400) give region
    payloads built by the wave kernel from either row; periphery vertices
    (deg 25-60) give list / Elias-Fano / region payloads built by one thread
    from the shorter row; self-loops on hubs, core and periphery."""
    rng = np.random.default_rng(2024)
    n, hubs, core = 2600, 10, 600
    E = set()
    for h in range(hubs):
        for v in np.nonzero(rng.random(n) < 0.8)[0]:
            if v != h:
                E.add((min(h, v), max(h, v)))
    for i in range(hubs, core):
        for j in np.nonzero(rng.random(core - i - 1) < 0.5)[0] + i + 1:
            E.add((i, int(j)))
    for u in range(core, n):
        for v in rng.choice(n, int(rng.integers(25, 61)), replace=False):
            if v != u:
                E.add((min(u, int(v)), max(u, int(v))))
    for v in list(range(0, 5)) + list(range(10, 41)) + list(range(600, 611)):
        E.add((v, v))
    with open(path, "w") as f:
        for a, b in sorted(E):
            f.write(f"{a} {b}\n")


@pytest.mark.parametrize("p,q", [(0.25, 4), (4, 0.25)])
def test_bitset_mixed_payload_modes_equal_oracle(gw, oracle, tmp_path, p, q):
    import torch
    from gwamd import _lib as C
    path = str(tmp_path / "mixed.edgelist")
    _mixed_mode_edgelist(path)
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), C.N2V_BITSET), G.handle)
    info = G.info()
    assert info.sampler_bytes > info.nnz * 64  # some slots hold regions
    n, L = G.n, 30
    begin, count = 123, 20000
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 5, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    ref, rl, rc = oracle.walks_bitset(G.export_csr(), p, q, 5, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])
    assert n == 2600


def _hub_edgelist(path):
    """A hub of degree 5,999 (> 4096: its regions keep the popcount directory
    in memory, the select path that reads directory words first) over a
    random graph of ~30 edges per vertex, so hub slots have many common
    neighbours (region payloads) and the periphery has list / Elias-Fano ones."""
    rng = np.random.default_rng(77)
    n = 6000
    E = {(0, v) for v in range(1, n)}
    for u in range(1, n):
        for v in rng.choice(np.arange(1, n), 15, replace=False):
            if v != u:
                E.add((min(u, int(v)), max(u, int(v))))
    with open(path, "w") as f:
        for a, b in sorted(E):
            f.write(f"{a} {b}\n")


def _multichunk_hub_edgelist(path):
    """Hub 0 of degree 13,999 (four 4,096-id hash chunks in the build) and a
    second hub 1 adjacent to ids 2..7000, so slot (0 -> 1) / (1 -> 0) has
    ~7,000 common neighbours spread over two of hub 0's chunks (region bits of
    the (v -> u) slot from several chunk windows, payloads OR-merged across
    chunks).  Every other vertex links to 8 ids within +-300 of itself, so the
    stream of N(v) for an edge (0, v) has nothing in most of hub 0's chunks:
    the build skips those (per-edge next element), which only happens for
    hubs with three or more chunks."""
    rng = np.random.default_rng(99)
    n = 14000
    E = {(0, v) for v in range(1, n)}
    E |= {(1, v) for v in range(2, 7001)}
    for u in range(2, n):
        lo, hi = max(2, u - 300), min(n - 1, u + 300)
        for v in rng.integers(lo, hi + 1, 8):
            if int(v) != u:
                E.add((min(u, int(v)), max(u, int(v))))
    with open(path, "w") as f:
        for a, b in sorted(E):
            f.write(f"{a} {b}\n")


@pytest.mark.parametrize("mode", ["bitset", "rejection"])
@pytest.mark.parametrize("p,q", [(0.25, 4), (4, 0.25)])
def test_multichunk_hub_builds_equal_oracle(gw, oracle, tmp_path, mode, p, q):
    """Walks over tables built for hubs spanning 4 hash chunks (chunk skips,
    cross-chunk merges) equal the oracle: bitset tables and the listed
    rejection sampler's lists-only build."""
    import torch
    from gwamd import _lib as C
    path = str(tmp_path / "mchub.edgelist")
    _multichunk_hub_edgelist(path)
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    if mode == "rejection":
        G.options(listed=1)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q),
                                   C.N2V_BITSET if mode == "bitset" else C.N2V_REJECTION), G.handle)
    inf = G.info()
    assert inf.max_degree > 3 * 4096
    if mode == "rejection":
        assert inf.listed == (1 if q < 1 else 0)  # q > 1: the mixture proposal needs no listed entries
    L, begin, count = 30, 123, 6000
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 5, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    csr = G.export_csr()
    if mode == "bitset":
        ref, rl, rc = oracle.walks_bitset(csr, p, q, 5, L, begin, count, nthreads=8)
    else:
        ref, rl, rc = oracle.walks_scale(dict(csr, weights=None), p, q, 5, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])
    o = out.cpu().numpy()
    assert (o == 0).sum() > count // 2 and (o == 1).sum() > 0  # the walks do pass through both hubs
    G.free()


@pytest.mark.parametrize("p,q", [(0.25, 4), (4, 0.25)])
def test_bitset_directory_hub_equals_oracle(gw, oracle, tmp_path, p, q):
    import torch
    from gwamd import _lib as C
    path = str(tmp_path / "hub.edgelist")
    _hub_edgelist(path)
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), C.N2V_BITSET), G.handle)
    assert G.info().max_degree > 4096
    L, begin, count = 30, 777, 4000
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 11, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    ref, rl, rc = oracle.walks_bitset(G.export_csr(), p, q, 11, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])
    assert (out.cpu().numpy() == 0).sum() > count // 8  # the hub (dense id 0) is visited often


def _selfloop_sparse_edgelist(path):
    """Sparse graph (a random tree plus a few extra edges, mean degree ~2.6)
    with self-loops on a third of the vertices: many edges u -> x with no
    common neighbour next to a self-looped u, where c(u -> x) = 0 but
    c(x -> u) = 1 (u's own loop) — the case the return elision must not
    stash.  Starts with the minimal instance (0,0), (0,1), (1,2)."""
    rng = np.random.default_rng(303)
    n = 3000
    E = {(0, 0), (0, 1), (1, 2)}
    for v in range(3, n):
        E.add((int(rng.integers(0, v)), v))
    for _ in range(n // 3):
        a, b = sorted(int(x) for x in rng.integers(0, n, 2))
        if a != b:
            E.add((a, b))
    for v in rng.choice(n, n // 3, replace=False):
        E.add((int(v), int(v)))
    with open(path, "w") as f:
        for a, b in sorted(E):
            f.write(f"{a} {b}\n")


def _ef_bucket_edgelist(path):
    """A hub (vertex 0) over leaves 1..3000 plus 45 vertices u_j = 3001 + j,
    each adjacent to the hub and to 43 consecutive leaves 64(j+1)+1 ..
    64(j+1)+43: slot (u_j -> 0) has c = 43 common neighbours in N(0)
    (deg 3045), an Elias-Fano payload with l = 6 whose bucket j+1 holds all
    43 of them — a run of more than 32 ones in the unary high parts."""
    E = {(0, v) for v in range(1, 3001)}
    for j in range(45):
        u = 3001 + j
        E.add((0, u))
        for v in range(64 * (j + 1) + 1, 64 * (j + 1) + 44):
            E.add((v, u))
    with open(path, "w") as f:
        for a, b in sorted(E):
            f.write(f"{a} {b}\n")


@pytest.mark.parametrize("mode", ["bitset", "rejection"])
@pytest.mark.parametrize("graph", ["selfloop_sparse", "ef_bucket"])
@pytest.mark.parametrize("p,q", [(0.25, 4), (4, 0.25)])
def test_bitset_edge_payloads_equal_oracle(gw, oracle, tmp_path, mode, graph, p, q):
    """Payload corner cases against the oracle: (a) return elision next to a
    self-looped vertex (the stash is valid only when the reverse slot has no
    common neighbour either); (b) an Elias-Fano bucket with more than 32
    elements (membership must read past the first 32-bit window).  Both the
    bitset kernel and the listed rejection sampler (same payloads)."""
    import torch
    from gwamd import _lib as C
    path = str(tmp_path / f"{graph}.edgelist")
    (_selfloop_sparse_edgelist if graph == "selfloop_sparse" else _ef_bucket_edgelist)(path)
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q),
                                   C.N2V_BITSET if mode == "bitset" else C.N2V_REJECTION), G.handle)
    n, L = G.n, 40
    begin, count = 5, 30 * n
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 9, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    csr = G.export_csr()
    if mode == "bitset":
        ref, rl, rc = oracle.walks_bitset(csr, p, q, 9, L, begin, count, nthreads=8)
    else:
        ref, rl, rc = oracle.walks_scale(dict(csr, weights=None), p, q, 9, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])
    G.free()


@pytest.mark.parametrize("p,q", [(1, 0.5), (0.25, 4), (1, 1)])
def test_rejection_rmat_equals_oracle(gw, oracle, p, q):
    """Rejection sampler (slot entries + per-row neighbour hash sets) and the
    first-order kernel on a power-law graph with hubs, walk windows and
    counters against the oracle."""
    import torch
    from gwamd import _lib as C
    G = gw.GWGraph.rmat(14, 16, 0.57, 0.19, 0.19, 3).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), C.N2V_REJECTION), G.handle)
    info = G.info()
    assert info.sampler_bytes >= info.nnz * 16  # slot entries built
    L, begin, count = 40, 3 * G.n + 5, 6000
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 21, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    ref, rl, rc = oracle.walks_scale(dict(G.export_csr(), weights=None), p, q, 21, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])


@pytest.mark.parametrize("graph", ["mixed", "hub"])
@pytest.mark.parametrize("p,q", [(1, 0.5), (0.25, 0.5), (4, 0.25)])
def test_rejection_listed_entries_equal_oracle(gw, oracle, tmp_path, graph, p, q):
    """k_walk_listed (REJECTION on an unweighted undirected graph): the lazy
    has_edge(x, prev) test answered from the list / inline / Elias-Fano
    payload of the entry that led to cur, region-size common sets and the
    outlier return (p < 1, no entry read) falling back to the neighbour-hash
    probe — the same walks as k_walk_scale, i.e. the oracle's walks_scale."""
    import torch
    from gwamd import _lib as C
    path = str(tmp_path / f"{graph}.edgelist")
    (_mixed_mode_edgelist if graph == "mixed" else _hub_edgelist)(path)
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), C.N2V_REJECTION), G.handle)
    info = G.info()
    assert info.sampler_bytes >= info.nnz * 64  # listed 64 B entries built
    L, begin, count = 30, 4 * G.n + 9, 12000
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 31, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    ref, rl, rc = oracle.walks_scale(dict(G.export_csr(), weights=None), p, q, 31, L, begin, count, nthreads=8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(lens.cpu().numpy(), rl)
    assert int(cnt[0]) == int(rc[0]) and int(cnt[1]) == int(rc[1])
    G.free()


@pytest.mark.parametrize("listed", [-1, 1])
def test_no_listed_entries_at_q_ge_1(gw, oracle, listed):
    """q >= 1: the rejection sampler never builds listed entries, whatever
    gw_options_t.listed says (q > 1 takes the mixture proposal, which has no
    lazy has_edge probe for them to answer; q = 1 has no probe at all), so the
    walks never depend on the option: == oracle.walks_scale."""
    import torch
    from gwamd import _lib as C
    G = gw.GWGraph.rmat(12, 16, 0.57, 0.19, 0.19, 9).to_device(0)
    G.options(listed=listed)
    for p, q in [(0.25, 4.0), (2.0, 1.0)]:
        C.check(C.lib().gw_n2v_prepare(G.handle, p, q, C.N2V_REJECTION), G.handle)
        assert G.info().listed == 0
        out = torch.empty((3000, 20), dtype=torch.int32, device="cuda")
        C.check(C.lib().gw_n2v_walks(G.handle, 20, 4, 100, 3000, 1, C.ptr(out), None, None, None), G.handle)
        torch.cuda.synchronize()
        ref, _, _ = oracle.walks_scale(dict(G.export_csr(), weights=None), p, q, 4, 20, 100, 3000, nthreads=4)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_native_comm_single_rank_allgather(gw):
    """gw_comm (RCCL loaded at run time): a one-rank communicator gathers
    int32 walk blocks and float64 score blocks unchanged."""
    import torch
    from gwamd import dist
    c = dist.NativeComm(dist.NativeComm.unique_id(), 1, 0, 0)
    try:
        w = torch.arange(12345, dtype=torch.int32, device="cuda")
        r = torch.empty_like(w)
        c.allgather(w, r, torch.cuda.current_stream())
        s = torch.rand(777, dtype=torch.float64, device="cuda")
        rs = torch.empty_like(s)
        c.allgather(s, rs)
        torch.cuda.synchronize()
        assert torch.equal(w, r) and torch.equal(s, rs)
    finally:
        c.close()


def test_cli_scale_two_ranks_equal_one(gw, tmp_path):
    """gwamd.cli --mode scale under torchrun: two ranks (gloo rehearsal on one
    GPU; RCCL on a multi-GPU node) walk their blocks and rank 0 writes a file
    byte-identical to the one-process run."""
    import socket
    import subprocess
    import sys
    from gwamd import cli
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-embedding_amd")
    common = ["--input", os.path.join(DATA, "moreno_crime_crime.txt"), "--delimiter", "\t", "--p", "0.25",
              "--q", "4", "--seed", "3", "--mode", "scale", "--num-walks", "3", "--walk-length", "30"]
    one = tmp_path / "one.txt"
    assert cli.main(common + ["--walks", str(one)]) == 0
    two = tmp_path / "two.txt"
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=pkg + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "gwamd.cli"] + common +
                       ["--walks", str(two), "--dist-backend", "gloo"], env=env, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    assert one.read_bytes() == two.read_bytes()


@pytest.mark.parametrize("sampler", ["auto", "rejection"])
def test_cli_scale_two_ranks_fail_together(gw, tmp_path, sampler):
    """A prepare that fails (p = 0: node2vec.py:70-76 divides by p) makes
    EVERY rank raise, promptly: under --sampler auto rank 0 broadcasts the
    failure sentinel instead of a mode, otherwise the ranks all-reduce a
    success flag before any walk collective (the other ranks used
    to wait in a collective until the NCCL timeout)."""
    import socket
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-embedding_amd")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=pkg + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "gwamd.cli",
                        "--input", os.path.join(DATA, "karate.edgelist"), "--delimiter", " ", "--p", "0",
                        "--q", "4", "--mode", "scale", "--sampler", sampler, "--num-walks", "1",
                        "--walks", str(tmp_path / "w.txt"), "--dist-backend", "gloo"],
                       env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode != 0
    assert r.stderr.count("p and q must be > 0") + r.stderr.count("failed to prepare") >= 2, r.stderr[-3000:]
    assert not (tmp_path / "w.txt").exists()


@pytest.mark.parametrize("mode", ["bitset", "rejection"])
def test_walks_host_pipeline_equals_device(gw, mode, monkeypatch):
    """gw_n2v_walks_host (chunked, kernel/copy overlapped on two streams):
    identical walks, lengths and counters to one device-buffer call, with
    small chunks so the double buffering wraps many times."""
    import torch
    from gwamd import _lib as C
    G = gw.GWGraph.rmat(13, 16, 0.57, 0.19, 0.19, 5).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, 0.25, 4.0, C.N2V_BITSET if mode == "bitset" else C.N2V_REJECTION),
            G.handle)
    L, begin, count = 40, 1234, 30001
    out = torch.empty((count, L), dtype=torch.int32, device="cuda")
    lens = torch.empty(count, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 9, begin, count, 1, C.ptr(out), C.ptr(lens), C.ptr(cnt), None),
            G.handle)
    torch.cuda.synchronize()
    G.options(host_chunk_bytes=1 << 20)  # 6,553 walks per chunk: 5 chunks
    W = np.empty((count, L), np.int32)
    ln = np.empty(count, np.int32)
    hc = np.zeros(2, np.uint64)
    C.check(C.lib().gw_n2v_walks_host(G.handle, L, 9, begin, count, 1, C.ptr(W), C.ptr(ln), C.ptr(hc)), G.handle)
    np.testing.assert_array_equal(W, out.cpu().numpy())
    np.testing.assert_array_equal(ln, lens.cpu().numpy())
    assert int(hc[0]) == int(cnt[0]) and int(hc[1]) == int(cnt[1])


@pytest.mark.parametrize("mode,p,q", [("bitset", 0.25, 4), ("rejection", 1, 0.5), ("rejection", 1, 1)])
def test_walk_shapes_edge_cases(gw, oracle, mode, p, q):
    """Partial waves and blocks (1, 63, 65, 257 walks), walk lengths around
    the 16-position flush (1, 15, 16, 17, 33) and zero walks: every sampler
    equals the oracle, including the cooperative flush's tail handling."""
    import torch
    from gwamd import _lib as C
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "moreno_crime_crime.txt"), "\t", "nx").to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q),
                                   C.N2V_BITSET if mode == "bitset" else C.N2V_REJECTION), G.handle)
    csr = G.export_csr()
    C.check(C.lib().gw_n2v_walks(G.handle, 8, 1, 0, 0, 1, None, None, None, None), G.handle)  # no walks: no-op
    for count in (1, 63, 65, 257):
        for L in (1, 15, 16, 17, 33):
            begin = 7 * count + L
            out = torch.full((count, L), -7, dtype=torch.int32, device="cuda")
            lens = torch.empty(count, dtype=torch.int32, device="cuda")
            C.check(C.lib().gw_n2v_walks(G.handle, L, 13, begin, count, 1, C.ptr(out), C.ptr(lens), None, None),
                    G.handle)
            torch.cuda.synchronize()
            if mode == "bitset":
                ref, rl, _ = oracle.walks_bitset(csr, p, q, 13, L, begin, count, nthreads=4)
            else:
                ref, rl, _ = oracle.walks_scale(dict(csr, weights=None), p, q, 13, L, begin, count, nthreads=4)
            np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"count={count} L={L}")
            np.testing.assert_array_equal(lens.cpu().numpy(), rl)


def test_calls_run_on_the_graph_device_and_keep_the_callers(gw, oracle):
    """Every C-ABI call runs on the graph's device and restores the caller's
    current device: the graph lives on the LAST visible device while
    the caller's current device is 0, the walk launch uses the NULL stream, and
    the walks still equal the oracle (on a one-GPU box both are device 0)."""
    import torch
    from gwamd import _lib as C
    dev = torch.cuda.device_count() - 1
    torch.cuda.set_device(0)
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "karate.edgelist"), " ", "nx").to_device(dev)
    assert torch.cuda.current_device() == 0
    C.check(C.lib().gw_n2v_prepare(G.handle, 0.25, 4.0, C.N2V_REJECTION), G.handle)
    assert torch.cuda.current_device() == 0
    nw, L = 200, 20
    out = torch.empty((nw, L), dtype=torch.int32, device=f"cuda:{dev}")
    C.check(C.lib().gw_n2v_walks(G.handle, L, 3, 0, nw, 1, C.ptr(out), None, None, None), G.handle)
    assert torch.cuda.current_device() == 0
    torch.cuda.synchronize(dev)
    ref, _, _ = oracle.walks_scale(dict(G.export_csr(), weights=None), 0.25, 4.0, 3, L, 0, nw)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    G.free()
    assert torch.cuda.current_device() == 0


def test_replay_sink_heavy_directed_many_walks(gw, oracle):
    """MT-replay on a directed graph where many walks stop at sinks (each one
    shifts the uniform offsets of every later walk): 200 walks per vertex ==
    the oracle's sequential replay, and the offset fixed point converges in a
    few passes (one pass per early-stopping walk was O(walks^2))."""
    import time
    from gwamd import _lib as C
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "directed_sinks.edgelist"), " ", "nx", True).to_device(0)
    C.check(C.lib().gw_n2v_prepare(G.handle, 0.5, 2.0, C.N2V_REPLAY), G.handle)
    csr = G.export_csr()
    n, nnz = G.n, G.nnz
    inf = G.info()
    nJ = np.empty(nnz, np.int32)
    nq = np.empty(nnz, np.float64)
    eoff = np.empty(nnz + 1, np.int64)
    C.check(C.lib().gw_n2v_export_alias(G.handle, C.ptr(nJ), C.ptr(nq), C.ptr(eoff), None, None), G.handle)
    ne = int(eoff[-1])
    eJ = np.empty(ne, np.int32)
    eq = np.empty(ne, np.float64)
    C.check(C.lib().gw_n2v_export_alias(G.handle, C.ptr(nJ), C.ptr(nq), C.ptr(eoff), C.ptr(eJ), C.ptr(eq)), G.handle)
    L = 20
    starts = np.tile(csr["node_order"], 200).astype(np.int32)
    U = np.random.RandomState(9).random_sample(2 * (L - 1) * len(starts))
    out = np.empty((len(starts), L), np.int32)
    lens = np.empty(len(starts), np.int32)
    used = C.I64(0)
    t0 = time.perf_counter()
    C.check(C.lib().gw_n2v_walks_replay(G.handle, L, len(starts), C.ptr(starts), C.ptr(U), len(U), C.ptr(out),
                                        C.ptr(lens), C.ctypes.byref(used)), G.handle)
    dt = time.perf_counter() - t0
    ref, rl, rused = oracle.walks_replay(csr["offsets"], csr["nbrs"], nJ, nq, eoff, eJ, eq, L, starts, U)
    assert (rl < L).sum() > len(starts) // 4  # sink-heavy: many walks stop early
    np.testing.assert_array_equal(out, ref)
    np.testing.assert_array_equal(lens, rl)
    assert used.value == rused
    assert dt < 20.0, dt
    del inf


def test_auto_sampler_choice_by_end_to_end_model(gw):
    """GW_N2V_AUTO: with the walk steps announced (gw_options_t.expected_steps)
    the library takes the rejection sampler when the bitset build cannot pay
    back and the bitset sampler when it can; unknown steps (0) keep the
    throughput choice (bitset); weighted graphs always take rejection; the
    choice is deterministic (pilot trials are counted, not timed)."""
    from gwamd import _lib as C
    G = gw.GWGraph.rmat(17, 16, seed=5).to_device(0)
    picks = []
    for steps in (0, 10**6, 10**13, 10**6):
        G.options(expected_steps=steps)
        C.check(C.lib().gw_n2v_prepare(G.handle, 0.25, 4.0, C.N2V_AUTO), G.handle)
        picks.append(G.info().n2v_mode)
    assert picks == [C.N2V_BITSET, C.N2V_REJECTION, C.N2V_BITSET, C.N2V_REJECTION], picks
    W = gw.GWGraph.from_edgelist(os.path.join(DATA, "weighted_quirks.edgelist"), " ", "nx", False, True).to_device(0)
    W.options(expected_steps=10**13)
    C.check(C.lib().gw_n2v_prepare(W.handle, 0.5, 2.0, C.N2V_AUTO), W.handle)
    assert W.info().n2v_mode == C.N2V_REJECTION
    # listed entries: never for q >= 1 under a known step count, on for q < 1 when they pay back
    G.options(expected_steps=10**6, listed=-1)
    C.check(C.lib().gw_n2v_prepare(G.handle, 1.0, 0.5, C.N2V_REJECTION), G.handle)
    assert G.info().listed == 0
    G.options(expected_steps=10**14)
    C.check(C.lib().gw_n2v_prepare(G.handle, 1.0, 0.5, C.N2V_REJECTION), G.handle)
    assert G.info().listed == 1
    G.options(expected_steps=10**14)
    C.check(C.lib().gw_n2v_prepare(G.handle, 0.25, 4.0, C.N2V_REJECTION), G.handle)
    assert G.info().listed == 0


def test_dropin_scale_mode_routes_through_auto(gw, oracle):
    """node2vec.Graph(..., mode="scale") defers the sampler to simulate_walks
    and prepares it with GW_N2V_AUTO for num_walks * n * (L - 1) steps
    (node2vec.py:83-113 then :41-59): at q = 4 with enough walks to pay the
    build back it takes the bitset sampler and returns exactly the bitset
    walks (== oracle); sampler="rejection" forces the rejection walks."""
    import networkx as nx
    from gwamd import _lib as C
    from gwamd import node2vec
    nxg = nx.read_edgelist(os.path.join(DATA, "moreno_crime_crime.txt"), nodetype=int, create_using=nx.DiGraph(),
                           delimiter="\t")
    for e in nxg.edges():
        nxg[e[0]][e[1]]["weight"] = 1
    nxg = nxg.to_undirected()
    n, L, r = nxg.number_of_nodes(), 40, 200
    G = node2vec.Graph(nxg, False, 0.25, 4.0, mode="scale", seed=11)
    G.preprocess_transition_probs()
    assert G.scale_sampler is None  # nothing built before the step count is known
    walks = G.simulate_walks(r, L)
    assert G.scale_sampler == C.N2V_BITSET
    assert G._g.options()["expected_steps"] == r * n * (L - 1)
    csr = G._g.export_csr()
    lab = csr["labels"]
    ref, rl, _ = oracle.walks_bitset(csr, 0.25, 4.0, 11, L, 0, r * n, nthreads=4)
    assert len(walks) == r * n
    for i in (0, 1, n, r * n // 2, r * n - 1):
        assert walks[i] == lab[ref[i, :rl[i]]].tolist()
    R = node2vec.Graph(nxg, False, 0.25, 4.0, mode="scale", seed=11, sampler="rejection")
    R.preprocess_transition_probs()
    wr = R.simulate_walks(2, L)
    assert R.scale_sampler == C.N2V_REJECTION
    ref2, rl2, _ = oracle.walks_scale(dict(csr, weights=None), 0.25, 4.0, 11, L, 0, 2 * n, nthreads=4)
    assert [lab[ref2[i, :rl2[i]]].tolist() for i in range(2 * n)] == wr
