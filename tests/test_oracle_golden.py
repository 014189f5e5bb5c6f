"""CPU: pin the oracle against the reference's golden vectors and fixtures.

Golden vectors: tests/golden/n2v_*.npz, produced by oracle/gen_goldens.py which
imports the reference node2vec.py.  SimRank fixture: the reference's committed
IsoMap_LE/data/0_333_5038_simrank_navie_top10.txt.sim.txt.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import DATA, golden_index, load_golden

CASES = golden_index()["cases"]


def _case_id(c):
    return c["file"]


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_nx_semantics_restatement(case, oracle):
    """read_graph (main.py:76-89) restated without networkx == golden CSR."""
    g = load_golden(case["file"])
    order, labels, offs, nbrs, w = oracle.read_graph_nx_semantics(
        os.path.join(DATA, case["graph"]), case["delimiter"], case["weighted"], case["directed"])
    np.testing.assert_array_equal(order, g["node_order"])
    np.testing.assert_array_equal(labels, g["labels"])
    np.testing.assert_array_equal(offs, g["offsets"])
    np.testing.assert_array_equal(labels[nbrs], g["nbrs"])
    np.testing.assert_array_equal(w, g["weights"])


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_alias_tables_bitwise(case, oracle):
    """alias_setup / preprocess_transition_probs (node2vec.py:83-147)."""
    g = load_golden(case["file"])
    rank = {int(x): i for i, x in enumerate(g["labels"])}
    nbrs = np.array([rank[int(x)] for x in g["nbrs"]], np.int32)
    w = g["weights"] if case["weighted"] else None
    J, q = oracle.alias_nodes(g["offsets"], w)
    np.testing.assert_array_equal(J, g["alias_node_J"])
    assert q.tobytes() == g["alias_node_q"].tobytes()
    eoff, eJ, eq = oracle.alias_edges(g["offsets"], nbrs, w, case["p"], case["q"])
    if "alias_edge_J" in g:
        np.testing.assert_array_equal(eoff, g["alias_edge_off"])
        np.testing.assert_array_equal(eJ, g["alias_edge_J"])
        assert eq.tobytes() == g["alias_edge_q"].tobytes()
    else:
        assert hashlib.sha256(eoff.tobytes()).digest() == bytes(g["alias_edge_off_sha256"])
        assert hashlib.sha256(eJ.tobytes()).digest() == bytes(g["alias_edge_J_sha256"])
        assert hashlib.sha256(eq.tobytes()).digest() == bytes(g["alias_edge_q_sha256"])


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_walks_replay_bitwise(case, oracle):
    """node2vec_walk/simulate_walks (node2vec.py:13-59) replayed from the
    np.random stream == the reference's own walks."""
    g = load_golden(case["file"])
    rank = {int(x): i for i, x in enumerate(g["labels"])}
    nbrs = np.array([rank[int(x)] for x in g["nbrs"]], np.int32)
    w = g["weights"] if case["weighted"] else None
    nJ, nq = oracle.alias_nodes(g["offsets"], w)
    eoff, eJ, eq = oracle.alias_edges(g["offsets"], nbrs, w, case["p"], case["q"])
    starts = np.array([rank[int(x)] for x in g["starts"]], np.int32)
    L = case["walk_length"]
    U = np.random.RandomState(case["seed"]).random_sample(2 * (L - 1) * len(starts))
    np.testing.assert_array_equal(U[:len(g["uniforms"])], g["uniforms"])
    out, lens, used = oracle.walks_replay(g["offsets"], nbrs, nJ, nq, eoff, eJ, eq, L, starts, U)
    assert used >= 0
    np.testing.assert_array_equal(lens, g["lens"])
    assert used == 2 * int((g["lens"] - 1).sum())
    lab = np.where(out >= 0, g["labels"][np.maximum(out, 0)], -1).astype(np.int64)
    if case["full_walks"]:
        np.testing.assert_array_equal(lab, g["walks"])
    else:
        np.testing.assert_array_equal(lab[:64], g["walks_head"])
        np.testing.assert_array_equal(lab[-64:], g["walks_tail"])
    assert hashlib.sha256(lab.tobytes()).hexdigest() == case["walks_sha256"]


def test_alias_setup_known_answer(oracle):
    """alias_setup on a hand-checkable distribution (node2vec.py:116-147)."""
    J, q = oracle.alias_setup([0.1, 0.2, 0.3, 0.4])
    # q = K*p = [.4,.8,1.2,1.6]; smaller=[0,1], larger=[2,3]
    # pop 1 & 3: J[1]=3, q[3]=1.6+0.8-1=1.4 -> larger=[2,3]
    # pop 0 & 3: J[0]=3, q[3]=1.4+0.4-1=0.8 -> smaller=[3]
    # pop 3 & 2: J[3]=2, q[2]=1.2+0.8-1=1.0 -> larger=[2]
    np.testing.assert_array_equal(J, [3, 3, 0, 2])
    np.testing.assert_allclose(q, [0.4, 0.8, 1.0, 0.8], rtol=0, atol=1e-15)


def _java_graph_csr(path, V, sep):
    adj = [[] for _ in range(V)]
    with open(path) as f:
        for line in f:
            a, b = line.rstrip("\r\n").split(sep)[:2]
            adj[int(a)].append(int(b))
            adj[int(b)].append(int(a))
    offs = np.zeros(V + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in adj])
    return offs, np.array([y for x in adj for y in x], np.int32)


def test_naive_simrank_fixture(oracle):
    """SimRank.java:36-77 restated == the reference's committed naive SimRank
    output (C=0.8, 30 iterations, Java graph semantics, top-10, %.8f)."""
    offs, nbrs = _java_graph_csr(os.path.join(DATA, "0_333_5038.txt"), 333, " ")
    sim = oracle.simrank_naive(offs, nbrs, 0.8, 30, nthreads=8)
    rows = 0
    with open(os.path.join(DATA, "0_333_5038_simrank_navie_top10.txt.sim.txt")) as f:
        for line in f:
            toks = line.strip().split(" ")
            v = int(toks[0])
            pairs = [(int(t.split(":")[0]), float(t.split(":")[1])) for t in toks[1:]]
            for (i, val) in pairs:
                assert abs(sim[v, i] - val) <= 5.1e-9, (v, i, sim[v, i], val)
            rows += 1
            if not pairs:  # vertex with no similar vertex: empty row
                assert sim[v].max() < 5e-9
                continue
            # the listed ids are a valid top-10 of the row (ties allowed)
            kth = pairs[-1][1]
            assert np.sum(sim[v] > kth + 1e-8) <= len(pairs)
    assert rows == 333


@pytest.mark.parametrize("step", [1, 2])
def test_topsim_deterministic_kat(oracle, step):
    """KAT: with SAMPLE large enough that every expansion
    enumerates, TopSim_singleSample / SAMPLE == naive SimRank after STEP
    Jacobi sweeps (C=0.6) on moreno (Java multigraph semantics)."""
    offs, nbrs = _java_graph_csr(os.path.join(DATA, "moreno_crime_crime.txt"), 1380, "\t")
    sample = 1000 if step == 1 else 200000
    rows, st = oracle.topsim(offs, nbrs, 0, sample, step, C=0.6, seed=1, nthreads=8)
    assert st["walkers"] == 0, "regime is not deterministic"
    naive = oracle.simrank_naive(offs, nbrs, 0.6, step, nthreads=8)
    np.testing.assert_allclose(rows / sample, naive, rtol=0, atol=1e-13)


def test_topsim_enumerate_equals_singlesample_in_det_regime(oracle):
    offs, nbrs = _java_graph_csr(os.path.join(DATA, "moreno_crime_crime.txt"), 1380, "\t")
    a, _ = oracle.topsim(offs, nbrs, 0, 1000, 1, sources=np.arange(0, 1380, 7))
    b, _ = oracle.topsim(offs, nbrs, 1, 1000, 1, sources=np.arange(0, 1380, 7))
    np.testing.assert_array_equal(a, b)


def test_java_random_lcg(oracle):
    # new Random(42).nextInt() == -1170105035 (well-known JDK value)
    mask = (1 << 48) - 1
    s = (42 ^ 0x5DEECE66D) & mask
    s = (s * 0x5DEECE66D + 0xB) & mask
    v = s >> 16
    v = v - (1 << 32) if v >= 1 << 31 else v
    assert v == -1170105035
    # power-of-two bound path: (bound * next(31)) >> 31
    seq = oracle.jrand_sequence(42, 1 << 30, 3)
    s = (42 ^ 0x5DEECE66D) & mask
    exp = []
    for _ in range(3):
        s = (s * 0x5DEECE66D + 0xB) & mask
        exp.append(((1 << 30) * (s >> 17)) >> 31)
    np.testing.assert_array_equal(seq, exp)
    # rejection path stays in range
    r = oracle.jrand_sequence(7, 1000, 10000)
    assert r.min() >= 0 and r.max() < 1000


def test_java_format_and_pq(oracle):
    f = oracle.java_format_fixed
    assert f(0.0) == "0.000000"
    assert f(0.1234565) == "0.123457"   # HALF_UP on the shortest repr digits
    assert f(1.0000005) == "1.000001"   # C printf would give 1.000000
    assert f(153.5) == "153.500000"
    assert f(0.0, 7) == "0.0000000"     # printByOrderAll's %.7f (Print.java:77)
    assert f(5e-08, 7) == "0.0000001"
    assert f(1.5e-08, 7) == "0.0000000"
    # FixedMaxPQ tie order: k=2, offers 1.0,1.0,2.0 -> root (id 0) evicted
    got = oracle.java_fixed_max_pq_row([1.0, 1.0, 2.0], 2)
    assert [i for i, _ in got] == [2, 1]


def _selfloop_csr():
    """A small undirected simple graph (sorted rows) with self-loops on a
    third of its vertices, hubs and leaves: both branches of the q > 1 mixture
    (deg prev < deg cur and not), prev drawn from N(prev) as its own
    self-loop, and cur's self-loop as a common neighbour."""
    rng = np.random.default_rng(17)
    n = 14
    E = set()
    for v in range(1, n):
        E.add((int(rng.integers(0, v)), v))
    for _ in range(12):
        a, b = sorted(int(x) for x in rng.integers(0, n, 2))
        if a != b:
            E.add((a, b))
    for v in range(0, n, 3):
        E.add((v, v))
    adj = [set() for _ in range(n)]
    for a, b in E:
        adj[a].add(b)
        adj[b].add(a)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(r) for r in adj])
    nbrs = np.concatenate([np.array(sorted(r), np.int32) for r in adj])
    return offs, nbrs


@pytest.mark.slow
@pytest.mark.parametrize("graph", ["karate", "selfloops"])
@pytest.mark.parametrize("p,q", [(0.25, 4), (4, 2), (0.5, 2), (1, 0.5), (4, 0.25)])
def test_scale_walks_match_second_order_distribution(oracle, graph, p, q):
    """The scale sampler reproduces the reference transition probabilities
    (alias_edges, node2vec.py:61-81) in distribution: the uniform-proposal
    rejection design (q <= 1) and, at q > 1, the mixture proposal taken when
    deg(prev) < deg(cur) — including 1/p < 1/q (a prev drawn from N(cur)
    accepted with probability q/p) and self-loops."""
    if graph == "karate":
        g = load_golden("n2v_karate_p0.25_q4_s0.npz")
        rank = {int(x): i for i, x in enumerate(g["labels"])}
        nbrs = np.array([rank[int(x)] for x in g["nbrs"]], np.int32)
        offs = g["offsets"]
    else:
        offs, nbrs = _selfloop_csr()
    csr = dict(offsets=offs, nbrs=nbrs, weights=None, node_order=np.arange(len(offs) - 1, dtype=np.int32))
    n = len(offs) - 1
    per = 20000 if graph == "karate" else 40000
    out, lens, cnt = oracle.walks_scale(csr, p, q, seed=3, L=3, walk_begin=0, walk_count=n * per,
                                        nthreads=8)
    # exact P(next | prev, cur) from the reference formula
    counts = {}
    mixed = 0
    deg = np.diff(offs)
    for a, b, c in out:
        counts.setdefault((a, b), {}).setdefault(c, 0)
        counts[(a, b)][c] += 1
    worst = 0.0
    for (a, b), dist in counts.items():
        tot = sum(dist.values())
        if tot < 4000:
            continue
        mixed += int(deg[a] < deg[b])
        row = nbrs[offs[b]:offs[b + 1]]
        na = set(nbrs[offs[a]:offs[a + 1]].tolist())
        un = np.array([1 / p if x == a else (1.0 if x in na else 1 / q) for x in row])
        pr = un / un.sum()
        emp = np.array([dist.get(int(x), 0) for x in row]) / tot
        sd = np.sqrt(pr * (1 - pr) / tot)
        worst = max(worst, float(np.max(np.abs(emp - pr) / np.maximum(sd, 1e-12))))
    assert worst < 5.5, worst
    assert mixed > 5  # the mixture branch is exercised (taken when deg prev < deg cur)


@pytest.mark.slow
@pytest.mark.parametrize("p,q", [(0.25, 4), (1, 0.5), (4, 0.25)])
def test_bitset_walks_match_second_order_distribution(oracle, p, q):
    """The GW_N2V_BITSET mixture (return / common / other) reproduces the
    reference transition probabilities of get_alias_edge (node2vec.py:61-81)."""
    g = load_golden("n2v_karate_p0.25_q4_s0.npz")
    rank = {int(x): i for i, x in enumerate(g["labels"])}
    nbrs = np.array([rank[int(x)] for x in g["nbrs"]], np.int32)
    offs = g["offsets"]
    n = len(offs) - 1
    csr = dict(offsets=offs, nbrs=nbrs, node_order=np.arange(n, dtype=np.int32))
    out, lens, cnt = oracle.walks_bitset(csr, p, q, seed=5, L=3, walk_begin=0, walk_count=n * 20000, nthreads=8)
    counts = {}
    for a, b, c in out:
        counts.setdefault((a, b), {}).setdefault(c, 0)
        counts[(a, b)][c] += 1
    worst = 0.0
    for (a, b), dist in counts.items():
        tot = sum(dist.values())
        if tot < 4000:
            continue
        row = nbrs[offs[b]:offs[b + 1]]
        na = set(nbrs[offs[a]:offs[a + 1]].tolist())
        un = np.array([1 / p if x == a else (1.0 if x in na else 1 / q) for x in row])
        pr = un / un.sum()
        emp = np.array([dist.get(int(x), 0) for x in row]) / tot
        sd = np.sqrt(pr * (1 - pr) / tot)
        worst = max(worst, float(np.max(np.abs(emp - pr) / np.maximum(sd, 1e-12))))
    assert worst < 5.5, worst


def test_fixed_cache_map_reference_main(oracle):
    """FixedCacheMap.main (FixedCacheMap.java:134-148): the reference's own
    example, capacity 3 -> drains (1, 1.1f), (2, 3f), (4, 16f)."""
    got = oracle.fcm_run(3, [1, 2, 3, 4, 4, 1, 5], [0.5, 3, 0.1, 8, 8, 0.6, 1])
    assert [k for k, _ in got] == [1, 2, 4]
    assert np.array_equal(np.float32([v for _, v in got]), np.float32([1.1, 3.0, 16.0]))
    py = oracle.PyFixedCacheMap(3)
    for k, v in zip([1, 2, 3, 4, 4, 1, 5], [0.5, 3, 0.1, 8, 8, 0.6, 1]):
        py.put(k, v)
    assert py.drain() == got


@pytest.mark.parametrize("nmax,nkeys,nput", [(5, 40, 400), (16, 30, 2000), (64, 1000, 5000), (200, 150, 3000)])
def test_fixed_cache_map_c_equals_python(oracle, nmax, nkeys, nput):
    """C restatement == literal Python port on random put streams (eviction,
    re-insertion of evicted keys, float accumulation, ties)."""
    rng = np.random.default_rng(nmax)
    keys = rng.integers(0, nkeys, nput).astype(np.int32)
    vals = (np.round(rng.random(nput) * 16) / 16 * rng.choice([1e-3, 1.0], nput)).astype(np.float32)
    got = oracle.fcm_run(nmax, keys, vals)
    py = oracle.PyFixedCacheMap(nmax)
    for k, v in zip(keys.tolist(), vals.tolist()):
        py.put(k, v)
    assert py.drain() == got


def test_topsim_m_oracle_no_eviction_matches_topsim(oracle):
    """TopSim_singleSample_M with a capacity that never evicts == float
    accumulation of TopSim_singleSample's updates / SAMPLE (same Philox walks)."""
    offs, nbrs = _java_graph_csr(os.path.join(DATA, "moreno_crime_crime.txt"), 1380, "\t")
    src = np.arange(0, 1380, 97, dtype=np.int32)
    keys, vals, size, st = oracle.topsim_m(offs, nbrs, 0, 300, 3, 4096, C=0.6, seed=5, sources=src, nthreads=8)
    rows, st2 = oracle.topsim(offs, nbrs, 0, 300, 3, C=0.6, seed=5, sources=src, nthreads=8)
    assert st["pair_updates"] == st2["pair_updates"] and st["extensions"] == st2["extensions"]
    for r in range(len(src)):
        ks = keys[r, :size[r]]
        assert set(ks.tolist()) == set(np.nonzero(rows[r])[0].tolist())
        np.testing.assert_allclose(vals[r, :size[r]], rows[r][ks] / 300, rtol=1e-5)
        assert np.all(np.diff(vals[r, :size[r]]) >= 0)  # ascending iteration


def _py_double_sample_levels(adj, src, SAMPLE, STEP):
    """Literal Python port of TopSim_doubleSample.sample/computePath
    (TopSim_doubleSample.java:71-164) for the deterministic regime (every
    queued path has mass >= degree, so no randNeighbor call happens)."""
    from collections import deque
    P = {}
    queue = deque([[(src, float(SAMPLE))]])
    pathLen, TopSim = 0, 1

    def computePath(step):
        for path in queue:
            target = path[step][0]
            if target == src:
                continue
            P[(target, step)] = path[step][1]

    while pathLen < STEP:
        if pathLen == TopSim:
            computePath(pathLen)
            TopSim += 1
        for _ in range(len(queue)):
            path = queue[0]
            cur, sample = path[pathLen]
            degree = len(adj[cur])
            assert degree != 0 and sample >= degree, "deterministic regime only"
            newSample = sample / degree
            for j in range(degree):
                queue.append(path + [(adj[cur][j], newSample)])
            queue.popleft()
        pathLen += 1
    computePath(pathLen)
    return P


def test_double_sample_levels_deterministic_kat(oracle):
    """or_topsim_levels == the literal Java-queue port (last path wins) on
    karate (Java multigraph semantics) with SAMPLE large enough that every
    path is enumerated."""
    path = os.path.join(DATA, "karate.edgelist")
    adj = [[] for _ in range(35)]
    with open(path) as f:
        for line in f:
            a, b = line.split()[:2]
            adj[int(a)].append(int(b))
            adj[int(b)].append(int(a))
    offs = np.zeros(36, np.int64)
    offs[1:] = np.cumsum([len(x) for x in adj])
    nbrs = np.array([y for x in adj for y in x], np.int32)
    M = oracle.topsim_levels(offs, nbrs, 10 ** 6, 3, np.arange(1, 35, dtype=np.int32))
    for t, src in enumerate(range(1, 35)):
        P = _py_double_sample_levels(adj, src, 10 ** 6, 3)
        got = {(x, s + 1): M[t, s, x] for s in range(3) for x in range(35) if M[t, s, x] > 0}
        assert got == P
