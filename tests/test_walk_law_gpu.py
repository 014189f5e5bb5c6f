"""GPU walks against the REFERENCE transition law (not only against the oracle).

The bitset and rejection samplers are Philox-keyed, so they cannot replay the
reference's own RNG stream; the oracle pins them bit-for-bit, but the oracle is
a restatement by the same author.  These tests check the GPU kernels' output
directly against the distribution the reference defines:

* second-order steps: get_alias_edge(src=prev, dst=cur) (node2vec.py:61-81):
  over sorted N(cur), weight w/p for the return edge, w when
  G.has_edge(dst_nbr, src) (the edge dst_nbr -> prev), w/q otherwise, with
  w = G[cur][dst_nbr]['weight'];
* the first step: alias_nodes[start] (node2vec.py:91-97), weights ∝ w;
* walks stop at sinks (node2vec.py:26-27 `if len(cur_nbrs) > 0 ... else break`).

Small graphs: per context (prev, cur) the empirical next-vertex frequencies
vs the exact probabilities (max |z| over contexts with enough samples).
The large mixed hub / self-loop graph (every bitset payload mode): aggregated
over all sampled steps, the return / common / other category counts and the
rank of the chosen vertex inside its category (uniform) vs expectation.
"""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu


def _walks(gw, G, mode, p, q, L, nwalks, seed):
    import torch
    from gwamd import _lib as C
    C.check(C.lib().gw_n2v_prepare(G.handle, float(p), float(q), mode), G.handle)
    out = torch.empty((nwalks, L), dtype=torch.int32, device="cuda")
    C.check(C.lib().gw_n2v_walks(G.handle, L, seed, 0, nwalks, 1, C.ptr(out), None, None, None), G.handle)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _law(csr, directed, p, q, prev, cur):
    """node2vec.py:61-81 for src=prev, dst=cur: probabilities over N(cur)."""
    offs, nbrs, w = csr["offsets"], csr["nbrs"], csr["weights"]
    row = nbrs[offs[cur]:offs[cur + 1]]
    wt = w[offs[cur]:offs[cur + 1]] if w is not None else np.ones(len(row))
    un = np.empty(len(row))
    for k, (x, wx) in enumerate(zip(row, wt)):
        if x == prev:
            un[k] = wx / p
        elif prev in set(nbrs[offs[x]:offs[x + 1]].tolist()):  # has_edge(x, prev)
            un[k] = wx
        else:
            un[k] = wx / q
    return row, un / un.sum()


def _max_z(counts, prob_of, min_n):
    worst, used = 0.0, 0
    for ctx, dist in counts.items():
        tot = sum(dist.values())
        if tot < min_n:
            continue
        used += 1
        row, pr = prob_of(ctx)
        emp = np.array([dist.get(int(x), 0) for x in row], float) / tot
        assert sum(dist.get(int(x), 0) for x in row) == tot, f"context {ctx}: a step leaves N(cur)"
        sd = np.sqrt(pr * (1 - pr) / tot)
        worst = max(worst, float(np.max(np.abs(emp - pr) / np.maximum(sd, 1e-12))))
    return worst, used


@pytest.mark.parametrize("name,directed,weighted,delim", [
    ("weighted_quirks.edgelist", False, True, " "),
    ("directed_sinks.edgelist", True, False, " "),
    ("karate.edgelist", False, False, " "),
])
@pytest.mark.parametrize("p,q", [(0.25, 4.0), (4.0, 0.25), (0.5, 2.0), (4.0, 2.0)])
def test_rejection_walks_follow_reference_law(gw, name, directed, weighted, delim, p, q):
    """k_walk_scale (GW_N2V_REJECTION): weighted rows (node alias proposal),
    directed rows (has_edge(x, prev) on x's out-row, sinks), the return-edge
    outlier envelope (p < 1) and, on the unweighted undirected graph at q > 1,
    the mixture proposal (steps with deg prev < deg cur; at p = 4, q = 2 a
    prev drawn from N(cur) is accepted with probability q/p) against
    get_alias_edge / alias_nodes."""
    from gwamd import _lib as C
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, name), delim, "nx", directed, weighted).to_device(0)
    csr = G.export_csr()
    if not weighted:
        csr["weights"] = None
    n = G.n
    L = 6
    W = _walks(gw, G, C.N2V_REJECTION, p, q, L, n * 6000, seed=17)
    offs, nbrs = csr["offsets"], csr["nbrs"]
    deg = np.diff(offs)
    # sinks stop walks; every other walk has all L positions
    for row in W[: 5000]:
        ln = int((row >= 0).sum())
        assert np.all(row[ln:] == -1)
        assert ln == L or deg[row[ln - 1]] == 0
    # first step: alias_nodes (weights of the start's row)
    first = {}
    for a, b in W[:, :2]:
        if b >= 0:
            first.setdefault(int(a), {}).setdefault(int(b), 0)
            first[int(a)][int(b)] += 1

    def node_law(v):
        row = nbrs[offs[v]:offs[v + 1]]
        wt = csr["weights"][offs[v]:offs[v + 1]] if csr["weights"] is not None else np.ones(len(row))
        return row, wt / wt.sum()
    z1, used1 = _max_z(first, node_law, 2000)
    assert used1 > 0 and z1 < 6.0, (z1, used1)
    # second-order steps
    trip = {}
    for t in range(L - 2):
        for a, b, c in W[:, t:t + 3]:
            if c >= 0:
                trip.setdefault((int(a), int(b)), {}).setdefault(int(c), 0)
                trip[(int(a), int(b))][int(c)] += 1
    z2, used2 = _max_z(trip, lambda ctx: _law(csr, directed, p, q, ctx[0], ctx[1]), 2000)
    assert used2 >= 10 and z2 < 6.0, (z2, used2)
    G.free()


@pytest.mark.parametrize("p,q", [(0.25, 4.0), (4.0, 2.0)])
def test_mixture_walks_follow_reference_law_selfloops(gw, tmp_path, p, q):
    """The q > 1 mixture proposal on a graph with self-loops on a third of its
    vertices, hubs and leaves: prev's own self-loop drawn from N(prev) is
    rejected, cur's self-loop is a common neighbour (has_edge(cur, prev))."""
    from gwamd import _lib as C
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
    path = str(tmp_path / "selfloops.edgelist")
    with open(path, "w") as f:
        for a, b in sorted(E):
            f.write(f"{a} {b}\n")
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    csr = dict(G.export_csr(), weights=None)
    L = 6
    W = _walks(gw, G, C.N2V_REJECTION, p, q, L, G.n * 20000, seed=23)
    deg = np.diff(csr["offsets"])
    trip = {}
    mixed = 0
    for t in range(L - 2):
        for a, b, c in W[:, t:t + 3]:
            trip.setdefault((int(a), int(b)), {}).setdefault(int(c), 0)
            trip[(int(a), int(b))][int(c)] += 1
    mixed = sum(1 for a, b in trip if deg[a] < deg[b])
    z2, used2 = _max_z(trip, lambda ctx: _law(csr, False, p, q, ctx[0], ctx[1]), 4000)
    assert used2 >= 20 and mixed >= 10 and z2 < 6.0, (z2, used2, mixed)
    G.free()


def _mixed_edgelist(path):
    """Superhubs (deg ~2000, region payloads with an in-entry directory), a
    dense core (deg ~300-400: inline bitsets and regions), a periphery (lists and
    Elias-Fano) and self-loops on hubs, core and periphery (test_n2v_gpu.py's
    mixed-mode graph)."""
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


@pytest.mark.parametrize("p,q", [(0.25, 4.0), (4.0, 0.25)])
def test_bitset_walks_follow_reference_law_mixed_graph(gw, tmp_path, p, q):
    """k_walk_bitset on a graph exercising every payload mode, hubs and
    self-loops: category frequencies (return / common neighbour / other) and
    the rank of the chosen vertex within its category, aggregated over all
    sampled second-order steps, against get_alias_edge's law."""
    from scipy import stats
    from gwamd import _lib as C
    path = str(tmp_path / "mixed.edgelist")
    _mixed_edgelist(path)
    G = gw.GWGraph.from_edgelist(path, " ", "nx").to_device(0)
    csr = G.export_csr()
    offs, nbrs = csr["offsets"], csr["nbrs"]
    n = G.n
    L = 4
    W = _walks(gw, G, C.N2V_BITSET, p, q, L, n * 40, seed=29)
    exp = np.zeros(3)
    var = np.zeros(3)
    obs = np.zeros(3)
    rank_hist = np.zeros((3, 10))
    bin_mass = np.zeros((3, 10))  # expected rank-bin mass of each category, summed over sampled contexts
    for t in range(L - 2):
        for a, b, c in W[:, t:t + 3]:
            row = nbrs[offs[b]:offs[b + 1]]
            ra = nbrs[offs[a]:offs[a + 1]]
            nota = row != a
            inb = np.isin(row, ra, assume_unique=False)  # has_edge(x, a) (undirected)
            common = row[nota & inb]
            others = row[nota & ~inb]
            un = np.array([1.0 / p, len(common), len(others) / q])  # a in N(b): the return edge exists
            pr = un / un.sum()
            exp += pr
            var += pr * (1 - pr)
            for cat, grp in ((1, common), (2, others)):
                m = len(grp)
                if m:
                    ks = np.minimum(9, ((np.arange(m) + 0.5) / m * 10).astype(int))
                    bin_mass[cat] += pr[cat] * np.bincount(ks, minlength=10) / m
            if c == a:
                obs[0] += 1
                continue
            cat, grp = (1, common) if c in common else (2, others)
            k = int(np.searchsorted(grp, c))
            assert k < len(grp) and grp[k] == c, "a step leaves N(cur)"
            obs[cat] += 1
            rank_hist[cat, min(9, int((k + 0.5) / len(grp) * 10))] += 1
    z = (obs - exp) / np.sqrt(var)
    assert np.all(np.abs(z) < 6.0), (obs, exp, z)
    # within the common and other categories the chosen position is uniform:
    # binned ranks against the exact binning expectation of the sampled rows
    for cat in (1, 2):
        tot = rank_hist[cat].sum()
        assert tot > 1000
        expct = tot * bin_mass[cat] / bin_mass[cat].sum()
        chi = stats.chisquare(rank_hist[cat], expct)
        assert chi.pvalue > 1e-6, (cat, rank_hist[cat], expct, chi)
    G.free()

