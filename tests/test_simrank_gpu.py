"""GPU parity for the naive SimRank ground-truth generator (SimRank.java:15-82)
against the oracle restatement (oracle.c or_simrank_naive, itself pinned to
the reference's committed 0_333_5038 naive SimRank output) and, at sizes the
oracle cannot finish, the one-round recurrence on sampled pairs.

Tolerance: fp64; the GPU sums neighbour pairs in a different order than the
Java double loop, so values agree to rtol 1e-12 (atol 1e-15), not bitwise."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu

GRAPHS = {"moreno": ("moreno_crime_crime.txt", 1380, "\t"),
          "g333": ("0_333_5038.txt", 333, " "),
          "blog": ("blog.txt", 10313, ",")}
RTOL, ATOL = 1e-12, 1e-15


def _graph(name):
    from gwamd import topsim
    f, V, sep = GRAPHS[name]
    return topsim.Graph(os.path.join(DATA, f), V, separator=sep)


def _gpu(g, C, iters):
    from gwamd import topsim
    sr = topsim.SimRank(g, C_=C, step=iters)
    sr.compute()
    return sr.getResult()


@pytest.mark.parametrize("name,C,iters", [("g333", 0.8, 30), ("g333", 0.6, 3), ("moreno", 0.6, 3),
                                          ("moreno", 0.8, 7)])
def test_naive_simrank_equals_oracle(gw, oracle, name, C, iters):
    g = _graph(name)
    sim = _gpu(g, C, iters)
    ref = oracle.simrank_naive(g._offs, g._nbrs, C, iters, nthreads=8)
    np.testing.assert_allclose(sim, ref, rtol=RTOL, atol=ATOL)
    assert np.array_equal(sim, sim.T)          # each pair computed once and mirrored
    assert np.all(np.diag(sim) == 0.0)         # postProcess


def test_naive_simrank_reference_fixture(gw):
    """GPU result == the reference's committed naive SimRank top-10 file
    (IsoMap_LE/data/0_333_5038_simrank_navie_top10.txt.sim.txt, %.8f)."""
    g = _graph("g333")
    sim = _gpu(g, 0.8, 30)
    with open(os.path.join(DATA, "0_333_5038_simrank_navie_top10.txt.sim.txt")) as f:
        for line in f:
            toks = line.strip().split(" ")
            v = int(toks[0])
            for t in toks[1:]:
                i, val = t.split(":")
                assert abs(sim[v, int(i)] - float(val)) <= 5.1e-9


def test_naive_simrank_global_row_path_bitwise(gw):
    """The HBM-row variant (n*8 > LDS budget) gives the same bits as the
    LDS-row variant (same reduction order)."""
    g = _graph("moreno")
    a = _gpu(g, 0.6, 3)
    g._g.options(simrank_hbm_row=1)
    b = _gpu(g, 0.6, 3)
    assert np.array_equal(a, b)


def test_naive_simrank_blog_recurrence(gw):
    """blog (10,313 vertices, 668K entries): too large for the oracle, so check
    the recurrence: S3 == one host round of SimRank.sim() over the GPU's S2
    (diag restored to 1) on sampled pairs, plus symmetry / range / isolated
    vertex 0."""
    g = _graph("blog")
    s2 = _gpu(g, 0.6, 2)
    s3 = _gpu(g, 0.6, 3)
    assert np.array_equal(s3, s3.T)
    assert np.all(np.diag(s3) == 0) and s3.min() >= 0 and s3.max() <= 0.6
    assert np.all(s3[0] == 0)  # vertex 0 is isolated in blog (ids 1..10312)
    s2 = s2.copy()
    np.fill_diagonal(s2, 1.0)
    rng = np.random.default_rng(5)
    offs, nbrs = g._offs, g._nbrs
    pairs = list(zip(rng.integers(1, 10313, 300), rng.integers(1, 10313, 300)))
    pairs += [(int(np.argmax(np.diff(offs))), 5), (17, 18)]
    for v, w in pairs:
        if v == w:
            continue
        nv, nw = nbrs[offs[v]:offs[v + 1]], nbrs[offs[w]:offs[w + 1]]
        exp = 0.6 * s2[np.ix_(nv, nw)].sum() / (len(nv) * len(nw)) if len(nv) and len(nw) else 0.0
        assert abs(s3[v, w] - exp) <= 1e-12 * max(exp, 1e-3), (v, w, s3[v, w], exp)


def test_naive_simrank_edge_cases(gw, oracle, tmp_path):
    """isolated vertices, self-loops, duplicate lines (multigraph counts),
    STEP=0 (all zeros) and the directed-graph refusal."""
    from gwamd import topsim
    from gwamd.graph import GWGraph
    from gwamd import _lib as C
    p = tmp_path / "g.txt"
    p.write_text("0,1\n1,2\n2,0\n2,3\n3,3\n1,2\n4,5\n")
    g = topsim.Graph(str(p), 8, separator=",")  # 6, 7 isolated
    for iters in (0, 1, 2, 5):
        sim = _gpu(g, 0.6, iters)
        ref = oracle.simrank_naive(g._offs, g._nbrs, 0.6, iters)
        np.testing.assert_allclose(sim, ref, rtol=RTOL, atol=ATOL)
    assert np.all(_gpu(g, 0.6, 0) == 0)
    sr = topsim.SimRank(g, step=3)
    sr.compute()
    # SimRank.sim(v, w) evaluates one more round from the final matrix (:67-77)
    S = sr.getResult()
    v, w = 0, 1
    nv, nw = g.neighbors(v), g.neighbors(w)
    assert sr.sim(v, w) == pytest.approx(0.6 * sum(S[a, b] for a in nv for b in nw) / (len(nv) * len(nw)))
    d = tmp_path / "d.txt"
    d.write_text("1 2\n2 3\n")
    gd = GWGraph.from_edgelist(str(d), delimiter=" ", semantics="nx", directed=True)
    gd.to_device(0)
    with pytest.raises(C.UnsupportedError):
        C.check(C.lib().gw_simrank_naive(gd.handle, 0.6, 3, None, None), gd.handle)


def test_print_by_order_all(gw, oracle, tmp_path):
    """Print.printByOrderAll (Print.java:55-84): %.7f with the exact
    FixedMaxPQ tie order, over the GPU matrix."""
    from gwamd import topsim
    g = _graph("g333")
    sr = topsim.SimRank(g)
    sr.compute()
    sim = sr.getResult()
    out = tmp_path / "sr.txt"
    topsim.printByOrderAll(sr, str(out), 1000, 10, separator=" ")
    lines = open(str(out) + ".sim.txt", "rb").read().split(b"\r\n")
    for v in (0, 1, 100, 332):
        exp = oracle.java_fixed_max_pq_row(sim[v], 1000)
        assert lines[v].decode() == f"{v}" + "".join(f" {i}:{oracle.java_format_fixed(x, 7)}" for i, x in exp)


def test_cpp_variants_driver_matches_python(gw, tmp_path):
    """The C++ host mirror (host/simrank_variants.cpp over topsim_host.hpp)
    produces the same files / matrices as the Python mirror for SimRank,
    TopSim_singleSample_M, SingleRandomWalk_M, TopSim_doubleSample, TopSim_Dev
    and DoubleRandomWalk (same library, same seeds)."""
    import subprocess
    from conftest import ROOT
    from gwamd import topsim
    exe = os.path.join(ROOT, "graph-embedding_amd", "bin", "simrank_variants")
    f, V, sep = GRAPHS["g333"]
    path = os.path.join(DATA, f)

    def run(algo, *extra):
        out = str(tmp_path / algo)
        subprocess.run([exe, "--graph", path, "--V", str(V), "--sep", sep, "--algo", algo, "--out", out,
                        "--seed", "3", *extra], check=True, timeout=600)
        return out

    g = _graph("g333")
    # SimRank.main: printByOrderAll(sim, out, 1000, 10) with MyConfiguration.SEPARATOR
    out = run("simrank", "--step", "3")
    sr = topsim.SimRank(g)
    sr.compute()
    topsim.printByOrderAll(sr, str(tmp_path / "py_sr"), 1000, 10, separator=sep)
    assert open(out + ".sim.txt", "rb").read() == open(str(tmp_path / "py_sr") + ".sim.txt", "rb").read()
    for algo, cls in (("topsim_m", topsim.TopSim_singleSample_M), ("srw_m", topsim.SingleRandomWalk_M)):
        out = run(algo, "--M", "2", "--sample", "500", "--step", "3")
        ts = cls(g, 2, 500, seed=3, step=3)
        ts.compute()
        topsim.printByOrder(ts, str(tmp_path / ("py_" + algo)), 20, separator=sep)
        assert open(out + ".sim.txt", "rb").read() == open(str(tmp_path / ("py_" + algo)) + ".sim.txt", "rb").read()
    out = run("double", "--sample", "100", "--step", "3")
    ds = topsim.TopSim_doubleSample(g, 100, 3, seed=3)
    ds.compute()
    assert np.array_equal(np.fromfile(out + ".bin").reshape(V, V), ds.getResult())
    out = run("drw", "--sample", "10", "--step", "3")
    dw = topsim.DoubleRandomWalk(g, 10, 3, seed=3)
    dw.compute()
    np.testing.assert_allclose(np.fromfile(out + ".bin").reshape(V, V), dw.getResult(), rtol=1e-12, atol=1e-15)
    out = run("dev", "--sample", "3000", "--step", "3", "--topk", "5", "--single", "1")
    dev = topsim.TopSim_Dev(g, 3000, 3, 5, 1, seed=3)
    sr2 = topsim.SimRank(g)
    sr2.compute()
    dev.compute(sr2.getResult())
    np.testing.assert_allclose(np.fromfile(out + ".bin").reshape(V, V), dev.getResult(), rtol=1e-12, atol=1e-15)
