"""GPU parity for the double-walk variants (§8f-4): TopSim_doubleSample,
TopSim_Dev and DoubleRandomWalk vs the oracle restatements (oracle.c
or_topsim_levels / or_topsim_double_sims / or_topsim_dev /
or_double_random_walk; the level rows are pinned by a literal Java-queue port
in test_oracle_golden.py).

Tolerance: fp64 with reassociated sums (MFMA tiles, atomics) — rtol 1e-12
plus atol 1e-12 x the matrix scale; the sparsity patterns must be identical."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu

GRAPHS = {"moreno": ("moreno_crime_crime.txt", 1380, "\t"),
          "g333": ("0_333_5038.txt", 333, " "),
          "karate": ("karate.edgelist", 35, " ")}


def _graph(name):
    from gwamd import topsim
    f, V, sep = GRAPHS[name]
    return topsim.Graph(os.path.join(DATA, f), V, separator=sep)


def _close(a, b):
    scale = max(float(np.abs(b).max()), 1e-300)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12 * scale)
    assert np.array_equal(a != 0, b != 0)


@pytest.mark.parametrize("name,sample,step", [("moreno", 200, 3), ("g333", 50, 2), ("karate", 10 ** 6, 3),
                                              ("moreno", 1000, 4)])
def test_topsim_double_sample_equals_oracle(gw, oracle, name, sample, step):
    from gwamd import topsim
    g = _graph(name)
    ts = topsim.TopSim_doubleSample(g, sample, step, seed=4)
    ts.compute()
    sim = ts.getResult()
    ref = oracle.topsim_double_sample(g._offs, g._nbrs, sample, step, C=0.6, seed=4, nthreads=8)
    _close(sim, ref)
    assert np.array_equal(sim, sim.T) and np.all(np.diag(sim) == 0)


@pytest.mark.parametrize("name,sample,step,K,single", [("moreno", 10000, 3, 10, 1), ("g333", 3000, 4, 5, 2)])
def test_topsim_dev_equals_oracle(gw, oracle, name, sample, step, K, single):
    from gwamd import topsim
    g = _graph(name)
    sr = topsim.SimRank(g)  # naive SimRank as the candidate matrix
    sr.compute()
    cand_m = sr.getResult()
    dev = topsim.TopSim_Dev(g, sample, step, K, single, seed=8)
    dev.compute(cand_m)
    sim = dev.getResult()
    cand = topsim.select_candidates(cand_m, K)
    ref = oracle.topsim_dev(g._offs, g._nbrs, dev.SAMPLE, step, cand, C=0.6, seed=8, nthreads=8)
    _close(sim, ref)
    # only (i, candidate) entries can be non-zero
    mask = np.zeros_like(sim, dtype=bool)
    for i in range(cand.shape[0]):
        mask[i, cand[i][cand[i] >= 0]] = True
    assert not np.any(sim[~mask])


@pytest.mark.parametrize("name,sample,step", [("moreno", 20, 3), ("g333", 10, 4), ("karate", 50, 5)])
def test_double_random_walk_equals_oracle(gw, oracle, name, sample, step):
    from gwamd import topsim
    g = _graph(name)
    drw = topsim.DoubleRandomWalk(g, sample, step, seed=2)
    drw.compute()
    sim = drw.getResult()
    ref = oracle.double_random_walk(g._offs, g._nbrs, sample, step, C=0.6, seed=2, nthreads=8)
    _close(sim, ref)
    assert np.array_equal(sim, sim.T) and np.all(np.diag(sim) == 0)
