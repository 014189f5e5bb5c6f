"""GPU parity for the bounded-memory variants (§8f-3): TopSim_singleSample_M
and SingleRandomWalk_M with lxctools.FixedCacheMap, against the oracle's
literal restatement (oracle.c or_topsim_m, FixedCacheMap pinned by the
reference's own FixedCacheMap.main example in test_oracle_golden.py).

Bar: bit-exact.  The walks use the same Philox keys, each update is the same
fp64 expression rounded to float, and the map sees the same put() sequence,
so keys, float values, sizes and iteration order must be identical."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu

GRAPHS = {"moreno": ("moreno_crime_crime.txt", 1380, "\t"),
          "g333": ("0_333_5038.txt", 333, " "),
          "blog": ("blog.txt", 10313, ",")}


def _graph(name):
    from gwamd import topsim
    f, V, sep = GRAPHS[name]
    return topsim.Graph(os.path.join(DATA, f), V, separator=sep)


def _run(cls, g, M, sample, step, sources, seed=9):
    ts = cls(g, M, sample, seed=seed, step=step)
    ts.compute(sources)
    return ts


@pytest.mark.parametrize("name,variant,M,sample,step,nsrc", [
    ("moreno", 0, 1, 1000, 5, None), ("moreno", 0, 5, 1000, 5, None), ("moreno", 2, 1, 2000, 3, None),
    ("g333", 0, 2, 2500, 3, None), ("g333", 2, 3, 500, 5, None), ("blog", 0, 10, 10000, 5, 48),
    ("blog", 2, 10, 10000, 5, 48)])
def test_topsim_m_equals_oracle(gw, oracle, name, variant, M, sample, step, nsrc):
    from gwamd import topsim
    g = _graph(name)
    V = g.getVCount()
    src = np.arange(V, dtype=np.int32) if nsrc is None else \
        np.linspace(1, V - 1, nsrc).astype(np.int32)
    cls = topsim.TopSim_singleSample_M if variant == 0 else topsim.SingleRandomWalk_M
    ts = _run(cls, g, M, sample, step, src)
    _, keys, vals, size = ts.raw()
    ok, ov, osz, st = oracle.topsim_m(g._offs, g._nbrs, variant, sample, step, 20 * M, C=0.6, seed=9,
                                      sources=src, nthreads=8)
    assert np.array_equal(size, osz)
    assert np.array_equal(keys, ok)
    assert np.array_equal(vals.view(np.uint32), ov.view(np.uint32))
    assert ts.stats["pair_updates"] == st["pair_updates"]
    assert ts.stats["extensions"] == st["extensions"]
    if variant == 0:
        assert ts.stats["walkers"] == st["walkers"]
        assert ts.stats["max_frontier"] == st["max_frontier"]


def test_topsim_m_print_by_order(gw, oracle, tmp_path):
    """Print.printByOrder(FixedCacheMap[], outPath, topk) (Print.java:94-124):
    the last topk entries of each ascending iteration, %.6f of the float."""
    from gwamd import topsim
    g = _graph("moreno")
    ts = _run(topsim.TopSim_singleSample_M, g, 2, 1000, 5, None)
    out = tmp_path / "m.txt"
    topsim.printByOrder(ts, str(out), 20)
    src, keys, vals, size = ts.raw()
    lines = open(str(out) + ".sim.txt", "rb").read().split(b"\r\n")
    ids = open(str(out), "rb").read().split(b"\r\n")
    maps = ts.getResult()
    for r in (0, 1, 17, 500, 1379):
        lo = max(0, size[r] - 20)
        exp = [(int(keys[r, i]), float(vals[r, i])) for i in range(lo, size[r])]
        assert lines[r].decode() == f"{r}" + "".join(f",{k}:{oracle.java_format_fixed(v)}" for k, v in exp)
        assert ids[r].decode() == f"{r}" + "".join(f",{k}" for k, _ in exp)
        assert maps[r].size() == size[r]
        assert [k for k, _ in maps[r]][lo:] == [k for k, _ in exp]


def test_topsim_m_capacity_limit(gw):
    from gwamd import topsim
    from gwamd import _lib as C
    g = _graph("g333")
    with pytest.raises(C.UnsupportedError):
        _run(topsim.TopSim_singleSample_M, g, 300, 100, 2, np.arange(4, dtype=np.int32))  # 6000 > 4096
