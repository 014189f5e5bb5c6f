"""oracle.topsim_topk (the CPU comparator for large graphs) == the top-k of
oracle.topsim's dense rows, bitwise: same walks, same sums, reused row.
(Print.printByOrder order: score desc, id asc; Print.java:25-53.)"""
import os

import numpy as np
import pytest

DATA = os.path.join(os.path.dirname(__file__), "golden", "data")


def _java_graph(path, V, sep):
    src, dst = [], []
    with open(path) as f:
        for line in f:
            p = line.strip().split(sep)
            if len(p) < 2:
                continue
            a, b = int(p[0]), int(p[1])
            src += [a, b]
            dst += [b, a]
    src, dst = np.array(src, np.int64), np.array(dst, np.int64)
    order = np.argsort(src, kind="stable")  # insertion order within a row (Graph.java)
    offs = np.zeros(V + 1, np.int64)
    np.add.at(offs, src + 1, 1)
    return np.cumsum(offs), dst[order].astype(np.int32)


@pytest.mark.parametrize("name,V,sep,sample,step,k", [
    ("moreno_crime_crime.txt", 1380, "\t", 500, 3, 20),
    ("blog.txt", 10313, ",", 1000, 3, 100),
])
def test_topsim_topk_equals_dense_rows(oracle, name, V, sep, sample, step, k):
    offs, nbrs = _java_graph(os.path.join(DATA, name), V, sep)
    srcs = np.arange(0, V, max(1, V // 97), dtype=np.int32)
    rows, st = oracle.topsim(offs, nbrs, 0, sample, step, C=0.6, seed=5, sources=srcs, nthreads=4)
    ids, sc, st2 = oracle.topsim_topk(offs, nbrs, 0, sample, step, k, C=0.6, seed=5, sources=srcs, nthreads=4)
    assert st == st2
    for r in range(len(srcs)):
        row = rows[r]
        nz = np.nonzero(row > 0)[0]
        top = nz[np.lexsort((nz, -row[nz]))][:k]
        m = len(top)
        np.testing.assert_array_equal(ids[r, :m], top)
        np.testing.assert_array_equal(sc[r, :m], row[top])
        assert np.all(ids[r, m:] == -1) and np.all(sc[r, m:] == 0.0)
