"""GPU parity for TopSim (H2): HIP kernel vs the Java-literal oracle
restatement (Philox-keyed random children), vs the naive-SimRank KAT, and the
top-k selection / writer path."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu

GRAPHS = {"moreno": ("moreno_crime_crime.txt", 1380, "\t"),
          "g333": ("0_333_5038.txt", 333, " "),
          "blog": ("blog.txt", 10313, ","),
          "arxiv": ("arxiv_author_pub.txt", 38741, "\t")}


def _graph(gw, name):
    f, V, sep = GRAPHS[name]
    from gwamd import topsim
    return topsim.Graph(os.path.join(DATA, f), V, separator=sep)


def _dense_gpu(g, variant, sample, step, sources, seed=11, C=0.6):
    import torch
    from gwamd import _lib as Cl
    g._ensure_device()
    src = torch.as_tensor(np.asarray(sources, np.int32), device="cuda")
    rows = torch.empty((len(src), g.getVCount()), dtype=torch.float64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    h = g._g.handle
    Cl.check(Cl.lib().gw_topsim_dense(h, variant, sample, step, C, seed, Cl.ptr(src), len(src), Cl.ptr(rows),
                                      Cl.ptr(st), None), h)
    return rows.cpu().numpy(), st.cpu().numpy()


def _oracle(oracle, g, variant, sample, step, sources, seed=11, C=0.6):
    return oracle.topsim(g._offs, g._nbrs, variant, sample, step, C=C, seed=seed, sources=sources, nthreads=8)


@pytest.mark.parametrize("name,sample,step", [("moreno", 1000, 5), ("moreno", 10000, 5), ("g333", 2500, 3),
                                              ("blog", 1000, 5), ("moreno", 40000, 2), ("g333", 100, 8),
                                              # the reference driver's largest SAMPLE at its STEP
                                              # (Test_u_u_TopSim_singleSample.java:36-38; bench config-3 sweep)
                                              ("moreno", 40000, 5), ("blog", 40000, 5)])
def test_topsim_dense_equals_oracle(gw, oracle, name, sample, step):
    g = _graph(gw, name)
    n = g.getVCount()
    sources = np.arange(n, dtype=np.int32) if n <= 1500 else np.arange(0, n, max(1, n // 600), dtype=np.int32)
    rows, st = _dense_gpu(g, 0, sample, step, sources)
    ref, rst = _oracle(oracle, g, 0, sample, step, sources)
    np.testing.assert_allclose(rows, ref, rtol=1e-12, atol=1e-12 * sample)
    assert np.array_equal(rows > 0, ref > 0)
    assert st[0] == rst["extensions"] and st[1] == rst["pair_updates"] and st[3] == rst["walkers"]


@pytest.mark.parametrize("sample,stride", [(5000, 97), (40000, 1931), (1000, 53), (2000, 211)])
def test_topsim_large_n_hash_accumulator(gw, oracle, sample, stride):
    """arxiv (n=38741 > LDS row) takes the LDS-hash path (overflow into the
    HBM hash is exercised by test_topsim_hash_overflow_rmat); SAMPLE <= 2048
    runs the pipelined kernel (wave 0 builds the next source's levels while
    the other waves walk): same rows, and the same extension / pair-update /
    walker counts as the reference's queue."""
    g = _graph(gw, "arxiv")
    sources = np.arange(0, 38741, stride, dtype=np.int32)
    rows, st = _dense_gpu(g, 0, sample, 5, sources)
    ref, rst = _oracle(oracle, g, 0, sample, 5, sources)
    np.testing.assert_allclose(rows, ref, rtol=1e-12, atol=1e-9)
    assert np.array_equal(rows > 0, ref > 0)
    assert st[1] == rst["pair_updates"]
    assert st[0] == rst["extensions"] and st[3] == rst["walkers"]


@pytest.mark.parametrize("step", [1, 2])
def test_topsim_kat_naive_simrank(gw, oracle, step):
    """Deterministic regime: TopSim / SAMPLE == naive SimRank after STEP sweeps."""
    g = _graph(gw, "moreno")
    sample = 1000 if step == 1 else 200000
    rows, st = _dense_gpu(g, 0, sample, step, np.arange(1380))
    assert st[3] == 0
    naive = oracle.simrank_naive(g._offs, g._nbrs, 0.6, step, nthreads=8)
    np.testing.assert_allclose(rows / sample, naive, rtol=0, atol=1e-13)


@pytest.mark.parametrize("variant,sample,step", [(1, 1, 3), (2, 2000, 5), (2, 300, 1)])
def test_topsim_variants(gw, oracle, variant, sample, step):
    g = _graph(gw, "moreno")
    sources = np.arange(0, 1380, 3, dtype=np.int32) if variant == 2 else np.array([0, 5, 17], np.int32)
    rows, st = _dense_gpu(g, variant, sample, step, sources)
    ref, rst = _oracle(oracle, g, variant, sample, step, sources)
    np.testing.assert_allclose(rows, ref, rtol=1e-12, atol=1e-15)
    assert st[1] == rst["pair_updates"]


@pytest.mark.parametrize("name,k", [("moreno", 20), ("blog", 20), ("arxiv", 100), ("arxiv", 3), ("blog", 200), ("blog", 256)])
def test_topk_selection(gw, oracle, name, k):
    import torch
    from gwamd import _lib as Cl
    g = _graph(gw, name)
    n = g.getVCount()
    sources = np.arange(0, n, max(1, n // 400), dtype=np.int32)
    g._ensure_device()
    src = torch.as_tensor(sources, device="cuda")
    ids = torch.empty((len(src), k), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(src), k), dtype=torch.float64, device="cuda")
    h = g._g.handle
    Cl.check(Cl.lib().gw_topsim(h, 0, 2500, 5, 0.6, 11, Cl.ptr(src), len(src), k, Cl.ptr(ids), Cl.ptr(sc),
                                None, None), h)
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    ref, _ = _oracle(oracle, g, 0, 2500, 5, sources)
    for r in range(len(sources)):
        row = ref[r]
        nz = np.nonzero(row > 0)[0]
        order = sorted(nz.tolist(), key=lambda i: (-row[i], i))[:k]
        got = [i for i in ids[r] if i >= 0]
        assert len(got) == len(order)
        np.testing.assert_allclose(sc[r, :len(got)], row[order], rtol=1e-12)
        # ids equal except where scores tie within fp noise
        for a, b in zip(got, order):
            if a != b:
                assert abs(row[a] - row[b]) <= 1e-12 * max(row[b], 1e-300)
        assert np.all(ids[r, len(got):] == -1) and np.all(sc[r, len(got):] == 0.0)


@pytest.mark.parametrize("sample,step,stride", [(1500, 5, 8), (1000, 3, 8)])
def test_topk_pipelined_many_sources_per_workgroup(gw, oracle, sample, step, stride):
    """The hash-mode pipelined kernel's deferred ordering (the last wave ranks
    source r's top-k while the workgroup walks source r+1) runs only when one
    workgroup handles two or more sources: arxiv at SAMPLE <= 2048 on every
    8th vertex (4,843 sources, ~5 per workgroup) against oracle.topsim_topk
    (same walks and sums; ranked score desc / id asc)."""
    import torch
    from gwamd import _lib as Cl
    g = _graph(gw, "arxiv")
    n, K = g.getVCount(), 20
    sources = np.arange(0, n, stride, dtype=np.int32)
    g._ensure_device()
    src = torch.as_tensor(sources, device="cuda")
    ids = torch.empty((len(src), K), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(src), K), dtype=torch.float64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    h = g._g.handle
    Cl.check(Cl.lib().gw_topsim(h, 0, sample, step, 0.6, 11, Cl.ptr(src), len(src), K, Cl.ptr(ids), Cl.ptr(sc),
                                Cl.ptr(st), None), h)
    I, S = ids.cpu().numpy(), sc.cpu().numpy()
    oi, osc, ost = oracle.topsim_topk(g._offs, g._nbrs, 0, sample, step, K, C=0.6, seed=11, sources=sources,
                                      nthreads=8)
    stg = st.cpu().numpy()
    assert int(stg[0]) == ost["extensions"] and int(stg[1]) == ost["pair_updates"]
    for r in range(len(sources)):
        m = int((oi[r] >= 0).sum())
        got = I[r][I[r] >= 0]
        assert len(got) == m
        np.testing.assert_allclose(S[r, :m], osc[r, :m], rtol=1e-12)
        omap = dict(zip(oi[r, :m].tolist(), osc[r, :m].tolist()))
        for k, (a, b) in enumerate(zip(got.tolist(), oi[r, :m].tolist())):  # ids equal except at fp-noise ties
            if a != b:
                sa = omap.get(a, S[r, k])
                assert abs(sa - osc[r, k]) <= 1e-12 * osc[r, k]
        assert np.all(I[r, m:] == -1) and np.all(S[r, m:] == 0.0)


def test_topsim_stretch_pipelined_overflow(gw, oracle):
    """SAMPLE above kPipeMaxSample on the pipelined kernel: a 1M-vertex
    Java-semantics R-MAT (config 5's generator, 1e7 lines) at config 5's
    stretch parameters, SAMPLE 10000 / STEP 5.  The host replay of the
    enumerated part gives W/E ~ 49 (>= 16: k_topsim_pipe<5>), and the sources'
    tens of thousands of distinct targets overflow the LDS table into the HBM
    hash, the compacted overflow list and the capped fold.  Top-100 rows and
    the exact counters against oracle.topsim_topk."""
    import torch
    from gwamd import _lib as Cl
    g = gw.GWGraph.rmat_java(1_000_000, 10_000_000, 0.57, 0.19, 0.19, 42)
    c = g.export_csr()
    offs, nbrs = c["offsets"], c["nbrs"]
    deg = np.diff(offs)
    nz = np.nonzero(deg > 0)[0]
    pick = np.concatenate([nz[np.argsort(deg[nz])[-2:]], nz[np.linspace(0, len(nz) - 1, 30).astype(np.int64)]])
    pick = pick.astype(np.int32)
    g.to_device(0)
    K, sample, step = 100, 10000, 5
    src = torch.as_tensor(pick, device="cuda")
    ids = torch.empty((len(pick), K), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(pick), K), dtype=torch.float64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    Cl.check(Cl.lib().gw_topsim(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), K, Cl.ptr(ids),
                                Cl.ptr(sc), Cl.ptr(st), None), g.handle)
    I, S = ids.cpu().numpy(), sc.cpu().numpy()
    oi, osc, ost = oracle.topsim_topk(offs, nbrs, 0, sample, step, K, C=0.6, seed=42, sources=pick, nthreads=8)
    stg = st.cpu().numpy()
    assert int(stg[0]) == ost["extensions"] and int(stg[1]) == ost["pair_updates"]
    assert int(stg[3]) == ost["walkers"]
    for r in range(len(pick)):
        m = int((oi[r] >= 0).sum())
        got = I[r][I[r] >= 0]
        assert len(got) == m
        np.testing.assert_allclose(S[r, :m], osc[r, :m], rtol=1e-12)
        omap = dict(zip(oi[r, :m].tolist(), osc[r, :m].tolist()))
        for k, (a, b) in enumerate(zip(got.tolist(), oi[r, :m].tolist())):  # ids equal except at fp-noise ties
            if a != b:
                sa = omap.get(a, S[r, k])
                assert abs(sa - osc[r, k]) <= 1e-12 * osc[r, k]


def test_topsim_stretch_many_sources_per_workgroup(gw, oracle):
    """The stretch parameters (SAMPLE 10000 / STEP 5) on 1,536 strided sources
    of the 1M-vertex Java R-MAT: more sources than resident workgroups, so each
    workgroup runs several in a row, mixing append-and-reduce sources (pair-
    update bound over 2x the LDS load limit: appended, partitioned, reduced in
    the emptied LDS table) with light ones (LDS table, HBM hash) — the
    append buffers, partition cursors, per-source overflow table size, LDS
    table and HBM hash must all come back clean between sources.  Top-100 rows
    and the exact counters against oracle.topsim_topk."""
    import torch
    from gwamd import _lib as Cl
    g = gw.GWGraph.rmat_java(1_000_000, 10_000_000, 0.57, 0.19, 0.19, 42)
    c = g.export_csr()
    offs, nbrs = c["offsets"], c["nbrs"]
    deg = np.diff(offs)
    nz = np.nonzero(deg > 0)[0]
    pick = nz[np.linspace(0, len(nz) - 1, 1536).astype(np.int64)].astype(np.int32)
    g.to_device(0)
    K, sample, step = 100, 10000, 5
    src = torch.as_tensor(pick, device="cuda")
    ids = torch.empty((len(pick), K), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(pick), K), dtype=torch.float64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    Cl.check(Cl.lib().gw_topsim(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), K, Cl.ptr(ids),
                                Cl.ptr(sc), Cl.ptr(st), None), g.handle)
    I, S = ids.cpu().numpy(), sc.cpu().numpy()
    oi, osc, ost = oracle.topsim_topk(offs, nbrs, 0, sample, step, K, C=0.6, seed=42, sources=pick, nthreads=16)
    stg = st.cpu().numpy()
    assert int(stg[0]) == ost["extensions"] and int(stg[1]) == ost["pair_updates"]
    assert int(stg[3]) == ost["walkers"]
    for r in range(len(pick)):
        m = int((oi[r] >= 0).sum())
        got = I[r][I[r] >= 0]
        assert len(got) == m
        np.testing.assert_allclose(S[r, :m], osc[r, :m], rtol=1e-12)
        omap = dict(zip(oi[r, :m].tolist(), osc[r, :m].tolist()))
        for k, (a, b) in enumerate(zip(got.tolist(), oi[r, :m].tolist())):  # ids equal except at fp-noise ties
            if a != b:
                sa = omap.get(a, S[r, k])
                assert abs(sa - osc[r, k]) <= 1e-12 * osc[r, k]


def _topk_match(I, S, oi, osc):
    for r in range(len(I)):
        m = int((oi[r] >= 0).sum())
        got = I[r][I[r] >= 0]
        assert len(got) == m
        np.testing.assert_allclose(S[r, :m], osc[r, :m], rtol=1e-12)
        omap = dict(zip(oi[r, :m].tolist(), osc[r, :m].tolist()))
        for k, (a, b) in enumerate(zip(got.tolist(), oi[r, :m].tolist())):  # ids equal except at fp-noise ties
            if a != b:
                sa = omap.get(a, S[r, k])
                assert abs(sa - osc[r, k]) <= 1e-12 * osc[r, k]


def test_topsim_small_hash_graph_more_pair_updates_than_append_room(gw, oracle):
    """A hash-mode graph with V just above the dense LDS row (V = 14,000: 112 KB
    > 96 KB) at the stretch parameters SAMPLE 10000 / STEP 5: the pipelined
    kernel runs (W/E ~ 49), touch_cap = 2^15 and the append buffer holds
    app_cap = 16,384 updates, while a source makes ~50k-75k pair updates.
    V <= app_cap bounds the DISTINCT keys only; the append-and-reduce choice
    must use the uncapped pair-update bound, else the appended updates
    overflow and the call fails with GW_ERR_CAPACITY (round-5 advisor
    finding).  Top-100 rows, dense rows and exact counters against the oracle."""
    import torch
    from gwamd import _lib as Cl
    g = gw.GWGraph.rmat_java(14_000, 350_000, 0.57, 0.19, 0.19, 42)
    c = g.export_csr()
    offs, nbrs = c["offsets"], c["nbrs"]
    deg = np.diff(offs)
    nz = np.nonzero(deg > 0)[0]
    pick = np.concatenate([nz[np.argsort(deg[nz])[-2:]], nz[np.linspace(0, len(nz) - 1, 46).astype(np.int64)]])
    pick = pick.astype(np.int32)
    g.to_device(0)
    K, sample, step = 100, 10000, 5
    src = torch.as_tensor(pick, device="cuda")
    ids = torch.empty((len(pick), K), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(pick), K), dtype=torch.float64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    Cl.check(Cl.lib().gw_topsim(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), K, Cl.ptr(ids),
                                Cl.ptr(sc), Cl.ptr(st), None), g.handle)
    assert Cl.lib().gw_topsim_kernel(g.handle) == b"k_topsim_pipe<5>"
    oi, osc, ost = oracle.topsim_topk(offs, nbrs, 0, sample, step, K, C=0.6, seed=42, sources=pick, nthreads=8)
    stg = st.cpu().numpy()
    assert int(stg[0]) == ost["extensions"] and int(stg[1]) == ost["pair_updates"]
    assert int(stg[3]) == ost["walkers"]
    assert ost["pair_updates"] > 16384 * len(pick)  # more updates per source than the append buffer holds
    _topk_match(ids.cpu().numpy(), sc.cpu().numpy(), oi, osc)
    rows = torch.empty((len(pick), len(deg)), dtype=torch.float64, device="cuda")
    st.zero_()
    Cl.check(Cl.lib().gw_topsim_dense(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), Cl.ptr(rows),
                                      Cl.ptr(st), None), g.handle)
    ref, rst = oracle.topsim(offs, nbrs, 0, sample, step, C=0.6, seed=42, sources=pick, nthreads=8)
    R = rows.cpu().numpy()
    np.testing.assert_allclose(R, ref, rtol=1e-12, atol=1e-12 * sample)
    assert np.array_equal(R > 0, ref > 0)
    assert int(st[1]) == rst["pair_updates"]


def test_topsim_stretch_heavy_sources_sparse_and_dense_rows(gw, oracle):
    """Sparse rows (gw_topsim_sparse, the Java-exact writer's input) and dense
    rows on the pipelined kernel with append-and-reduce sources: the 1M-vertex
    Java R-MAT at SAMPLE 10000 / STEP 5, the two hubs and six strided sources
    (each makes ~50k pair updates: over 2x the LDS load limit and within the
    131,072-entry append buffer).  Rows against the oracle's dense rows
    (rtol 1e-12, identical support) and exact counters; the capacity
    protocol of the sparse rows (too small -> GW_ERR_CAPACITY, *used = room
    needed)."""
    import torch
    from gwamd import _lib as Cl
    g = gw.GWGraph.rmat_java(1_000_000, 10_000_000, 0.57, 0.19, 0.19, 42)
    c = g.export_csr()
    offs, nbrs = c["offsets"], c["nbrs"]
    n = len(offs) - 1
    deg = np.diff(offs)
    nz = np.nonzero(deg > 0)[0]
    pick = np.concatenate([nz[np.argsort(deg[nz])[-2:]], nz[np.linspace(0, len(nz) - 1, 6).astype(np.int64)]])
    pick = pick.astype(np.int32)
    g.to_device(0)
    sample, step = 10000, 5
    src = torch.as_tensor(pick, device="cuda")
    ref, rst = oracle.topsim(offs, nbrs, 0, sample, step, C=0.6, seed=42, sources=pick, nthreads=8)

    def sparse(capacity):
        b = torch.empty(len(pick), dtype=torch.int64, device="cuda")
        ln = torch.empty(len(pick), dtype=torch.int32, device="cuda")
        ids = torch.empty(max(capacity, 1), dtype=torch.int32, device="cuda")
        sc = torch.empty(max(capacity, 1), dtype=torch.float64, device="cuda")
        used = torch.zeros(1, dtype=torch.int64, device="cuda")
        st = torch.zeros(4, dtype=torch.int64, device="cuda")
        rc = Cl.lib().gw_topsim_sparse(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), capacity,
                                       Cl.ptr(b), Cl.ptr(ln), Cl.ptr(ids), Cl.ptr(sc), Cl.ptr(used), Cl.ptr(st), None)
        return rc, b.cpu().numpy(), ln.cpu().numpy(), ids.cpu().numpy(), sc.cpu().numpy(), int(used.cpu()[0]), \
            st.cpu().numpy()

    rc, b, ln, ids, sc, used, st = sparse(20000)
    assert rc == Cl.GW_ERR_CAPACITY and used > 20000
    rc, b, ln, ids, sc, used2, st = sparse(used)
    assert rc == 0 and used2 == used and int(ln.sum()) == used
    assert Cl.lib().gw_topsim_kernel(g.handle) == b"k_topsim_pipe<5>"
    assert int(st[0]) == rst["extensions"] and int(st[1]) == rst["pair_updates"] and int(st[3]) == rst["walkers"]
    for r in range(len(pick)):
        row_ids = ids[b[r]:b[r] + ln[r]]
        assert len(np.unique(row_ids)) == ln[r]
        nzr = np.nonzero(ref[r])[0]
        assert np.array_equal(np.sort(row_ids), nzr)
        np.testing.assert_allclose(sc[b[r]:b[r] + ln[r]], ref[r][row_ids], rtol=1e-12, atol=0)
    rows = torch.empty((len(pick), n), dtype=torch.float64, device="cuda")
    st2 = torch.zeros(4, dtype=torch.int64, device="cuda")
    Cl.check(Cl.lib().gw_topsim_dense(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), Cl.ptr(rows),
                                      Cl.ptr(st2), None), g.handle)
    R = rows.cpu().numpy()
    np.testing.assert_allclose(R, ref, rtol=1e-12, atol=0)
    assert np.array_equal(R > 0, ref > 0)
    assert int(st2[1]) == rst["pair_updates"]


def test_topsim_partition_overflow_reruns_without_append(gw, oracle):
    """The append path's fallback: with gw_options_t.topsim_part_shrink = 5 a
    heavy source's key-hash partitions get 1/32 of their room, so they fill
    (flag 8) and gw_dev_topsim re-runs the launch without the append path,
    from the caller's counters and sparse-row cursor as they were.  Top-k
    rows, sparse rows and exact counters against the oracle (1M-vertex Java
    R-MAT, SAMPLE 10000 / STEP 5, hubs + strided sources)."""
    import torch
    from gwamd import _lib as Cl
    g = gw.GWGraph.rmat_java(1_000_000, 10_000_000, 0.57, 0.19, 0.19, 42)
    c = g.export_csr()
    offs, nbrs = c["offsets"], c["nbrs"]
    deg = np.diff(offs)
    nz = np.nonzero(deg > 0)[0]
    pick = np.concatenate([nz[np.argsort(deg[nz])[-2:]], nz[np.linspace(0, len(nz) - 1, 14).astype(np.int64)]])
    pick = pick.astype(np.int32)
    g.to_device(0)
    assert g.options(topsim_part_shrink=5)["topsim_part_shrink"] == 5
    K, sample, step = 100, 10000, 5
    src = torch.as_tensor(pick, device="cuda")
    ids = torch.empty((len(pick), K), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(pick), K), dtype=torch.float64, device="cuda")
    st = torch.full((4,), 7, dtype=torch.int64, device="cuda")  # accumulated onto, as the caller's counters
    Cl.check(Cl.lib().gw_topsim(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), len(pick), K, Cl.ptr(ids),
                                Cl.ptr(sc), Cl.ptr(st), None), g.handle)
    oi, osc, ost = oracle.topsim_topk(offs, nbrs, 0, sample, step, K, C=0.6, seed=42, sources=pick, nthreads=8)
    stg = st.cpu().numpy()
    assert int(stg[0]) == 7 + ost["extensions"] and int(stg[1]) == 7 + ost["pair_updates"]
    assert int(stg[3]) == 7 + ost["walkers"]
    _topk_match(ids.cpu().numpy(), sc.cpu().numpy(), oi, osc)
    # sparse rows through the re-run: the cursor restarts where the caller left it
    ref, rst = oracle.topsim(offs, nbrs, 0, sample, step, C=0.6, seed=42, sources=pick[:4], nthreads=8)
    cap = 400_000
    b = torch.empty(4, dtype=torch.int64, device="cuda")
    ln = torch.empty(4, dtype=torch.int32, device="cuda")
    sid = torch.empty(cap, dtype=torch.int32, device="cuda")
    ssc = torch.empty(cap, dtype=torch.float64, device="cuda")
    used = torch.zeros(1, dtype=torch.int64, device="cuda")
    st2 = torch.zeros(4, dtype=torch.int64, device="cuda")
    Cl.check(Cl.lib().gw_topsim_sparse(g.handle, 0, sample, step, 0.6, 42, Cl.ptr(src), 4, cap, Cl.ptr(b), Cl.ptr(ln),
                                       Cl.ptr(sid), Cl.ptr(ssc), Cl.ptr(used), Cl.ptr(st2), None), g.handle)
    B, LN, I, S = b.cpu().numpy(), ln.cpu().numpy(), sid.cpu().numpy(), ssc.cpu().numpy()
    assert int(used.cpu()[0]) == int(LN.sum()) and int(st2[1]) == rst["pair_updates"]
    for r in range(4):
        row_ids = I[B[r]:B[r] + LN[r]]
        assert np.array_equal(np.sort(row_ids), np.nonzero(ref[r])[0])
        np.testing.assert_allclose(S[B[r]:B[r] + LN[r]], ref[r][row_ids], rtol=1e-12, atol=0)
    g.options(topsim_part_shrink=0)


def test_mirror_compute_and_print(gw, oracle, tmp_path):
    """TopSim_singleSample mirror + printByOrder on GPU dense rows == Java
    emulation over the oracle rows."""
    from gwamd import topsim
    g = _graph(gw, "moreno")
    ts = topsim.TopSim_singleSample(g, 1000, 1, seed=3)
    ts.compute()
    sim = ts.getResult()
    naive = oracle.simrank_naive(g._offs, g._nbrs, 0.6, 1, nthreads=8)
    np.testing.assert_allclose(sim / 1000, naive, rtol=0, atol=1e-13)
    out = tmp_path / "m.txt"
    topsim.printByOrder(ts, str(out), 20)
    lines = open(str(out) + ".sim.txt", "rb").read().split(b"\r\n")
    for v in (0, 1, 2, 700, 1379):
        exp = oracle.java_fixed_max_pq_row(sim[v], 20)
        assert lines[v].decode() == f"{v}" + "".join(f",{i}:{oracle.java_format_fixed(x)}" for i, x in exp)


def test_enumerate_capacity_error(gw):
    from gwamd import _lib as Cl
    g = _graph(gw, "blog")
    with pytest.raises(Cl.CapacityError):
        _dense_gpu(g, 1, 1, 4, np.array([1], np.int32))


def test_cpp_driver_matches_oracle(gw, oracle, tmp_path):
    """The C++ host mirror's driver (port of Test_u_u_TopSim_singleSample.java)
    writes the same .sim.txt as the Java emulation over the oracle rows, and
    Eval.precision against a naive-SimRank gold file is ~1 in the
    deterministic regime."""
    import subprocess
    from conftest import PKG
    from gwamd import topsim
    exe = os.path.join(PKG, "bin", "test_u_u_topsim_singlesample")
    g = _graph(gw, "moreno")
    naive = oracle.simrank_naive(g._offs, g._nbrs, 0.6, 1, nthreads=8)
    gold = tmp_path / "gold"
    # MyConfiguration.SEPARATOR drives input parsing AND output (Print/Eval)
    topsim.printByOrder(naive, str(gold), 20, separator="\t")
    r = subprocess.run([exe, "--graph", os.path.join(DATA, "moreno_crime_crime.txt"), "--V", "1380", "--sep", "tab",
                        "--steps", "1", "--samples", "1000", "--seed", "3", "--gold", str(gold),
                        "--out", str(tmp_path / "o")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    # ties broken differently by 1-ulp differences cost a few rows
    pre = float(r.stdout.strip().splitlines()[-1])
    assert pre >= 0.99, r.stdout
    rows, _ = oracle.topsim(g._offs, g._nbrs, 0, 1000, 1, seed=3)
    got = open(str(tmp_path / "o_topSimSingle_top20_step1_sample1000.txt.sim.txt"), "rb").read().split(b"\r\n")
    for v in (0, 3, 500, 1379):
        exp = oracle.java_fixed_max_pq_row(rows[v], 20)
        assert got[v].decode() == f"{v}" + "".join(f"\t{i}:{oracle.java_format_fixed(x)}" for i, x in exp)


@pytest.mark.parametrize("sample,step", [(20000, 3), (2000, 4)])
def test_topsim_hash_overflow_rmat(gw, oracle, sample, step):
    """Hub sources of a Java-semantics R-MAT-15 graph reach > 6144 distinct
    targets: the LDS hash overflows into the HBM hash, results unchanged
    (SAMPLE 2000: the pipelined kernel)."""
    import torch
    from gwamd import _lib as Cl
    G = gw.GWGraph.rmat(15, 8, seed=3)
    c = G.export_csr()
    deg = np.diff(c["offsets"])
    rows = np.repeat(np.arange(len(deg)), deg)
    m = rows < c["nbrs"]
    J = gw.GWGraph.from_edges(rows[m], c["nbrs"][m], semantics="java", vcount=len(deg))
    jc = J.export_csr()
    J.to_device(0)
    top = np.argsort(-np.diff(jc["offsets"]))[:16].astype(np.int32)
    ref, rst = oracle.topsim(jc["offsets"], jc["nbrs"], 0, sample, step, seed=9, sources=top, nthreads=8)
    assert (ref > 0).sum(axis=1).max() > 4608  # past the 6144-slot LDS hash's load limit
    src = torch.as_tensor(top, device="cuda")
    out = torch.empty((len(top), len(deg)), dtype=torch.float64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    Cl.check(Cl.lib().gw_topsim_dense(J.handle, 0, sample, step, 0.6, 9, Cl.ptr(src), len(top), Cl.ptr(out),
                                      Cl.ptr(st), None), J.handle)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-12, atol=1e-9)
    assert int(st[1]) == rst["pair_updates"]
    # top-k path over the same overflowing rows
    k = 100
    ids = torch.empty((len(top), k), dtype=torch.int32, device="cuda")
    sc = torch.empty((len(top), k), dtype=torch.float64, device="cuda")
    Cl.check(Cl.lib().gw_topsim(J.handle, 0, sample, step, 0.6, 9, Cl.ptr(src), len(top), k, Cl.ptr(ids), Cl.ptr(sc),
                                None, None), J.handle)
    for r in range(len(top)):
        row = ref[r]
        order = sorted(np.nonzero(row > 0)[0].tolist(), key=lambda i: (-row[i], i))[:k]
        np.testing.assert_allclose(sc.cpu().numpy()[r], row[order], rtol=1e-12)


def _sparse_gpu(g, sample, step, sources, capacity, seed=11):
    import torch
    from gwamd import _lib as Cl
    g._ensure_device()
    src = torch.as_tensor(np.asarray(sources, np.int32), device="cuda")
    b = torch.empty(len(src), dtype=torch.int64, device="cuda")
    ln = torch.empty(len(src), dtype=torch.int32, device="cuda")
    ids = torch.empty(max(capacity, 1), dtype=torch.int32, device="cuda")
    sc = torch.empty(max(capacity, 1), dtype=torch.float64, device="cuda")
    used = torch.full((1,), 123, dtype=torch.int64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    h = g._g.handle
    rc = Cl.lib().gw_topsim_sparse(h, 0, sample, step, 0.6, seed, Cl.ptr(src), len(src), capacity, Cl.ptr(b),
                                   Cl.ptr(ln), Cl.ptr(ids), Cl.ptr(sc), Cl.ptr(used), Cl.ptr(st), None)
    return rc, b.cpu().numpy(), ln.cpu().numpy(), ids.cpu().numpy(), sc.cpu().numpy(), int(used.cpu()[0]), \
        st.cpu().numpy()


def _scatter(n, b, ln, ids, sc):
    rows = np.zeros((len(b), n))
    for r in range(len(b)):
        rows[r, ids[b[r]:b[r] + ln[r]]] = sc[b[r]:b[r] + ln[r]]
    return rows


@pytest.mark.parametrize("name,sample,step", [("moreno", 10000, 5), ("blog", 2500, 5), ("arxiv", 5000, 5)])
def test_sparse_rows_equal_oracle_and_write_exact(gw, oracle, tmp_path, name, sample, step):
    """gw_topsim_sparse: every nonzero entry of each row (== the oracle's rows
    at rtol 1e-12, identical support, same counters); the capacity protocol
    (too small -> GW_ERR_CAPACITY, *used = room needed, rows that did not fit
    marked -1); and gw_write_sim_text_sparse on those rows byte-identical to
    the Java-exact dense writer on the same values (Print.java:25-53)."""
    from gwamd import _lib as Cl
    g = _graph(gw, name)
    n = g.getVCount()
    sources = np.arange(n, dtype=np.int32) if n <= 1500 else np.arange(3, n, max(1, n // 500), dtype=np.int32)
    rc, b, ln, ids, sc, used, st = _sparse_gpu(g, sample, step, sources, 1000)
    assert rc == Cl.GW_ERR_CAPACITY and used > 1000
    assert np.all((ln == -1) == (b == -1)) and (ln == -1).any()
    ok = ln >= 0
    assert int(ln[ok].sum()) <= 1000
    rc, b, ln, ids, sc, used2, st = _sparse_gpu(g, sample, step, sources, used)
    assert rc == 0 and used2 == used and int(ln.sum()) == used and np.all(ln >= 0)
    rows = _scatter(n, b, ln, ids, sc)
    ref, rst = _oracle(oracle, g, 0, sample, step, sources)
    np.testing.assert_allclose(rows, ref, rtol=1e-12, atol=0)
    assert np.array_equal(rows > 0, ref > 0)
    assert st[0] == rst["extensions"] and st[1] == rst["pair_updates"] and st[3] == rst["walkers"]
    for topk in (20, 100):
        d, s = tmp_path / f"d{topk}", tmp_path / f"s{topk}"
        Cl.check(Cl.lib().gw_write_sim_text_dense(str(d).encode(), Cl.ptr(rows), Cl.ptr(sources), len(sources), n,
                                                  topk, b",", 6))
        Cl.check(Cl.lib().gw_write_sim_text_sparse(str(s).encode(), Cl.ptr(b), Cl.ptr(ln), Cl.ptr(ids), Cl.ptr(sc),
                                                   Cl.ptr(sources), len(sources), n, topk, b",", 6))
        assert open(str(s) + ".sim.txt", "rb").read() == open(str(d) + ".sim.txt", "rb").read()
        assert open(s, "rb").read() == open(d, "rb").read()


@pytest.mark.parametrize("name,sample,step,topk", [("moreno", 1000, 5, 20), ("blog", 1000, 3, 100),
                                                   ("arxiv", 2500, 5, 20),
                                                   # the reference driver's largest SAMPLE, its STEP and
                                                   # topK (Test_u_u_TopSim_singleSample.java:36-38, testTopK)
                                                   ("moreno", 40000, 5, 20), ("blog", 40000, 5, 20),
                                                   ("arxiv", 40000, 5, 20)])
def test_write_text_matches_java_print_on_oracle_rows(gw, oracle, tmp_path, name, sample, step, topk):
    """gw_topsim_write_text (compute + Print.printByOrder at any V, the path
    of config 5 and the JNI writer) against Print.printByOrder's Java
    emulation over the oracle's rows (Java-literal summation order): min(topk,
    V) entries per row including zero-score ids, same ids in the same order
    except where two oracle values are equal within fp64 accumulation noise
    (the GPU adds with atomics: rtol 1e-12), same %.6f strings except where
    the value sits on a HALF_UP rounding boundary (C = 0.6 and integer SAMPLE
    and degrees make exact decimal halves common, and an ulp decides them)."""
    from gwamd import topsim
    g = _graph(gw, name)
    n = g.getVCount()
    sources = np.arange(n, dtype=np.int32) if n <= 1500 else np.arange(1, n, max(1, n // 300), dtype=np.int32)
    ts = topsim.TopSim_singleSample(g, sample, step, seed=11)
    out = tmp_path / "w.txt"
    ts.writeText(str(out), topk, sources=sources)
    ref, rst = _oracle(oracle, g, 0, sample, step, sources)
    assert ts.stats["pair_updates"] == rst["pair_updates"]
    got = open(str(out) + ".sim.txt", "rb").read().decode().split("\r\n")
    assert got[-1] == "" and len(got) == len(sources) + 1
    diff_vals = 0
    for r, v in enumerate(sources):
        exp = oracle.java_fixed_max_pq_row(ref[r], topk)
        toks = got[r].split(",")
        assert toks[0] == str(v) and len(toks) - 1 == len(exp) == min(topk, n)
        for t, (i, x) in zip(toks[1:], exp):
            gi, gs = t.split(":")
            if int(gi) != i:
                assert abs(ref[r][int(gi)] - x) <= 1e-12 * max(x, 1e-300), (v, gi, i)
            es = oracle.java_format_fixed(x)
            if gs != es:
                diff_vals += 1
                assert abs(float(gs) - float(es)) <= 1.000001e-6, (v, gs, es)
                frac = x * 1e6 - np.floor(x * 1e6)
                assert abs(frac - 0.5) < 1e-4, (v, gs, es, x)
    assert diff_vals <= max(2, len(sources) * topk // 1000)
