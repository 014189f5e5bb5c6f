"""CPU: the C-ABI library loads, exports every declared symbol, and its host
logic (graph semantics, generators, writers) matches the reference formats.
No compute (GPU) calls are made here."""
import os
import re

import numpy as np
import pytest

from conftest import DATA, ROOT, golden_index, load_golden

CASES = golden_index()["cases"]


def test_exports_every_declared_symbol(gw):
    with open(os.path.join(ROOT, "include", "graphwalk.h")) as f:
        hdr = f.read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = sorted(set(re.findall(r"\b(gw_[a-z0-9_]+)\s*\(", hdr)))
    assert len(declared) >= 20
    L = gw.lib()
    for name in declared:
        assert hasattr(L, name), name
    from gwamd._lib import SIGNATURES
    assert sorted(SIGNATURES) == declared


def test_version_and_errors(gw):
    L = gw.lib()
    assert b"gfx950" in L.gw_version()
    assert L.gw_strerror(-11) == b"capacity exceeded"


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["file"])
def test_nx_loader_matches_networkx(case, gw):
    """gw_graph_load_edgelist(NX_SIMPLE) == read_graph (main.py:76-89) as
    networkx built it when the goldens were generated."""
    g = load_golden(case["file"])
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, case["graph"]), delimiter=case["delimiter"],
                                 semantics="nx", directed=case["directed"], weighted=case["weighted"])
    c = G.export_csr()
    np.testing.assert_array_equal(c["labels"], g["labels"])
    np.testing.assert_array_equal(c["offsets"], g["offsets"])
    np.testing.assert_array_equal(c["labels"][c["nbrs"]], g["nbrs"])
    np.testing.assert_array_equal(c["weights"], g["weights"])
    np.testing.assert_array_equal(c["labels"][c["node_order"]], g["node_order"])
    assert G.info().device == -1


def test_from_networkx_matches_loader(gw):
    import networkx as nx
    path = os.path.join(DATA, "weighted_quirks.edgelist")
    G = nx.read_edgelist(path, nodetype=int, data=(("weight", float),), create_using=nx.DiGraph(),
                         delimiter=" ").to_undirected()
    a = gw.GWGraph.from_networkx(G).export_csr()
    b = gw.GWGraph.from_edgelist(path, " ", "nx", False, True).export_csr()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize("fname,V,sep", [("moreno_crime_crime.txt", 1380, "\t"),
                                         ("blog.txt", 10313, ","), ("0_333_5038.txt", 333, " ")])
def test_java_loader(fname, V, sep, gw):
    """gw_graph_load_edgelist(JAVA_MULTI) == structures.Graph (Graph.java:28-57)."""
    adj = [[] for _ in range(V)]
    with open(os.path.join(DATA, fname)) as f:
        for line in f:
            a, b = line.rstrip("\r\n").split(sep)[:2]
            adj[int(a)].append(int(b))
            adj[int(b)].append(int(a))
    c = gw.GWGraph.from_edgelist(os.path.join(DATA, fname), delimiter=sep, semantics="java",
                                 vcount=V).export_csr()
    np.testing.assert_array_equal(np.diff(c["offsets"]), [len(x) for x in adj])
    np.testing.assert_array_equal(c["nbrs"], [y for x in adj for y in x])


def test_java_loader_errors(gw, tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("0,1\n2,7\n")
    with pytest.raises(IndexError):  # ArrayIndexOutOfBounds: id >= V
        gw.GWGraph.from_edgelist(str(p), ",", "java", vcount=5)
    p.write_text("0\t1\n")
    with pytest.raises(ValueError):  # shipped SEPARATOR "," cannot parse tab files
        gw.GWGraph.from_edgelist(str(p), ",", "java", vcount=5)
    p.write_text("0,1\n\n1,2\n")
    with pytest.raises(ValueError):  # blank line -> ids[1] out of bounds in Java
        gw.GWGraph.from_edgelist(str(p), ",", "java", vcount=5)


def test_nx_loader_quirks(gw, tmp_path):
    p = tmp_path / "e.txt"
    # comments, blank lines, '\r', trailing-delimiter error
    p.write_text("# header\n5 7\n\n7 9 # c\n")
    with pytest.raises(ValueError):  # "7 9 " -> extra empty data token (networkx TypeError)
        gw.GWGraph.from_edgelist(str(p), " ", "nx")
    p.write_text("# header\n5 7\r\n\n7 9\n9 5\n")
    c = gw.GWGraph.from_edgelist(str(p), " ", "nx").export_csr()
    np.testing.assert_array_equal(c["labels"], [5, 7, 9])
    np.testing.assert_array_equal(c["offsets"], [0, 2, 4, 6])
    # default delimiter ',' on a space file parses zero edges
    c = gw.GWGraph.from_edgelist(os.path.join(DATA, "karate.edgelist"), ",", "nx").export_csr()
    assert len(c["labels"]) == 0


def test_rmat_generator(gw):
    G = gw.GWGraph.rmat(12, 16, seed=42)
    c = G.export_csr()
    n = len(c["labels"])
    offs, nbrs = c["offsets"], c["nbrs"]
    deg = np.diff(offs)
    assert deg.min() >= 1  # isolated vertices removed
    rows = np.repeat(np.arange(n), deg)
    assert not np.any(rows == nbrs)  # no self loops
    for v in range(0, n, 97):
        r = nbrs[offs[v]:offs[v + 1]]
        assert np.all(np.diff(r) > 0)  # sorted, deduplicated
    key = set(zip(rows.tolist(), nbrs.tolist()))
    assert all((b, a) in key for (a, b) in list(key)[:5000])  # symmetric
    c2 = gw.GWGraph.rmat(12, 16, seed=42).export_csr()
    np.testing.assert_array_equal(c2["nbrs"], nbrs)  # deterministic
    c3 = gw.GWGraph.rmat(12, 16, seed=43).export_csr()
    assert len(c3["nbrs"]) != len(nbrs) or not np.array_equal(c3["nbrs"], nbrs)


def test_walk_writer_format(gw, tmp_path):
    """DeepSim save_list (DeepSim/src/main.py:237-243): 'id\\t' per id."""
    from gwamd import io
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "karate.edgelist"), " ", "nx")
    lab = G.export_csr()["labels"]
    walks = np.array([[0, 1, 2, -1], [3, 3, 4, 5]], np.int32)
    p1 = tmp_path / "a.txt"
    p2 = tmp_path / "b.txt"
    io.save_walks(G, p1, walks)
    io.save_list([[int(lab[0]), int(lab[1]), int(lab[2])], [int(lab[i]) for i in (3, 3, 4, 5)]], p2)
    assert p1.read_bytes() == p2.read_bytes()
    assert io.read_list(p1)[1] == [str(int(lab[i])) for i in (3, 3, 4, 5)]


def test_sim_writer_java_exact(gw, oracle, tmp_path):
    """Print.printByOrder (Print.java:25-53): FixedMaxPQ tie order and Java
    %.6f HALF_UP, CRLF line ends."""
    from gwamd import topsim
    rng = np.random.RandomState(0)
    rows = np.round(rng.rand(40, 57) * 8) / 8  # many ties
    rows[3] = 0.0
    rows[5, :5] = 1.0000005
    out = tmp_path / "s.txt"
    topsim.printByOrder(rows, str(out), topk=20)
    lines = open(str(out) + ".sim.txt", "rb").read().split(b"\r\n")
    ids_lines = open(out, "rb").read().split(b"\r\n")
    for v in range(40):
        exp = oracle.java_fixed_max_pq_row(rows[v], 20)
        s = f"{v}" + "".join(f",{i}:{oracle.java_format_fixed(x)}" for i, x in exp)
        assert lines[v].decode() == s
        assert ids_lines[v].decode() == f"{v}" + "".join(f",{i}" for i, _ in exp)


def _sparse_of(rows, rng):
    """Nonzero entries of each row, shuffled within the row (the device emits
    them in accumulator order), packed with gaps like claimed offsets."""
    begin, ln, ids, sc = [], [], [], []
    pos = 0
    for r in range(rows.shape[0]):
        nz = np.nonzero(rows[r])[0]
        nz = nz[rng.permutation(len(nz))]
        pos += int(rng.integers(0, 3))  # unused room between rows
        while len(ids) < pos:
            ids.append(-7)
            sc.append(-1.0)
        begin.append(pos)
        ln.append(len(nz))
        ids.extend(nz.tolist())
        sc.extend(rows[r, nz].tolist())
        pos += len(nz)
    return (np.array(begin, np.int64), np.array(ln, np.int32), np.array(ids, np.int32),
            np.array(sc, np.float64))


@pytest.mark.parametrize("topk", [0, 1, 7, 20, 57, 80])
def test_sim_writer_sparse_equals_dense(gw, oracle, tmp_path, topk):
    """gw_write_sim_text_sparse (the exact top-k path, rows given as their
    nonzero entries only) == gw_write_sim_text_dense on the same rows, byte
    for byte: FixedMaxPQ's fill with zero-score ids, strict replacement and
    sortedElement() tie order (Print.java:30-47, FixedMaxPQ.java:30-39,
    72-76).  Rows with many ties, few nonzeros (fewer than topk: zero ids
    included), all-zero rows, and topk above the row length."""
    from gwamd import _lib as C
    rng = np.random.default_rng(5)
    n = 57
    rows = np.round(rng.random((60, n)) * 6) / 6  # many ties, ~1/12 zeros
    rows[rng.random((60, n)) < 0.5] = 0.0
    rows[3] = 0.0
    rows[4] = 0.0
    rows[4, [50, 2, 40]] = [0.5, 0.5, 0.25]  # fewer nonzeros than topk
    rows[6, :] = 0.0
    rows[6, 56] = 1.0
    rid = np.arange(100, 160, dtype=np.int32)
    dense = tmp_path / "d.txt"
    sparse = tmp_path / "s.txt"
    C.check(C.lib().gw_write_sim_text_dense(str(dense).encode(), C.ptr(np.ascontiguousarray(rows)), C.ptr(rid),
                                            rows.shape[0], n, topk, b",", 6))
    b, ln, ids, sc = _sparse_of(rows, rng)
    C.check(C.lib().gw_write_sim_text_sparse(str(sparse).encode(), C.ptr(b), C.ptr(ln), C.ptr(ids), C.ptr(sc),
                                             C.ptr(rid), rows.shape[0], n, topk, b",", 6))
    assert open(sparse, "rb").read() == open(dense, "rb").read()
    assert open(str(sparse) + ".sim.txt", "rb").read() == open(str(dense) + ".sim.txt", "rb").read()
    lines = open(str(sparse) + ".sim.txt", "rb").read().split(b"\r\n")
    for v in range(rows.shape[0]):
        exp = oracle.java_fixed_max_pq_row(rows[v], topk) if topk else []
        assert lines[v].decode() == f"{rid[v]}" + "".join(f",{i}:{oracle.java_format_fixed(x)}" for i, x in exp)
        assert len(exp) == min(topk, n)


def test_sim_writer_sparse_rejects_bad_rows(gw, tmp_path):
    from gwamd import _lib as C
    b = np.array([0], np.int64)
    for ln, ids, sc in [([-1], [0], [1.0]), ([2], [3, 3], [1.0, 2.0]), ([1], [9], [1.0]), ([1], [2], [0.0])]:
        ln, ids, sc = np.array(ln, np.int32), np.array(ids, np.int32), np.array(sc)  # alive across the call
        rc = C.lib().gw_write_sim_text_sparse(str(tmp_path / "x").encode(), C.ptr(b), C.ptr(ln), C.ptr(ids),
                                              C.ptr(sc), None, 1, 5, 3, b",", 6)
        assert rc in (C.GW_ERR_INVALID, C.GW_ERR_RANGE)


def test_sim_writer_print_by_order_all(gw, oracle, tmp_path):
    """Print.printByOrderAll (Print.java:55-84): %.7f, topk 1000 > row length."""
    from gwamd import topsim
    rng = np.random.RandomState(1)
    rows = np.round(rng.rand(12, 30) * 64) / 64 * 1e-6
    rows[2, 3] = 5e-08
    out = tmp_path / "a.txt"
    topsim.printByOrderAll(rows, str(out), 1000, 10)
    lines = open(str(out) + ".sim.txt", "rb").read().split(b"\r\n")
    for v in range(12):
        exp = oracle.java_fixed_max_pq_row(rows[v], 1000)
        assert lines[v].decode() == f"{v}" + "".join(f",{i}:{oracle.java_format_fixed(x, 7)}" for i, x in exp)


def test_precision_metric(tmp_path):
    """Eval.precision (Eval.java:81-131)."""
    from gwamd import topsim
    g = tmp_path / "g.sim.txt"
    t = tmp_path / "t.sim.txt"
    g.write_text("0,1:0.5,2:0.4,3:0.0\r\n1,0:0.0\r\n")
    t.write_text("0,2:0.9,5:0.3\r\n1,4:0.2\r\n")
    pre = topsim.precision(str(g), str(t), str(tmp_path / "p.txt"), 20)
    assert pre == pytest.approx((0.5 + 1.0) / 2)


def test_compute_calls_fail_loudly_without_gpu(gw):
    """No CPU fallback: on a host without a GPU the device calls raise."""
    from gwamd._lib import DeviceError
    if gw.device_count() > 0:
        pytest.skip("a GPU is visible")
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "karate.edgelist"), " ", "nx")
    with pytest.raises(DeviceError):
        G.to_device(0)
    with pytest.raises(Exception):
        from gwamd.node2vec import alias_setup
        alias_setup([0.5, 0.5])
    # naive SimRank refuses a graph that is not on a device (no host compute)
    import numpy as np
    from gwamd import _lib as C
    out = np.zeros(34 * 34)
    with pytest.raises(C.StateError):
        C.check(C.lib().gw_simrank_naive_host(G.handle, 0.6, 3, C.ptr(out)), G.handle)


def test_select_fixed_max_pq_for_topsim_dev(gw, oracle):
    """TopSim_Dev's candidate choice (TopSim_Dev.java:64-71): FixedMaxPQ over
    entries >= MIN in j order, sortedElement() order (ties included)."""
    from gwamd import topsim
    rng = np.random.RandomState(3)
    cand = np.round(rng.rand(30, 41) * 6) / 6
    cand[cand < 0.2] = 1e-12  # below MyConfiguration.MIN
    cand[4] = 0.0
    ids = topsim.select_candidates(cand, 7)
    for i in range(30):
        exp = [j for j, _ in oracle.java_fixed_max_pq_row(cand[i], 7, min_score=topsim.MIN)]
        assert ids[i].tolist() == exp + [-1] * (7 - len(exp))


def test_cachemap_writer_format(gw, oracle, tmp_path):
    """Print.printByOrder(FixedCacheMap[], outPath, topk) (Print.java:94-124):
    the last topk entries of each ascending iteration, %.6f of the float
    value widened to double, CRLF; rows of fewer than topk print whole."""
    from gwamd import _lib as C
    cap = 6
    keys = np.array([[5, 2, 9, 1, -1, -1], [3, 4, 7, 8, 0, 6], [-1] * 6], np.int32)
    vals = np.array([[0.1, 0.25, 0.3, 1.5, 0, 0], [1e-7, 2e-7, 0.5, 0.5, 0.75, 3.0], [0] * 6], np.float32)
    size = np.array([4, 6, 0], np.int32)
    out = tmp_path / "c.txt"
    C.check(C.lib().gw_write_sim_text_cachemap(str(out).encode(), C.ptr(keys), C.ptr(vals), C.ptr(size), None, 3,
                                               cap, 4, b","))
    lines = open(str(out) + ".sim.txt", "rb").read().split(b"\r\n")
    ids = open(out, "rb").read().split(b"\r\n")
    for r in range(3):
        lo = max(0, size[r] - 4)
        exp = [(int(keys[r, i]), float(vals[r, i])) for i in range(lo, size[r])]
        assert lines[r].decode() == f"{r}" + "".join(f",{k}:{oracle.java_format_fixed(v)}" for k, v in exp)
        assert ids[r].decode() == f"{r}" + "".join(f",{k}" for k, _ in exp)


def test_walk_writer_large_and_range(gw, tmp_path):
    """The parallel writer (label text table, chunked formatting overlapped
    with ordered writes) equals Python's save_list across many chunks and
    batches, and refuses entries outside the graph (GW_ERR_RANGE)."""
    from gwamd import io
    G = gw.GWGraph.rmat(10, 8, seed=7)
    lab = G.export_csr()["labels"]
    rng = np.random.default_rng(3)
    nw, L = 2_100_000 // 20, 20  # 105,000 walks: 13 chunks of 8,192
    W = rng.integers(0, G.n, (nw, L)).astype(np.int32)
    cut = rng.integers(1, L + 1, nw)
    W[np.arange(L)[None, :] >= cut[:, None]] = -1  # ragged walks, -1 padded
    p1 = tmp_path / "a.txt"
    io.save_walks(G, p1, W)
    expect = "".join("".join(f"{int(lab[x])}\t" for x in row[row >= 0]) + "\n" for row in W)
    assert p1.read_text() == expect
    W[nw // 2, 0] = G.n  # outside the graph
    with pytest.raises(IndexError):  # GW_ERR_RANGE
        io.save_walks(G, tmp_path / "b.txt", W)


def test_comm_argument_errors(gw):
    """gw_comm_* without a GPU: argument checks and error strings (RCCL is
    loaded only on first use; no collective runs here)."""
    import ctypes
    from gwamd import _lib as C
    L = gw.lib()
    uid = (ctypes.c_uint8 * 128)()
    h = ctypes.c_void_p()
    p_uid = ctypes.cast(uid, ctypes.c_void_p)
    assert L.gw_comm_init(p_uid, 2, 2, 0, ctypes.byref(h)) == C.GW_ERR_INVALID  # rank >= nranks
    assert L.gw_comm_init(p_uid, 0, 0, 0, ctypes.byref(h)) == C.GW_ERR_INVALID
    assert L.gw_comm_init(None, 1, 0, 0, ctypes.byref(h)) == C.GW_ERR_INVALID
    assert L.gw_last_error(None) is not None
    assert L.gw_comm_last_error(None) == b"bad arguments"
    assert L.gw_comm_allgather(None, None, None, 4, 0, None) == C.GW_ERR_INVALID
    assert L.gw_comm_free(None) == C.GW_OK
    assert L.gw_comm_unique_id(None) == C.GW_ERR_INVALID


def test_release_library_has_no_diagnostic_knobs(gw):
    """The GW_DIAG_* timing knobs (some return wrong walks on purpose) are
    compiled only into the -DGW_DIAG library (build.py --diag): the release
    libgraphwalk.so neither names nor reads them."""
    from gwamd import _lib
    if os.path.basename(_lib.LIB_PATH) != "libgraphwalk.so":
        pytest.skip("GW_LIB points at a non-release library")
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"GW_DIAG" not in blob


def test_release_library_reads_no_environment_knobs(gw):
    """Sizing / sampler choices are per-handle options (gw_graph_set_options),
    not environment variables: no source of the library calls getenv except
    through the -DGW_DIAG-only GW_DIAG_ENV macro, and the release binary names
    none of the former knobs.  (The only getenv left in the binary is rocPRIM's
    own ROCPRIM_USE_ATOMIC_BLOCK_ID, inside its device scan.)"""
    import glob
    from gwamd import _lib
    srcs = glob.glob(os.path.join(ROOT, "graph-embedding_amd", "csrc", "*"))
    for f in srcs:
        txt = open(f).read()
        for m in re.finditer(r"\bgetenv\s*\(", txt):
            line = txt[:m.start()].count("\n") + 1
            assert f.endswith("gw_internal.h") and "GW_DIAG_ENV" in txt.splitlines()[line - 1], (f, line)
    if os.path.basename(_lib.LIB_PATH) != "libgraphwalk.so":
        pytest.skip("GW_LIB points at a non-release library")
    blob = open(_lib.LIB_PATH, "rb").read()
    for knob in (b"GW_SENT_MAX_GB", b"GW_BITSET_BUDGET_GB", b"GW_HOST_CHUNK_MB", b"GW_SIMRANK_HBM_ROW"):
        assert knob not in blob


def test_options_roundtrip_and_validation(gw):
    import ctypes
    from gwamd import _lib as C
    G = gw.GWGraph.from_edgelist(os.path.join(DATA, "karate.edgelist"), " ", "nx")
    d = G.options()
    assert d == dict(table_budget_bytes=0, expected_steps=0, listed=-1, simrank_hbm_row=0, host_chunk_bytes=0,
                     topsim_part_shrink=0, reserved0=0)
    d = G.options(expected_steps=123, listed=0, host_chunk_bytes=1 << 20, topsim_part_shrink=3)
    assert d["expected_steps"] == 123 and d["listed"] == 0 and d["host_chunk_bytes"] == 1 << 20
    assert d["topsim_part_shrink"] == 3
    for bad in (C.Options(0, 0, 2, 0, 0, 0, 0), C.Options(0, 0, 0, 0, 0, 9, 0), C.Options(0, 0, 0, 0, 0, -1, 0),
                C.Options(0, 0, 0, 0, 0, 0, 1)):
        assert C.lib().gw_graph_set_options(G.handle, ctypes.byref(bad)) == C.GW_ERR_INVALID
    assert C.lib().gw_graph_set_options(G.handle, None) == 0
    assert G.options()["listed"] == -1


def test_java_double_to_string_matches_java(gw, oracle):
    """gw_format_java_double == Java's Double.toString (Eval.java:118 writes
    precision values this way) on known Java outputs and random doubles."""
    import ctypes
    from gwamd import _lib as C

    def fmt(v):
        buf = ctypes.create_string_buffer(64)
        C.check(C.lib().gw_format_java_double(float(v), buf, 64))
        return buf.value.decode()
    known = [(1.0, "1.0"), (0.0, "0.0"), (-0.0, "-0.0")] + list({0.5: "0.5", 0.001: "0.001", 1e-4: "1.0E-4",
             1e7: "1.0E7", 9999999.0: "9999999.0", 123456789.0: "1.23456789E8", 0.1 + 0.2: "0.30000000000000004",
             2 / 3: "0.6666666666666666", -2.5: "-2.5", 100.0: "100.0", 0.05: "0.05", 1234.5678: "1234.5678",
             -3.2e-5: "-3.2E-5", 1.5e300: "1.5E300", float("nan"): "NaN", float("inf"): "Infinity"}.items())
    for v, s in known:
        assert fmt(v) == s, (v, fmt(v), s)
        assert oracle.java_double_to_string(v) == s, (v, s)
    rng = np.random.default_rng(5)
    for v in np.concatenate([rng.random(300), rng.random(200) * 10.0 ** rng.integers(-8, 12, 200),
                             -rng.random(50) * 1e3, np.arange(0, 21) / 20.0]):
        assert fmt(v) == oracle.java_double_to_string(v), v
    buf = ctypes.create_string_buffer(3)
    assert C.lib().gw_format_java_double(0.123, buf, 3) == C.GW_ERR_RANGE


def test_read_simrank_reads_topk_writer_output(gw, tmp_path):
    """gwamd.io.read_simrank (DeepSim/src/main.py:83-107) on a .sim.txt that
    gw_write_sim_text_topk wrote: rows in order, ids in score order, values
    <= 1e-8 (printed 0.000000) dropped."""
    from gwamd import _lib as C
    from gwamd.io import read_simrank
    ids = np.array([[4, 1, 2], [0, 3, 2], [1, 0, 4]], np.int32)
    sc = np.array([[0.75, 0.125, 0.0], [3.5, 1e-9, 0.0], [2.0000005, 0.0, 0.0]], np.float64)
    rid = np.array([0, 1, 2], np.int32)
    path = str(tmp_path / "topk")
    C.check(C.lib().gw_write_sim_text_topk(path.encode(), C.ptr(ids), C.ptr(sc), C.ptr(rid), 3, 3, b",", 6))
    got = read_simrank(path + ".sim.txt")
    assert [[i for i, _ in row] for row in got] == [["4", "1"], ["0"], ["1"]]
    assert [[float(v) for _, v in row] for row in got] == [[0.75, 0.125], [3.5], [2.000001]]


MALFORMED = [
    b"", b"\n\n\n", b"# only a comment\n", b"1", b"1 ", b"1 2 3 4 5\n", b"a b\n", b"1 b\n", b"1 2\n3",
    b"99999999999999999999999 1\n", b"-1 2\n", b"1 -2\n", b"1\x002\n", b"\xff\xfe 1\n", b"1 2 nan\n", b"1 2 inf\n",
    b"1 2 1e999\n", b"1 2 -0.5\n", b"1\t2\n", b"1  2\n", b"\r\r\r", b"1 2\r3 4\r", b" 1 2\n", b"1 2 \n",
    b"1" * 100000 + b" 2\n", (b"1 2\n" * 50000)[:-3],
]


@pytest.mark.parametrize("blob", MALFORMED, ids=[str(i) for i in range(len(MALFORMED))])
@pytest.mark.parametrize("sem", ["nx", "java"])
def test_loaders_survive_malformed_input(gw, tmp_path, blob, sem):
    """Malformed, truncated and oversized edge lists (Graph.java:38-39 and
    networkx read_edgelist error cases): the loaders either build a graph or
    raise a library error — never crash (tools/sanitize.sh runs this under
    ASan/UBSan)."""
    from gwamd import _lib as C
    p = tmp_path / "m.txt"
    p.write_bytes(blob)
    for weighted in (False, True):
        try:
            g = gw.GWGraph.from_edgelist(str(p), " ", sem, False, weighted, vcount=5 if sem == "java" else -1)
        except (C.GraphWalkError, ValueError, IndexError, KeyError, OSError, ZeroDivisionError):
            continue
        csr = g.export_csr()
        assert csr["offsets"][-1] == len(csr["nbrs"]) and np.all(np.diff(csr["offsets"]) >= 0)
        if len(csr["nbrs"]):
            assert csr["nbrs"].min() >= 0 and csr["nbrs"].max() < len(csr["offsets"]) - 1
        g.free()


def test_generators_and_csr_reject_bad_sizes(gw):
    from gwamd import _lib as C
    for scale, ef in ((-1, 16), (0, 16), (63, 16), (10, -3), (10, 0)):
        try:
            gw.GWGraph.rmat(scale, ef).free()
        except (C.GraphWalkError, ValueError, MemoryError):
            pass
    with pytest.raises(Exception):
        gw.GWGraph.from_csr(np.array([0, 3, 2], np.int64), np.array([1, 0, 1], np.int32))  # offsets decrease
    with pytest.raises(Exception):
        gw.GWGraph.from_csr(np.array([0, 1, 2], np.int64), np.array([1, 7], np.int32))  # neighbour id >= n


def test_jni_shim_calls_only_exported_abi(gw):
    """graph-embedding_amd/jni/graphwalk_jni.c (built only where a JDK exists,
    untested here): every gw_* function it calls is declared in
    include/graphwalk.h and exported by libgraphwalk.so, and every native
    method of simrank.GraphWalkNative has its Java_simrank_GraphWalkNative_* C
    definition.  Every Java-facing writer must emit Print.printByOrder's bytes
    (Print.java:25-53, FixedMaxPQ.java:30-39, 72-76): the shim may reach the
    sim-file writers only through gw_topsim_write_text (sparse rows, FixedMaxPQ
    replayed), never the score-desc/id-asc top-k writer."""
    from gwamd import _lib as C
    jni = open(os.path.join(ROOT, "graph-embedding_amd", "jni", "graphwalk_jni.c")).read()
    hdr = open(os.path.join(ROOT, "include", "graphwalk.h")).read()
    called = set(re.findall(r"\b(gw_[a-z0-9_]+)\(", jni)) - {"gw_graph_info_t"}
    declared = set(re.findall(r"\bint (gw_[a-z0-9_]+)\(", hdr)) | set(re.findall(r"\b(gw_last_error)\(", hdr))
    assert called and called <= declared, called - declared
    lib = C.lib()
    for f in called:
        getattr(lib, f)
    java = open(os.path.join(ROOT, "graph-embedding_amd", "jni", "simrank", "GraphWalkNative.java")).read()
    natives = set(re.findall(r"public static native \w+ (\w+)\(", java))
    defined = set(re.findall(r"Java_simrank_GraphWalkNative_(\w+)\(", jni))
    assert natives and natives == defined, (natives, defined)
    writers = {f for f in called if f.startswith("gw_write_sim_text") or f.endswith("write_text")}
    assert writers == {"gw_topsim_write_text"}, writers
    assert "writeTopK" not in natives
