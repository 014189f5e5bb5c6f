"""The JNI shim (graph-embedding_amd/jni/graphwalk_jni.c) compiled and driven
without a JVM.

This image has no JDK, so the shim is compiled with -Wall -Wextra -Werror
against a test-only stand-in for <jni.h> (tests/jni_stub/jni.h: the JNIEnv
members the shim calls, JNI signatures and names) together with a fake JNIEnv
(tests/jni_stub/fake_jni_env.c) that copies on every pin, so release modes
matter, counts pins, records the pending exception and can fail the k-th pin
with an OutOfMemoryError.  Every Java_simrank_GraphWalkNative_* entry point is
called through ctypes:

* CPU: the exception mapping the reference's Java code shows on the same
  inputs (Graph.java:28-42: IOException for an unreadable file,
  NumberFormatException for a separator that does not split a line,
  ArrayIndexOutOfBoundsException for ids >= V), IllegalArgumentException for
  null / short arrays, a pin failure at every pin of every entry point (the
  shim releases what it pinned and returns with the OutOfMemoryError
  pending), and no input array written back;
* GPU: load -> topsimWriteText equal to gw_topsim_write_text on the same
  graph (two device runs differ only by fp64-atomic summation order: ids
  swap only at ties, %.6f strings only at an ulp-decided HALF_UP boundary),
  topsimTopK / topsimDense equal to gw_topsim_host (rtol 1e-12) and
  simrankNaive bitwise equal to gw_simrank_naive_host (deterministic)
  (Test_u_u_TopSim_singleSample.java:46-64's sequence).

The JVM itself stays unverified (N1 "partial"): the stand-in's function-table
order is not the JVM's.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import DATA, PKG, ROOT

STUB = os.path.join(ROOT, "tests", "jni_stub")
SHIM = os.path.join(PKG, "jni", "graphwalk_jni.c")
LIBDIR = os.path.join(PKG, "gwamd")

I32, I64, F64 = 2, 3, 4


@pytest.fixture(scope="module")
def jni(gw, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("jni") / "libgraphwalk_jni_fake.so")
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", "-fPIC", "-shared",
           f"-I{STUB}", f"-I{os.path.join(ROOT, 'include')}", SHIM, os.path.join(STUB, "fake_jni_env.c"),
           f"-L{LIBDIR}", "-lgraphwalk", f"-Wl,-rpath,{LIBDIR}", "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    L = ctypes.CDLL(out)
    P, J, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
    I = ctypes.c_int32
    sig = {
        "fake_env": (P, []), "fake_string": (P, [ctypes.c_char_p]), "fake_array": (P, [ctypes.c_int, I, P]),
        "fake_object_array": (P, [I, P]), "fake_data": (P, [P]), "fake_free": (None, [P]),
        "fake_exception_class": (ctypes.c_char_p, []), "fake_exception_msg": (ctypes.c_char_p, []),
        "fake_pins": (ctypes.c_int, []), "fake_abort_copyback": (ctypes.c_int, []), "fake_clear": (None, [ctypes.c_int]),
        "Java_simrank_GraphWalkNative_loadGraph": (J, [P, P, P, P, I, I]),
        "Java_simrank_GraphWalkNative_freeGraph": (None, [P, P, J]),
        "Java_simrank_GraphWalkNative_vertexCount": (I, [P, P, J]),
        "Java_simrank_GraphWalkNative_topsimTopK": (None, [P, P, J, I, I, I, D, J, P, I, P, P, P]),
        "Java_simrank_GraphWalkNative_topsimWriteText": (None, [P, P, J, I, I, I, D, J, P, I, P, P, P]),
        "Java_simrank_GraphWalkNative_topsimDense": (None, [P, P, J, I, I, I, D, J, P, P, P]),
        "Java_simrank_GraphWalkNative_simrankNaive": (None, [P, P, J, D, I, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    L.env = L.fake_env()
    return L


class _Objs:
    """Fake Java objects made for one call, freed afterwards."""

    def __init__(self, L):
        self.L, self.objs = L, []

    def s(self, text):
        o = self.L.fake_string(text.encode())
        self.objs.append(o)
        return o

    def a(self, kind, arr=None, n=None):
        if arr is not None:
            arr = np.ascontiguousarray(arr, {I32: np.int32, I64: np.int64, F64: np.float64}[kind])
            o = self.L.fake_array(kind, len(arr), arr.ctypes.data)
        else:
            o = self.L.fake_array(kind, n, None)
        self.objs.append(o)
        return o

    def rows(self, nrows, n):
        rs = [self.a(F64, n=n) for _ in range(nrows)]
        arr = (ctypes.c_void_p * max(nrows, 1))(*rs)
        o = self.L.fake_object_array(nrows, arr)
        self.objs.append(o)
        return o, rs

    def np(self, o, kind, n):
        ct = {I32: ctypes.c_int32, I64: ctypes.c_int64, F64: ctypes.c_double}[kind]
        return np.ctypeslib.as_array(ctypes.cast(self.L.fake_data(o), ctypes.POINTER(ct)), shape=(n,)).copy()

    def free(self):
        for o in self.objs:
            self.L.fake_free(o)
        self.objs = []


def _exc(L):
    return L.fake_exception_class().decode()


def _load(L, O, path, sep, V, fail_at=-1):
    L.fake_clear(fail_at)
    return L.Java_simrank_GraphWalkNative_loadGraph(L.env, None, O.s(path), O.s(sep), V, 0)


def test_shim_compiles_and_exports_every_native(jni):
    java = open(os.path.join(PKG, "jni", "simrank", "GraphWalkNative.java")).read()
    import re
    for m in re.findall(r"public static native \w+ (\w+)\(", java):
        assert getattr(jni, f"Java_simrank_GraphWalkNative_{m}")


def test_load_exceptions_match_graph_java(jni, tmp_path):
    L, O = jni, _Objs(jni)
    try:
        h = _load(L, O, str(tmp_path / "missing.txt"), "\t", 10)
        assert h == 0 and _exc(L) == "java/io/IOException" and L.fake_pins() == 0
        # blog.txt is comma-separated: a tab does not split its lines (Graph.java:38-39 Integer.parseInt)
        h = _load(L, O, os.path.join(DATA, "blog.txt"), "\t", 10313)
        assert h == 0 and _exc(L) == "java/lang/NumberFormatException" and L.fake_pins() == 0
        # moreno has ids up to 1379: V = 100 overruns Graph.java's adjacency array
        h = _load(L, O, os.path.join(DATA, "moreno_crime_crime.txt"), "\t", 100)
        assert h == 0 and _exc(L) == "java/lang/ArrayIndexOutOfBoundsException" and L.fake_pins() == 0
        assert L.fake_exception_msg()  # gw_last_error's text travels as the message
        L.fake_clear(-1)
        assert L.Java_simrank_GraphWalkNative_loadGraph(L.env, None, None, O.s("\t"), 10, 0) == 0
        assert _exc(L) == "java/lang/IllegalArgumentException"
        for k in (0, 1):  # the path's / the separator's pin fails: OOM pending, nothing left pinned
            h = _load(L, O, os.path.join(DATA, "moreno_crime_crime.txt"), "\t", 1380, fail_at=k)
            assert h == 0 and _exc(L) == "java/lang/OutOfMemoryError" and L.fake_pins() == 0
    finally:
        O.free()


def test_load_without_gpu_is_runtime_exception(jni):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the load succeeds (test_jni_gpu_*)")
    L, O = jni, _Objs(jni)
    try:
        h = _load(L, O, os.path.join(DATA, "moreno_crime_crime.txt"), "\t", 1380)
        assert h == 0 and _exc(L) == "java/lang/RuntimeException" and L.fake_pins() == 0
    finally:
        O.free()


def _topk_call(L, O, h, k=5, ids_n=None, stats_n=4, ns=3):
    src = O.a(I32, np.arange(ns))
    ids = O.a(I32, n=ns * k if ids_n is None else ids_n)
    sc = O.a(F64, n=ns * k)
    st = O.a(I64, n=stats_n) if stats_n else None
    L.Java_simrank_GraphWalkNative_topsimTopK(L.env, None, h, 0, 100, 3, 0.6, 11, src, k, ids, sc, st)
    return src, ids, sc, st


def test_argument_checks_and_pin_failures(jni):
    """Every entry point: null / short arrays -> IllegalArgumentException
    before anything is pinned; a NULL handle -> the C ABI's GW_ERR_INVALID as
    RuntimeException with every pin released and no input written back; a
    failed pin at each position -> OutOfMemoryError pending, every earlier
    pin released, the C ABI not called."""
    L, O = jni, _Objs(jni)
    try:
        L.fake_clear(-1)
        _topk_call(L, O, 0, ids_n=4)
        assert _exc(L) == "java/lang/IllegalArgumentException" and L.fake_pins() == 0
        L.fake_clear(-1)
        _topk_call(L, O, 0, stats_n=3)
        assert _exc(L) == "java/lang/IllegalArgumentException" and L.fake_pins() == 0
        L.fake_clear(-1)
        _topk_call(L, O, 0)
        assert _exc(L) == "java/lang/RuntimeException" and L.fake_pins() == 0 and L.fake_abort_copyback() == 0
        for k in range(4):  # sources, ids, scores, stats
            L.fake_clear(k)
            _topk_call(L, O, 0)
            assert _exc(L) == "java/lang/OutOfMemoryError" and L.fake_pins() == 0, k
        for k in range(4):  # path, separator, sources, stats
            L.fake_clear(k)
            L.Java_simrank_GraphWalkNative_topsimWriteText(L.env, None, 0, 0, 100, 3, 0.6, 11, O.a(I32, np.arange(3)),
                                                           5, O.s("/nonexistent/x"), O.s(","), O.a(I64, n=4))
            assert _exc(L) == "java/lang/OutOfMemoryError" and L.fake_pins() == 0, k
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_topsimWriteText(L.env, None, 0, 0, 100, 3, 0.6, 11, O.a(I32, np.arange(3)),
                                                       5, O.s("/nonexistent/x"), O.s(","), None)
        assert _exc(L) == "java/lang/RuntimeException" and L.fake_pins() == 0
        L.fake_clear(-1)
        rows, _ = O.rows(3, 4)
        L.Java_simrank_GraphWalkNative_topsimDense(L.env, None, 0, 0, 100, 3, 0.6, 11, O.a(I32, np.arange(3)), rows,
                                                   None)
        assert _exc(L) == "java/lang/RuntimeException" and L.fake_pins() == 0
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_simrankNaive(L.env, None, 0, 0.8, 3, O.a(F64, n=16))
        assert _exc(L) == "java/lang/RuntimeException" and L.fake_pins() == 0
        L.fake_clear(-1)
        assert L.Java_simrank_GraphWalkNative_vertexCount(L.env, None, 0) == 0
        assert _exc(L) == "java/lang/RuntimeException"
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_freeGraph(L.env, None, 0)  # freeing NULL is a no-op
        assert _exc(L) == ""
    finally:
        O.free()


@pytest.mark.gpu
def test_jni_gpu_driver_sequence_equals_c_abi(jni, gw, tmp_path):
    """Test_u_u_TopSim_singleSample.java:46-64 through the shim on moreno
    (tab, V = 1380): loadGraph -> topsimWriteText equal to
    gw_topsim_write_text on the same graph (up to fp64-atomic order noise);
    topsimTopK, topsimDense and simrankNaive equal to gw_topsim_host /
    gw_simrank_naive_host; inputs never written back; every pin released."""
    from gwamd import _lib as C
    L, O = jni, _Objs(jni)
    path = os.path.join(DATA, "moreno_crime_crime.txt")
    try:
        h = _load(L, O, path, "\t", 1380)
        assert h != 0 and _exc(L) == "" and L.fake_pins() == 0
        L.fake_clear(-1)
        assert L.Java_simrank_GraphWalkNative_vertexCount(L.env, None, h) == 1380
        G = gw.GWGraph.from_edgelist(path, "\t", "java", vcount=1380).to_device(0)
        src = np.arange(0, 1380, 7, dtype=np.int32)
        ns = len(src)
        sample, step, seed, topk = 1000, 5, 11, 20
        # writer
        jp, cp = str(tmp_path / "jni"), str(tmp_path / "capi")
        st = O.a(I64, n=4)
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_topsimWriteText(L.env, None, h, 0, sample, step, 0.6, seed, O.a(I32, src), topk,
                                                       O.s(jp), O.s(","), st)
        assert _exc(L) == "" and L.fake_pins() == 0 and L.fake_abort_copyback() == 0
        cst = np.zeros(4, np.int64)
        C.check(C.lib().gw_topsim_write_text(G.handle, 0, sample, step, 0.6, seed, C.ptr(src), ns, topk, cp.encode(),
                                             b",", 6, C.ptr(cst)), G.handle)
        # two runs of the device sums differ in the last bits (fp64 atomics): the
        # files are equal line by line up to a %.6f HALF_UP boundary decided by
        # an ulp, and ids equal except where two scores tie within that noise
        for suf in ("", ".sim.txt"):
            a = open(jp + suf, "rb").read().decode().split("\r\n")
            b = open(cp + suf, "rb").read().decode().split("\r\n")
            assert len(a) == len(b) == ns + 1 and a[-1] == b[-1] == ""
            ndiff = 0
            for la, lb in zip(a[:-1], b[:-1]):
                if la == lb:
                    continue
                ta, tb = la.split(","), lb.split(",")
                assert ta[0] == tb[0] and len(ta) == len(tb)
                for x, y in zip(ta[1:], tb[1:]):
                    if x != y:
                        ndiff += 1
                        if ":" in x:  # the .sim.txt file: id:score
                            (ia, va), (ib, vb) = x.split(":"), y.split(":")
                            assert abs(float(va) - float(vb)) <= 1.000001e-6, (x, y)
            assert ndiff <= max(2, ns * topk // 1000), ndiff
        assert np.array_equal(O.np(st, I64, 4), cst)
        # top-k
        k = 50
        L.fake_clear(-1)
        s_o = O.a(I32, src)
        ids_o, sc_o, st_o = O.a(I32, n=ns * k), O.a(F64, n=ns * k), O.a(I64, n=4)
        L.Java_simrank_GraphWalkNative_topsimTopK(L.env, None, h, 0, sample, step, 0.6, seed, s_o, k, ids_o, sc_o, st_o)
        assert _exc(L) == "" and L.fake_pins() == 0 and L.fake_abort_copyback() == 0
        ci, cs, cst = np.zeros(ns * k, np.int32), np.zeros(ns * k), np.zeros(4, np.int64)
        C.check(C.lib().gw_topsim_host(G.handle, 0, sample, step, 0.6, seed, C.ptr(src), ns, k, C.ptr(ci), C.ptr(cs),
                                       None, C.ptr(cst)), G.handle)
        gi, gs = O.np(ids_o, I32, ns * k), O.np(sc_o, F64, ns * k)
        np.testing.assert_allclose(gs, cs, rtol=1e-12)
        swap = gi != ci  # ids equal except where two scores tie within fp64 atomic-order noise
        assert np.all(np.abs(cs[swap] - gs[swap]) <= 1e-12 * np.abs(cs[swap]))
        assert np.array_equal(O.np(st_o, I64, 4)[[0, 1, 3]], cst[[0, 1, 3]])
        # dense rows
        rows, rs = O.rows(ns, 1380)
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_topsimDense(L.env, None, h, 0, sample, step, 0.6, seed, O.a(I32, src), rows,
                                                   None)
        assert _exc(L) == "" and L.fake_pins() == 0
        cr = np.zeros((ns, 1380))
        C.check(C.lib().gw_topsim_host(G.handle, 0, sample, step, 0.6, seed, C.ptr(src), ns, 0, None, None, C.ptr(cr),
                                       None), G.handle)
        got = np.stack([O.np(r, F64, 1380) for r in rs])
        np.testing.assert_allclose(got, cr, rtol=1e-12, atol=0)
        # a row shorter than V
        short, _ = O.rows(ns, 10)
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_topsimDense(L.env, None, h, 0, sample, step, 0.6, seed, O.a(I32, src), short,
                                                   None)
        assert _exc(L) == "java/lang/IllegalArgumentException" and L.fake_pins() == 0
        # a source id >= V
        L.fake_clear(-1)
        bad = O.a(I32, np.array([0, 1380], np.int32))
        L.Java_simrank_GraphWalkNative_topsimTopK(L.env, None, h, 0, sample, step, 0.6, seed, bad, 5, O.a(I32, n=10),
                                                  O.a(F64, n=10), None)
        assert _exc(L) == "java/lang/ArrayIndexOutOfBoundsException" and L.fake_pins() == 0
        # naive SimRank
        sim = O.a(F64, n=1380 * 1380)
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_simrankNaive(L.env, None, h, 0.6, 3, sim)
        assert _exc(L) == "" and L.fake_pins() == 0
        csim = np.zeros(1380 * 1380)
        C.check(C.lib().gw_simrank_naive_host(G.handle, 0.6, 3, C.ptr(csim)), G.handle)
        assert np.array_equal(O.np(sim, F64, 1380 * 1380), csim)
        L.fake_clear(-1)
        L.Java_simrank_GraphWalkNative_freeGraph(L.env, None, h)
        assert _exc(L) == ""
    finally:
        O.free()
