"""Owning Python handle over a libgraphwalk graph (gw_graph*)."""
import ctypes

import numpy as np

from . import _lib as C


class GWGraph:
    """A CSR graph living in libgraphwalk (host copy + optional HBM copy).

    Construction mirrors the two reference graph semantics:
      * `from_edgelist(..., semantics="nx")`  == read_graph (node2vec/src/main.py:76-89)
      * `from_edgelist(..., semantics="java")` == structures.Graph(path, V) (Graph.java:28-42)
    """

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle) if not isinstance(handle, ctypes.c_void_p) else handle
        self._info = None

    # ---- constructors -------------------------------------------------------
    @classmethod
    def from_edgelist(cls, path, delimiter=None, semantics="nx", directed=False,
                      weighted=False, vcount=-1):
        sem = C.SEM_NX_SIMPLE if semantics == "nx" else C.SEM_JAVA_MULTI
        h = ctypes.c_void_p()
        d = None if delimiter is None else delimiter.encode()
        rc = C.lib().gw_graph_load_edgelist(str(path).encode(), d, sem, int(directed),
                                            int(weighted), int(vcount), ctypes.byref(h))
        C.check(rc)
        return cls(h)

    @classmethod
    def from_edges(cls, src, dst, weights=None, semantics="nx", directed=False, vcount=-1):
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        sem = C.SEM_NX_SIMPLE if semantics == "nx" else C.SEM_JAVA_MULTI
        h = ctypes.c_void_p()
        rc = C.lib().gw_graph_from_edges(len(src), C.ptr(src), C.ptr(dst), C.ptr(w), sem,
                                         int(directed), int(vcount), ctypes.byref(h))
        C.check(rc)
        return cls(h)

    @classmethod
    def from_csr(cls, offsets, nbrs, weights=None, labels=None, node_order=None,
                 semantics="nx", directed=False):
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        nbrs = np.ascontiguousarray(nbrs, dtype=np.int32)
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.int64)
        order = None if node_order is None else np.ascontiguousarray(node_order, dtype=np.int32)
        sem = C.SEM_NX_SIMPLE if semantics == "nx" else C.SEM_JAVA_MULTI
        h = ctypes.c_void_p()
        rc = C.lib().gw_graph_from_csr(len(offsets) - 1, C.ptr(offsets), C.ptr(nbrs), C.ptr(w),
                                       C.ptr(lab), C.ptr(order), sem, int(directed), ctypes.byref(h))
        C.check(rc)
        g = cls(h)
        g._keep = (offsets, nbrs, w, lab, order)
        return g

    @classmethod
    def from_networkx(cls, G, directed=None):
        """CSR of a networkx graph exactly as node2vec.Graph sees it: draw order
        = sorted(G.neighbors(v)) (node2vec.py:25,67,94), start order = G.nodes()."""
        if directed is None:
            directed = G.is_directed()
        labels = np.array(sorted(G.nodes()), dtype=np.int64)
        rank = {int(x): i for i, x in enumerate(labels)}
        offs = np.zeros(len(labels) + 1, np.int64)
        nbrs, wts = [], []
        weighted = False
        for i, u in enumerate(labels):
            ns = sorted(G.neighbors(int(u)))
            for v in ns:
                nbrs.append(rank[v])
                w = G[int(u)][v].get("weight", 1)
                if w != 1:
                    weighted = True
                wts.append(float(w))
            offs[i + 1] = len(nbrs)
        order = np.array([rank[int(x)] for x in G.nodes()], np.int32)
        return cls.from_csr(offs, np.array(nbrs, np.int32),
                            np.array(wts, np.float64) if weighted else None,
                            labels, order, "nx", directed)

    @classmethod
    def rmat(cls, scale, edge_factor=16, a=0.57, b=0.19, c=0.19, seed=42):
        h = ctypes.c_void_p()
        C.check(C.lib().gw_graph_rmat(int(scale), int(edge_factor), a, b, c, int(seed), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def rmat_java(cls, n, m, a=0.57, b=0.19, c=0.19, seed=42):
        """Java-multigraph R-MAT over n vertices (RMATGraphGenerator.java:119-145)."""
        h = ctypes.c_void_p()
        C.check(C.lib().gw_graph_rmat_java(int(n), int(m), a, b, c, int(seed), ctypes.byref(h)))
        return cls(h)

    # ---- accessors ------------------------------------------------------------
    @property
    def handle(self):
        return self._h

    def info(self):
        inf = C.GraphInfo()
        C.check(C.lib().gw_graph_info(self._h, ctypes.byref(inf)), self._h)
        return inf

    def options(self, **kw):
        """Read, and with keyword arguments update, the handle's gw_options_t
        (table_budget_bytes, expected_steps, listed, simrank_hbm_row,
        host_chunk_bytes).  Returns the options in effect as a dict."""
        o = C.Options()
        C.check(C.lib().gw_graph_get_options(self._h, ctypes.byref(o)), self._h)
        for k, v in kw.items():
            if not hasattr(o, k):
                raise TypeError(f"unknown option {k!r}")
            setattr(o, k, int(v))
        if kw:
            C.check(C.lib().gw_graph_set_options(self._h, ctypes.byref(o)), self._h)
        return {f: getattr(o, f) for f, _ in C.Options._fields_}

    @property
    def n(self):
        return self.info().n

    @property
    def nnz(self):
        return self.info().nnz

    def export_csr(self):
        inf = self.info()
        offs = np.empty(inf.n + 1, np.int64)
        nbrs = np.empty(inf.nnz, np.int32)
        w = np.empty(inf.nnz, np.float64)
        lab = np.empty(inf.n, np.int64)
        order = np.empty(inf.n, np.int32)
        C.check(C.lib().gw_graph_export_csr(self._h, C.ptr(offs), C.ptr(nbrs), C.ptr(w), C.ptr(lab),
                                            C.ptr(order)), self._h)
        return dict(offsets=offs, nbrs=nbrs, weights=w, labels=lab, node_order=order)

    def to_device(self, device=0):
        C.check(C.lib().gw_graph_to_device(self._h, int(device)), self._h)
        return self

    def free(self):
        if self._h is not None and self._h.value:
            C.lib().gw_graph_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
