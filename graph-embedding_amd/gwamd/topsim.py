"""Drop-in for the reference's TopSim side (DeepSim/TopSimAll/src), GPU-backed.

    g = Graph(path, V, separator=",")              # structures.Graph (Graph.java:28-42)
    ts = TopSim_singleSample(g, sample, step)     # TopSim_singleSample.java:35-44
    ts.compute()                                  # :47-54 (all sources, on the GPU)
    sim = ts.getResult()                          # :235-237 dense V x V (small V only)
    ids, scores = ts.topK(k)                      # sparse top-k rows (any V)
    printByOrder(ts, outPath, topk, testTopK)     # utils/Print.java:25-53
    precision(gold, test, prePath, K)             # utils/Eval.java:81-131

`TopSim_Enumerate` (TopSim_Enumerate.java, walks source 0 only by default)
and `SingleRandomWalk` (SingleRandomWalk.java) use the same kernel.
`SimRank` (SimRank.java, the naive all-pairs ground truth) runs on the GPU
as two sparse row-gather passes per round; `printByOrderAll` is its writer.

Randomness: the reference draws from an unseeded static java.util.Random
(Graph.java:17); here every random child is a Philox draw keyed by
(seed, source, walker index, level), so runs are reproducible.
"""
import ctypes

import numpy as np

from . import _lib as C
from .graph import GWGraph

MIN = 0.000000001   # MyConfiguration.MIN (MyConfiguration.java:20)
C_DEFAULT = 0.6     # MyConfiguration.C (:21)
TOPK = 20           # MyConfiguration.TOPK (:19)
SEPARATOR = ","     # MyConfiguration.SEPARATOR (:16)
DENSE_LIMIT = 1 << 28  # bytes of dense result a getResult() may allocate


class Graph:
    """structures.Graph: undirected multigraph, insertion-order adjacency."""

    def __init__(self, graphPath, V, separator=SEPARATOR, device=0):
        self.vCount = int(V)
        self._g = GWGraph.from_edgelist(graphPath, delimiter=separator, semantics="java",
                                        vcount=int(V))
        csr = self._g.export_csr()
        self._offs = csr["offsets"]
        self._nbrs = csr["nbrs"]
        self.eCount = len(self._nbrs) // 2
        self.device = device
        self._on_device = False

    def _ensure_device(self):
        if not self._on_device:
            self._g.to_device(self.device)
            self._on_device = True

    def degree(self, v):
        return int(self._offs[v + 1] - self._offs[v])

    def neighbors(self, v):
        return self._nbrs[self._offs[v]:self._offs[v + 1]].tolist()

    def getVCount(self):
        return self.vCount

    def getECount(self):
        return self.eCount


class _TopSimBase:
    VARIANT = C.TOPSIM_SINGLE_SAMPLE

    def __init__(self, g, sample, step, C_=C_DEFAULT, seed=0):
        self.g = g
        self.SAMPLE = int(sample)
        self.STEP = int(step)
        self.C = float(C_)
        self.seed = int(seed)
        self.COUNT = g.getVCount()
        self.stats = None
        self._sources = None
        self._rows = None
        self._topk = None

    def _default_sources(self):
        return np.arange(self.COUNT, dtype=np.int32)

    def _run(self, sources, topk=None, dense=False):
        import torch
        g = self.g
        g._ensure_device()
        dev = torch.device("cuda", g.device)
        src = torch.as_tensor(np.ascontiguousarray(sources, np.int32), device=dev)
        stats = torch.zeros(4, dtype=torch.int64, device=dev)
        h = g._g.handle
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        if dense:
            rows = torch.empty((len(src), self.COUNT), dtype=torch.float64, device=dev)
            C.check(C.lib().gw_topsim_dense(h, self.VARIANT, self.SAMPLE, self.STEP, self.C, self.seed,
                                            C.ptr(src), len(src), C.ptr(rows), C.ptr(stats), stream), h)
            out = rows.cpu().numpy()
        else:
            k = int(topk)
            ids = torch.empty((len(src), k), dtype=torch.int32, device=dev)
            sc = torch.empty((len(src), k), dtype=torch.float64, device=dev)
            C.check(C.lib().gw_topsim(h, self.VARIANT, self.SAMPLE, self.STEP, self.C, self.seed,
                                      C.ptr(src), len(src), k, C.ptr(ids), C.ptr(sc), C.ptr(stats), stream), h)
            out = (ids.cpu().numpy(), sc.cpu().numpy())
        s = stats.cpu().numpy()
        self.stats = dict(extensions=int(s[0]), pair_updates=int(s[1]), max_frontier=int(s[2]),
                          walkers=int(s[3]))
        return out

    def compute(self, sources=None):
        """compute() over all sources (or the given ones).  Keeps dense rows
        when they fit DENSE_LIMIT, else top-TOPK rows."""
        src = self._default_sources() if sources is None else np.asarray(sources, np.int32)
        self._sources = src
        if len(src) * self.COUNT * 8 <= DENSE_LIMIT:
            self._rows = self._run(src, dense=True)
        else:
            self._topk = self._run(src, topk=TOPK)

    def getResult(self):
        """double[V][V] (TopSim_singleSample.java:235); rows not computed are 0."""
        if self._rows is None:
            raise MemoryError("dense result too large for this graph; use topK()")
        if len(self._sources) == self.COUNT and np.all(self._sources == np.arange(self.COUNT)):
            return self._rows
        full = np.zeros((self.COUNT, self.COUNT))
        full[self._sources] = self._rows
        return full

    def sparse(self, sources=None, capacity=None):
        """Nonzero (id, score) entries of each source's row (gw_topsim_sparse):
        returns (row_begin, row_len, ids, scores) host arrays, entries of a row
        in no particular order."""
        import torch
        src = self._default_sources() if sources is None else np.asarray(sources, np.int32)
        g = self.g
        g._ensure_device()
        dev = torch.device("cuda", g.device)
        h = g._g.handle
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        s_dev = torch.as_tensor(np.ascontiguousarray(src, np.int32), device=dev)
        cap = int(capacity) if capacity is not None else max(1, min(len(src) * self.COUNT, 1 << 24))
        while True:
            begin = torch.empty(len(src), dtype=torch.int64, device=dev)
            ln = torch.empty(len(src), dtype=torch.int32, device=dev)
            ids = torch.empty(cap, dtype=torch.int32, device=dev)
            sc = torch.empty(cap, dtype=torch.float64, device=dev)
            used = torch.zeros(1, dtype=torch.int64, device=dev)
            stats = torch.zeros(4, dtype=torch.int64, device=dev)
            rc = C.lib().gw_topsim_sparse(h, self.VARIANT, self.SAMPLE, self.STEP, self.C, self.seed,
                                          C.ptr(s_dev), len(src), cap, C.ptr(begin), C.ptr(ln), C.ptr(ids),
                                          C.ptr(sc), C.ptr(used), C.ptr(stats), stream)
            need = int(used.cpu()[0])
            if rc == C.GW_ERR_CAPACITY and need > cap:
                cap = need
                continue
            C.check(rc, h)
            break
        s = stats.cpu().numpy()
        self.stats = dict(extensions=int(s[0]), pair_updates=int(s[1]), max_frontier=int(s[2]),
                          walkers=int(s[3]))
        return begin.cpu().numpy(), ln.cpu().numpy(), ids[:need].cpu().numpy(), sc[:need].cpu().numpy()

    def writeText(self, outPath, topk=TOPK, sources=None, separator=SEPARATOR, decimals=6):
        """compute() + Print.printByOrder in one native call
        (gw_topsim_write_text): Java-exact bytes at any V."""
        src = self._sources if sources is None else np.asarray(sources, np.int32)
        if src is None:
            src = self._default_sources()
        src = np.ascontiguousarray(src, np.int32)
        self.g._ensure_device()
        st = np.zeros(4, np.int64)
        h = self.g._g.handle
        C.check(C.lib().gw_topsim_write_text(h, self.VARIANT, self.SAMPLE, self.STEP, self.C, self.seed,
                                             C.ptr(src), len(src), int(topk), str(outPath).encode(),
                                             separator.encode(), int(decimals), C.ptr(st)), h)
        self.stats = dict(extensions=int(st[0]), pair_updates=int(st[1]), max_frontier=int(st[2]),
                          walkers=int(st[3]))

    def topK(self, k=TOPK, sources=None):
        src = self._default_sources() if sources is None else np.asarray(sources, np.int32)
        return self._run(src, topk=k)


class TopSim_singleSample(_TopSimBase):
    VARIANT = C.TOPSIM_SINGLE_SAMPLE


class TopSim_Basic(TopSim_singleSample):
    """TopSim_Basic.java: the same algorithm as TopSim_singleSample."""


class TopSim_Enumerate(_TopSimBase):
    """TopSim_Enumerate.java:46-53: compute() walks source 0 only."""
    VARIANT = C.TOPSIM_ENUMERATE

    def _default_sources(self):
        return np.array([0], np.int32)

    def getResult(self):
        full = np.zeros((self.COUNT, self.COUNT))
        full[self._sources] = self._rows
        return full


class SingleRandomWalk(_TopSimBase):
    """SingleRandomWalk.java:28-92 (scores divided by SAMPLE)."""
    VARIANT = C.TOPSIM_SINGLE_RW


class FixedCacheMap:
    """lxctools.FixedCacheMap contents as produced on the GPU: the entries in
    iteration order (ascending value, FixedCacheMap.java:104-127).  Iterating
    empties it, as the Java iterator does (delMin)."""

    def __init__(self, keys, vals, capacity):
        self._items = [(int(k), float(v)) for k, v in zip(keys, vals)]
        self.NMAX = int(capacity)

    def size(self):
        return len(self._items)

    def isEmpty(self):
        return not self._items

    def __iter__(self):
        while self._items:
            yield self._items.pop(0)


class _TopSimM:
    """Shared by TopSim_singleSample_M / SingleRandomWalk_M (STEP = 5 as in
    the reference; `step` overrides it)."""
    VARIANT = C.TOPSIM_SINGLE_SAMPLE
    STEP = 5

    def __init__(self, g, M, sample, C_=C_DEFAULT, seed=0, step=None, topk=TOPK):
        self.g = g
        self.COUNT = g.getVCount()
        self.capacity = int(topk) * int(M)  # capacity = topk * M (:37)
        self.SAMPLE = int(sample)
        self.STEP = type(self).STEP if step is None else int(step)
        self.C = float(C_)
        self.seed = int(seed)
        self.stats = None
        self._raw = None

    def compute(self, sources=None):
        import torch
        g = self.g
        g._ensure_device()
        dev = torch.device("cuda", g.device)
        src_np = np.arange(self.COUNT, dtype=np.int32) if sources is None else np.asarray(sources, np.int32)
        src = torch.as_tensor(src_np, device=dev)
        cap = self.capacity
        keys = torch.empty((len(src), cap), dtype=torch.int32, device=dev)
        vals = torch.empty((len(src), cap), dtype=torch.float32, device=dev)
        size = torch.empty(len(src), dtype=torch.int32, device=dev)
        st = torch.zeros(4, dtype=torch.int64, device=dev)
        h = g._g.handle
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        C.check(C.lib().gw_topsim_m(h, self.VARIANT, cap, self.SAMPLE, self.STEP, self.C, self.seed,
                                    C.ptr(src), len(src), C.ptr(keys), C.ptr(vals), C.ptr(size), C.ptr(st),
                                    stream), h)
        s = st.cpu().numpy()
        self.stats = dict(extensions=int(s[0]), pair_updates=int(s[1]), max_frontier=int(s[2]),
                          walkers=int(s[3]))
        self._raw = (src_np, keys.cpu().numpy(), vals.cpu().numpy(), size.cpu().numpy())

    def raw(self):
        """(sources, keys[nsrc, capacity], values float32, sizes) in iteration order."""
        if self._raw is None:
            raise RuntimeError("call compute() first")
        return self._raw

    def getResult(self):
        """FixedCacheMap[] (one per vertex; rows not computed are empty)."""
        src, keys, vals, size = self.raw()
        out = [FixedCacheMap([], [], self.capacity) for _ in range(self.COUNT)]
        for r, v in enumerate(src):
            out[int(v)] = FixedCacheMap(keys[r, :size[r]], vals[r, :size[r]], self.capacity)
        return out


class TopSim_singleSample_M(_TopSimM):
    """simrank.TopSim_singleSample_M (TopSim_singleSample_M.java:21-243)."""
    VARIANT = C.TOPSIM_SINGLE_SAMPLE


class SingleRandomWalk_M(_TopSimM):
    """simrank.SingleRandomWalk_M (SingleRandomWalk_M.java:15-102)."""
    VARIANT = C.TOPSIM_SINGLE_RW


class _DoubleBase:
    def __init__(self, g, C_=C_DEFAULT, seed=0):
        self.g = g
        self.COUNT = g.getVCount()
        self.C = float(C_)
        self.seed = int(seed)
        self._sim = None

    def _dense(self, fn, *args):
        import torch
        g = self.g
        g._ensure_device()
        dev = torch.device("cuda", g.device)
        sim = torch.empty((self.COUNT, self.COUNT), dtype=torch.float64, device=dev)
        h = g._g.handle
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        C.check(fn(h, *args, C.ptr(sim), stream), h)
        self._sim = sim.cpu().numpy()

    def getResult(self):
        if self._sim is None:
            raise RuntimeError("call compute() first")
        return self._sim


class TopSim_doubleSample(_DoubleBase):
    """simrank.TopSim_doubleSample (TopSim_doubleSample.java:20-197)."""

    def __init__(self, g, sample, step, C_=C_DEFAULT, seed=0):
        super().__init__(g, C_, seed)
        self.SAMPLE, self.STEP = int(sample), int(step)

    def compute(self):
        self._dense(C.lib().gw_topsim_double, self.SAMPLE, self.STEP, self.C, self.seed)


class DoubleRandomWalk(_DoubleBase):
    """simrank.DoubleRandomWalk (DoubleRandomWalk.java:15-95)."""

    def __init__(self, g, sample, step, C_=C_DEFAULT, seed=0):
        super().__init__(g, C_, seed)
        self.SAMPLE, self.STEP = int(sample), int(step)

    def compute(self):
        self._dense(C.lib().gw_double_random_walk, self.SAMPLE, self.STEP, self.C, self.seed)


def select_candidates(candidate, k, min_score=MIN):
    """TopSim_Dev's candidate choice (TopSim_Dev.java:64-71): FixedMaxPQ(k)
    over candidate[i][j] >= MIN, sortedElement() order -> int32 [n, k], -1 padded."""
    cand = np.ascontiguousarray(candidate, np.float64)
    out = np.full((cand.shape[0], int(k)), -1, np.int32)
    C.check(C.lib().gw_select_fixed_max_pq(C.ptr(cand), cand.shape[0], cand.shape[1], int(k), float(min_score),
                                           C.ptr(out)))
    return out


class TopSim_Dev(_DoubleBase):
    """simrank.TopSim_Dev (TopSim_Dev.java:24-101): candidate refinement."""

    def __init__(self, g, sample, step, topK, singleStep, C_=C_DEFAULT, seed=0):
        super().__init__(g, C_, seed)
        self.sample_total, self.STEP = int(sample), int(step)
        self.singleK, self.singleStep = int(topK), int(singleStep)
        # SAMPLE = (int)(((step-singleStep)*sample*2.0)/((double)step*(topK+1.0))) (:33)
        self.SAMPLE = int(((step - singleStep) * sample * 2.0) / (float(step) * (topK + 1.0)))

    def compute(self, candidate):
        import torch
        cand = candidate if (isinstance(candidate, np.ndarray) and candidate.dtype == np.int32
                             and candidate.ndim == 2 and candidate.shape[1] == self.singleK) \
            else select_candidates(candidate, self.singleK)
        dev = torch.device("cuda", self.g.device)
        cd = torch.as_tensor(np.ascontiguousarray(cand, np.int32), device=dev)
        self._dense(C.lib().gw_topsim_dev, self.sample_total, self.STEP, self.singleK, self.singleStep, self.C,
                    self.seed, C.ptr(cd))


class SimRank:
    """simrank.SimRank (SimRank.java:15-82): naive SimRank, STEP = 3 rounds
    (the reference's private field; `step` overrides it), C from
    MyConfiguration.C.  getResult() is the dense V x V matrix with a zero
    diagonal (postProcess, :62-65).  Needs V*V doubles on the device."""
    STEP = 3

    def __init__(self, g, C_=C_DEFAULT, step=None):
        self.g = g
        self.COUNT = g.getVCount()
        self.C = float(C_)
        self.STEP = SimRank.STEP if step is None else int(step)
        self._sim = None

    def compute(self):
        import torch
        g = self.g
        g._ensure_device()
        dev = torch.device("cuda", g.device)
        sim = torch.empty((self.COUNT, self.COUNT), dtype=torch.float64, device=dev)
        h = g._g.handle
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        C.check(C.lib().gw_simrank_naive(h, self.C, self.STEP, C.ptr(sim), stream), h)
        self._sim = sim.cpu().numpy()

    def sim(self, v, w):
        """SimRank.java:67-77: one round for the pair (v, w) from the current
        matrix (the identity before compute(); host arithmetic, O(deg^2))."""
        if v == w:
            return 1.0
        g = self.g
        dv, dw = g.degree(v), g.degree(w)
        if dv == 0 or dw == 0:
            return 0.0
        S = self._sim if self._sim is not None else np.eye(self.COUNT)
        result = 0.0
        for vn in g.neighbors(v):
            for wn in g.neighbors(w):
                result += float(S[vn, wn])
        return self.C * result / (dv * dw)

    def getResult(self):
        if self._sim is None:
            raise RuntimeError("call compute() first")
        return self._sim


def printByOrderAll(sim, outPath, topk=1000, testTopK=10, separator=SEPARATOR):
    """Print.printByOrderAll (Print.java:55-84): printByOrder with `%.7f`."""
    if isinstance(sim, SimRank):
        sim = sim.getResult()
    printByOrder(sim, outPath, topk, testTopK, separator=separator, decimals=7)


def printByOrder(sim, outPath, topk=TOPK, testTopK=None, separator=SEPARATOR, decimals=6):
    """Print.printByOrder (Print.java:25-53): `outPath` gets "v,id,...\\r\\n" and
    `outPath.sim.txt` gets "v,id:%.6f,...\\r\\n".  `sim` is a dense V x V array
    (exact Java FixedMaxPQ tie order and %.6f HALF_UP), a TopSim object, or a
    TopSim_M object (the FixedCacheMap[] overload, Print.java:94-124: last
    `topk` entries of each map's ascending iteration)."""
    if isinstance(sim, _TopSimM):
        src, keys, vals, size = sim.raw()
        C.check(C.lib().gw_write_sim_text_cachemap(
            str(outPath).encode(), C.ptr(np.ascontiguousarray(keys)), C.ptr(np.ascontiguousarray(vals)),
            C.ptr(np.ascontiguousarray(size)), C.ptr(np.ascontiguousarray(src, np.int32)), keys.shape[0],
            keys.shape[1], int(topk), separator.encode()))
        return
    if isinstance(sim, _TopSimBase):
        if sim._rows is not None:
            rows, ids = sim._rows, sim._sources
            rows = np.ascontiguousarray(rows, np.float64)
            C.check(C.lib().gw_write_sim_text_dense(str(outPath).encode(), C.ptr(rows),
                                                    C.ptr(np.ascontiguousarray(ids, np.int32)),
                                                    rows.shape[0], rows.shape[1], int(topk),
                                                    separator.encode(), int(decimals)))
            return
        # rows too large to keep dense: recompute the same Philox walks as
        # sparse rows and replay FixedMaxPQ exactly (gw_topsim_write_text)
        sim.writeText(outPath, topk, separator=separator, decimals=decimals)
        return
    rows = np.ascontiguousarray(sim, np.float64)
    C.check(C.lib().gw_write_sim_text_dense(str(outPath).encode(), C.ptr(rows), None, rows.shape[0],
                                            rows.shape[1], int(topk), separator.encode(), int(decimals)))


def precision(path1, path2, prePath, K, separator=SEPARATOR, topk=TOPK):
    """Eval.precision (Eval.java:81-131): mean over rows of
    |gold ∩ test| / min(TOPK, |gold|) with ids whose score >= MIN; 1.0 when
    the gold row is empty.  Writes "v,pre\\r\\n" lines to prePath."""
    total, s, mn = 0, 0.0, float("inf")
    with open(path1) as f1, open(path2) as f2, open(prePath, "w", newline="") as out:
        for line1 in f1:
            line2 = f2.readline()
            line1 = line1.rstrip("\r\n")
            line2 = line2.rstrip("\r\n")
            t1 = [t for t in line1.split(separator)]
            t2 = [t for t in line2.split(separator)]
            while t1 and t1[-1] == "":
                t1.pop()
            while t2 and t2[-1] == "":
                t2.pop()
            if t1[0] != t2[0]:
                print("error !" + t1[0] + "\t" + t2[0])
                continue
            s1 = {x.split(":")[0] for x in t1[1:] if float(x.split(":")[1]) >= MIN}
            s2 = {x.split(":")[0] for x in t2[1:] if float(x.split(":")[1]) >= MIN}
            realK = min(topk, len(s1))
            pre = 1.0 if realK == 0 else len(s1 & s2) / realK
            s += pre
            out.write(f"{t1[0]}{separator}{pre}\r\n")
            total += 1
            mn = min(mn, pre)
    return s / total if total else float("nan")
