"""Parity oracle — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference algorithms on the hot path, used as the
checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Nothing under graph-embedding_amd/ imports this package.

* liboracle.so (oracle/oracle.c, built by `make -C oracle`): alias tables,
  exact-replay walks, Philox scale walks, TopSim (Java-literal queue
  formulation), naive SimRank, java.util.Random.
* pure-Python restatements (small inputs): networkx `read_graph` semantics
  without networkx, Java FixedMaxPQ / PriorityQueue tie order, Java
  `String.format("%.6f")`.

Pinning: see DESIGN.md §Oracle (golden vectors from the imported reference
node2vec.py under tests/golden/, the reference's committed naive-SimRank
fixture, and the deterministic-regime TopSim == truncated naive SimRank KAT).
"""
import ctypes
import decimal
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("GW_ORACLE_LIB", os.path.join(HERE, "liboracle.so"))  # (sanitizer runs: tools/sanitize.sh)
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if LIB == os.path.join(HERE, "liboracle.so") and (
                not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "oracle.c"))):
            build()
        L = ctypes.CDLL(LIB)
        v, i64, i32, d, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_uint64
        ci = ctypes.c_int
        L.or_alias_setup.argtypes = [v, i64, v, v]
        L.or_alias_nodes.argtypes = [i64, v, v, v, v]
        L.or_alias_edges_offsets.argtypes = [i64, v, v, v]
        L.or_alias_edges_offsets.restype = i64
        L.or_alias_edges.argtypes = [i64, v, v, v, d, d, v, v, v]
        L.or_walks_replay.argtypes = [i64, v, v, v, v, v, v, v, ci, i64, v, v, i64, v, v]
        L.or_walks_replay.restype = i64
        L.or_walks_scale.argtypes = [i64, v, v, v, v, v, v, v, ci, d, d, u64, ci, i64, i64, ci, v, v, v, ci]
        L.or_jrand_sequence.argtypes = [i64, i32, i64, v]
        L.or_walks_bitset.argtypes = [i64, v, v, v, d, d, u64, ci, i64, i64, ci, v, v, v, ci]
        L.or_topsim.argtypes = [i64, v, v, ci, ci, ci, d, u64, ci, i64, v, i64, v, v, ci]
        L.or_simrank_naive.argtypes = [i64, v, v, d, ci, v, ci]
        L.or_topsim_topk.argtypes = [i64, v, v, ci, ci, ci, d, u64, v, i64, ci, v, v, v, ci]
        L.or_topsim_m.argtypes = [i64, v, v, ci, ci, ci, d, u64, ci, v, i64, v, v, v, v, ci]
        L.or_fcm_run.argtypes = [ci, i64, v, v, v, v]
        L.or_topsim_levels.argtypes = [i64, v, v, ci, ci, u64, v, v, i64, v, ci]
        L.or_topsim_double_sims.argtypes = [i64, v, ci, d, v, ci]
        L.or_topsim_dev.argtypes = [i64, v, v, ci, ci, d, u64, v, ci, v, ci]
        L.or_double_random_walk.argtypes = [i64, v, v, ci, ci, d, u64, v, ci]
        L.or_fcm_run.restype = ci
        L.or_simrank_round_rows.argtypes = [i64, v, v, d, v, i64, i64, v, ci]
        L.or_simrank_round_rows.restype = i64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


# ---- node2vec ----------------------------------------------------------------
def alias_setup(probs):
    p = np.ascontiguousarray(probs, np.float64)
    J = np.zeros(len(p), np.int64)
    q = np.zeros(len(p), np.float64)
    lib().or_alias_setup(_p(p), len(p), _p(J), _p(q))
    return J, q


def alias_nodes(offsets, weights=None):
    offsets = np.ascontiguousarray(offsets, np.int64)
    nnz = int(offsets[-1])
    w = None if weights is None else np.ascontiguousarray(weights, np.float64)
    J = np.zeros(nnz, np.int64)
    q = np.zeros(nnz, np.float64)
    lib().or_alias_nodes(len(offsets) - 1, _p(offsets), _p(w), _p(J), _p(q))
    return J, q


def alias_edges(offsets, nbrs, weights, p, q):
    offsets = np.ascontiguousarray(offsets, np.int64)
    nbrs = np.ascontiguousarray(nbrs, np.int32)
    w = None if weights is None else np.ascontiguousarray(weights, np.float64)
    n = len(offsets) - 1
    eoff = np.zeros(len(nbrs) + 1, np.int64)
    tot = lib().or_alias_edges_offsets(n, _p(offsets), _p(nbrs), _p(eoff))
    J = np.zeros(tot, np.int64)
    qq = np.zeros(tot, np.float64)
    lib().or_alias_edges(n, _p(offsets), _p(nbrs), _p(w), float(p), float(q), _p(eoff), _p(J), _p(qq))
    return eoff, J, qq


def walks_replay(offsets, nbrs, nJ, nq, eoff, eJ, eq, L, starts, U):
    offsets = np.ascontiguousarray(offsets, np.int64)
    nbrs = np.ascontiguousarray(nbrs, np.int32)
    starts = np.ascontiguousarray(starts, np.int32)
    U = np.ascontiguousarray(U, np.float64)
    out = np.empty((len(starts), L), np.int32)
    lens = np.empty(len(starts), np.int32)
    used = lib().or_walks_replay(len(offsets) - 1, _p(offsets), _p(nbrs), _p(np.ascontiguousarray(nJ, np.int64)),
                                 _p(np.ascontiguousarray(nq, np.float64)), _p(np.ascontiguousarray(eoff, np.int64)),
                                 _p(np.ascontiguousarray(eJ, np.int64)), _p(np.ascontiguousarray(eq, np.float64)),
                                 int(L), len(starts), _p(starts), _p(U), len(U), _p(out), _p(lens))
    return out, lens, used


def walks_scale(csr, p, q, seed, L, walk_begin, walk_count, shuffle=True, directed=False,
                node_alias=None, nthreads=0):
    """csr: dict(offsets, nbrs, weights or None, node_order)."""
    off = np.ascontiguousarray(csr["offsets"], np.int64)
    nbrs = np.ascontiguousarray(csr["nbrs"], np.int32)
    w = csr.get("weights")
    w = None if w is None else np.ascontiguousarray(w, np.float64)
    n = len(off) - 1
    wsum = None
    nJ = nq = None
    if w is not None:
        wsum = np.array([w[off[v]:off[v + 1]].sum() if off[v + 1] > off[v] else 0.0 for v in range(n)])
        # sequential left-to-right sums (as the kernel)
        for v in range(n):
            s = 0.0
            for k in range(off[v], off[v + 1]):
                s += w[k]
            wsum[v] = s
        if node_alias is None:
            J64, qn = alias_nodes(off, w)
            node_alias = (J64.astype(np.int32), qn)
        nJ = np.ascontiguousarray(node_alias[0], np.int32)
        nq = np.ascontiguousarray(node_alias[1], np.float64)
    order = np.ascontiguousarray(csr["node_order"], np.int32)
    out = np.empty((walk_count, L), np.int32)
    lens = np.empty(walk_count, np.int32)
    cnt = np.zeros(2, np.uint64)
    lib().or_walks_scale(n, _p(off), _p(nbrs), _p(w), _p(wsum), _p(nJ), _p(nq), _p(order), int(directed),
                         float(p), float(q), int(seed), int(L), int(walk_begin), int(walk_count), int(shuffle),
                         _p(out), _p(lens), _p(cnt), int(nthreads))
    return out, lens, cnt


def walks_bitset(csr, p, q, seed, L, walk_begin, walk_count, shuffle=True, nthreads=0):
    """GW_N2V_BITSET restatement (exact 3-way mixture; unweighted undirected)."""
    off = np.ascontiguousarray(csr["offsets"], np.int64)
    nbrs = np.ascontiguousarray(csr["nbrs"], np.int32)
    order = np.ascontiguousarray(csr["node_order"], np.int32)
    out = np.empty((walk_count, L), np.int32)
    lens = np.empty(walk_count, np.int32)
    cnt = np.zeros(2, np.uint64)
    lib().or_walks_bitset(len(off) - 1, _p(off), _p(nbrs), _p(order), float(p), float(q), int(seed), int(L),
                          int(walk_begin), int(walk_count), int(shuffle), _p(out), _p(lens), _p(cnt),
                          int(nthreads))
    return out, lens, cnt


def jrand_sequence(seed, bound, k):
    out = np.empty(k, np.int32)
    lib().or_jrand_sequence(int(seed), int(bound), int(k), _p(out))
    return out


# ---- TopSim / SimRank ----------------------------------------------------------
def topsim(offsets, nbrs, variant, sample, step, C=0.6, seed=0, sources=None, rng="philox",
           java_seed=0, nthreads=0):
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    src = np.arange(n, dtype=np.int32) if sources is None else np.ascontiguousarray(sources, np.int32)
    rows = np.zeros((len(src), n), np.float64)
    st = np.zeros(4, np.int64)
    lib().or_topsim(n, _p(off), _p(nb), int(variant), int(sample), int(step), float(C), int(seed),
                    0 if rng == "philox" else 1, int(java_seed), _p(src), len(src), _p(rows), _p(st),
                    int(nthreads))
    return rows, dict(extensions=int(st[0]), pair_updates=int(st[1]), max_frontier=int(st[2]),
                      walkers=int(st[3]))


def topsim_topk(offsets, nbrs, variant, sample, step, topk, C=0.6, seed=0, sources=None, nthreads=0):
    """Per-source top-k (score desc, id asc; padded with id -1 / score 0) of the
    same TopSim rows as topsim(), without materialising n-wide rows per source
    (oracle.c or_topsim_topk): the CPU comparator for large graphs."""
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    src = np.arange(n, dtype=np.int32) if sources is None else np.ascontiguousarray(sources, np.int32)
    ids = np.empty((len(src), topk), np.int32)
    sc = np.empty((len(src), topk), np.float64)
    st = np.zeros(4, np.int64)
    lib().or_topsim_topk(n, _p(off), _p(nb), int(variant), int(sample), int(step), float(C), int(seed),
                         _p(src), len(src), int(topk), _p(ids), _p(sc), _p(st), int(nthreads))
    return ids, sc, dict(extensions=int(st[0]), pair_updates=int(st[1]), max_frontier=int(st[2]),
                         walkers=int(st[3]))


def simrank_naive(offsets, nbrs, C, iters, nthreads=0):
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    sim = np.zeros((n, n), np.float64)
    lib().or_simrank_naive(n, _p(off), _p(nb), float(C), int(iters), _p(sim), int(nthreads))
    return sim


def topsim_m(offsets, nbrs, variant, sample, step, capacity, C=0.6, seed=0, sources=None, nthreads=0):
    """TopSim_singleSample_M (variant 0) / SingleRandomWalk_M (variant 2) with
    FixedCacheMap(capacity): per source the drained (ascending) keys/values
    and sizes, plus stats."""
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    src = np.arange(n, dtype=np.int32) if sources is None else np.ascontiguousarray(sources, np.int32)
    keys = np.full((len(src), capacity), -1, np.int32)
    vals = np.zeros((len(src), capacity), np.float32)
    size = np.zeros(len(src), np.int32)
    st = np.zeros(4, np.int64)
    lib().or_topsim_m(n, _p(off), _p(nb), int(variant), int(sample), int(step), float(C), int(seed),
                      int(capacity), _p(src), len(src), _p(keys), _p(vals), _p(size), _p(st), int(nthreads))
    return keys, vals, size, dict(extensions=int(st[0]), pair_updates=int(st[1]), max_frontier=int(st[2]),
                                  walkers=int(st[3]))


def topsim_levels(offsets, nbrs, sample, step, tasks_v, tasks_call=None, seed=0, nthreads=0):
    """TopSim_doubleSample/TopSim_Dev sample(): per task the last-wins mass
    rows M[task, s-1, x] (0 = absent)."""
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    tv = np.ascontiguousarray(tasks_v, np.int32)
    tc = np.zeros_like(tv) if tasks_call is None else np.ascontiguousarray(tasks_call, np.int32)
    out = np.zeros((len(tv), step, n), np.float64)
    lib().or_topsim_levels(n, _p(off), _p(nb), int(sample), int(step), int(seed), _p(tv), _p(tc), len(tv),
                           _p(out), int(nthreads))
    return out


def topsim_double_sample(offsets, nbrs, sample, step, C=0.6, seed=0, nthreads=0):
    """TopSim_doubleSample(g, sample, step).compute() -> dense sim."""
    n = len(offsets) - 1
    M = topsim_levels(offsets, nbrs, sample, step, np.arange(n, dtype=np.int32), seed=seed, nthreads=nthreads)
    sim = np.zeros((n, n), np.float64)
    lib().or_topsim_double_sims(n, _p(M), int(step), float(C), _p(sim), int(nthreads))
    return sim


def topsim_dev(offsets, nbrs, sample, step, cand, C=0.6, seed=0, nthreads=0):
    """TopSim_Dev.compute(candidate) with candidate lists cand[n, K] (-1 pad);
    `sample` is TopSim_Dev's derived SAMPLE."""
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    cd = np.ascontiguousarray(cand, np.int32)
    sim = np.zeros((n, n), np.float64)
    lib().or_topsim_dev(n, _p(off), _p(nb), int(sample), int(step), float(C), int(seed), _p(cd), cd.shape[1],
                        _p(sim), int(nthreads))
    return sim


def double_random_walk(offsets, nbrs, sample, step, C=0.6, seed=0, nthreads=0):
    """DoubleRandomWalk(g, sample, step).compute() -> dense sim."""
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    sim = np.zeros((n, n), np.float64)
    lib().or_double_random_walk(n, _p(off), _p(nb), int(sample), int(step), float(C), int(seed), _p(sim),
                                int(nthreads))
    return sim


def fcm_run(nmax, keys, vals):
    """FixedCacheMap(nmax): put (keys[i], vals[i]) in order, then iterate
    (delMin, ascending) -> list of (key, value)."""
    k = np.ascontiguousarray(keys, np.int32)
    v = np.ascontiguousarray(vals, np.float32)
    ok = np.zeros(nmax, np.int32)
    ov = np.zeros(nmax, np.float32)
    c = lib().or_fcm_run(int(nmax), len(k), _p(k), _p(v), _p(ok), _p(ov))
    return [(int(ok[i]), float(ov[i])) for i in range(c)]


class PyFixedCacheMap:
    """Pure-Python literal FixedCacheMap (FixedCacheMap.java:14-127), float32
    arithmetic via numpy; cross-checks the C restatement."""

    def __init__(self, nmax):
        self.NMAX, self.N = nmax, 0
        self.keys = [0] * (nmax + 1)
        self.values = [np.float32(0)] * (nmax + 1)
        self.key2Index = {}

    def put(self, key, value):
        value = np.float32(value)
        index = self.key2Index.get(key)
        if index is not None:
            self.values[index] = np.float32(self.values[index] + value)
            self._sink(index)
        elif self.N < self.NMAX:
            self.N += 1
            self.keys[self.N], self.values[self.N] = key, value
            self.key2Index[key] = self.N
            self._swim(self.N)
        elif value > self.values[1]:
            del self.key2Index[self.keys[1]]
            self.keys[1], self.values[1] = key, value
            self.key2Index[key] = 1
            self._sink(1)

    def _sink(self, i):
        while 2 * i <= self.N:
            j = 2 * i
            if j < self.N and self.values[j] > self.values[j + 1]:
                j += 1
            if not self.values[i] > self.values[j]:
                break
            self._exch(i, j)
            i = j

    def _swim(self, i):
        while i > 1 and self.values[i // 2] > self.values[i]:
            self._exch(i, i // 2)
            i //= 2

    def _exch(self, a, b):
        self.key2Index[self.keys[a]] = b
        self.key2Index[self.keys[b]] = a
        self.keys[a], self.keys[b] = self.keys[b], self.keys[a]
        self.values[a], self.values[b] = self.values[b], self.values[a]

    def drain(self):
        out = []
        while self.N > 0:
            out.append((self.keys[1], float(self.values[1])))
            self.key2Index.pop(self.keys[1], None)
            self._exch(1, self.N)
            self.N -= 1
            self._sink(1)
        return out


def simrank_round_rows(offsets, nbrs, C, S, rb, re, nthreads=0):
    """One SimRank.java sweep for rows [rb, re) from matrix S -> (rows, pairs)."""
    off = np.ascontiguousarray(offsets, np.int64)
    nb = np.ascontiguousarray(nbrs, np.int32)
    n = len(off) - 1
    S = np.ascontiguousarray(S, np.float64)
    out = np.zeros((re - rb, n), np.float64)
    pairs = lib().or_simrank_round_rows(n, _p(off), _p(nb), float(C), _p(S), int(rb), int(re), _p(out),
                                        int(nthreads))
    return out, int(pairs)


# ---- pure-Python restatements ---------------------------------------------------
def read_graph_nx_semantics(path, delimiter, weighted, directed):
    """read_graph (node2vec/src/main.py:76-89) semantics WITHOUT networkx:
    returns (node_order labels, sorted labels, offsets, nbrs (dense), weights)."""
    order, seen = [], set()
    di = {}  # (u, v) -> weight, insertion order of first insert (DiGraph)
    succ = {}
    with open(path, "rb") as f:
        for raw in f:
            line = raw.decode()
            p = line.find("#")
            if p >= 0:
                line = line[:p]
                if not line:
                    continue
            s = line.rstrip("\n").split(delimiter)
            if len(s) < 2:
                continue
            u, v, d = int(s[0]), int(s[1]), s[2:]
            if weighted:
                if len(d) != 1:
                    raise IndexError("edge data length")
                w = float(d[0])
            else:
                if d:
                    raise TypeError("extra edge data")
                w = 1
            for x in (u, v):
                if x not in seen:
                    seen.add(x)
                    order.append(x)
            if (u, v) not in di:
                succ.setdefault(u, []).append(v)
            di[(u, v)] = w
    if directed:
        adj = {x: {} for x in order}
        for (u, v), w in di.items():
            adj[u][v] = w
    else:
        # to_undirected: iterate u in node order, v in succ insertion order;
        # the later processed directed edge's data wins for the pair
        adj = {x: {} for x in order}
        for u in order:
            for v in succ.get(u, []):
                w = di[(u, v)]
                adj[u][v] = w
                adj[v][u] = w
    labels = sorted(order)
    rank = {x: i for i, x in enumerate(labels)}
    offs, nbrs, wts = [0], [], []
    for u in labels:
        for v in sorted(adj[u]):
            nbrs.append(rank[v])
            wts.append(float(adj[u][v]))
        offs.append(len(nbrs))
    return (np.array(order, np.int64), np.array(labels, np.int64), np.array(offs, np.int64),
            np.array(nbrs, np.int32), np.array(wts, np.float64))


def java_double_to_string(v):
    """Java Double.toString(v) / "" + v (JLS): shortest round-trip digits
    (Python repr's), plain with >= 1 fraction digit for 1e-3 <= |v| < 1e7,
    else "d.dddE[-]n".  (JDK <= 18 printed a few values, e.g. subnormals, with
    extra digits; not emulated.)"""
    import math
    v = float(v)
    if v != v:
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    sign, digits, exp = decimal.Decimal(repr(v)).normalize().as_tuple()
    ds = "".join(map(str, digits))
    e = len(ds) - 1 + exp
    if 1e-3 <= abs(v) < 1e7:
        if e >= 0:
            body = ds[:e + 1].ljust(e + 1, "0") + "." + (ds[e + 1:] or "0")
        else:
            body = "0." + "0" * (-e - 1) + ds
    else:
        body = ds[0] + "." + (ds[1:] or "0") + "E" + str(e)
    return ("-" if sign else "") + body


def java_format_fixed(v, decimals=6):
    """Java 8 String.format("%.Nf", v): shortest repr digits, HALF_UP."""
    d = decimal.Decimal(repr(float(v)))
    q = decimal.Decimal(1).scaleb(-decimals)
    return format(d.quantize(q, rounding=decimal.ROUND_HALF_UP), "f")


def java_fixed_max_pq_row(row, topk, min_score=None):
    """FixedMaxPQ.offer over (i, row[i]) for i in order (only row[i] >=
    min_score when given, as TopSim_Dev.java:66-68), then sortedElement()
    (FixedMaxPQ.java:30-39,72-76; java.util.PriorityQueue siftUp/siftDown;
    Collections.sort(reverseOrder()) is stable)."""
    q = []

    def sift_up(k, x):
        while k > 0:
            parent = (k - 1) >> 1
            if x[1] >= q[parent][1]:
                break
            q[k] = q[parent]
            k = parent
        q[k] = x

    def poll():
        n = len(q) - 1
        x = q.pop()
        if n == 0:
            return
        k, half = 0, n >> 1
        while k < half:
            child = 2 * k + 1
            c = q[child]
            right = child + 1
            if right < n and c[1] > q[right][1]:
                child = right
                c = q[child]
            if x[1] <= c[1]:
                break
            q[k] = c
            k = child
        q[k] = x

    for i, val in enumerate(row):
        if min_score is not None and not float(val) >= min_score:
            continue
        e = (i, float(val))
        if len(q) < topk:
            q.append(None)
            sift_up(len(q) - 1, e)
        elif topk > 0 and q[0][1] < e[1]:
            poll()
            q.append(None)
            sift_up(len(q) - 1, e)
    out = list(q)
    out.sort(key=lambda t: -t[1])  # stable
    return out
