"""Drop-in for the reference `node2vec` module (node2vec/src/node2vec.py).

Same names, argument meaning and side effects:

    G = node2vec.Graph(nx_G, is_directed, p, q)     # node2vec.py:7-11
    G.preprocess_transition_probs()                  # node2vec.py:83-113  (GPU)
    walks = G.simulate_walks(num_walks, walk_length) # node2vec.py:41-59   (GPU)
    J, q = alias_setup(probs)                        # node2vec.py:116-147 (GPU)
    idx = alias_draw(J, q)                           # node2vec.py:150-160

Exact replay: like the reference, `simulate_walks` shuffles `list(G.nodes())`
in place with the global `random` module once per iteration and draws every
step's two uniforms from the global `np.random` stream; the global states
advance exactly as the reference's would.  The uniforms are generated on the
host by numpy (they ARE the reference's stream), the walks and alias tables
are computed by the HIP kernels of libgraphwalk.

`mode="scale"` instead runs the Philox-keyed scale samplers (reproducible by
`seed`, identical for any GPU count).  `preprocess_transition_probs` then only
uploads the graph: the sampler is prepared by the first `simulate_walks`, once
num_walks * n * (walk_length - 1) steps are known, with GW_N2V_AUTO by default
(the per-edge bitset sampler when its build pays back over those steps, else
the rejection sampler; `sampler="bitset"` / `"rejection"` force one).

Walk bits in scale mode: both samplers draw every walk from the reference's
law, but with different draws, so for a given `seed` the walk at a given
index depends on the sampler — and under the default `sampler="auto"` the
sampler depends on the FIRST `simulate_walks` call's workload (the choice
then sticks for later calls on the same Graph).  Callers that need walks that
are bit-stable across different `num_walks` (e.g. a prefix of a larger run)
pass `sampler="rejection"` or `sampler="bitset"` explicitly.
"""
import random
from collections.abc import Mapping

import numpy as np

from . import _lib as C
from .graph import GWGraph


class _AliasNodes(Mapping):
    def __init__(self, owner):
        self._o = owner

    def __getitem__(self, node):
        o = self._o
        i = o._rank(node)
        b, e = o._csr["offsets"][i], o._csr["offsets"][i + 1]
        return o._node_J[b:e].astype(np.int64), o._node_q[b:e].copy()

    def __iter__(self):
        return iter(self._o.G.nodes())

    def __len__(self):
        return self._o.G.number_of_nodes()


class _AliasEdges(Mapping):
    def __init__(self, owner):
        self._o = owner

    def _slot(self, key):
        o = self._o
        u, v = key
        i, j = o._rank(u), o._rank(v)
        offs, nbrs = o._csr["offsets"], o._csr["nbrs"]
        row = nbrs[offs[i]:offs[i + 1]]
        k = np.searchsorted(row, j)
        if k >= len(row) or row[k] != j:
            raise KeyError(key)
        return offs[i] + k

    def __getitem__(self, key):
        o = self._o
        s = self._slot(key)
        b, e = o._edge_off[s], o._edge_off[s + 1]
        return o._edge_J[b:e].astype(np.int64), o._edge_q[b:e].copy()

    def __iter__(self):
        o = self._o
        offs, nbrs, lab = o._csr["offsets"], o._csr["nbrs"], o._csr["labels"]
        for i in range(len(offs) - 1):
            for k in range(offs[i], offs[i + 1]):
                yield (int(lab[i]), int(lab[nbrs[k]]))

    def __len__(self):
        return int(self._o._csr["nnz"])


class Graph:
    """node2vec.Graph (node2vec.py:6-113) on the GPU."""

    def __init__(self, nx_G, is_directed, p, q, device=0, mode="replay", seed=0, sampler="auto"):
        if sampler not in ("auto", "bitset", "rejection"):
            raise ValueError("sampler must be 'auto', 'bitset' or 'rejection'")
        self.sampler = sampler
        self.G = nx_G
        self.is_directed = is_directed
        self.p = p
        self.q = q
        self.device = device
        self.mode = mode
        self.seed = seed
        self._g = GWGraph.from_networkx(nx_G, directed=bool(is_directed))
        csr = self._g.export_csr()
        csr["nnz"] = len(csr["nbrs"])
        self._csr = csr
        self._lab2rank = {int(x): i for i, x in enumerate(csr["labels"])}
        self._prepared = False

    def _rank(self, label):
        try:
            return self._lab2rank[int(label)]
        except (KeyError, TypeError, ValueError):
            raise KeyError(label)

    # -- node2vec.py:83-113 ----------------------------------------------------
    def preprocess_transition_probs(self):
        self._g.to_device(self.device)
        self._prepared = True
        if self.mode != "replay":
            # scale mode: the sampler is chosen and built by the first
            # simulate_walks, when the number of walk steps is known
            self._scale_mode = None
            return
        mode = C.N2V_REPLAY
        C.check(C.lib().gw_n2v_prepare(self._g.handle, float(self.p), float(self.q), mode),
                self._g.handle)
        if mode == C.N2V_REPLAY:
            inf = self._g.info()
            nnz, E = inf.nnz, inf.edge_alias_entries
            self._node_J = np.empty(nnz, np.int32)
            self._node_q = np.empty(nnz, np.float64)
            self._edge_off = np.empty(nnz + 1, np.int64)
            self._edge_J = np.empty(E, np.int32)
            self._edge_q = np.empty(E, np.float64)
            C.check(C.lib().gw_n2v_export_alias(self._g.handle, C.ptr(self._node_J), C.ptr(self._node_q),
                                                C.ptr(self._edge_off), C.ptr(self._edge_J),
                                                C.ptr(self._edge_q)), self._g.handle)
            self.alias_nodes = _AliasNodes(self)
            self.alias_edges = _AliasEdges(self)
        return

    # -- node2vec.py:41-59 -----------------------------------------------------
    def simulate_walks(self, num_walks, walk_length):
        if not self._prepared:
            raise AttributeError("'Graph' object has no attribute 'alias_nodes' "
                                 "(call preprocess_transition_probs first)")
        if self.mode != "replay":
            return self._simulate_scale(num_walks, walk_length)
        nodes = list(self.G.nodes())
        starts = []
        for _ in range(num_walks):
            random.shuffle(nodes)  # in place, cumulative (node2vec.py:49-51)
            starts.extend(self._rank(x) for x in nodes)
        return self._replay(np.asarray(starts, np.int32), walk_length)

    # -- node2vec.py:13-39 -----------------------------------------------------
    def node2vec_walk(self, walk_length, start_node):
        if not self._prepared:
            raise AttributeError("call preprocess_transition_probs first")
        return self._replay(np.asarray([self._rank(start_node)], np.int32), walk_length)[0]

    def _replay(self, starts, L):
        nw = len(starts)
        if nw == 0:
            return []
        upper = 2 * max(L - 1, 0) * nw
        st = np.random.get_state()
        U = np.random.random_sample(upper) if upper else np.zeros(0)
        out = np.empty((nw, L), np.int32)
        lens = np.empty(nw, np.int32)
        used = C.I64(0)
        h = self._g.handle
        C.check(C.lib().gw_n2v_walks_replay(h, int(L), nw, C.ptr(starts), C.ptr(U), len(U),
                                            C.ptr(out), C.ptr(lens), C.ctypes.byref(used)), h)
        # advance the global stream by exactly what the reference would draw
        np.random.set_state(st)
        if used.value:
            np.random.random_sample(int(used.value))
        lab = self._csr["labels"]
        return [lab[out[i, :lens[i]]].tolist() for i in range(nw)]

    @property
    def scale_sampler(self):
        """GW_N2V_* the scale sampler was prepared with (None before the first
        simulate_walks)."""
        return getattr(self, "_scale_mode", None)

    def _prepare_scale(self, steps):
        if self._scale_mode is not None:
            return
        mode = {"auto": C.N2V_AUTO, "bitset": C.N2V_BITSET, "rejection": C.N2V_REJECTION}[self.sampler]
        self._g.options(expected_steps=int(steps))
        h = self._g.handle
        C.check(C.lib().gw_n2v_prepare(h, float(self.p), float(self.q), mode), h)
        self._scale_mode = self._g.info().n2v_mode

    def _simulate_scale(self, num_walks, walk_length):
        import torch
        n = self._csr["labels"].shape[0]
        nw = num_walks * n
        self._prepare_scale(nw * max(int(walk_length) - 1, 0))
        dev = torch.device("cuda", self.device)
        out = torch.empty((nw, walk_length), dtype=torch.int32, device=dev)
        lens = torch.empty(nw, dtype=torch.int32, device=dev)
        h = self._g.handle
        stream = torch.cuda.current_stream(dev).cuda_stream
        C.check(C.lib().gw_n2v_walks(h, int(walk_length), int(self.seed), 0, nw, 1, C.ptr(out), C.ptr(lens),
                                     None, C.ctypes.c_void_p(stream)), h)
        o = out.cpu().numpy()
        ln = lens.cpu().numpy()
        lab = self._csr["labels"]
        return [lab[o[i, :ln[i]]].tolist() for i in range(nw)]


def alias_setup(probs, device=0):
    """node2vec.py:116-147 on the GPU: returns (J int64, q float64)."""
    p = np.ascontiguousarray(probs, dtype=np.float64)
    K = len(p)
    J = np.zeros(K, np.int64)
    q = np.zeros(K, np.float64)
    if K:
        C.check(C.lib().gw_alias_setup(int(device), C.ptr(p), K, C.ptr(J), C.ptr(q)))
    return J, q


def alias_draw(J, q):
    """node2vec.py:150-160: one draw with two np.random.rand() values (host
    utility; the walk kernels never call this)."""
    K = len(J)
    kk = int(np.floor(np.random.rand() * K))
    if np.random.rand() < q[kk]:
        return kk
    return J[kk]
