"""Expected fabric reads per second-order step of the rejection sampler:
uniform proposal (envelope + lazy has_edge probe) vs the q > 1 mixture
proposal, over walks of the exact law (oracle.walks_bitset) on
R-MAT-<scale>.  CPU only.

    python tools/mixture_cost_model.py [scale] [p] [q] [edge_factor]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'graph-embedding_amd'))
from gwamd import GWGraph
import oracle
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
p, q = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25, float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
ef = int(sys.argv[4]) if len(sys.argv) > 4 else 16
G = GWGraph.rmat(scale, ef)
csr = G.export_csr()
off, nb = csr['offsets'], csr['nbrs']
n = len(off) - 1
deg = np.diff(off)
print('n', n, 'nnz', len(nb))
t = time.time()
W, lens, cnt = oracle.walks_bitset(csr, p, q, 7, 80, 0, 4000)
print('walks', time.time() - t)
sets = {}
def N(v):
    s = sets.get(v)
    if s is None:
        s = set(nb[off[v]:off[v+1]].tolist()); sets[v] = s
    return s
a_p, a_q = 1/p, 1/q
old = new = best = 0.0; steps = 0; frac_new = 0
for w in range(W.shape[0]):
    row = W[w]
    for t in range(2, lens[w]):
        prev, cur = int(row[t-2]), int(row[t-1])
        dc, dp = deg[cur], deg[prev]
        Np = N(prev); Nc = N(cur)
        c = len(Nc & Np) - (1 if prev in Nc and prev in Np else 0)
        Z = a_p + c + (dc - 1 - c) * a_q
        # old: envelope M = max(1, 1/q); candidate reads + lazy probes
        M = max(1.0, a_q); lo = min(1.0, a_q)
        extra = max(0.0, a_p - M)
        Hold = M * dc + extra
        reads_old = dc * (1 + (1 - lo / M))  # per unit proposal mass: 1 read + probe w.p. 1-lo/M
        o = reads_old / Hold * (Hold / Z)  # reads per trial * trials
        # new mixture (q > 1): cur-branch mass dc/q, prev-branch (1-1/q) dp, outlier 1/p - 1/q
        Hn = dc * a_q + (1 - a_q) * dp + max(0.0, a_p - a_q)
        nr = (dc * a_q * 1 + (1 - a_q) * dp * 2) / Z
        old += o; new += nr; best += min(o, nr); steps += 1; frac_new += nr < o
print('steps', steps, 'old reads/step %.3f new %.3f best %.3f  new-chosen %.2f' % (old/steps, new/steps, best/steps, frac_new/steps))
print('trials/step old', cnt[1]/max(cnt[0],1))
