"""CPU model: would a 128-bit Bloom filter of N(prev), carried in the rejection
sampler's slot entry, spare the has_edge probes?  Samples edge-stationary
(prev, cur, x) triples on R-MAT and reports P(x in N(prev)) and the filter's
false-positive rate.   python tools/bloom_probe_model.py 20 16
"""
import sys, numpy as np
sys.path.insert(0,'graph-embedding_amd'); sys.path.insert(0,'.')
import gwamd
sc, ef = int(sys.argv[1]), int(sys.argv[2])
G = gwamd.GWGraph.rmat(sc, ef, 0.57, 0.19, 0.19, 42)
csr = G.export_csr(); off, nb = csr["offsets"].astype(np.int64), csr["nbrs"]
n = len(off)-1; deg = np.diff(off)
rng = np.random.default_rng(1)
# stationary edge-uniform: pick random slots (prev->cur), then uniform x in N(cur)
S = 200000
slots = rng.integers(0, len(nb), S)
prev = np.searchsorted(off, slots, side='right')-1
cur = nb[slots]
dc = deg[cur]
x = nb[off[cur] + (rng.random(S)*dc).astype(np.int64)]
keep = x != prev
prev, cur, x = prev[keep], cur[keep], x[keep]
def h(v, salt):
    return ((v.astype(np.uint64) * np.uint64(salt)) & np.uint64(0xFFFFFFFF)) >> np.uint64(25)  # 7 bits
adj = np.zeros(len(x), bool); fp1 = np.zeros(len(x), bool); fp2 = np.zeros(len(x), bool)
for i in range(len(x)):
    row = nb[off[prev[i]]:off[prev[i]+1]]
    adj[i] = x[i] in set(row.tolist()) if len(row) < 64 else np.any(row == x[i])
    if not adj[i]:
        b1 = set(h(row, 0x9E3779B1).tolist()); b2 = set(h(row, 0x85EBCA6B).tolist())
        hx1 = int(h(np.array([x[i]]), 0x9E3779B1)[0]); hx2 = int(h(np.array([x[i]]), 0x85EBCA6B)[0])
        fp1[i] = hx1 in b1
        fp2[i] = (hx1 in b1) and (hx2 in (b1 | b2))  # 2 hashes in one 128-bit filter
    if i > 60000: break
m = slice(0, i+1)
a = adj[m].mean(); f1 = fp1[m][~adj[m]].mean(); 
# k=2 in one filter: bits = union of h1,h2 of row
print(f"R-MAT-{sc} ef{ef}: P(x in N(prev)) = {a:.3f}; k=1 FP = {f1:.3f}; maybe-rate k=1 = {a + (1-a)*f1:.3f}")
