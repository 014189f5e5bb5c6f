"""Would a neighbour-set filter in the slot entry cut the one-shot sampler's
requests?  (round-6 review item: hybrids that avoid the two-request
from_prev rejects).  CPU only.

The rejection sampler (k_walk_scale) pays per trial one slot
entry and, for some trials, one probe of a neighbour hash:

  mixture step (q > 1, dp < dc), from_prev trial: x uniform over N(prev)
      (prev's slot entry of x), accepted iff x in N(cur): entry + probe of
      cur's hash;
  uniform step (dp >= dc, or q < 1): x uniform over N(cur), lazy probe of
      prev's hash for "x in N(prev)".

Both probes ask whether an edge {x, y} exists for y = cur or prev, and the
entry just read is x's own.  Here x's entry would carry a B-bit one-hash
filter of N(x) (a Bloom filter: bit h(y) set for every y in N(x)); a clear
bit proves {x, y} absent and skips the probe.  A filter cannot widen the
16 B entry without a second load instruction per entry (the
cost is per instruction and line), so B = 32 (4 B left in a 12 B-packed
entry) is what fits for free; 96 / 224 bits are priced as if a 32 / 64 B
entry cost nothing extra (upper bounds on the gain).

For walks of the exact law (oracle.walks_scale) the expected requests per
step are computed in closed form per step: with FP(x) = 1 - (1 - 1/B)^deg(x)
the probability that a non-member's bit is set,

  from_prev probes = (c + sum_{x in N(prev) \\ N(cur)} FP(x)) / dp per trial,
  uniform probes  = (lazy share) * (c' + sum_{x in N(cur) \\ N(prev), x != prev} FP(x)) / (dc - 1).

    python tools/mixture_filter_model.py [scale] [p] [q] [edge_factor] [walks]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'graph-embedding_amd'))
from gwamd import GWGraph  # noqa: E402
import oracle  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
q = float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
ef = int(sys.argv[4]) if len(sys.argv) > 4 else 16
nw = int(sys.argv[5]) if len(sys.argv) > 5 else 1000
BITS = [0, 32, 96, 224]
G = GWGraph.rmat(scale, ef, 0.57, 0.19, 0.19, 42)
csr = G.export_csr()
off, nb = csr['offsets'], csr['nbrs']
deg = np.diff(off).astype(np.int64)
t0 = time.time()
W, lens, cnt = oracle.walks_scale(dict(csr, weights=None), p, q, 42, 80, 0, nw, nthreads=8)
print(f'n {len(deg)} nnz {len(nb)}; {nw} walks in {time.time() - t0:.1f} s', file=sys.stderr)
FP = {B: (1.0 - (1.0 - 1.0 / B) ** deg.astype(np.float64)) if B else np.ones(len(deg)) for B in BITS}
# S[B][v] = sum over x in N(v) of FP_B(x)
rowid = np.repeat(np.arange(len(deg)), deg)
S = {B: np.bincount(rowid, weights=FP[B][nb], minlength=len(deg)) for B in BITS}
a_p, a_q = 1 / p, 1 / q
mo = max(0.0, a_p - a_q)
mprev = min(1.0, a_p / a_q)
M = max(1.0, a_q)
lo = min(1.0, a_q)
ext = max(0.0, a_p - M)
acc = {B: dict(ent=0.0, probe=0.0) for B in BITS}
steps = 0
sets = {}


def N(v):
    s = sets.get(v)
    if s is None:
        s = nb[off[v]:off[v + 1]]
        sets[v] = (s, set(s.tolist()))
        s = sets[v]
    return s


for w in range(W.shape[0]):
    row = W[w]
    ln = int(lens[w])
    if ln > 1:
        steps += 1
        for B in BITS:
            acc[B]['ent'] += 1
    for t in range(2, ln):
        prev, cur = int(row[t - 2]), int(row[t - 1])
        dc, dp = int(deg[cur]), int(deg[prev])
        (ap, Np), (ac, Nc) = N(prev), N(cur)
        common = Nc & Np
        c = len(common) - (1 if prev in Np else 0)
        comm_arr = np.fromiter((x for x in common if x != prev), dtype=np.int64, count=c) if c else None
        steps += 1
        if q > 1.0 and dp < dc:
            Z = mo + (dc - 1 + mprev) * a_q + (1 - a_q) * c
            tc, tp = dc * a_q / Z, (1 - a_q) * dp / Z
            for B in BITS:
                # x in N(prev): members (common, incl. cur's own self-loop case ignored) always probe
                s_non = S[B][prev] - (FP[B][comm_arr].sum() if c else 0.0)
                if prev in Np:  # prev's self-loop: x = prev, in N(cur); counted as a member probe
                    s_non -= FP[B][prev]
                pr = (c + (1 if prev in Np else 0) + s_non) / dp
                acc[B]['ent'] += tc + tp
                acc[B]['probe'] += tp * pr
        else:
            Z = ext + min(a_p, M) + c + (dc - 1 - c) * a_q
            te = M * dc / Z
            lazy = (1 - lo / M)  # share of candidates whose draw needs the probe
            for B in BITS:
                # candidates x in N(cur), x != prev: members of N(prev) always probe
                s_non = S[B][cur] - (FP[B][comm_arr].sum() if c else 0.0) - (FP[B][prev] if prev in Nc else 0.0)
                pr_c = M * lazy * (c + s_non) / Z
                acc[B]['ent'] += te
                acc[B]['probe'] += pr_c
res = {'graph': f'R-MAT-{scale} ef {ef}', 'p': p, 'q': q, 'walks': nw, 'steps': steps,
       'requests_per_step': {str(B) if B else 'no filter': round((acc[B]['ent'] + acc[B]['probe']) / steps, 4)
                             for B in BITS},
       'probes_per_step': {str(B) if B else 'no filter': round(acc[B]['probe'] / steps, 4) for B in BITS},
       'entries_per_step': round(acc[0]['ent'] / steps, 4)}
print(json.dumps(res, indent=1))
