"""Where the rejection sampler's requests go (k_walk_scale, q > 1:
the mixture proposal when deg(prev) < deg(cur), the uniform proposal with the
lazy has_edge probe otherwise).  CPU only.

For every second-order step of walks of the exact law (oracle.walks_scale,
the same sampler the GPU runs) the expected trials and random requests are
computed in closed form from (deg prev, deg cur, common neighbours):

  mixture  (dp < dc): H = o + dc/q + (1-1/q) dp      (o = max(0, 1/p - 1/q))
           trials = H / (o + (dc - 1 + min(1, q/p))/q + (1-1/q) c)
           from_cur trial: 1 slot entry; from_prev trial: 1 slot entry + 1
           probe of cur's neighbour hash (x in N(cur))
  uniform  (dp >= dc): A = M dc + e  (M = max(1, 1/q), e = max(0, 1/p - M))
           candidate: 1 slot entry; x != prev and u M >= min(1, 1/q): 1 probe
           of prev's neighbour hash (x in N(prev))

and split by branch, by the degree of the probed row, and by the size of the
probed hash row.  At q < 1 (config 4) every step takes the uniform proposal.

    python tools/mixture_access_model.py [scale] [p] [q] [edge_factor] [walks]
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
nw = int(sys.argv[5]) if len(sys.argv) > 5 else 3000
G = GWGraph.rmat(scale, ef, 0.57, 0.19, 0.19, 42)
csr = G.export_csr()
off, nb = csr['offsets'], csr['nbrs']
deg = np.diff(off)
t0 = time.time()
W, lens, cnt = oracle.walks_scale(dict(csr, weights=None), p, q, 42, 80, 0, nw, nthreads=8)
print(f'n {len(deg)} nnz {len(nb)}; {nw} walks in {time.time() - t0:.1f} s; oracle trials/step '
      f'{cnt[1] / max(cnt[0], 1):.3f}', file=sys.stderr)

sets = {}


def N(v):
    s = sets.get(v)
    if s is None:
        s = set(nb[off[v]:off[v + 1]].tolist())
        sets[v] = s
    return s


a_p, a_q = 1 / p, 1 / q
# q < 1 (config 4): the uniform proposal with the lazy probe at every step
mo = max(0.0, a_p - a_q)
mprev = min(1.0, a_p / a_q)
M = max(1.0, a_q)
lo = min(1.0, a_q)
ext = max(0.0, a_p - M)
acc = dict(steps=0, first=0, mix_steps=0, uni_steps=0, trials=0.0, ent=0.0, probe=0.0,
           mix_ent_cur=0.0, mix_ent_prev=0.0, mix_probe=0.0, uni_ent=0.0, uni_probe=0.0,
           probe_rows_le16=0.0, probe_rows_le64=0.0, mix_rej_prev=0.0)
hub_rank = np.argsort(-deg, kind='stable')
rank_of = np.empty_like(hub_rank)
rank_of[hub_rank] = np.arange(len(deg))
probe_rank_hist = np.zeros(8)  # probed vertex rank < 16, 64, 256, 1024, 4096, 16384, 65536, rest
edges = [16, 64, 256, 1024, 4096, 16384, 65536]
for w in range(W.shape[0]):
    row = W[w]
    ln = int(lens[w])
    if ln > 1:
        acc['first'] += 1
        acc['ent'] += 1  # step 1: one slot entry
    for t in range(2, ln):
        prev, cur = int(row[t - 2]), int(row[t - 1])
        dc, dp = int(deg[cur]), int(deg[prev])
        Np, Nc = N(prev), N(cur)
        c = len(Nc & Np) - (1 if prev in Np else 0)  # x in N(cur), x != prev, x in N(prev)
        acc['steps'] += 1
        if q > 1.0 and dp < dc:  # the mixture proposal exists only at q > 1
            H = mo + dc * a_q + (1 - a_q) * dp
            Z = mo + (dc - 1 + mprev) * a_q + (1 - a_q) * c
            T = H / Z
            tc, tp = dc * a_q / Z, (1 - a_q) * dp / Z  # expected trials per branch
            acc['mix_steps'] += 1
            acc['mix_ent_cur'] += tc
            acc['mix_ent_prev'] += tp
            acc['mix_probe'] += tp
            acc['mix_rej_prev'] += (1 - a_q) * (dp - c) / Z
            pr, pv = tp, cur
        else:
            A = M * dc + ext
            # accepted mass (a candidate's proposal mass is M): the outlier ext,
            # prev min(1/p, M), a common neighbour 1, any other 1/q
            Z = ext + min(a_p, M) + c + (dc - 1 - c) * a_q
            T = A / Z
            te = M * dc / Z
            pr = M * (dc - 1) * (1 - lo / M) / Z
            pv = prev
            acc['uni_steps'] += 1
            acc['uni_ent'] += te
            acc['uni_probe'] += pr
        acc['trials'] += T
        dpr = int(deg[pv])
        if dpr <= 16:
            acc['probe_rows_le16'] += pr
        if dpr <= 64:
            acc['probe_rows_le64'] += pr
        k = int(np.searchsorted(edges, rank_of[pv], side='right'))
        probe_rank_hist[k] += pr
S = acc['steps'] + acc['first']
ent = acc['ent'] + acc['mix_ent_cur'] + acc['mix_ent_prev'] + acc['uni_ent']
probe = acc['mix_probe'] + acc['uni_probe']
res = {
    'graph': f'R-MAT-{scale} ef {ef}', 'p': p, 'q': q, 'walks': nw, 'steps': S,
    'oracle_trials_per_step': cnt[1] / max(cnt[0], 1),
    'model_trials_per_step': (acc['trials'] + acc['first']) / S,
    'requests_per_step': (ent + probe) / S,
    'entries_per_step': ent / S, 'probes_per_step': probe / S,
    'mixture_share_of_steps': acc['mix_steps'] / S,
    'mixture': {'from_cur_entries': acc['mix_ent_cur'] / S, 'from_prev_entries': acc['mix_ent_prev'] / S,
                'from_prev_probes': acc['mix_probe'] / S, 'from_prev_rejected': acc['mix_rej_prev'] / S},
    'uniform': {'entries': acc['uni_ent'] / S, 'probes': acc['uni_probe'] / S},
    'probes_into_rows_le16': acc['probe_rows_le16'] / S, 'probes_into_rows_le64': acc['probe_rows_le64'] / S,
    'probes_by_degree_rank_of_probed_row': dict(zip(['<16', '<64', '<256', '<1024', '<4096', '<16384', '<65536',
                                                     'rest'], (probe_rank_hist / S).round(4).tolist())),
}
print(json.dumps(res, indent=1))
