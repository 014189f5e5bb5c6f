"""Access model of k_walk_bitset: replays a sample of walks exactly (same
Philox draws as the kernel and the oracle) and counts, per step, the random
64 B sectors the kernel reads beyond the step's entry — region membership
words the draw filter cannot answer, region selects (block, and directory
words at hubs with d > 4096) — by payload mode and branch.  CPU only; the
sum is compared with the measured fabric read requests per step
(profiles/pmc_summary.json).

    python tools/bitset_access_model.py [--scale 20] [--walks 600]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))
sys.path.insert(0, ROOT)

M32 = 0xFFFFFFFF
TAG_STEP = 0x6E327632  # GW_TAG_N2V_STEP


def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (csrc/gw_philox.h)."""
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        hi0, lo0 = p0 >> 32, p0 & M32
        hi1, lo1 = p1 >> 32, p1 & M32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & M32, lo1, (hi0 ^ c3 ^ k1) & M32, lo0
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def index64(hi, lo, d):
    """gw_index (csrc/gw_philox.h): floor((hi * 2^32 + lo) * d / 2^64)."""
    return ((hi << 32 | lo) * d) >> 64


def bounded(x, d):
    return (x * d) >> 32


def mode_of(c, d, list_max=22, bits=352, inline_bits=None):
    """Payload mode of a slot (gw_internal.h): d < 65536 entries pack kp | c in
    one word and carry 11 payload words (352 bits, lists of 22), others 10."""
    if d >= 65536:
        bits = bits - 32
    if c <= list_max and d < 65536:
        return "list"
    if d <= (inline_bits or bits):
        return "inline"
    if c > 0:
        l = int(np.floor(np.log2(d // c))) if d // c > 0 else 0
        if c * l + c + ((d - 1) >> l) + 1 <= bits:
            return "ef"
    return "region"


def dir_reads(common, d, c, j, ndir, how):
    """Directory reads of a region select of the j-th common neighbour at a
    row with ndir > kPDir 512-bit blocks (the directory dir[g] = commons in
    blocks < g lives in the region).  Both searches start from the
    interpolated block g0 = floor(j * ndir / c):
    * "pair" (the shipped kernel): read dir[g], dir[g+1]; step g by -1 / +1
      until dir[g] <= j < dir[g+1] (one read per probe);
    * "sector" (round 3's degree-ordered library): read the 64 B sector of 16
      entries holding g, move one sector back / forward until the block is
      inside (one read per sector);
    * "one": a single read per select (round 3's model)."""
    if how == "one":
        return 1
    blocks = np.bincount(np.asarray(common, dtype=np.int64) // 512, minlength=ndir)[:ndir]
    dirv = np.concatenate([[0], np.cumsum(blocks)[:-1]])  # commons before block g
    g = min(int(j * ndir // max(c, 1)), ndir - 1)
    if how == "pair":
        reads = 1
        while True:
            lo = dirv[g]
            hi = dirv[g + 1] if g + 1 < ndir else c
            if j < lo:
                g -= 1
            elif j >= hi:
                g += 1
            else:
                return reads
            reads += 1
    # "sector"
    K = 16
    g &= ~(K - 1)
    reads, dmv = 0, 0
    while True:
        reads += 1
        E = dirv[g:g + K]
        cnt = int((E <= j).sum())
        if cnt == 0:
            if dmv == 1:
                return reads
            g -= K
            dmv = 2
        elif cnt == K and g + K < ndir and dmv != 2:
            g += K
            dmv = 1
        else:
            return reads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--p", type=float, default=0.25)
    ap.add_argument("--q", type=float, default=4.0)
    ap.add_argument("--walks", type=int, default=600)
    ap.add_argument("--seed", type=int, default=42)
    # what-if knobs (defaults = the built kernel): payload bits, list length,
    # filter buckets with / without an in-entry directory, in-entry directory limit
    ap.add_argument("--payload-bits", type=int, default=352)
    ap.add_argument("--list-max", type=int, default=22)
    ap.add_argument("--inline-bits", type=int, default=None,
                    help="inline bitsets up to this degree (default: --payload-bits)")
    ap.add_argument("--filter-dir", type=int, default=192)
    ap.add_argument("--filter-nodir", type=int, default=320)
    ap.add_argument("--tail-list", type=int, default=0,
                    help="what-if: entries with c <= this also carry their commons as positions in N(u)")
    ap.add_argument("--pdir", type=int, default=8, help="directory blocks kept in the entry (0: none)")
    ap.add_argument("--hub-bits", type=int, default=0,
                    help="what-if: every entry (u -> x) whose payload has room carries a bitmap of x's "
                         "adjacency to the H highest-degree vertices, answering membership of a hub prev")
    ap.add_argument("--order", default="id", choices=["id", "degree"],
                    help="what-if: positions of each row in degree-descending order, ties by id, instead of id "
                         "order")
    ap.add_argument("--hybrid-prefix", type=int, default=0,
                    help="what-if (with --order degree): region slots whose commons all lie below the payload's "
                         "bit count become inline ('prefix' mode); the others carry a bitset of positions < P and a "
                         "--tail-filter-bucket filter over positions >= P; selects of the j-th common below the "
                         "prefix count and membership of k < P are answered in registers")
    ap.add_argument("--tail-filter", type=int, default=64)
    ap.add_argument("--dir-search", default="pair", choices=["pair", "sector", "one"],
                    help="directory reads of a hub select: the shipped kernel's pair probes, round 3's "
                         "degree-ordered library's 64 B sectors, or one read (round 3's model)")
    ap.add_argument("--hybrid-dir", type=int, default=1,
                    help="1: entries with 512 < d <= 4096 keep the 128-bit in-entry directory (prefix shrinks by 128)")
    a = ap.parse_args()
    import gwamd
    import oracle
    G = gwamd.GWGraph.rmat(a.scale, 16, 0.57, 0.19, 0.19, 42)
    csr = G.export_csr()
    off, nbrs = csr["offsets"], csr["nbrs"]
    n = len(off) - 1
    deg = np.diff(off)
    hub_rank = np.full(n, n, dtype=np.int64)
    hub_rank[np.argsort(-deg, kind="stable")] = np.arange(n)
    L = 80
    begin = 7 * n + 11  # a window inside the bench's first step
    W, lens, _ = oracle.walks_bitset(csr, a.p, a.q, a.seed, L, begin, a.walks, nthreads=8)
    ap_, aq = 1.0 / a.p, 1.0 / a.q
    k0, k1 = a.seed & M32, ((a.seed >> 32) ^ TAG_STEP) & M32
    cnt = {}
    steps = 0

    def add(key, v=1):
        cnt[key] = cnt.get(key, 0) + v

    iters = np.zeros(a.walks)  # loop iterations each walk occupies (trials + region phases)
    for i in range(a.walks):
        w = begin + i
        iters[i] = 1
        c0, c1 = w & M32, (w >> 32) & M32
        last_ret = False
        for t in range(2, int(lens[i])):
            prev, cur = int(W[i, t - 2]), int(W[i, t - 1])
            row = nbrs[off[cur]:off[cur + 1]]
            if a.order == "degree":  # the same multiset, positions re-ranked by degree
                row = row[np.lexsort((row, -deg[row]))]
            d = len(row)
            prow = nbrs[off[prev]:off[prev + 1]]
            kp = int(np.nonzero(row == prev)[0][0])
            common = np.nonzero(np.isin(row, prow, assume_unique=True) & (row != prev))[0]
            c = len(common)
            mode = mode_of(c, d, a.list_max, a.payload_bits, a.inline_bits)
            if mode == "region" and a.hybrid_prefix and c and int(common.max()) < a.payload_bits - 32:
                mode = "prefix"  # every common position fits a prefix bitset in the payload: no region reads
            ndir = (d + 511) // 512 if d > 512 else 0
            F = a.filter_dir if 0 < ndir <= a.pdir else a.filter_nodir
            fset = set()
            if mode == "region":
                for k in common:
                    ulo = (int(k) << 32) // d  # high words y of the 64-bit draws with index k
                    uhi = (((int(k) + 1) << 32) + d - 1) // d - 1
                    for b in range(bounded(ulo, F), bounded(uhi, F) + 1):
                        fset.add(b)
            cset = set(common.tolist())
            steps += 1
            add(f"mode_{mode}")
            trial = 0
            while True:
                u = philox(c0, c1, t, trial, k0, k1)
                trial += 1
                iters[i] += 1
                if trial == 1:
                    Z = (ap_ + c) + (d - 1 - c) * aq
                    r = u[0] * 2.3283064365386963e-10 * Z
                    if r < ap_:
                        add("branch_return")
                        if c == 0 and d < 65536 and len(prow) < 65536:
                            add("entry_elided_return")  # return elision: the reverse entry is the stash
                        if last_ret:
                            add("return_after_return")  # entry = the one read two steps earlier
                        last_ret = True
                        break
                    last_ret = False
                    if r - ap_ < c:
                        add("branch_common")
                        jsel = min(int(r - ap_), c - 1)
                        Pp = a.hybrid_prefix if not (a.hybrid_dir and 512 < d <= 4096) else max(a.hybrid_prefix - 128, 0)
                        if mode == "region" and a.hybrid_prefix and int(common[jsel]) < Pp:
                            add("select_answered_by_prefix")
                            break
                        if mode == "region":
                            add("sectors_region_select_block")
                            iters[i] += 1
                            if ndir > a.pdir:
                                nrd = dir_reads(common, d, c, jsel, ndir, a.dir_search)
                                add("sectors_region_directory", nrd)
                                add("region_directory_selects")
                                iters[i] += nrd
                        break
                    add("branch_other")
                k = index64(u[1], u[2], d)  # the kernel's 64-bit "other" draw (u.y:u.z)
                if mode == "region" and a.hybrid_prefix and k != kp:
                    P = a.hybrid_prefix if not (a.hybrid_dir and 512 < d <= 4096) else max(a.hybrid_prefix - 128, 0)
                    if k < P:
                        add("membership_answered_by_prefix")
                    else:  # tail filter: buckets over positions P..d-1
                        tail = [int(x) for x in common if x >= P]
                        TB = a.tail_filter
                        b = (k - P) * TB // max(d - P, 1)
                        if any((x - P) * TB // max(d - P, 1) == b for x in tail):
                            add("sectors_region_membership_word")
                elif mode == "region" and k != kp and bounded(u[1], F) in fset:
                    add("sectors_region_membership_word")
                    if k in cset:  # the candidate's entry, loaded beside the word, is dropped
                        add("speculative_entry_dropped")
                    if a.tail_list:  # would the candidate's entry (cur -> x) carry a tail-indexed list?
                        x = int(row[k])
                        rx = nbrs[off[x]:off[x + 1]]
                        cx = int(np.isin(rx, row, assume_unique=True).sum()) - int(cur in set(rx.tolist()))
                        if cx <= a.tail_list and d < 65536:
                            add("membership_word_answered_by_candidate_tail_list")
                    if a.hub_bits:
                        if hub_rank[prev] < a.hub_bits:
                            add(f"membership_word_prev_in_top{a.hub_bits}")
                            x = int(row[k])
                            rx = nbrs[off[x]:off[x + 1]]
                            cx = int(np.isin(rx, row, assume_unique=True).sum()) - int(cur in set(rx.tolist()))
                            # room: a list of cx u16 beside the bitmap, or the other modes' payload bits
                            room = (16 * cx + a.hub_bits <= a.payload_bits) if cx <= a.list_max else False
                            if room and len(rx) < 65536:
                                add("membership_word_answered_by_candidate_hub_bitmap")
                if k != kp and k not in cset:
                    break
                add("other_retries")
    # a wave's 64 lanes run until its slowest walk ends: lane occupancy
    g = iters[: len(iters) // 64 * 64].reshape(-1, 64)
    occupancy = float(g.mean() / g.max(axis=1).mean()) if len(g) else None
    res = {"graph": f"R-MAT-{a.scale}", "p": a.p, "q": a.q, "walks": a.walks, "steps_modelled": steps}
    for k, v in sorted(cnt.items()):
        res[k + "_per_step"] = v / steps
    extra = sum(v for k, v in cnt.items() if k.startswith("sectors_")) / steps
    res["extra_region_sectors_per_step"] = extra
    elided = cnt.get("entry_elided_return", 0) / steps
    res["model_read_sectors_per_step"] = 1.0 - elided + extra + 2.0 / L  # + entry (less elided returns); + walk starts
    res["iterations_per_walk_mean"] = float(iters.mean())
    res["wave_lane_occupancy"] = occupancy
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
        e = pmc.get(f"n2v_rmat{a.scale}_ef16_p{a.p}_q{a.q}_L80_r10_bitset") or pmc[f"n2v_rmat{a.scale}_p{a.p}_q{a.q}_L80_r10_bitset"]
        units = e.get("units_per_launch") or e["walk_steps_per_launch"]
        res["measured_fabric_read_requests_per_step"] = e["fabric_read_requests_per_launch"] / units
        res["measured_lib_sha256"] = e.get("lib_sha256")
    except Exception:
        pass
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
