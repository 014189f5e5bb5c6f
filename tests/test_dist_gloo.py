"""CPU, world_size 2 over gloo: the data-parallel split used by bench.py and
the multi-GPU path.  The per-rank compute is the oracle's restatement of the
walk kernel (a CPU stand-in for the HIP call, which the GPU tests cover); what
is tested here is the shard arithmetic, the keyed-by-global-index invariance
and the all-gather plumbing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import DATA, PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _csr():
    import sys
    sys.path.insert(0, PKG)
    import gwamd
    G = gwamd.GWGraph.from_edgelist(os.path.join(DATA, "moreno_crime_crime.txt"), "\t", "nx")
    c = G.export_csr()
    c["weights"] = None
    return c


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from gwamd import dist as gd
        csr = _csr()
        n = len(csr["offsets"]) - 1
        total = 3 * n + 5
        b, c = gd.shard_range(total, world, rank)
        walks, lens, _ = oracle.walks_scale(csr, 0.25, 4.0, 17, 12, b, c)
        full = gd.allgather_rows(torch.from_numpy(walks), world)
        # weak scaling blocks: rank r step s -> (s*world + r)*B
        B = 100
        w0 = gd.weak_block(1, world, rank, B)
        wk, _, _ = oracle.walks_scale(csr, 0.25, 4.0, 17, 12, w0, B)
        weak = gd.allgather_rows(torch.from_numpy(wk), world)
        # TopSim sources sharded
        from conftest import DATA as D
        offs, nbrs = _java(os.path.join(D, "moreno_crime_crime.txt"), 1380)
        sb, sc = gd.shard_range(1380, world, rank)
        rows, _ = oracle.topsim(offs, nbrs, 0, 300, 2, seed=4, sources=np.arange(sb, sb + sc))
        tops = gd.allgather_rows(torch.from_numpy(rows), world)
        if rank == 0:
            q.put((full.numpy(), weak.numpy(), tops.numpy()))
    finally:
        dist.destroy_process_group()


def _java(path, V):
    adj = [[] for _ in range(V)]
    for line in open(path):
        a, b = line.split("\t")[:2]
        adj[int(a)].append(int(b))
        adj[int(b)].append(int(a))
    offs = np.zeros(V + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in adj])
    return offs, np.array([y for x in adj for y in x], np.int32)


def test_shard_range_partitions():
    from gwamd.dist import shard_range, weak_block
    for total in (0, 1, 7, 1000, 12345):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (b0, c0), (b1, _) in zip(spans, spans[1:]):
                assert b0 + c0 == b1
            assert sum(c for _, c in spans) == total
    assert [weak_block(s, 4, r, 10) for s in range(2) for r in range(4)] == list(range(0, 80, 10))


def test_two_rank_gloo_matches_single_process(oracle):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, weak, tops = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    csr = _csr()
    n = len(csr["offsets"]) - 1
    ref, _, _ = oracle.walks_scale(csr, 0.25, 4.0, 17, 12, 0, 3 * n + 5)
    np.testing.assert_array_equal(full, ref)
    refw, _, _ = oracle.walks_scale(csr, 0.25, 4.0, 17, 12, 200, 200)
    np.testing.assert_array_equal(weak, refw)
    offs, nbrs = _java(os.path.join(DATA, "moreno_crime_crime.txt"), 1380)
    rt, _ = oracle.topsim(offs, nbrs, 0, 300, 2, seed=4)
    np.testing.assert_array_equal(tops, rt)
