"""node2vec walk-generation CLI, flag-compatible with node2vec/src/main.py.

    python -m gwamd.cli --input graph.edgelist --delimiter ' ' --p 0.25 --q 4 \
        --walk-length 80 --num-walks 10 --walks walks.txt [--mode replay|scale]

main.py:20-73 flags are accepted with the same names, defaults and quirks
(`--delimiter` defaults to ',' (:59); `--unweighted`/`--undirected` write to
their own dests and never clear `weighted`/`directed` (:64, :69)).
The embedding flags (--output, --dimensions, --window-size, --iter,
--workers) belong to gensim's Word2Vec (main.py:92-101), which is out of
scope: they are accepted and ignored.  Walks are written in DeepSim's
save_list format (DeepSim/src/main.py:237-243) or as .npy.

--mode replay : reference-exact (networkx graph, global random/np.random
                seeded with --seed, per-edge alias tables on the GPU);
--mode scale  : Philox samplers (any size; identical for any GPU count):
                --sampler auto (GW_N2V_AUTO) picks the per-edge bitset
                sampler or the rejection sampler by modelled end-to-end
                time for this run's walks (a one-pass run on R-MAT-20:
                rejection, 0.05 s vs 0.22 s, the bitset build dominating).

Multi-GPU (scale mode): launch one process per GPU with torchrun; rank r
walks its contiguous block of the global walk indices on GPU LOCAL_RANK, the
blocks are all-gathered over RCCL (gwamd.dist.allgather_rows) and rank 0
writes the file, identical to a one-GPU run.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m gwamd.cli --mode scale ...
"""
import argparse
import random
import sys
import time

import numpy as np


def parse_args(argv=None, p=1.0, q=1.0):
    ap = argparse.ArgumentParser(description="Run node2vec walk generation on MI355X.")
    ap.add_argument("--input", nargs="?", default="../graph/karate.edgelist", help="Input graph path")
    ap.add_argument("--output", nargs="?", default=None, help="(embeddings path; gensim step not run)")
    ap.add_argument("--walks", default="walks.txt", help="walks output (save_list format, or .npy)")
    ap.add_argument("--dimensions", type=int, default=128)
    ap.add_argument("--walk-length", type=int, default=80)
    ap.add_argument("--num-walks", type=int, default=10)
    ap.add_argument("--window-size", type=int, default=10)
    ap.add_argument("--iter", default=10, type=int)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--p", type=float, default=p)
    ap.add_argument("--q", type=float, default=q)
    ap.add_argument("--delimiter", type=str, default=",")
    ap.add_argument("--weighted", dest="weighted", action="store_true")
    ap.add_argument("--unweighted", dest="unweighted", action="store_false")
    ap.set_defaults(weighted=False)
    ap.add_argument("--directed", dest="directed", action="store_true")
    ap.add_argument("--undirected", dest="undirected", action="store_false")
    ap.set_defaults(directed=False)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--mode", choices=["replay", "scale"], default="replay")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--sampler", choices=["auto", "bitset", "rejection"], default="auto",
                    help="scale mode: second-order sampler")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend when launched with several ranks (nccl = RCCL)")
    return ap.parse_args(argv)


def read_graph(args):
    """main.py:76-89 read_graph (networkx)."""
    import networkx as nx
    if args.weighted:
        G = nx.read_edgelist(args.input, nodetype=int, data=(("weight", float),), create_using=nx.DiGraph(),
                             delimiter=args.delimiter)
    else:
        G = nx.read_edgelist(args.input, nodetype=int, create_using=nx.DiGraph(), delimiter=args.delimiter)
        for edge in G.edges():
            G[edge[0]][edge[1]]["weight"] = 1
    if not args.directed:
        G = G.to_undirected()
    return G


def _scale(args):
    """--mode scale on one GPU or, under torchrun, one block of walks per rank."""
    import os
    import torch
    from . import _lib as C
    from . import dist as gd
    from . import io
    from .graph import GWGraph
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    device = args.device
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        device = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)
    g = GWGraph.from_edgelist(args.input, args.delimiter, "nx", args.directed, args.weighted)
    g.to_device(device)
    # the walks this rank will run on this preparation: the sampler's optional
    # tables are built only when they pay back within them (gw_options_t)
    g.options(expected_steps=gd.shard_range(args.num_walks * g.n, world, rank)[1] * (args.walk_length - 1))
    if world > 1:
        import torch.distributed as dist
        dev = torch.device("cuda", device) if args.dist_backend == "nccl" else torch.device("cpu")
    err = None
    if args.sampler == "auto":
        # the library picks bitset or rejection by modelled end-to-end time for
        # the walks announced above (the rejection sampler's pilot trials
        # against the bitset build model); with several ranks rank 0 decides
        # for all, so every shard comes from the same sampler.  A failure on
        # rank 0 is broadcast as mode -2 so no rank waits in a collective for it.
        chosen = -1
        if world == 1 or rank == 0:
            try:
                C.check(C.lib().gw_n2v_prepare(g.handle, args.p, args.q, C.N2V_AUTO), g.handle)
                chosen = g.info().n2v_mode
            except Exception as e:  # noqa: BLE001 - re-raised below on every rank
                if world == 1:
                    raise
                err, chosen = e, -2
        if world > 1:
            m = torch.tensor([chosen if rank == 0 else -1], dtype=torch.int64, device=dev)
            dist.broadcast(m, 0)
            chosen = int(m.item())
            if chosen == -2 and err is None:
                err = RuntimeError("rank 0 failed to prepare the sampler (GW_N2V_AUTO)")
            if rank != 0 and err is None:
                try:
                    C.check(C.lib().gw_n2v_prepare(g.handle, args.p, args.q, chosen), g.handle)
                except Exception as e:  # noqa: BLE001
                    err = e
    else:
        mode = C.N2V_BITSET if args.sampler == "bitset" else C.N2V_REJECTION
        try:
            C.check(C.lib().gw_n2v_prepare(g.handle, args.p, args.q, mode), g.handle)
        except Exception as e:  # noqa: BLE001
            if world == 1:
                raise
            err = e
    if world > 1:
        # every rank prepared (or every rank raises): no rank enters the walk
        # all-gather while another has already failed
        ok = torch.tensor([0 if err is not None else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            dist.destroy_process_group()
            raise err if err is not None else RuntimeError("another rank failed to prepare the sampler")
    nwalks = args.num_walks * g.n
    L = args.walk_length
    begin, count = gd.shard_range(nwalks, world, rank)
    W = torch.empty((count, L), dtype=torch.int32, device=f"cuda:{device}")
    lens = torch.empty(count, dtype=torch.int32, device=f"cuda:{device}")
    st = torch.cuda.current_stream(device)
    C.check(C.lib().gw_n2v_walks(g.handle, L, args.seed, begin, count, 1, C.ptr(W), C.ptr(lens), None,
                                 C.ctypes.c_void_p(st.cuda_stream)), g.handle)
    torch.cuda.synchronize(device)
    if world > 1:
        if args.dist_backend != "nccl":  # (gloo rehearsals gather host tensors)
            W, lens = W.cpu(), lens.cpu()
        W = gd.allgather_rows(W, world)
        lens = gd.allgather_rows(lens.view(-1, 1), world).view(-1)
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
        if rank != 0:
            return None
    W, lens = W.cpu().numpy(), lens.cpu().numpy()
    if args.walks.endswith(".npy"):
        lab = g.export_csr()["labels"]
        np.save(args.walks, np.where(W >= 0, lab[np.maximum(W, 0)], -1))
    else:
        io.save_walks(g, args.walks, W, lens)
    return nwalks


def main(argv=None):
    args = parse_args(argv)
    t0 = time.time()
    from . import io
    if args.mode == "replay":
        from . import node2vec
        random.seed(args.seed)
        np.random.seed(args.seed)
        nx_G = read_graph(args)
        G = node2vec.Graph(nx_G, args.directed, args.p, args.q, device=args.device)
        G.preprocess_transition_probs()
        walks = G.simulate_walks(args.num_walks, args.walk_length)
        if args.walks.endswith(".npy"):
            W = np.full((len(walks), args.walk_length), -1, np.int64)
            for i, w in enumerate(walks):
                W[i, :len(w)] = w
            np.save(args.walks, W)
        else:
            io.save_list(walks, args.walks)
        nwalks = len(walks)
    else:
        nwalks = _scale(args)
        if nwalks is None:  # not rank 0
            return 0
    print(f"{nwalks} walks -> {args.walks} in {time.time() - t0:.2f}s", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
