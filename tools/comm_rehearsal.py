"""Rehearse gw_comm with N processes (default 2), one per visible GPU (RCCL
refuses two ranks on one GPU: "invalid usage", so N > 1 needs N GPUs).  Rank 0 creates the id and
passes it through a pipe; every rank gathers a block of int32 "walks" that
encodes its rank and checks the concatenation.

    python tools/comm_rehearsal.py [N]
"""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-embedding_amd"))


def rank_main(uid, n, r, q):
    try:
        q.put(_rank(uid, n, r))
    except Exception as e:  # report, do not leave the parent waiting
        q.put((r, False, str(e)))


def _rank(uid, n, r):
    import torch
    from gwamd import dist
    dev = r % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    c = dist.NativeComm(uid, n, r, dev)
    blk = 1 << 20
    send = torch.full((blk,), r, dtype=torch.int32, device="cuda") + torch.arange(blk, dtype=torch.int32,
                                                                                  device="cuda") * n
    recv = torch.empty(n * blk, dtype=torch.int32, device="cuda")
    c.allgather(send, recv, torch.cuda.current_stream())
    torch.cuda.synchronize()
    want = torch.cat([torch.full((blk,), k, dtype=torch.int32, device="cuda") +
                      torch.arange(blk, dtype=torch.int32, device="cuda") * n for k in range(n)])
    ok = bool(torch.equal(recv, want))
    c.close()
    return (r, ok, "")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from gwamd import dist
    uid = dist.NativeComm.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(uid, n, r, q)) for r in range(n)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(n))
    for p in ps:
        p.join(30)
    print("ranks", res)
    sys.exit(0 if all(ok for _, ok, _ in res) else 1)


if __name__ == "__main__":
    main()
