"""Data-parallel sharding over GPUs (one process per GPU, torch.distributed).

The graph is replicated on every rank (RMAT-24 CSR ~8.5 GB of 288 GB HBM).
Units are independent:

* node2vec: global walk index w in [0, num_walks * n); walk w is a pure
  function of (seed, w) (Philox keyed), so a rank computes any contiguous
  block with no communication and the concatenation over ranks is identical
  to a single-GPU run.
* TopSim: query sources; each source's row depends only on (seed, source).

The only exchange step is optional: an all-gather of the emitted walks
(north_star: RCCL all-gather over xGMI), for consumers that need every walk
on every rank.  With backend "nccl" (= RCCL on ROCm) the tensors live in HBM;
the same code runs on "gloo" for CPU tests.
"""
import torch
import torch.distributed as dist


def shard_range(total, world, rank):
    """Contiguous block [begin, begin+count) of `total` units for `rank`
    (strong scaling: blocks differ by at most one unit)."""
    base, rem = divmod(int(total), int(world))
    begin = rank * base + min(rank, rem)
    count = base + (1 if rank < rem else 0)
    return begin, count


def weak_block(step, world, rank, block):
    """First global unit of (step, rank) when every rank processes `block`
    units per step (weak scaling): steps never overlap across ranks."""
    return (int(step) * int(world) + int(rank)) * int(block)


def allgather_rows(local, world, group=None):
    """All-gather row blocks of possibly different lengths (strong-scaling
    shards differ by one row): pads to the longest block, gathers with one
    collective, strips the padding.  Returns the concatenation in rank
    order."""
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    if local.shape[0] < mx:
        pad = torch.full((mx - local.shape[0],) + tuple(local.shape[1:]), -1, dtype=local.dtype,
                         device=local.device)
        local = torch.cat([local, pad])
    out = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if hasattr(dist, "all_gather_into_tensor") and local.device.type == "cuda":
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    else:
        chunks = list(out.chunk(world))
        dist.all_gather(chunks, local.contiguous(), group=group)
    parts = [out[r * mx:r * mx + sizes[r]] for r in range(world)]
    return torch.cat(parts)


class NativeComm:
    """The C ABI's RCCL communicator (include/graphwalk.h gw_comm_*): the same
    all-gather for hosts that do not run torch.distributed (JNI, C++ drivers).
    Rank 0 creates the id with NativeComm.unique_id() and distributes it."""

    def __init__(self, uid, nranks, rank, device):
        import ctypes
        from . import _lib as C
        self._C = C
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
        h = ctypes.c_void_p()
        rc = C.lib().gw_comm_init(ctypes.cast(buf, ctypes.c_void_p), nranks, rank, device, ctypes.byref(h))
        if rc != C.GW_OK:
            raise C.DeviceError(rc, C.lib().gw_comm_last_error(None).decode(errors="replace"))
        self.handle, self.nranks, self.rank = h, nranks, rank

    @staticmethod
    def unique_id():
        import ctypes
        from . import _lib as C
        buf = (ctypes.c_uint8 * 128)()
        rc = C.lib().gw_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p))
        if rc != C.GW_OK:
            raise C.DeviceError(rc, C.lib().gw_comm_last_error(None).decode(errors="replace"))
        return bytes(buf)

    def allgather(self, send, recv, stream=None):
        """recv[nranks * n] = every rank's send[n] in rank order (int32 or float64 CUDA tensors)."""
        C = self._C
        dt = {torch.int32: 0, torch.float64: 1}[send.dtype]
        assert recv.dtype == send.dtype and recv.numel() == self.nranks * send.numel()
        st = None if stream is None else C.ctypes.c_void_p(stream.cuda_stream)
        rc = C.lib().gw_comm_allgather(self.handle, C.ptr(send), C.ptr(recv), send.numel(), dt, st)
        if rc != C.GW_OK:
            raise C.DeviceError(rc, C.lib().gw_comm_last_error(self.handle).decode(errors="replace"))

    def close(self):
        if self.handle:
            self._C.lib().gw_comm_free(self.handle)
            self.handle = None
