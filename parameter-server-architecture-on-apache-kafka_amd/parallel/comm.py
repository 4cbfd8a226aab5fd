"""Native RCCL communicator for the BSP collectives (csrc/comm/rccl_comm.h).

The reference's push/pull bus is Kafka (WorkerApp.java:60-80, ServerApp.java:46-70);
here the BSP schedules of :mod:`psx.parallel.dist` are RCCL collectives over
xGMI.  torch.distributed spends ~30 us of host time per collective call, which
at a ~100 us round keeps the per-rank loop host-bound, so the hot collectives go
through a communicator driven from C++ (a few us per call).  torch.distributed
stays the control plane: rendezvous, the unique-id exchange through its store,
barriers and the bootstrap broadcast.

``make_comm`` returns None (callers fall back to torch.distributed) on the CPU /
gloo paths, when PSX_NATIVE_RCCL=0, or when no RCCL library is mapped.
"""
from __future__ import annotations

import itertools
import os

import torch
import torch.distributed as dist

from .. import _native

F32, I32, U8 = 0, 1, 2
_seq = itertools.count()


def exchange_unique_id(rank: int, make_id, key: str | None = None) -> bytes:
    """Rank 0's ``make_id()`` bytes, handed to every rank through the c10d store."""
    store = dist.distributed_c10d._get_default_store()
    key = key or f"psx_rccl_uid_{next(_seq)}"
    if rank == 0:
        uid = bytes(make_id())
        store.set(key, uid)
        return uid
    return bytes(store.get(key))


def _dtype(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.int32:
        return I32
    if t.dtype == torch.uint8:
        return U8
    raise TypeError(f"unsupported collective dtype {t.dtype}")


class NativeComm:
    """RCCL communicator on this rank's GPU; collectives take torch tensors and run
    on the caller's current stream, or on the communicator's side stream between
    :meth:`fork` and :meth:`join` (overlap with compute)."""

    def __init__(self, rank: int, world: int, device):
        h = _native.hip()
        self.rank, self.world, self.device = int(rank), int(world), torch.device(device)
        uid = exchange_unique_id(self.rank, h.RcclComm.unique_id)
        self.c = h.RcclComm(uid, self.world, self.rank, self.device.index or 0)
        self.side = self.c.side_stream
        self._cs = None  # cached handle of the compute stream

    # -- streams ---------------------------------------------------------------
    def compute_stream(self) -> int:
        if self._cs is None:
            self._cs = torch.cuda.current_stream(self.device).cuda_stream
        return self._cs

    def refresh_stream(self):
        self._cs = None

    def fork(self):
        self.c.fork(self.compute_stream())

    def join(self):
        self.c.join(self.compute_stream())

    def _s(self, side: bool) -> int:
        return self.side if side else self.compute_stream()

    # -- collectives (sum) -----------------------------------------------------
    def all_reduce(self, t: torch.Tensor, side: bool = False):
        self.c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _dtype(t), self._s(side))

    def reduce(self, t: torch.Tensor, root: int = 0, side: bool = False):
        self.c.reduce(t.data_ptr(), t.data_ptr(), t.numel(), _dtype(t), root, self._s(side))

    def broadcast(self, t: torch.Tensor, root: int = 0, side: bool = False):
        self.c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _dtype(t), root, self._s(side))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, side: bool = False):
        if inp.numel() != out.numel() * self.world:
            raise ValueError("reduce_scatter: input must be world x output")
        self.c.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), _dtype(out), self._s(side))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, side: bool = False):
        """``out`` = concat over ranks of ``inp`` (in place when inp is out's own rank slice)."""
        if out.numel() != inp.numel() * self.world:
            raise ValueError("all_gather: output must be world x input")
        self.c.all_gather(inp.data_ptr(), out.data_ptr(), inp.numel(), _dtype(inp), self._s(side))

    # -- point-to-point (SSP / ASP pushes and pulls) -----------------------------
    def send(self, t: torch.Tensor, peer: int, side: bool = False):
        self.c.send(t.data_ptr(), t.numel(), _dtype(t), int(peer), self._s(side))

    def recv(self, t: torch.Tensor, peer: int, side: bool = False):
        self.c.recv(t.data_ptr(), t.numel(), _dtype(t), int(peer), self._s(side))

    def close(self):
        torch.cuda.current_stream(self.device).synchronize()
        self.c.close()


class IpcNativeComm(NativeComm):
    """Ranks sharing ONE GPU (PSX_GPU_OVERSUBSCRIBE=1, gloo control plane): the
    same-device IPC transport of csrc/comm/ipc_comm.h -- HIP IPC-mapped staging
    buffers, stream-ordered flags -- with NativeComm's interface for the dense
    collectives (all-reduce, reduce, broadcast).  RCCL refuses two ranks on one
    device; this is what lets the multi-rank lanes loop (1 server rank + worker
    ranks) run on a one-GPU box."""

    kind = "ipc"

    def __init__(self, rank: int, world: int, device, max_bytes: int = 1 << 22):
        h = _native.hip()
        self.rank, self.world, self.device = int(rank), int(world), torch.device(device)
        self.c = h.IpcComm(self.world, self.rank, self.device.index or 0, int(max_bytes))
        store = dist.distributed_c10d._get_default_store()
        tag = f"psx_ipc_{next(_seq)}"
        store.set(f"{tag}_{self.rank}", bytes(self.c.handle()))
        self.c.connect([bytes(store.get(f"{tag}_{r}")) for r in range(self.world)])
        dist.barrier()  # every rank mapped every area before the first collective
        self.side = None
        self._cs = None

    def fork(self):  # no side stream: collectives run on the compute stream
        pass

    def join(self):
        pass

    def _s(self, side: bool) -> int:
        return self.compute_stream()

    def reduce_scatter(self, out, inp, side=False):
        raise NotImplementedError("IpcNativeComm carries the dense BSP collectives only")

    all_gather = send = recv = reduce_scatter

    def close(self):
        torch.cuda.current_stream(self.device).synchronize()
        dist.barrier()  # nobody unmaps an area a peer may still read
        self.c.close()


NativeComm.kind = "rccl"


def oversubscribed() -> bool:
    """Every rank on GPU 0 over gloo (psx.parallel.dist.init_from_env)."""
    return os.environ.get("PSX_GPU_OVERSUBSCRIBE") == "1"


def make_comm(rank: int, world: int, device, ipc: bool = False) -> NativeComm | None:
    """The native transport of this rank: RCCL (nccl backend, one rank per GPU), or
    with ``ipc`` and ranks sharing one GPU the IPC transport; None: the caller uses
    torch.distributed."""
    device = torch.device(device)
    if device.type != "cuda" or not dist.is_initialized():
        return None
    if dist.get_backend() != "nccl":
        if ipc and oversubscribed() and os.environ.get("PSX_IPC_COMM", "1") != "0":
            return IpcNativeComm(rank, world, device)
        return None
    if os.environ.get("PSX_NATIVE_RCCL", "1") == "0":
        return None
    if not _native.hip().RcclComm.available():
        return None
    return NativeComm(rank, world, device)
