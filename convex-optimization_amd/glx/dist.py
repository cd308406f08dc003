"""Multi-GPU plumbing: one process per GPU, A and b row-sharded, RCCL inside libglx.

The bootstrap (exchanging RCCL's unique id) rides on ``torch.distributed`` with whatever
backend the launcher initialised (gloo is enough); every GPU collective of the solve itself
is issued by libglx on the compute stream (csrc/comm.cpp). ProxGD's row-sharded schedule
(the default where n divides by the world size): a reduce-scatter of the n x l gradient per
A^T r and one grouped all-gather of the new iterate's rows with every rank's partial sums per
trial; otherwise one sum all-reduce of the gradient plus 8-byte all-reduces of squared
residual norms.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import torch

from . import _lib
from ._lib import check, lib


def shard_rows(m: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous row range [r0, r1) of rank ``rank`` (sizes differ by at most one row)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return (m * rank) // world, (m * (rank + 1)) // world


class Comm:
    """An RCCL communicator created from a unique id broadcast over torch.distributed."""

    def __init__(self, handle: ctypes.c_void_p, world: int, rank: int, keep=None):
        self.handle = handle
        self.world = world
        self.rank = rank
        self._keep = keep   # the host transport's ctypes callback must outlive the handle

    @classmethod
    def host_staged(cls, group=None) -> "Comm":
        """A communicator whose all-reduces go through pinned host memory and
        ``torch.distributed.all_reduce`` on ``group`` (gloo). For several ranks on ONE GPU (tests,
        one-GPU rehearsal of the sharded solver): RCCL requires one rank per device."""
        import numpy as np
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)

        def _allreduce(buf, count, dtype, _user):
            try:
                ct = ctypes.c_double if dtype == _lib.GLX_F64 else ctypes.c_float
                arr = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ct)), shape=(int(count),))
                t = torch.from_numpy(arr)   # shares the pinned staging buffer
                dist.all_reduce(t, group=group)
                return 0
            except Exception:   # never unwind through C
                return 1

        cb = _lib.HOST_ALLREDUCE_FN(_allreduce)
        h = ctypes.c_void_p()
        check(lib().glx_comm_create_host(ctypes.byref(h), world, rank, ctypes.cast(cb, ctypes.c_void_p), None))
        return cls(h, world, rank, keep=cb)

    @classmethod
    def from_torch_distributed(cls, group=None) -> "Comm":
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = torch.zeros(_lib.COMM_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            arr = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
            check(lib().glx_comm_unique_id(arr))
            uid.copy_(torch.tensor(list(bytes(arr)), dtype=torch.uint8))
        if dist.get_backend(group) == "nccl":
            dev_uid = uid.cuda()
            dist.broadcast(dev_uid, src=0, group=group)
            uid = dev_uid.cpu()
        else:
            dist.broadcast(uid, src=0, group=group)
        arr = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)(*uid.tolist())
        h = ctypes.c_void_p()
        check(lib().glx_comm_create(ctypes.byref(h), arr, world, rank))
        return cls(h, world, rank)

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum all-reduce of a contiguous float32/float64 device tensor."""
        dt = _lib.GLX_F64 if t.dtype == torch.float64 else _lib.GLX_F32
        stream = ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
        check(lib().glx_comm_allreduce(self.handle, ctypes.c_void_p(t.data_ptr()), t.numel(), dt, stream))
        return t

    def _chunked(self, fn, t: torch.Tensor) -> torch.Tensor:
        if t.numel() % self.world:
            raise ValueError("the tensor must hold world-size equal chunks")
        dt = _lib.GLX_F64 if t.dtype == torch.float64 else _lib.GLX_F32
        stream = ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
        check(fn(self.handle, ctypes.c_void_p(t.data_ptr()), t.numel() // self.world, dt, stream))
        return t

    def reduce_scatter_(self, t: torch.Tensor) -> torch.Tensor:
        """In place over world-size chunks: chunk ``rank`` becomes the sum over ranks of that
        chunk (the other chunks are left undefined)."""
        return self._chunked(lib().glx_comm_reduce_scatter, t)

    def all_gather_(self, t: torch.Tensor) -> torch.Tensor:
        """In place over world-size chunks: chunk ``rank`` is sent, every chunk received."""
        return self._chunked(lib().glx_comm_all_gather, t)

    def progress(self):
        """Thread-safe progress record (glx_comm_progress): collectives issued, completed by the
        host transport (-1 for RCCL), kind of the last one, RCCL's asynchronous error."""
        if not self.handle:
            return {"closed": 1}
        out = (ctypes.c_int64 * 4)()
        check(lib().glx_comm_progress(self.handle, out))
        return {"issued": out[0], "host_done": out[1], "last_kind": out[2], "async_error": out[3]}

    def close(self):
        if self.handle:
            lib().glx_comm_destroy(self.handle)
            self.handle = None
