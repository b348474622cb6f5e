"""The data-parallel gradient all-reduce of the C-ABI (kanode_comm_*, include/kanode.h) from Python.

Python drivers normally all-reduce with torch.distributed (kanode.Trainer, bench.py); this wrapper is the
path a Julia / C host takes through libkanode.so alone, exposed here so the GPU tests
drive it: rank 0 makes the 128-byte unique id, the host hands it to every rank, every rank joins with
its rank and device, then `allreduce_sum_` sums a device tensor over the ranks in place on a stream.
"""
import ctypes as C

import torch

from . import _lib as L


def unique_id() -> bytes:
    buf = (C.c_uint8 * L.COMM_ID_BYTES)()
    _check(L.lib().kanode_comm_unique_id(buf), None, "kanode_comm_unique_id")
    return bytes(buf)


def _check(status, comm, what):
    if status != 0:
        msg = L.lib().kanode_comm_last_error(comm)
        raise L.KanodeError(f"{what} failed (status {status}): {msg.decode() if msg else ''}")


class Comm:
    """One RCCL communicator per process (kanode_comm_create); `close()` or garbage collection frees it."""

    def __init__(self, nranks: int, rank: int, uid: bytes, device: int = 0):
        if len(uid) != L.COMM_ID_BYTES:
            raise ValueError(f"the unique id is {L.COMM_ID_BYTES} bytes, got {len(uid)}")
        buf = (C.c_uint8 * L.COMM_ID_BYTES).from_buffer_copy(uid)
        out = C.c_void_p()
        _check(L.lib().kanode_comm_create(int(nranks), int(rank), buf, int(device), C.byref(out)), None,
               "kanode_comm_create")
        self._c = out
        self.size = int(L.lib().kanode_comm_size(self._c))
        self.rank = int(L.lib().kanode_comm_rank(self._c))

    def allreduce_sum_(self, x: torch.Tensor, stream=None) -> torch.Tensor:
        """x (device, contiguous, f32/f64) <- Σ over the ranks, stream-ordered on `stream` (default: torch's
        current stream)."""
        if not (x.is_cuda and x.is_contiguous()) or x.dtype not in (torch.float32, torch.float64):
            raise ValueError("allreduce_sum_ takes a contiguous float32/float64 device tensor")
        st = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
        dt = 1 if x.dtype == torch.float64 else 0
        _check(L.lib().kanode_comm_allreduce_sum(self._c, C.c_void_p(x.data_ptr()), x.numel(), dt, C.c_void_p(st)),
               self._c, "kanode_comm_allreduce_sum")
        return x

    def close(self):
        if getattr(self, "_c", None):
            L.lib().kanode_comm_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
