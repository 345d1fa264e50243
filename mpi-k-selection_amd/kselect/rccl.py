"""Direct RCCL communicator for the sharded protocol (ctypes over librccl).

Why not ``torch.distributed`` for the per-step collectives: ProcessGroupNCCL
runs every collective on its own internal stream, fenced with events against
the caller's stream.  Each of the five collectives of one selection then costs
two cross-queue hops (~10 us of GPU idle per collective, measured with a
one-rank group: 0.824 vs 0.779 ms per 2^30 select).  Here the collectives are
enqueued with ncclAllReduce / ncclAllGather on the SAME stream as the kth_dist_*
kernels, the way the C driver (apps/kth_cgm.c) does it, so a step's kernel is
followed directly by its collective.

The communicator is created once per DistSelector from a unique id that rank 0
generates and ``torch.distributed`` broadcasts (any backend).  The library is
the librccl that torch itself loaded (torch/lib), so one RCCL copy serves both.
"""
import ctypes
import os

import torch
import torch.distributed as dist

_NCCL_UINT32, _NCCL_UINT64, _NCCL_SUM = 3, 5, 0  # rccl.h: ncclDataType_t, ncclRedOp_t


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_ubyte * 128)]  # NCCL_UNIQUE_ID_BYTES


_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"), "librccl.so.1", "librccl.so"]
    err = None
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            break
        except OSError as e:
            err = e
    else:
        raise RuntimeError(f"librccl not loadable: {err}")
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ci, _UniqueId, ci]
    lib.ncclAllReduce.argtypes = [vp, vp, sz, ci, ci, vp, vp]
    lib.ncclAllGather.argtypes = [vp, vp, sz, ci, vp, vp]
    lib.ncclCommDestroy.argtypes = [vp]
    lib.ncclGetErrorString.argtypes = [ci]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclAllGather", "ncclCommDestroy"):
        getattr(lib, f).restype = ci
    _lib = lib
    return lib


def _check(r, what):
    if r != 0:
        raise RuntimeError(f"{what}: {_lib.ncclGetErrorString(r).decode()} ({r})")


class RcclComm:
    """One RCCL communicator over the ranks of ``group``, bound to ``stream``.

    Collectives are enqueued on ``stream`` (a torch.cuda.Stream) and never
    synchronise the host.  Every rank of ``group`` must construct it together."""

    def __init__(self, device, stream, group=None):
        lib = _load()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.stream = stream
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        obj = [ctypes.string_at(ctypes.addressof(uid), 128) if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group,
                                   device=torch.device("cuda", device) if dist.get_backend(group) == "nccl" else None)
        if len(obj[0]) != 128:
            raise RuntimeError("RCCL unique id: bad broadcast")
        ctypes.memmove(ctypes.addressof(uid), obj[0], 128)
        self._comm = ctypes.c_void_p()
        self._eps = None
        with torch.cuda.device(device):
            _check(lib.ncclCommInitRank(ctypes.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")

    def _s(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def all_reduce_sum_(self, t):
        """In-place uint64 SUM of an int64 tensor (the stats slot)."""
        _check(_lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), _NCCL_UINT64, _NCCL_SUM, self._comm,
                                  self._s()), "ncclAllReduce")

    def all_gather(self, out, inp):
        """out[r * inp.numel() ..] = rank r's inp (int32 / uint32 words)."""
        _check(_lib.ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), _NCCL_UINT32, self._comm,
                                  self._s()), "ncclAllGather")

    def entry_points(self):
        """(communicator, ncclAllReduce, ncclAllGather) addresses of the RCCL copy
        this communicator came from (kth_dist_select_rccl calls through them)."""
        if self._eps is None or self._eps[0] != self._comm.value:
            self._eps = (self._comm.value, ctypes.cast(_lib.ncclAllReduce, ctypes.c_void_p).value,
                         ctypes.cast(_lib.ncclAllGather, ctypes.c_void_p).value)
        return self._eps

    def close(self):
        if self._comm:
            _lib.ncclCommDestroy(self._comm)
            self._comm = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass


class HostComm:
    """The two collectives of device tensors staged through host memory over a
    CPU process group (gloo): device -> host copy (which waits for the stream's
    work so far), the collective on host tensors, host -> device copy.  The
    host waits at every collective; this is the transport of ranks that share
    one GPU (bench.py / tests with KTH_SHARE_GPU=1, where RCCL refuses two ranks
    on one device), the way apps/kth_cgm.c --comm mpi stages through MPI."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)

    def all_reduce_sum_(self, t):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
        t.copy_(h)

    def all_gather(self, out, inp):
        h = inp.cpu()
        o = torch.empty(out.numel(), dtype=out.dtype)
        dist.all_gather_into_tensor(o, h, group=self.group)
        out.copy_(o)

    def close(self):
        pass


class TorchComm:
    """The same two collectives through torch.distributed (gloo tests, fallback)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)

    def all_reduce_sum_(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def all_gather(self, out, inp):
        dist.all_gather_into_tensor(out, inp, group=self.group)

    def close(self):
        pass
