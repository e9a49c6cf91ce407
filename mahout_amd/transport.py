"""A caller-supplied communicator for SketchTable.comm_init_transport over
torch.distributed (any backend: gloo here, or whatever a Spark / MPI host
offers), staged through host memory.

This is the integration route for hosts that already own the process group
(spark-itemsimilarity executors, an MPI job) and the way the multi-rank logic
(packed merge, delta-log exchange, collective top-k) is exercised with several
processes on ONE GPU, where RCCL refuses to put two ranks on one device.  The
RCCL path (SketchTable.comm_init) stays the data path on an 8-GPU node.
"""
import ctypes

import numpy as np

_hip = None


def _hip_runtime():
    """The HIP runtime already mapped into this process (the one torch and
    libmahout_cms.so share) for the staging copies."""
    global _hip
    if _hip is None:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split()[-1]
                if "libamdhip64.so" in path:
                    lib = ctypes.CDLL(path)
                    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
                    lib.hipMemcpy.restype = ctypes.c_int
                    _hip = lib
                    break
        if _hip is None:
            raise RuntimeError("libamdhip64 is not mapped into this process")
    return _hip


_D2H, _H2D = 2, 1


def _d2h(host, ptr, nbytes):
    if _hip_runtime().hipMemcpy(host.ctypes.data, ptr, nbytes, _D2H) != 0:
        raise RuntimeError("hipMemcpy device->host failed")


def _h2d(ptr, host, nbytes):
    if _hip_runtime().hipMemcpy(ptr, host.ctypes.data, nbytes, _H2D) != 0:
        raise RuntimeError("hipMemcpy host->device failed")


def _host_copy(dst, src, nbytes):
    ctypes.memmove(dst, src, nbytes)


class TorchDistTransport:
    """allreduce / allgather callables for SketchTable.comm_init_transport.

    The library hands device pointers (staged through host memory with
    hipMemcpy); host=True takes host pointers instead (the same collective
    logic without a GPU: tests/test_dist_gloo.py)."""

    def __init__(self, group=None, host=False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.host = host
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.bytes_moved = 0
        self.calls = []

    def allreduce(self, ptr, count):
        import torch
        host = np.empty(count, np.int64)
        self._in(host, ptr, count * 8)
        t = torch.from_numpy(host)
        self.dist.all_reduce(t, group=self.group)  # u64 sums: two's complement gives the same bits
        self._out(ptr, host, count * 8)
        self.bytes_moved += count * 8
        self.calls.append(("allreduce", count * 8))

    def allgather(self, send, recv, nbytes):
        import torch
        host = np.empty(nbytes, np.uint8)
        self._in(host, send, nbytes)
        out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
        self.dist.all_gather(out, torch.from_numpy(host), group=self.group)
        allh = np.ascontiguousarray(torch.cat(out).numpy())
        self._out(recv, allh, nbytes * self.world)
        self.bytes_moved += nbytes * self.world
        self.calls.append(("allgather", nbytes))

    def _in(self, host, ptr, nbytes):
        if self.host:
            _host_copy(host.ctypes.data, ptr, nbytes)
        else:
            _d2h(host, ptr, nbytes)

    def _out(self, ptr, host, nbytes):
        if self.host:
            _host_copy(ptr, host.ctypes.data, nbytes)
        else:
            _h2d(ptr, host, nbytes)

    def attach(self, table):
        table.comm_init_transport(self.rank, self.world, self.allreduce, self.allgather)
        return table
