"""Halo-exchange transports for the native slab solver.

Reference: two blocking ``MPI_Sendrecv`` per step over host-staged (or
CUDA-aware) buffers (fortran/hip/heat.F90:196-230, fortran/mpi+cuda/heat.F90:143-195).
Here a transport is a native object the solver calls once per cycle:

* :class:`SelfTransport`  — one rank, no exchange.
* :class:`RcclTransport`  — RCCL over xGMI, zero-copy rows, grouped send/recv on the
  solver's comm stream (device-direct; the production path, one process or one
  host thread per GPU). The 128-byte ``ncclUniqueId`` is created by rank 0 and
  broadcast through ``torch.distributed`` (any backend) or passed explicitly.
* :class:`RcclLoopTransport` — 1-rank periodic self-exchange: perf rehearsal of the
  multi-GPU schedule on one GPU.
* :class:`TorchDistTransport` — host callbacks over ``torch.distributed`` point-to-point
  (gloo on CPU): runs the *same native schedule* in CPU-only multi-process CI.
* :class:`CallbackTransport` — any Python callables (tests, custom fabrics).
* :class:`IpcTransport` — process per GPU WITHOUT RCCL: the neighbours' fields are
  mapped once through hipIpc handles and halos are pulled by device copies on the
  solver's exchange stream, ordered by stream-side counters in host-shared memory
  (csrc/runtime/ipc_transport.cpp, kernels/ipc_sync.hip); capturable into hipGraphs.
  Host collectives over ``torch.distributed`` (gloo), so several processes may
  share one GPU (``bench.py --transport peer --share-gpu``).
"""
from __future__ import annotations

import ctypes as C
import traceback
from typing import Callable, Optional

import numpy as np

from ..ops import _native as N


class Transport:
    """Owns a native transport handle."""

    def __init__(self, handle, rank: int, size: int, name: str):
        self._h = handle
        self.rank = rank
        self.size = size
        self.name = name

    @property
    def handle(self):
        return self._h

    def abort(self, reason: str = "aborted by the caller") -> None:
        """Fail fast (RCCL: ncclCommAbort): blocked exchanges return and the
        solver's next synchronisation raises ``reason``."""
        N.call("heat2d_transport_abort", self._h, reason.encode())

    def close(self) -> None:
        if self._h:
            N.call("heat2d_transport_free", self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


class SelfTransport(Transport):
    def __init__(self):
        h = C.c_void_p()
        N.call("heat2d_transport_self", C.byref(h))
        super().__init__(h, 0, 1, "self")


class RcclTransport(Transport):
    """RCCL communicator created from an ncclUniqueId (collective over all ranks).

    A watchdog thread aborts the communicator when outstanding exchanges stop
    completing for ``$HEAT2D_COMM_TIMEOUT`` seconds (default 600, 0 = off) or
    RCCL reports an async error; the rank then raises instead of hanging."""

    def __init__(self, rank: int, size: int, device: int, uid: Optional[bytes] = None, group=None):
        if uid is None:
            uid = broadcast_unique_id(rank, group)
        buf = (C.c_ubyte * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        N.call("heat2d_transport_rccl", buf, rank, size, device, C.byref(h))
        super().__init__(h, rank, size, "rccl")


class RcclLoopTransport(Transport):
    """1-rank RCCL communicator exchanging the slab's boundary rows with ITSELF
    (periodic wrap): rehearses the multi-GPU schedule — boundary bands and RCCL
    send/recv kernels on the comm stream beside a CU-masked interior — on one
    GPU, with the same message sizes. Performance only: it overwrites the
    Dirichlet frame rows, so the physics is not the problem's."""

    def __init__(self, device: int):
        h = C.c_void_p()
        N.call("heat2d_transport_rccl_loop", device, C.byref(h))
        super().__init__(h, 0, 1, "rccl-loop")


def broadcast_unique_id(rank: int, group=None) -> bytes:
    """Rank 0 creates the RCCL unique id; everyone receives it via torch.distributed."""
    import torch
    import torch.distributed as dist
    t = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        t.copy_(torch.frombuffer(bytearray(N.rccl_unique_id()), dtype=torch.uint8))
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        td = t.to(dev)
        dist.broadcast(td, src=0, group=group)
        t = td.cpu()
    else:
        dist.broadcast(t, src=0, group=group)
    return bytes(t.numpy().tobytes())


_NP_DTYPES = {N.F32: np.float32, N.F64: np.float64}


class CallbackTransport(Transport):
    """Transport driven by Python callables on host buffers.

    exchange(send_lo, send_hi, recv_lo, recv_hi) receives numpy arrays (or None at the
    domain ends) of ``k*ncols`` elements; allreduce(vals, op) gets a float64 numpy array
    to reduce in place (op 0 sum, 1 max, 2 min); barrier() blocks.
    """

    def __init__(self, rank: int, size: int, exchange: Callable, allreduce: Callable, barrier: Callable,
                 name: str = "callback"):
        self._py = (exchange, allreduce, barrier)

        def _arr(ptr, count, dtype):
            if not ptr:
                return None
            ct = C.c_float if dtype == N.F32 else C.c_double
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(count,))

        def ex(ctx, s_lo, s_hi, r_lo, r_hi, count, dtype):
            try:
                exchange(_arr(s_lo, count, dtype), _arr(s_hi, count, dtype), _arr(r_lo, count, dtype),
                         _arr(r_hi, count, dtype))
                return 0
            except Exception:
                traceback.print_exc()
                return 1

        def ar(ctx, vals, n, op):
            try:
                allreduce(np.ctypeslib.as_array(vals, shape=(n,)), int(op))
                return 0
            except Exception:
                traceback.print_exc()
                return 1

        def br(ctx):
            try:
                barrier()
                return 0
            except Exception:
                traceback.print_exc()
                return 1

        # keep the CFUNCTYPE objects alive as long as the native transport exists
        self._cbs = (N.EXCHANGE_FN(ex), N.ALLREDUCE_FN(ar), N.BARRIER_FN(br))
        h = C.c_void_p()
        N.call("heat2d_transport_callback", self._cbs[0], self._cbs[1], self._cbs[2], None, rank, size,
               C.byref(h))
        super().__init__(h, rank, size, name)


class TorchDistTransport(CallbackTransport):
    """Host-side halo exchange over torch.distributed point-to-point (gloo)."""

    TAG_DOWN, TAG_UP = 11, 12

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        self._group = group

        def exchange(s_lo, s_hi, r_lo, r_hi):
            ops = []
            if s_lo is not None:  # my first rows -> rank-1 (its high ghost rows)
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(s_lo), rank - 1, group, self.TAG_DOWN))
            if r_hi is not None:
                ops.append(dist.P2POp(dist.irecv, torch.from_numpy(r_hi), rank + 1, group, self.TAG_DOWN))
            if s_hi is not None:  # my last rows -> rank+1 (its low ghost rows)
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(s_hi), rank + 1, group, self.TAG_UP))
            if r_lo is not None:
                ops.append(dist.P2POp(dist.irecv, torch.from_numpy(r_lo), rank - 1, group, self.TAG_UP))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()

        def allreduce(vals, op):
            t = torch.from_numpy(vals)
            rop = {0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MAX, 2: dist.ReduceOp.MIN}[op]
            dist.all_reduce(t, op=rop, group=group)

        def barrier():
            dist.barrier(group=group)

        super().__init__(rank, size, exchange, allreduce, barrier, name="torch-dist")


def _dist_ops(group):
    """allgather(bytes) / allreduce(doubles) / barrier over torch.distributed as
    native callbacks (CPU tensors on gloo, device tensors on nccl)."""
    import torch
    import torch.distributed as dist
    size = dist.get_world_size(group)
    dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
           else torch.device("cpu"))

    def ag(ctx, mine, out, nbytes):
        try:
            t = torch.frombuffer(bytearray(C.string_at(mine, nbytes)), dtype=torch.uint8).to(dev)
            outs = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(size)]
            dist.all_gather(outs, t, group=group)
            buf = b"".join(bytes(o.cpu().numpy().tobytes()) for o in outs)
            C.memmove(out, buf, len(buf))
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def ar(ctx, vals, n, op):
        try:
            t = torch.from_numpy(np.ctypeslib.as_array(vals, shape=(n,)).copy()).to(dev)
            rop = {0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MAX, 2: dist.ReduceOp.MIN}[int(op)]
            dist.all_reduce(t, op=rop, group=group)
            np.ctypeslib.as_array(vals, shape=(n,))[:] = t.cpu().numpy()
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def br(ctx):
        try:
            dist.barrier(group=group)
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    return N.ALLGATHER_FN(ag), N.ALLREDUCE_FN(ar), N.BARRIER_FN(br)


class IpcTransport(Transport):
    """Process per GPU (or processes sharing one GPU) without RCCL: halos pulled
    out of the neighbours' fields through hipIpc mappings, ordered on the
    stream by counters in host-shared memory (no host wait per cycle), and
    capturable into hipGraphs. The fields are mapped when the solver is built
    (Transport.attach, collective). Host collectives: ``torch.distributed``."""

    def __init__(self, device: int, group=None):
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        self._cbs = _dist_ops(group)  # keep the CFUNCTYPE objects alive
        h = C.c_void_p()
        N.call("heat2d_transport_ipc", self._cbs[0], self._cbs[1], self._cbs[2], None, rank, size, device,
               C.byref(h))
        super().__init__(h, rank, size, "ipc")


class IpcLoopTransport(Transport):
    """1-rank IPC transport exchanging the slab's boundary rows with itself
    (periodic wrap): one rank's IPC cycle — counter kernels, two pulls, graph
    capture — rehearsed on one GPU (like :class:`RcclLoopTransport`).
    Performance only: it overwrites the Dirichlet frame rows."""

    def __init__(self, device: int):
        h = C.c_void_p()
        N.call("heat2d_transport_ipc_loop", device, C.byref(h))
        super().__init__(h, 0, 1, "ipc-loop")


def default_transport(backend: str, device: Optional[int] = None) -> Transport:
    """Pick the transport for the current process: self if not distributed, RCCL for
    device fields, torch.distributed host callbacks for CPU fields."""
    try:
        import torch.distributed as dist
        distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    except Exception:  # pragma: no cover
        distributed = False
    if not distributed:
        return SelfTransport()
    import torch.distributed as dist
    rank, size = dist.get_rank(), dist.get_world_size()
    if backend == "hip":
        import torch
        dev = torch.cuda.current_device() if device is None else device
        return RcclTransport(rank, size, dev)
    return TorchDistTransport()
