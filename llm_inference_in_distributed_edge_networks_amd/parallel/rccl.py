"""Native RCCL transport for boundary messages (``csrc/comm/rccl_comm.cpp``).

An alternative to ``torch.distributed`` p2p for the stage hand-off: one communicator over all ranks
(bootstrapped with a unique id broadcast through the default process group), a dedicated
non-blocking HIP comm stream, and event-only ordering with the compute stream.  ``send``/``recv``
return handles whose ``wait()`` makes the *current* stream wait on the GPU (no host blocking),
mirroring ``torch.distributed.Work.wait`` for NCCL.  Buffers are tied to the comm stream with
``record_stream`` so the caching allocator never recycles them while RCCL still uses them.
"""
from __future__ import annotations

import ctypes
import os

import torch

from ..ops._native import LIB_PATH as _KLIB

COMM_LIB_PATH = os.path.join(os.path.dirname(_KLIB), "libedge_comm.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(COMM_LIB_PATH):
            raise RuntimeError(f"{COMM_LIB_PATH} missing: run the build (__graft_entry__.build())")
        L = ctypes.CDLL(COMM_LIB_PATH)
        p, i, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
        sig = {"edge_rccl_id_bytes": [], "edge_rccl_unique_id": [ctypes.c_char_p],
               "edge_rccl_init": [ctypes.POINTER(p), i, ctypes.c_char_p, i, i], "edge_rccl_destroy": [p],
               "edge_rccl_wait_for": [p, p], "edge_rccl_signal_to": [p, p], "edge_rccl_group_start": [],
               "edge_rccl_group_end": [], "edge_rccl_send": [p, p, ll, i], "edge_rccl_recv": [p, p, ll, i],
               "edge_rccl_allreduce_sum_f64": [p, p, ll], "edge_rccl_stream_sync": [p], "edge_rccl_stream": [p]}
        for n, a in sig.items():
            f = getattr(L, n)
            f.argtypes = a
            f.restype = ll if n == "edge_rccl_stream" else i
        _lib = L
    return _lib


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc}; >=1000 is an RCCL ncclResult_t + 1000)")


class _Handle:
    def __init__(self, comm, is_recv):
        self.comm, self.is_recv = comm, is_recv

    def wait(self):
        # the current stream waits (GPU-side) for the comm stream's work so far: a receive's data is visible, or
        # a send has finished reading its buffer (the pipeline reuses graph output buffers after this)
        _ok(lib().edge_rccl_signal_to(self.comm.h, torch.cuda.current_stream().cuda_stream), "signal_to")


class RcclComm:
    def __init__(self, rank: int, world: int, device: int, unique_id: bytes | None = None):
        L = lib()
        if unique_id is None:
            unique_id = self.make_unique_id() if world == 1 else self._bootstrap_id(rank)
        h = ctypes.c_void_p()
        _ok(L.edge_rccl_init(ctypes.byref(h), world, unique_id, rank, device), "ncclCommInitRank")
        self.h, self.rank, self.world = h, rank, world
        self.stream = torch.cuda.ExternalStream(L.edge_rccl_stream(h), device=torch.device("cuda", device))

    @staticmethod
    def make_unique_id() -> bytes:
        L = lib()
        buf = ctypes.create_string_buffer(L.edge_rccl_id_bytes())
        _ok(L.edge_rccl_unique_id(buf), "ncclGetUniqueId")
        return buf.raw

    @staticmethod
    def _bootstrap_id(rank: int) -> bytes:
        from .dist import broadcast_object
        return broadcast_object(RcclComm.make_unique_id() if rank == 0 else None, src=0)

    def _after_compute(self):
        _ok(lib().edge_rccl_wait_for(self.h, torch.cuda.current_stream().cuda_stream), "wait_for")

    def send(self, t: torch.Tensor, peer: int) -> _Handle:
        self._after_compute()
        t.record_stream(self.stream)
        _ok(lib().edge_rccl_send(self.h, t.data_ptr(), t.numel() * t.element_size(), peer), "ncclSend")
        return _Handle(self, False)

    def recv(self, t: torch.Tensor, peer: int) -> _Handle:
        self._after_compute()
        t.record_stream(self.stream)
        _ok(lib().edge_rccl_recv(self.h, t.data_ptr(), t.numel() * t.element_size(), peer), "ncclRecv")
        return _Handle(self, True)

    def sendrecv(self, send_t, recv_t, peer):
        """Grouped send+recv with one peer (self-loopback when peer == rank)."""
        L = lib()
        self._after_compute()
        send_t.record_stream(self.stream)
        recv_t.record_stream(self.stream)
        _ok(L.edge_rccl_group_start(), "group_start")
        _ok(L.edge_rccl_send(self.h, send_t.data_ptr(), send_t.numel() * send_t.element_size(), peer), "send")
        _ok(L.edge_rccl_recv(self.h, recv_t.data_ptr(), recv_t.numel() * recv_t.element_size(), peer), "recv")
        _ok(L.edge_rccl_group_end(), "group_end")
        return _Handle(self, True)

    def all_reduce_sum_f64(self, t: torch.Tensor):
        assert t.dtype == torch.float64
        self._after_compute()
        _ok(lib().edge_rccl_allreduce_sum_f64(self.h, t.data_ptr(), t.numel()), "allreduce")
        _Handle(self, True).wait()
        return t

    def close(self):
        if self.h:
            lib().edge_rccl_destroy(self.h)
            self.h = None


class _HostSend:
    def __init__(self, work, host):
        self.work, self.host = work, host     # keeps the staging buffer alive until the send completes

    def wait(self):
        self.work.wait()


class _HostRecv:
    def __init__(self, work, host, dst):
        self.work, self.host, self.dst = work, host, dst

    def wait(self):
        self.work.wait()
        self.dst.copy_(self.host)


class TorchP2P:
    """The default transport: torch.distributed isend/irecv (RCCL via ProcessGroupNCCL, or gloo).

    CUDA tensors over a gloo group (the EDGE_SHARED_GPU rehearsal) are staged through host memory."""

    @staticmethod
    def _host_staged(t) -> bool:
        import torch.distributed as dist
        return t.is_cuda and dist.get_backend() == "gloo"

    def send(self, t, peer):
        import torch.distributed as dist
        if self._host_staged(t):
            h = t.to("cpu")
            return _HostSend(dist.isend(h, peer), h)
        return dist.isend(t, peer)

    def recv(self, t, peer):
        import torch.distributed as dist
        if self._host_staged(t):
            h = torch.empty(t.shape, dtype=t.dtype)
            return _HostRecv(dist.irecv(h, peer), h, t)
        return dist.irecv(t, peer)


class P2PIntegrityError(RuntimeError):
    """A boundary message arrived corrupted, truncated or out of order (checked transport only)."""


def fingerprint(t: torch.Tensor, seq: int) -> torch.Tensor:
    """[seq, nbytes, sum(b), sum(b * w)] int64 of a tensor's bytes, ``w = 1 + (pos mod 251)``.

    The position weight catches swapped or shifted byte ranges, which a plain byte sum misses."""
    b = t.detach().contiguous().view(-1).view(torch.uint8).to(torch.int64)
    w = torch.arange(b.numel(), device=b.device, dtype=torch.int64).remainder_(251).add_(1)
    head = torch.tensor([seq, b.numel()], dtype=torch.int64, device=b.device)
    return torch.cat([head, b.sum().view(1), (b * w).sum().view(1)])


class _CheckedRecv:
    def __init__(self, tr, t, fp, reqs, seq, peer):
        self.tr, self.t, self.fp, self.reqs, self.seq, self.peer = tr, t, fp, reqs, seq, peer

    def wait(self):
        for r in self.reqs:
            r.wait()
        got = self.fp.cpu().tolist()
        want = fingerprint(self.t, self.seq).cpu().tolist()
        if got != want:
            raise P2PIntegrityError(f"message {self.seq} from rank {self.peer}: sender fingerprint "
                                    f"[seq, bytes, sum, wsum]={got}, received data gives {want}")


class _CheckedSend:
    def __init__(self, reqs):
        self.reqs = reqs

    def wait(self):
        for r in self.reqs:
            r.wait()


class CheckedTransport:
    """Debug wrapper (SURVEY §5.2 "P2P ordering tests with payload checksums"): every message is followed by
    a 32-byte fingerprint carrying a per-peer sequence number; the receiver recomputes it after the
    transfer and raises :class:`P2PIntegrityError` on any mismatch.  Costs a host sync per receive, so it
    is opt-in (``EDGE_P2P_CHECK=1`` or ``DistributedPipeline(..., check=True)``)."""

    def __init__(self, inner):
        self.inner = inner
        self.sent: dict[int, int] = {}
        self.recvd: dict[int, int] = {}

    def send(self, t, peer):
        seq = self.sent.get(peer, 0)
        self.sent[peer] = seq + 1
        fp = fingerprint(t, seq)
        return _CheckedSend([self.inner.send(t, peer), self.inner.send(fp, peer)])

    def recv(self, t, peer):
        seq = self.recvd.get(peer, 0)
        self.recvd[peer] = seq + 1
        fp = torch.empty(4, dtype=torch.int64, device=t.device)
        reqs = [self.inner.recv(t, peer), self.inner.recv(fp, peer)]
        return _CheckedRecv(self, t, fp, reqs, seq, peer)
