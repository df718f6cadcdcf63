"""Native RCCL transport for boundary messages (``csrc/comm/rccl_comm.cpp``).

An alternative to ``torch.distributed`` p2p for the stage hand-off: one 2-rank communicator per pipeline edge
(its unique id handed over through the process group's store), each with its own non-blocking HIP stream, and
event-only ordering with the compute stream.  ``send``/``recv`` return handles holding an event recorded right
after that operation; ``wait()`` makes the *current* stream wait for that operation only (no host blocking),
mirroring ``torch.distributed.Work.wait`` for NCCL.  Because a middle stage's receive from ``prev`` and its send
to ``next`` live on different streams, the receive it posts ahead for micro-batch i+1 never delays the send of
micro-batch i.  Buffers are tied to the channel stream with ``record_stream`` so the caching allocator never
recycles them while RCCL still uses them.
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
    """One RCCL operation: an event recorded on its channel's stream right after the operation was enqueued.

    ``wait()`` makes the *current* stream wait (GPU-side) for exactly that operation: a receive's data is
    visible, or a send has finished reading its buffer.  Later operations queued on the same or other channels
    are not waited for."""

    def __init__(self, stream, keep=()):
        self.ev = torch.cuda.Event()
        self.ev.record(stream)
        self.keep = keep

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)

    def query(self) -> bool:
        return self.ev.query()


class _Channel:
    """A communicator over a rank set (a pipeline edge = 2 ranks, or this rank alone for loopback) and its
    own non-blocking HIP stream."""

    def __init__(self, ranks: tuple, me: int, device: int, unique_id: bytes):
        L = lib()
        h = ctypes.c_void_p()
        _ok(L.edge_rccl_init(ctypes.byref(h), len(ranks), unique_id, ranks.index(me), device), "ncclCommInitRank")
        self.h, self.ranks, self.device = h, ranks, device
        self._stream = None

    @property
    def stream(self):
        """The channel's HIP stream as a torch stream (created on first use)."""
        if self._stream is None:
            self._stream = torch.cuda.ExternalStream(lib().edge_rccl_stream(self.h),
                                                     device=torch.device("cuda", self.device))
        return self._stream

    def peer_index(self, peer: int) -> int:
        return self.ranks.index(peer)

    def after_compute(self):
        _ok(lib().edge_rccl_wait_for(self.h, torch.cuda.current_stream().cuda_stream), "wait_for")

    def close(self):
        if self.h:
            lib().edge_rccl_destroy(self.h)
            self.h = None


def channel_key(rank: int, peer: int) -> tuple:
    """The channel an operation between ``rank`` and ``peer`` runs on: one per unordered rank pair.  A pipeline
    stage receives from ``prev`` and sends to ``next`` on two different channels (two streams), so a send never
    queues behind a receive posted ahead of it (and vice versa)."""
    return (min(rank, peer), max(rank, peer))


class RcclComm:
    """Native RCCL transport with one 2-rank communicator and one stream per pipeline edge.

    ``peers``: the ranks this rank exchanges messages with (its pipeline neighbours).  Every edge's unique id is
    created by its lower rank and handed to the other through the process group's key-value store (no
    collective), and the edges are initialised in one global order (sorted rank pairs), so the blocking
    ``ncclCommInitRank`` calls of a chain of stages cannot wait on each other in a cycle.  ``peers=None`` with
    ``world == 1`` is the single-GPU loopback (``sendrecv`` to itself, ``all_reduce_sum_f64``).

    The store keys of one construction live under a namespace rank 0 draws and broadcasts, so keys never depend on
    how many communicators each rank built before; the reader deletes a key once it has the id.  That broadcast
    makes construction with ``world > 1`` a COLLECTIVE over the default process group: every rank must construct its
    ``RcclComm`` at the same point of the program (``DistributedPipeline`` does, at its construction), or the ranks
    hang in the broadcast."""

    def __init__(self, rank: int, world: int, device: int, unique_id: bytes | None = None, peers=None):
        self.rank, self.world, self.device = rank, world, device
        self.channels: dict = {}
        if peers is None:
            if world != 1:
                raise ValueError("RcclComm over several ranks needs its peers (the pipeline neighbours)")
            peers = [rank]
        gen = self._namespace() if world > 1 else ""
        for key in sorted({channel_key(rank, p) for p in peers if p is not None}):
            ranks = tuple(sorted(set(key)))
            if len(ranks) == 1:
                uid = unique_id if unique_id is not None else self.make_unique_id()
            else:
                uid = self._exchange_id(gen, ranks)
            self.channels[key] = _Channel(ranks, rank, device, uid)
        # the loopback/all-reduce channel (world == 1), or the first edge: what ``stream`` / ``h`` refer to
        self.h = next(iter(self.channels.values())).h if self.channels else None

    @property
    def stream(self):
        return next(iter(self.channels.values())).stream

    @staticmethod
    def make_unique_id() -> bytes:
        L = lib()
        buf = ctypes.create_string_buffer(L.edge_rccl_id_bytes())
        _ok(L.edge_rccl_unique_id(buf), "ncclGetUniqueId")
        return buf.raw

    @staticmethod
    def _namespace() -> str:
        import secrets

        from .dist import broadcast_object
        import torch.distributed as dist
        return broadcast_object(secrets.token_hex(8) if dist.get_rank() == 0 else None, src=0)

    def _exchange_id(self, gen: str, ranks: tuple) -> bytes:
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
        k = f"edge_rccl/{gen}/{ranks[0]}-{ranks[1]}"
        if self.rank == ranks[0]:
            uid = self.make_unique_id()
            store.set(k, uid)
            return uid
        uid = bytes(store.get(k))
        try:
            store.delete_key(k)
        except (AttributeError, RuntimeError, NotImplementedError):
            pass
        return uid

    def _channel(self, peer: int) -> _Channel:
        try:
            return self.channels[channel_key(self.rank, peer)]
        except KeyError:
            raise ValueError(f"rank {self.rank} has no RCCL channel to rank {peer}") from None

    def send(self, t: torch.Tensor, peer: int) -> _Handle:
        ch = self._channel(peer)
        ch.after_compute()
        t.record_stream(ch.stream)
        _ok(lib().edge_rccl_send(ch.h, t.data_ptr(), t.numel() * t.element_size(), ch.peer_index(peer)), "ncclSend")
        return _Handle(ch.stream, (t,))

    def recv(self, t: torch.Tensor, peer: int) -> _Handle:
        ch = self._channel(peer)
        ch.after_compute()
        t.record_stream(ch.stream)
        _ok(lib().edge_rccl_recv(ch.h, t.data_ptr(), t.numel() * t.element_size(), ch.peer_index(peer)), "ncclRecv")
        return _Handle(ch.stream, (t,))

    def sendrecv(self, send_t, recv_t, peer):
        """Grouped send+recv with one peer (self-loopback when peer == rank)."""
        L = lib()
        ch = self._channel(peer)
        ch.after_compute()
        send_t.record_stream(ch.stream)
        recv_t.record_stream(ch.stream)
        p = ch.peer_index(peer)
        _ok(L.edge_rccl_group_start(), "group_start")
        _ok(L.edge_rccl_send(ch.h, send_t.data_ptr(), send_t.numel() * send_t.element_size(), p), "send")
        _ok(L.edge_rccl_recv(ch.h, recv_t.data_ptr(), recv_t.numel() * recv_t.element_size(), p), "recv")
        _ok(L.edge_rccl_group_end(), "group_end")
        return _Handle(ch.stream, (send_t, recv_t))

    def all_reduce_sum_f64(self, t: torch.Tensor):
        """In-place sum over the loopback channel's ranks (world == 1 self-test)."""
        assert t.dtype == torch.float64
        ch = self.channels[channel_key(self.rank, self.rank)]
        ch.after_compute()
        _ok(lib().edge_rccl_allreduce_sum_f64(ch.h, t.data_ptr(), t.numel()), "allreduce")
        _Handle(ch.stream).wait()
        return t

    def close(self):
        for ch in self.channels.values():
            ch.close()
        self.channels.clear()
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
