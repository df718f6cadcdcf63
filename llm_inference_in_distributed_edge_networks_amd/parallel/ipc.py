"""Peer-copy transport for boundary messages: the sender copies straight into the receiver's memory.

The RCCL alternative SURVEY §5.8 asks to compare against (``hipMemcpyPeerAsync`` over xGMI / IPC).  Every
receiving stage allocates a ring of ``slots`` receive buffers once and hands their IPC handles to its upstream
neighbour (``torch.multiprocessing`` CUDA IPC = hipIpcGetMemHandle on dmabuf; /dev/shm mappings for CPU tensors).
A message then moves as

  sender   : [wait credit for the slot's previous message] -> copy into the peer's slot (copy engine over xGMI,
             no CUs, stream-ordered) -> flag (seq, bytes) via the process group
  receiver : flag -> local copy out of the slot into the stage's buffer -> credit back

so RCCL (or gloo) carries only 16-byte flags.  Slot reuse: message m goes into slot m % slots, which held message
m - slots.  With RCCL the receiver posts its receive for flag m' only after it enqueued the copy-out of message
m' - RECV_AHEAD (RCCL's stream waits for that), so the completion of the send of flag m - slots + RECV_AHEAD proves
the slot is free: the
sender's stream waits for it (``Work.wait``, no host blocking) - no backward messages, which would serialize
against the flags on RCCL's one stream per peer pair and deadlock.  With gloo (CPU runs, the one-GPU rehearsal,
asynchronous host-side sends) the receiver returns explicit credits instead, and the copies are synchronized on the
host before a flag or credit goes out.  A message larger than the
slot capacity falls back to a plain process-group send/recv (both sides decide the same way from the byte count).
"""
from __future__ import annotations

import os
import uuid

import torch
import torch.distributed as dist

DEFAULT_CAPACITY = int(os.environ.get("EDGE_IPC_SLOT_BYTES", str(64 << 20)))
DEFAULT_SLOTS = 8
# receives a stage posts ahead of consuming (boundary message + aggregate carry, each with a checked-transport
# fingerprint): the completion of flag m proves the copy-out of message m - RECV_AHEAD
RECV_AHEAD = 4


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _bytes_view(t: torch.Tensor) -> torch.Tensor:
    return t.view(-1).view(torch.uint8) if t.numel() else t.view(torch.uint8)


class _Done:
    def wait(self):
        pass


class _Work:
    def __init__(self, works, keep=None):
        self.works, self.keep = works, keep

    def wait(self):
        for w in self.works:
            w.wait()


class _IpcRecv:
    def __init__(self, tr, peer, t, seq, flag, work):
        self.tr, self.peer, self.t, self.seq, self.flag, self.work = tr, peer, t, seq, flag, work

    def wait(self):
        self.work.wait()
        tr = self.tr
        n = _nbytes(self.t)
        if not tr.nccl:
            seq, nb = int(self.flag[0]), int(self.flag[1])
            if seq != self.seq or nb != n:
                raise RuntimeError(f"ipc transport: expected message {self.seq} ({n} B) from rank {self.peer}, "
                                   f"got {seq} ({nb} B)")
        slot = tr.rx_slots[self.peer][self.seq % tr.slots]
        _bytes_view(self.t).copy_(slot[:n], non_blocking=True)
        if not tr.nccl:
            tr._credit(self.peer, self.seq)


class IpcP2P:
    """Transport with the ``send(t, peer)`` / ``recv(t, peer)`` interface of ``TorchP2P`` / ``RcclComm``.

    ``setup(prev, next)`` is collective over all ranks (every rank calls it once, with its pipeline neighbours)."""

    def __init__(self, device: torch.device, slots: int = DEFAULT_SLOTS, capacity: int = DEFAULT_CAPACITY):
        if slots <= RECV_AHEAD:
            raise ValueError(f"ipc transport needs more than {RECV_AHEAD} slots")
        self.device, self.slots, self.capacity = torch.device(device), slots, capacity
        self.nccl = dist.get_backend() == "nccl"
        self.sig_dev = self.device if self.nccl else torch.device("cpu")
        self.rx_slots: dict = {}     # peer -> my receive slots (written by that peer)
        self.tx_slots: dict = {}     # peer -> that peer's receive slots, mapped here
        self.tx_seq: dict = {}       # messages sent to a peer
        self.cred_seen: dict = {}    # credits received from it (= messages it has copied out of its slots)
        self.rx_seq: dict = {}
        self._credits: dict = {}     # peer -> pending credit sends (gloo; kept alive)
        self._flags: dict = {}       # peer -> {seq: flag send work} (RCCL: slot-free proof)
        self._files: list = []

    # ---- setup -----------------------------------------------------------------------------------------------
    def _alloc_slots(self):
        if self.device.type == "cuda":
            from torch.multiprocessing.reductions import reduce_tensor
            bufs = [torch.empty(self.capacity, dtype=torch.uint8, device=self.device) for _ in range(self.slots)]
            return bufs, [("cuda", reduce_tensor(b)) for b in bufs]
        tag = uuid.uuid4().hex[:12]
        bufs, descs = [], []
        for i in range(self.slots):
            path = f"/dev/shm/edge_ipc_{os.getpid()}_{tag}_{i}"
            bufs.append(torch.from_file(path, shared=True, size=self.capacity, dtype=torch.uint8))
            self._files.append(path)
            descs.append(("file", path))
        return bufs, descs

    @staticmethod
    def _open(desc, capacity):
        kind, payload = desc
        if kind == "cuda":
            fn, args = payload
            return fn(*args)
        return torch.from_file(payload, shared=True, size=capacity, dtype=torch.uint8)

    def setup(self, rank: int, prev: int | None, next_: int | None):
        """Allocate this rank's receive ring for ``prev`` and map ``next_``'s ring (all ranks call this)."""
        desc = None
        if prev is not None:
            bufs, desc = self._alloc_slots()
            self.rx_slots[prev] = bufs
            self.rx_seq[prev] = 0
        gathered = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, (prev, desc))
        if next_ is not None:
            nprev, ndesc = gathered[next_]
            if nprev != rank or ndesc is None:
                raise RuntimeError(f"ipc transport: rank {next_} does not receive from rank {rank}")
            self.tx_slots[next_] = [self._open(d, self.capacity) for d in ndesc]
            self.tx_seq[next_] = 0
            self.cred_seen[next_] = 0
        dist.barrier()

    # ---- data path ---------------------------------------------------------------------------------------------
    def _sig(self, seq, nbytes):
        return torch.tensor([seq, nbytes], dtype=torch.int64, device=self.sig_dev)

    def send(self, t: torch.Tensor, peer: int):
        n = _nbytes(t)
        if n > self.capacity:          # oversized: plain process-group send (the receiver takes the same branch)
            return dist.isend(t if (self.nccl or not t.is_cuda) else t.cpu(), peer)
        seq = self.tx_seq[peer]
        self.tx_seq[peer] = seq + 1
        flags = self._flags.setdefault(peer, {})
        if self.nccl:
            # its completion: the receiver copied message seq - slots out of the slot
            w = flags.pop(seq - self.slots + RECV_AHEAD, None)
            if w is not None:
                w.wait()
        else:
            self._take_credits(peer, seq - self.slots + 1)
        slot = self.tx_slots[peer][seq % self.slots]
        slot[:n].copy_(_bytes_view(t), non_blocking=True)     # peer copy (same device: D2D; CPU: shared memory)
        if t.is_cuda and not self.nccl:
            torch.cuda.current_stream().synchronize()           # gloo flags are host-ordered
        flag = self._sig(seq, n)
        work = dist.isend(flag, peer)
        if self.nccl:
            flags[seq] = work
        return _Work([work], keep=(flag, t))

    def recv(self, t: torch.Tensor, peer: int):
        n = _nbytes(t)
        if n > self.capacity:
            if self.nccl or not t.is_cuda:
                return dist.irecv(t, peer)
            from .rccl import _HostRecv
            h = torch.empty(t.shape, dtype=t.dtype)
            return _HostRecv(dist.irecv(h, peer), h, t)
        seq = self.rx_seq[peer]
        self.rx_seq[peer] = seq + 1
        flag = torch.empty(2, dtype=torch.int64, device=self.sig_dev)
        return _IpcRecv(self, peer, t, seq, flag, dist.irecv(flag, peer))

    def _take_credits(self, peer: int, upto: int):
        """Receive credits until ``upto`` messages are known to be copied out of ``peer``'s slots."""
        while self.cred_seen[peer] < upto:
            credit = torch.empty(2, dtype=torch.int64, device=self.sig_dev)
            dist.irecv(credit, peer).wait()
            self.cred_seen[peer] += 1

    def _credit(self, peer: int, seq: int):
        if self.device.type == "cuda" and not self.nccl:
            torch.cuda.current_stream().synchronize()           # the copy-out is done before the slot is freed
        c = self._sig(seq, 0)
        pend = self._credits.setdefault(peer, [])
        pend.append((dist.isend(c, peer), c))
        while len(pend) > 2 * self.slots:
            w, _ = pend.pop(0)
            w.wait()

    def quiesce(self):
        """gloo: consume every outstanding credit and finish the credit sends (end of an evaluation run: both
        neighbours call it, so no credit is left unmatched).  RCCL: nothing is outstanding but flag sends."""
        if self.nccl:
            for flags in self._flags.values():
                for w in flags.values():
                    w.wait()
                flags.clear()
            return
        for peer in self.tx_seq:
            self._take_credits(peer, self.tx_seq[peer])
        for pend in self._credits.values():
            for w, _ in pend:
                w.wait()
            pend.clear()

    def close(self):
        self.quiesce()
        for p in self._files:
            try:
                os.unlink(p)
            except OSError:
                pass
        self._files.clear()
