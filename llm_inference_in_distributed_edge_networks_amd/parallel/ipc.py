"""Peer-copy transport for boundary messages: the sender copies straight into the receiver's memory.

The RCCL alternative SURVEY §5.8 asks to compare against (``hipMemcpyPeerAsync`` over xGMI / IPC).  Every
receiving stage allocates a ring of ``slots`` receive buffers once and hands their IPC handles to its upstream
neighbour (``torch.multiprocessing`` CUDA IPC = hipIpcGetMemHandle on dmabuf; /dev/shm mappings for CPU tensors).
A message then moves as

  sender   : [wait for the credit of the slot's previous message] -> copy into the peer's slot (copy engine over
             xGMI, no CUs, stream-ordered) -> flag (seq, bytes) via the process group
  receiver : flag -> local copy out of the slot into the stage's buffer -> credit back

so the process group carries only 16-byte flags and credits.  Slot reuse: message m goes into slot m % slots, which
held message m - slots; the sender copies it only after the receiver's credit for m - slots arrived, and the
receiver sends that credit only after its copy-out of m - slots (stream order on RCCL: the credit send waits for
the copy-out on the GPU, and the sender's stream waits for the credit receive before its copy - no host blocking;
host-synchronous on gloo).  Credits travel on their own process group: with RCCL a group is one communicator and one
stream per rank pair, and credits queued on the flags' stream would sit behind receives posted ahead and deadlock.
A completed flag *send* proves nothing about the receiver (RCCL may finish a small send into the peer's FIFO before
the matching receive runs), so it is never used as a slot-free signal.  A message larger than the slot capacity
falls back to a plain process-group send/recv (both sides decide the same way from the byte count).
"""
from __future__ import annotations

import os
import uuid

import torch
import torch.distributed as dist

DEFAULT_CAPACITY = int(os.environ.get("EDGE_IPC_SLOT_BYTES", str(64 << 20)))
DEFAULT_SLOTS = 8
# receives a stage posts ahead of consuming (boundary message + aggregate carry, each with a checked-transport
# fingerprint); the ring needs more slots than that so the sender never waits on a credit the receiver can only
# send after a receive the sender has not fed yet
RECV_AHEAD = 4


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _bytes_view(t: torch.Tensor) -> torch.Tensor:
    return t.view(-1).view(torch.uint8) if t.numel() else t.view(torch.uint8)


class _Done:
    def wait(self):
        pass


class _Work:
    """Idempotent wait: a gloo send's ``wait()`` consumes one completion of its buffer, so waiting the same work
    twice (the pipeline and the transport's own bookkeeping) would block for a completion that never comes."""

    def __init__(self, works, keep=None):
        self.works, self.keep, self.done = works, keep, False

    def wait(self):
        if not self.done:
            for w in self.works:
                w.wait()
            self.done = True


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
        self._credits: dict = {}     # peer -> pending credit sends (kept alive until done)
        self._flags: dict = {}       # peer -> pending flag sends
        self._files: list = []
        self.credit_pg = None        # process group of the credits (set up collectively in ``setup``)

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
        self.credit_pg = dist.new_group(backend="nccl" if self.nccl else "gloo")
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
        self._take_credits(peer, seq - self.slots + 1)       # the slot's previous message was copied out
        slot = self.tx_slots[peer][seq % self.slots]
        slot[:n].copy_(_bytes_view(t), non_blocking=True)     # peer copy (same device: D2D; CPU: shared memory)
        if t.is_cuda and not self.nccl:
            torch.cuda.current_stream().synchronize()           # gloo flags are host-ordered
        flag = self._sig(seq, n)
        work = _Work([dist.isend(flag, peer)], keep=(flag, t))
        pend = self._flags.setdefault(peer, [])
        pend.append(work)
        while len(pend) > 2 * self.slots:
            pend.pop(0).wait()
        return work

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
        """Receive credits until ``upto`` messages are known to be copied out of ``peer``'s slots (RCCL: the
        current stream waits for each credit on the GPU; gloo: the host waits)."""
        while self.cred_seen[peer] < upto:
            credit = torch.empty(2, dtype=torch.int64, device=self.sig_dev)
            dist.irecv(credit, peer, group=self.credit_pg).wait()
            self.cred_seen[peer] += 1

    def _credit(self, peer: int, seq: int):
        if self.device.type == "cuda" and not self.nccl:
            torch.cuda.current_stream().synchronize()           # the copy-out is done before the slot is freed
        c = self._sig(seq, 0)          # RCCL: the credit send is stream-ordered after the copy-out
        pend = self._credits.setdefault(peer, [])
        pend.append(_Work([dist.isend(c, peer, group=self.credit_pg)], keep=c))
        while len(pend) > 2 * self.slots:
            pend.pop(0).wait()

    def quiesce(self):
        """Consume every outstanding credit and finish the flag and credit sends (end of an evaluation run: both
        neighbours call it, so no credit is left unmatched)."""
        for peer in self.tx_seq:
            self._take_credits(peer, self.tx_seq[peer])
        for pend in list(self._credits.values()) + list(self._flags.values()):
            for w in pend:
                w.wait()
            pend.clear()

    def close(self):
        self.quiesce()
        if self.credit_pg is not None:    # the credit group's communicator / streams (one per transport)
            try:
                dist.destroy_process_group(self.credit_pg)
            except (RuntimeError, ValueError):
                pass
            self.credit_pg = None
        for p in self._files:
            try:
                os.unlink(p)
            except OSError:
                pass
        self._files.clear()
