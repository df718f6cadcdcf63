"""Pipeline-stage runtime: layer-wise split inference with a quantized boundary.

This is the real version of what the reference simulates in one process
(``QwenPointFiveBModel.activation_quantization``, ``qwen_layer_wise.py:42-76``):
stage ``s`` runs its contiguous layer range, scores the tokens at its last layer,
encodes the hidden state with the boundary codec into one byte message and ships
it to stage ``s+1`` (RCCL ``isend``/``irecv`` over xGMI between GPU processes,
or a direct hand-off when all stages live in one process).  The last stage
computes the per-window NLL of the scored rows.

* ``StageRunner``      - executes one stage for one micro-batch (shared by both runtimes)
* ``LocalPipeline``    - every stage in this process (1 GPU, CPU, tests, sweeps)
* ``DistributedPipeline`` - one stage per rank, ``dp`` replicas of ``pp`` stages; the
  receive for micro-batch i+1 is posted before micro-batch i is computed, so the
  transfer overlaps compute, and consecutive micro-batches keep every stage busy
  (forward-only GPipe fill/drain).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .. import codec as C
from ..eval.windows import PPLAccumulator, WindowBatch, window_nll
from ..importance import ImportanceTracker, canonical
from ..models.model import DecoderLM
from ..utils import trace
from ..utils.graphs import GraphCache, prerun_active
from ..utils.watchdog import from_env as watchdog_from_env
from .dist import Grid, all_reduce_sum
from .plan import PipelinePlan


@dataclass
class BoundaryConfig:
    codec: str = "passthrough"
    ratio: float = 0.0
    method: str = "last_row"
    head_weights: torch.Tensor | None = None
    selection: str = "ratio"      # "ratio": int(ratio*S) least important; "top_rho": keep mass 1 - ratio
    # head-group codecs (rgroup, mixed_rgroup_int8): the relevance pass's channel-group tables of the residual stream
    # entering each layer - {"relevance", "sensitivity"} (codec.wire.load_group_tables) or a plain [layers][H / 64]
    # relevance list - and the average bits per channel; without a table every group gets the same width
    group_relevance: object = None
    group_avg_bits: float = 4.0

    @property
    def spec(self) -> C.CodecSpec:
        return C.get_codec(self.codec)

    def spec_for(self, boundary: int | None, hidden: int) -> C.CodecSpec:
        """The codec of the boundary after layer ``boundary``: with its relevance-allocated group plan for the
        head-group codecs (the tensor crossing it enters layer boundary + 1)."""
        spec = self.spec
        if boundary is None or not C.wire.needs_plan(spec):
            return spec
        G = hidden // C.wire.GROUP
        return C.wire.with_plan(spec, C.wire.boundary_group_plan(self.group_relevance, boundary, G,
                                                                 self.group_avg_bits))

    @property
    def kvar(self) -> bool:
        return C.wire.uses_kvar(self.spec, self.selection)

    def needs_importance(self, S: int) -> bool:
        if self.kvar:
            return self.spec.needs_importance and self.ratio < 1.0
        k = C.wire.num_lo(self.spec, self.ratio, S)
        return self.spec.needs_importance and 0 < k < S


@dataclass
class StageStats:
    tokens: int = 0
    windows: int = 0
    wire_bytes: int = 0          # bytes this stage sent across its outgoing boundary
    wire_tokens: int = 0
    compute_s: float = 0.0
    kvar_bytes: torch.Tensor | None = None   # variable-k messages: payload bytes summed on the device

    @property
    def bytes_per_token(self) -> float:
        b, t = self.totals()
        return b / t if t else 0.0

    def totals(self) -> tuple[float, float]:
        """(bytes sent across the outgoing boundary, tokens they carried) since this runner was created."""
        return self.wire_bytes + (float(self.kvar_bytes) if self.kvar_bytes is not None else 0.0), float(self.wire_tokens)


class StageRunner:
    def __init__(self, model: DecoderLM, plan: PipelinePlan, stage: int, bcfg: BoundaryConfig):
        self.model, self.plan, self.stage, self.bcfg = model, plan, stage, bcfg
        self.layers = plan.stage_layers(stage)
        self.first = stage == 0
        self.last = stage == plan.num_stages - 1
        self.boundary = None if self.last else self.layers[-1]
        self.stats = StageStats()
        self.scored_rows_only = os.environ.get("EDGE_LAST_LAYER_ALL_ROWS", "0") in ("", "0")
        self.rows_only = False
        # LRP head table resident on the stage's device once (no host->device copy inside a captured graph)
        hw = bcfg.head_weights
        self.head_weights = None if hw is None else torch.as_tensor(hw).to(model.device, torch.float32).contiguous()
        H = model.cfg.hidden_size
        self.spec_out = bcfg.spec_for(self.boundary, H)
        self.spec_in = bcfg.spec_for(None if self.first else self.layers[0] - 1, H)

    def _tracker(self, S: int):
        if self.boundary is None or not self.bcfg.needs_importance(S):
            return None
        return ImportanceTracker(self.bcfg.method, [self.boundary], self.model.cfg.num_heads, self.head_weights)

    def carries_state(self) -> bool:
        return canonical(self.bcfg.method) in ("aggregate_till", "maximum_aggregation")

    def run(self, batch: WindowBatch, x: torch.Tensor | None = None, carry: torch.Tensor | None = None):
        """Returns (x_out, importance or None, carry_out or None)."""
        m, B, S = self.model, batch.B, batch.S
        if self.first:
            x = m.embed(batch.ids)
        tr = self._tracker(S)
        if tr is not None and carry is not None:
            tr.load_carry(carry, self.layers[0])
        self.rows_only = False
        for i in self.layers:
            need = tr.stats_for(i) if tr is not None else None
            if self.last and i == m.cfg.num_layers - 1 and need is None and self.scored_rows_only:
                # the model's last layer feeds only the LM head: evaluate it at the scored rows only
                x = m.layer_rows(i, x, B, S, batch.rows, batch.n_rows)
                self.rows_only = True
                continue
            x, st = m.layer(i, x, B, S, stats=need)
            if need is not None:
                tr.observe(i, st, S)
        imp = tr.importance(self.boundary) if tr is not None else None
        return x, imp, (tr.carry() if tr is not None else None)

    def encode(self, x, batch: WindowBatch, imp, out=None):
        msg, L = C.encode(x, self.spec_out, batch.B, batch.S, self.bcfg.ratio, imp, out=out,
                          selection=self.bcfg.selection)
        if L.kvar and not prerun_active():   # compact message payload, summed on the device (capturable, no sync)
            kt = msg[L.off_kvec:L.off_kvec + 4 * L.B].view(torch.int32).sum().to(torch.float64)
            rl, rh = L.row_bytes(L.lo_fmt), L.row_bytes(L.hi_fmt)
            pay = L.off_lo + torch.ceil(kt * rl / 16) * 16 + (L.B * L.S - kt) * rh
            if self.stats.kvar_bytes is None or self.stats.kvar_bytes.device != msg.device:
                self.stats.kvar_bytes = torch.zeros((), dtype=torch.float64, device=msg.device)
            self.stats.kvar_bytes += pay
        return msg, L

    def account(self, batch: WindowBatch) -> None:
        """Wire-byte accounting of the outgoing boundary (outside any captured graph)."""
        if not self.last:
            L = self.layout(batch)
            if not L.kvar:
                self.stats.wire_bytes += L.total
            self.stats.wire_tokens += batch.B * batch.S
        self.stats.windows += batch.B
        self.stats.tokens += batch.tokens

    def forward(self, ids, rows, targets, row_window, n_rows, msg_in=None, carry_in=None):
        """Graph-capturable stage step on tensors only.

        Non-last stage -> (msg_out, carry_out or empty); last stage -> per-window NLL [B]."""
        b = WindowBatch(ids, None, rows, targets, row_window, n_rows, None)
        x = None
        if not self.first:
            L = self.layout_in(b)
            x = C.decode(msg_in, self.spec_in, L, self.model.dtype)
        x, imp, c = self.run(b, x, carry_in if (carry_in is not None and carry_in.numel()) else None)
        if self.last:
            return self.finish(x, b)
        msg, _ = self.encode(x, b, imp)
        return msg, (c if c is not None else torch.empty(0, device=msg.device))

    def layout_in(self, batch) -> C.Layout:
        return self.layout(batch, self.spec_in)

    def layout(self, batch: WindowBatch, spec: C.CodecSpec | None = None) -> C.Layout:
        spec = self.spec_out if spec is None else spec
        if self.bcfg.kvar:
            return C.layout(spec, batch.B, batch.S, self.model.cfg.hidden_size, -1, self.model.dtype, kvar=True)
        k = C.wire.num_lo(spec, self.bcfg.ratio, batch.S)
        return C.layout(spec, batch.B, batch.S, self.model.cfg.hidden_size, k, self.model.dtype)

    def finish(self, x, batch: WindowBatch) -> torch.Tensor:
        """Per-window mean NLL [B] (last stage)."""
        rows = batch.rows
        if self.rows_only:           # x already holds just the scored rows, in batch.rows order
            rows = torch.arange(x.shape[0], device=x.device)
        nll = self.model.row_nll(x, rows, batch.targets)
        return window_nll(nll, batch)


class LocalPipeline:
    """All stages in one process.  ``run_batch`` is the split runner of the reference.

    On a GPU the whole multi-stage step (all layers, importance, boundary encode/decode, head) is
    captured into one HIP graph per batch signature (``use_graphs``)."""

    def __init__(self, model: DecoderLM, plan: PipelinePlan, bcfg: BoundaryConfig, use_graphs: bool = True):
        self.model, self.plan, self.bcfg = model, plan, bcfg
        self.stages = [StageRunner(model, plan, s, bcfg) for s in range(plan.num_stages)]
        self.graphs = GraphCache(self._step, enabled=use_graphs and model.device.type == "cuda")

    def set_boundary(self, bcfg: BoundaryConfig) -> None:
        """Switch the boundary codec / importance / ratio (fresh stage runners and byte counters; graphs of the old
        configuration are dropped)."""
        self.bcfg = bcfg
        self.stages = [StageRunner(self.model, self.plan, s, bcfg) for s in range(self.plan.num_stages)]
        self.graphs.clear()

    def _step(self, ids, rows, targets, row_window, n_rows):
        msg = carry = None
        for st in self.stages:
            out = st.forward(ids, rows, targets, row_window, n_rows, msg, carry)
            if st.last:
                return out
            msg, carry = out
        raise AssertionError

    def run_batch(self, batch: WindowBatch) -> torch.Tensor:
        for st in self.stages:
            st.account(batch)
        with trace.range("local/step"):
            return self.graphs(batch.ids, batch.rows, batch.targets, batch.row_window, batch.n_rows)

    def evaluate(self, batches, acc: PPLAccumulator | None = None, on_batch=None) -> PPLAccumulator:
        acc = acc or PPLAccumulator()
        for b in batches:
            b = b.to(self.model.device)
            wn = self.run_batch(b)
            acc.add(wn, b)
            if on_batch:
                on_batch(b, wn)
        return acc

    def wire_bytes_per_token(self) -> list[float]:
        return [s.stats.bytes_per_token for s in self.stages[:-1]]

    def wire_totals(self) -> tuple[float, float]:
        """(bytes, tokens) summed over the boundaries since the last ``set_boundary``: their ratio is the mean
        wire bytes per token per boundary."""
        tot = [s.stats.totals() for s in self.stages[:-1]]
        return sum(b for b, _ in tot), sum(t for _, t in tot)


class DistributedPipeline:
    """One pipeline stage per rank; ``grid.dp`` replicas share the window batches round-robin.

    Construction is COLLECTIVE over the default process group when ``transport`` is ``"rccl"`` (``RcclComm`` draws
    its store namespace with a broadcast from rank 0) or ``"ipc"`` (the slot rings are exchanged): every rank must
    build its pipeline at the same point of the program, as ``bench.py`` and the pipeline driver do."""

    def __init__(self, model: DecoderLM, plan: PipelinePlan, bcfg: BoundaryConfig, grid: Grid, rank: int,
                 use_graphs: bool = True, transport="torch", check: bool | None = None):
        self.model, self.plan, self.bcfg, self.grid, self.rank = model, plan, bcfg, grid, rank
        self.dp_idx, self.stage = grid.coords(rank)
        if plan.num_stages != grid.pp:
            raise ValueError("plan stages != grid pp")
        self.runner = StageRunner(model, plan, self.stage, bcfg)
        self.prev = grid.rank_of(self.dp_idx, self.stage - 1) if self.stage > 0 else None
        self.next = grid.rank_of(self.dp_idx, self.stage + 1) if self.stage < grid.pp - 1 else None
        self.device = model.device
        self.graphs = GraphCache(self._stage_step, enabled=use_graphs and model.device.type == "cuda")
        if not isinstance(transport, str):       # a transport object with send(t, peer) / recv(t, peer)
            self.tr = transport
        elif transport == "rccl":
            from .rccl import RcclComm
            self.tr = RcclComm(rank, grid.world, model.device.index or 0, peers=[self.prev, self.next])
        elif transport == "torch":
            from .rccl import TorchP2P
            self.tr = TorchP2P()
        elif transport == "ipc":
            from .ipc import IpcP2P
            self.tr = IpcP2P(model.device)
            self.tr.setup(rank, self.prev, self.next)
        else:
            raise ValueError(f"unknown transport {transport!r}")
        if check is None:
            check = os.environ.get("EDGE_P2P_CHECK", "0") not in ("", "0")
        if check:
            from .rccl import CheckedTransport
            self.tr = CheckedTransport(self.tr)

    def set_boundary(self, bcfg: BoundaryConfig) -> None:
        """Switch the boundary configuration, keeping the transport (RCCL channels, IPC slot rings) and process
        layout.  Every rank must switch to the same configuration before its next ``evaluate``."""
        self.bcfg = bcfg
        self.runner = StageRunner(self.model, self.plan, self.stage, bcfg)
        self.graphs.clear()

    def _stage_step(self, ids, rows, targets, row_window, n_rows, msg_in=None, carry_in=None):
        return self.runner.forward(ids, rows, targets, row_window, n_rows, msg_in, carry_in)

    def probe_p2p(self, sizes, iters: int = 10, warm: int = 2) -> list[dict]:
        """Time the active transport on every pipeline edge (SURVEY §5.8 p2p latency / bandwidth), before a run:
        per message size, the sender streams ``iters`` messages to its next stage and stops its clock when the
        receiver's acknowledgement (a 4-byte process-group message, after the receiver's stream is synchronised)
        arrives.  ``warm`` untimed messages first (RCCL connects a channel on its first message).  Edges are
        probed in stage order, every replica at once; collective over all ranks.  Returns the sender's rows
        ``{edge, stage, bytes, p2p_us, p2p_GBps}`` (one per size; receivers and the last stage return [])."""
        import torch.distributed as dist
        dev = self.device
        cuda = dev.type == "cuda"
        ctl_dev = dev if (cuda and dist.get_backend() == "nccl") else torch.device("cpu")

        def sync():
            if cuda:
                torch.cuda.synchronize(dev)

        rows = []
        for s in range(self.grid.pp - 1):
            if self.stage not in (s, s + 1):
                continue
            for nbytes in sizes:
                buf = torch.zeros(int(nbytes), dtype=torch.uint8, device=dev)
                ctl = torch.zeros(1, dtype=torch.int32, device=ctl_dev)
                for n, timed in ((warm, False), (iters, True)):
                    if self.stage == s:
                        dist.recv(ctl, self.next)            # the receiver has posted nothing yet: start together
                        sync()
                        t0 = time.perf_counter()
                        hs = [self.tr.send(buf, self.next) for _ in range(n)]
                        for h in hs:
                            h.wait()
                        dist.recv(ctl, self.next)            # acknowledgement: all n arrived
                        sync()
                        dt = time.perf_counter() - t0
                        if timed:
                            rows.append({"edge": [self.rank, self.next], "stage": s, "bytes": int(nbytes),
                                         "p2p_us": round(1e6 * dt / n, 2),
                                         "p2p_GBps": round(n * nbytes / dt / 1e9, 3)})
                    else:
                        dist.send(ctl, self.prev)
                        hs = [self.tr.recv(buf, self.prev) for _ in range(n)]
                        for h in hs:
                            h.wait()
                        sync()
                        dist.send(ctl, self.prev)
                if hasattr(self.tr, "quiesce"):              # IPC: both ends of the edge settle their credits
                    self.tr.quiesce()
        return rows

    def my_batches(self, batches):
        for i, b in enumerate(batches):
            if i % self.grid.dp == self.dp_idx:
                yield b

    def _recv_bufs(self, batch: WindowBatch):
        r = self.runner
        L = r.layout_in(batch)
        msg = torch.empty(L.total, dtype=torch.uint8, device=self.device)
        carry = torch.empty(0, dtype=torch.float32, device=self.device)
        if r.carries_state() and self.bcfg.needs_importance(batch.S):
            carry = torch.empty(batch.B, batch.S, dtype=torch.float32, device=self.device)
        return msg, carry

    def _post_recv(self, batch):
        msg, carry = self._recv_bufs(batch)
        reqs = [self.tr.recv(msg, self.prev)]
        if carry.numel():
            reqs.append(self.tr.recv(carry, self.prev))
        return msg, carry, reqs

    def evaluate(self, batches, timing: bool = False) -> tuple[PPLAccumulator, dict]:
        """Run this rank's share of ``batches`` as one continuous pipeline (no flush between batches).

        Returns the globally reduced accumulator (valid on every rank) and this rank's stage report.  With
        ``timing`` the report carries a GPU-event breakdown of the stage's stream: ``compute_ms`` (stage
        graphs), ``recv_wait_ms`` (stream stalled on the incoming boundary message), ``send_post_ms`` (host
        time posting sends) and ``bubble_frac`` = 1 - compute / wall."""
        mine = [b.to(self.device) for b in self.my_batches(batches)]
        acc_local = torch.zeros(2, dtype=torch.float64, device=self.device)
        wd = watchdog_from_env(f"stage{self.stage}")
        tag = f"stage{self.stage}"
        cuda = self.device.type == "cuda"
        timing = timing and cuda
        evs = []
        send_post = 0.0
        # two graph slots: the boundary message of micro-batch i lives in slot i % 2's static buffer, so the
        # send of i overlaps the compute of i + 1; before slot i % 2 is replayed again (i + 2) the stream waits
        # for the send that still reads it (GPU-side wait, no host sync, no copy of the message)
        in_flight: list = [None, None]
        # EDGE_DUMP_NLL=<prefix>: the last stage saves every micro-batch's per-window NLL (debug: a wrong PPL is then
        # traced to the windows / micro-batches that differ from a reference run)
        dump = [] if (self.next is None and os.environ.get("EDGE_DUMP_NLL")) else None
        recv_next = self._post_recv(mine[0]) if (self.prev is not None and mine) else None
        t0 = time.perf_counter()
        if timing:
            ev_begin = torch.cuda.Event(enable_timing=True)
            ev_begin.record()
        for i, b in enumerate(mine):
            msg_in = carry_in = None
            slot = i & 1
            if wd:
                wd.beat()
            if timing:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            # the send that still reads this slot's message buffer (micro-batch i - 2) must be done before the slot
            # is replayed; waited for before the next receive is posted, so the wait can never cover that receive
            if in_flight[slot] is not None:
                for r in in_flight[slot]:
                    r.wait()
                in_flight[slot] = None
            if self.prev is not None:
                msg_in, carry_in, reqs = recv_next
                with trace.range(f"{tag}/recv_wait"):
                    for r in reqs:
                        r.wait()
                if i + 1 < len(mine):
                    recv_next = self._post_recv(mine[i + 1])  # prefetch: overlap next transfer with compute
            if timing:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
            self.runner.account(b)
            with trace.range(f"{tag}/compute"):
                out = self.graphs(b.ids, b.rows, b.targets, b.row_window, b.n_rows,
                                  *(() if self.prev is None else (msg_in, carry_in)), slot=slot)
            if timing:
                e2 = torch.cuda.Event(enable_timing=True)
                e2.record()
                evs.append((e0, e1, e2))
            if self.next is not None:
                msg, c = out
                trace.counter(f"{tag}/wire_bytes", msg.numel() + 4 * c.numel())
                ts = time.perf_counter()
                with trace.range(f"{tag}/send_post"):
                    reqs = [self.tr.send(msg, self.next)] + ([self.tr.send(c, self.next)] if c.numel() else [])
                send_post += time.perf_counter() - ts
                if self.graphs.enabled:
                    in_flight[slot] = reqs
                else:
                    in_flight[slot] = None
                    self._eager_sends = getattr(self, "_eager_sends", [])
                    self._eager_sends.append(reqs)
                    while len(self._eager_sends) > 2:
                        for r in self._eager_sends.pop(0):
                            r.wait()
            else:
                w = b.weights.to(self.device)
                acc_local[0] += (out.double() * w).sum()
                acc_local[1] += w.sum()
                if dump is not None:
                    dump.append(out.detach().double().clone())
        for reqs in in_flight + getattr(self, "_eager_sends", []):
            for r in reqs or ():
                r.wait()
        self._eager_sends = []
        report = {"stage": self.stage, "dp": self.dp_idx, "layers": [self.runner.layers.start,
                                                                     self.runner.layers.stop - 1]}
        if timing:
            ev_end = torch.cuda.Event(enable_timing=True)
            ev_end.record()
            torch.cuda.synchronize()
            comp = sum(e1.elapsed_time(e2) for _, e1, e2 in evs)
            wait = sum(e0.elapsed_time(e1) for e0, e1, _ in evs)
            wall = ev_begin.elapsed_time(ev_end)
            report.update(compute_ms=round(comp, 3), recv_wait_ms=round(wait, 3), send_post_ms=round(1e3 * send_post, 3),
                          wall_ms=round(wall, 3), bubble_frac=round(max(0.0, 1.0 - comp / wall), 4) if wall else None,
                          microbatches=len(evs))
        if wd:
            wd.stop()
        if dump:
            path = f"{os.environ['EDGE_DUMP_NLL']}.rank{self.rank}.{getattr(self, '_dumps', 0)}.pt"
            self._dumps = getattr(self, "_dumps", 0) + 1
            torch.save(torch.stack([d.cpu() for d in dump]), path)
        self.runner.stats.compute_s += time.perf_counter() - t0
        if hasattr(self.tr, "quiesce"):      # peer-copy transport: no flow-control message left unmatched
            self.tr.quiesce()
        all_reduce_sum(acc_local)
        acc = PPLAccumulator()
        acc.total_nll, acc.n_tokens = float(acc_local[0]), float(acc_local[1])
        report["wire_bytes_per_token"] = self.runner.stats.bytes_per_token
        # this rank's cumulative counters since set_boundary (the last stage sends nothing)
        report["wire_bytes"], report["wire_tokens"] = self.runner.stats.totals() if not self.runner.last else (0.0, 0.0)
        return acc, report

    def close(self) -> None:
        """Release the transport (IPC slot rings and their /dev/shm files, RCCL channels).  Idempotent."""
        tr = getattr(self, "tr", None)
        inner = getattr(tr, "inner", tr)
        if inner is not None and hasattr(inner, "close"):
            inner.close()
        self.tr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
