"""Worker for multi-process pipeline tests (gloo on CPU; same code path as RCCL on GPUs)."""
import json
import os
import sys

import torch
import torch.distributed as dist


def run(rank, world, port, pp, codec, ratio, method, out_path, split):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, build_model
    from llm_inference_in_distributed_edge_networks_amd.parallel import (BoundaryConfig, DistributedPipeline, Grid,
                                                                          PipelinePlan, init_distributed, shutdown)
    env = init_distributed("cpu", timeout_s=120)
    cfg = TINY_QWEN2.replace(num_layers=int(os.environ.get("EDGE_TEST_LAYERS", TINY_QWEN2.num_layers)))
    grid = Grid(world, pp)
    plan = PipelinePlan.from_split_layers(cfg.num_layers, split) if split else PipelinePlan.balanced(cfg, pp, 128)
    _, stage = grid.coords(rank)
    model, _ = build_model(cfg, "cpu", torch.float32, seed=0, layers=plan.stage_layers(stage),
                           with_embed=stage == 0, with_head=stage == pp - 1)
    hw = torch.linspace(-1, 2, cfg.num_layers * cfg.num_heads).view(cfg.num_layers, cfg.num_heads)
    pipe = DistributedPipeline(model, plan, BoundaryConfig(codec, ratio, method, hw), grid, rank,
                               transport=os.environ.get("EDGE_TEST_TRANSPORT", "torch"))
    toks = synthetic_stream(1500, cfg.vocab_size, 2)
    bl = list(batches(toks, sliding_windows(1500, 128, 32), 3))
    acc, info = pipe.evaluate(bl)
    if os.environ.get("EDGE_TEST_TWICE"):          # a second run on the same transport state (sequence numbers go on)
        acc, info = pipe.evaluate(bl)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"ppl": acc.ppl(), "n": acc.n_tokens}, f)
    shutdown()


def run_checked(rank, world, port, out_path, corrupt):
    """Fingerprinted p2p: rank 0 sends 3 messages (the 2nd corrupted in flight if ``corrupt``)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llm_inference_in_distributed_edge_networks_amd.parallel import init_distributed, shutdown
    from llm_inference_in_distributed_edge_networks_amd.parallel.rccl import (CheckedTransport, P2PIntegrityError,
                                                                             TorchP2P)

    class Flip(TorchP2P):  # flips one bit of the 2nd payload after the sender fingerprinted it
        n = 0

        def send(self, t, peer):
            if t.dtype == torch.uint8:
                Flip.n += 1
                if corrupt and Flip.n == 2:
                    t = t.clone()
                    t[77] ^= 4
            return super().send(t, peer)

    init_distributed("cpu", timeout_s=60)
    tr = CheckedTransport(Flip())
    msgs = [torch.randint(0, 256, (1000 + 13 * i,), dtype=torch.uint8, generator=torch.Generator().manual_seed(i))
            for i in range(3)]
    if rank == 0:
        for h in [tr.send(m, 1) for m in msgs]:
            h.wait()
    else:
        res = {"ok": 0, "error": None}
        for m in msgs:
            buf = torch.empty_like(m)
            try:
                tr.recv(buf, 0).wait()
                res["ok"] += int(torch.equal(buf, m))
            except P2PIntegrityError as e:
                res["error"] = str(e)
        with open(out_path, "w") as f:
            json.dump(res, f)
    shutdown()


class LaneP2P:
    """Host model of a stream-ordered transport (the native RCCL layer's semantics on gloo): every operation runs
    on a *lane* - a worker thread executing its lane's operations strictly in posting order, like a HIP stream
    running ncclSend / ncclRecv kernels that block until matched.  ``lanes="per_peer"`` puts each peer on its own
    lane (``RcclComm``: one channel and stream per pipeline edge, ``rccl.channel_key``); ``lanes="single"`` is the
    round-2 layout (every operation on one comm stream)."""

    def __init__(self, rank, lanes, on_recv=None, before_send=None):
        import queue
        import threading
        from llm_inference_in_distributed_edge_networks_amd.parallel.rccl import channel_key
        self.rank, self.lanes, self.on_recv, self.before_send = rank, lanes, on_recv, before_send
        self.key = (lambda peer: channel_key(rank, peer)) if lanes == "per_peer" else (lambda peer: 0)
        self.queues, self.threads, self.sent, self.recvd = {}, [], {}, {}
        self._queue, self._threading = queue, threading

    def _lane(self, peer):
        k = self.key(peer)
        if k not in self.queues:
            q = self._queue.Queue()

            def loop():
                while True:
                    item = q.get()
                    if item is None:
                        return
                    fn, done = item
                    fn()
                    done.set()
            th = self._threading.Thread(target=loop, daemon=True)
            th.start()
            self.queues[k] = q
            self.threads.append(th)
        return self.queues[k]

    def _post(self, peer, fn):
        done = self._threading.Event()
        self._lane(peer).put((fn, done))

        class H:
            def wait(self_inner):
                if not done.wait(60):
                    raise TimeoutError("lane operation did not complete")
        return H()

    def send(self, t, peer):
        seq = self.sent.get(peer, 0)
        self.sent[peer] = seq + 1
        t = t.clone()

        def fn():
            if self.before_send:
                self.before_send(peer, seq)
            dist.send(t, peer)
        return self._post(peer, fn)

    def recv(self, t, peer):
        seq = self.recvd.get(peer, 0)
        self.recvd[peer] = seq + 1

        def fn():
            dist.recv(t, peer)
            if self.on_recv:
                self.on_recv(peer, seq)
        return self._post(peer, fn)

    def close(self):
        for q in self.queues.values():
            q.put(None)


def run_lanes(rank, world, port, lanes, out_path):
    """3 stages; stage 0 holds micro-batch i >= 1 back until the LAST stage has received micro-batch i - 1.  The
    middle stage therefore has to get send(i - 1) out while its receive of micro-batch i (posted ahead) is still
    pending: with one lane for both (``lanes="single"``) this deadlocks, with a lane per edge it completes."""
    import datetime
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, build_model
    from llm_inference_in_distributed_edge_networks_amd.parallel import (BoundaryConfig, DistributedPipeline, Grid,
                                                                          PipelinePlan, init_distributed, shutdown)
    init_distributed("cpu", timeout_s=30)
    store = dist.distributed_c10d._get_default_store()
    cfg = TINY_QWEN2
    grid = Grid(world, 3)
    plan = PipelinePlan.from_split_layers(cfg.num_layers, [0, 2])
    stage = rank
    model, _ = build_model(cfg, "cpu", torch.float32, seed=0, layers=plan.stage_layers(stage),
                           with_embed=stage == 0, with_head=stage == 2)

    def gate(peer, seq):          # stage 0: micro-batch seq waits until the last stage got seq - 1
        if seq >= 1:
            store.wait([f"got/{seq - 1}"], datetime.timedelta(seconds=15))

    def got(peer, seq):
        store.set(f"got/{seq}", "1")

    tr = LaneP2P(rank, lanes, on_recv=got if stage == 2 else None, before_send=gate if stage == 0 else None)
    pipe = DistributedPipeline(model, plan, BoundaryConfig("mixed_int4_int8", 0.5, "regular_importance"), grid,
                               rank, transport=tr)
    toks = synthetic_stream(1500, cfg.vocab_size, 2)
    bl = list(batches(toks, sliding_windows(1500, 128, 32), 3))[:5]
    acc, _ = pipe.evaluate(bl)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"ppl": acc.ppl()}, f)
    tr.close()
    shutdown()


def run_driver(rank, world, port, params, crash_at, out_dir):
    """pipeline_experiment on one rank of a gloo job; crash_at > 0: the job dies (every rank, before its crash_at-th
    evaluate call, so no rank is left inside a collective) after writing its per-rank checkpoints."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llm_inference_in_distributed_edge_networks_amd.config import Params
    from llm_inference_in_distributed_edge_networks_amd.eval import experiments as E
    from llm_inference_in_distributed_edge_networks_amd.parallel import pipeline as P
    from llm_inference_in_distributed_edge_networks_amd.parallel import shutdown
    if crash_at:
        orig, calls = P.DistributedPipeline.evaluate, {"n": 0}

        def flaky(self, *a, **k):
            calls["n"] += 1
            if calls["n"] == crash_at:
                raise KeyboardInterrupt("simulated crash")
            return orig(self, *a, **k)
        P.DistributedPipeline.evaluate = flaky
    try:
        E.pipeline_experiment(Params.from_dict(dict(params, output_dir=out_dir)), "qwen2-0.5b")
    except KeyboardInterrupt:
        pass
    shutdown()


class FakeRcclLib:
    """Stand-in for libedge_comm.so (ctypes): records every call instead of touching RCCL / HIP."""

    def __init__(self, rank):
        self.rank, self.n_ids, self.inits, self.destroyed = rank, 0, [], []

    def edge_rccl_id_bytes(self):
        return 128

    def edge_rccl_unique_id(self, buf):
        self.n_ids += 1
        buf.value = f"uid-made-by-{self.rank}-#{self.n_ids}".encode()
        return 0

    def edge_rccl_init(self, href, nranks, uid, idx, device):
        h = 1000 * self.rank + len(self.inits) + 1
        href._obj.value = h
        self.inits.append({"h": h, "nranks": nranks, "uid": uid.rstrip(b"\0").decode(), "idx": idx, "device": device})
        return 0

    def edge_rccl_destroy(self, h):
        self.destroyed.append(h.value if hasattr(h, "value") else h)
        return 0


def run_rccl_bootstrap(rank, world, port, out_path):
    """RcclComm's store bootstrap on a pp chain 0-1-..-(world-1) with the RCCL library mocked: two constructions in a
    row, every rank reports its namespace, channels (in init order), the ids / comm indices it initialised with, and
    whether the store keys it read are gone."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llm_inference_in_distributed_edge_networks_amd.parallel import init_distributed, shutdown
    from llm_inference_in_distributed_edge_networks_amd.parallel import rccl as R
    init_distributed("cpu", timeout_s=60)
    fake = FakeRcclLib(rank)
    R._lib = fake
    gens = []
    orig_ns = R.RcclComm._namespace

    def ns():
        g = orig_ns()
        gens.append(g)
        return g

    R.RcclComm._namespace = staticmethod(ns)
    prev = rank - 1 if rank > 0 else None
    nxt = rank + 1 if rank < world - 1 else None
    report = []
    for _ in range(2):
        start = len(fake.inits)
        comm = R.RcclComm(rank, world, device=rank % 8, peers=[prev, nxt])
        chans = list(comm.channels.keys())
        report.append({"gen": gens[-1], "channels": [list(k) for k in chans], "inits": fake.inits[start:],
                       "peer_index": {str(p): comm.channels[R.channel_key(rank, p)].peer_index(p)
                                      for p in (prev, nxt) if p is not None},
                       "h": [comm.channels[k].h.value for k in chans]})
        dist.barrier()
        store = dist.distributed_c10d._get_default_store()
        report[-1]["keys_left"] = [f"{a}-{b}" for a, b in chans
                                   if store.check([f"edge_rccl/{gens[-1]}/{a}-{b}"])]
        comm.close()
        report[-1]["destroyed"] = list(fake.destroyed)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(report, f)
    shutdown()
