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
