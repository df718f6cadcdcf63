"""Can RCCL run several ranks on ONE GPU?  (If so, the nccl-backend pipeline paths - torch p2p over RCCL, the native
RcclComm, IPC credits over RCCL - can be rehearsed on a one-GPU box.)  Launch with
``torchrun --nproc-per-node N tools/rccl_shared_probe.py``; every rank uses cuda:0.  Prints one JSON line per rank."""
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    out = {"rank": rank, "world": world}
    t0 = time.time()
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["all_reduce"] = float(x[0])
        y = torch.empty(1 << 20, device="cuda")
        if rank == 0:
            dist.send(torch.full((1 << 20,), 7.0, device="cuda"), 1)
        elif rank == 1:
            dist.recv(y, 0)
            torch.cuda.synchronize()
            out["recv"] = float(y[0])
        dist.barrier()
        out["ok"] = True
    except Exception as e:   # recorded: a duplicate-GPU refusal is the expected negative answer
        out["ok"] = False
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    out["s"] = round(time.time() - t0, 2)
    print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
