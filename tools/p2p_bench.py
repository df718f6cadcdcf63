"""Point-to-point transport microbenchmark between pipeline stages (p2p latency/bandwidth).

``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/p2p_bench.py``
Ping-pong latency (half round trip) and one-way streaming bandwidth of isend/irecv for message sizes
covering the boundary payloads (Qwen2-0.5B, 32 windows x 512 tokens: passthrough bf16 29.4 MB,
mixed int4/int8 11.1 MB).  RCCL over xGMI on GPUs, gloo on CPUs."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd.parallel.dist import init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,65536,1048576,11075584,29360128")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--transport", default="torch", choices=["torch", "ipc", "rccl"],
                    help="torch: isend/irecv (RCCL); ipc: peer copies into the receiver's IPC-mapped slot ring "
                         "(parallel/ipc.py, the hipMemcpyPeerAsync baseline); rccl: the native per-edge RCCL "
                         "channels (parallel/rccl.py)")
    a = ap.parse_args()
    env = init_distributed("auto")
    assert env.world_size == 2, "run with exactly 2 ranks"
    dev = env.device
    peer = 1 - env.rank
    res = []
    for n in [int(x) for x in a.sizes.split(",")]:
        buf = torch.zeros(n, dtype=torch.uint8, device=dev)
        for _ in range(3):
            if env.rank == 0:
                dist.send(buf, peer); dist.recv(buf, peer)
            else:
                dist.recv(buf, peer); dist.send(buf, peer)
        sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
        sync()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if env.rank == 0:
                dist.send(buf, peer); dist.recv(buf, peer)
            else:
                dist.recv(buf, peer); dist.send(buf, peer)
        sync()
        lat = (time.perf_counter() - t0) / a.iters / 2
        dist.barrier()
        t0 = time.perf_counter()
        reqs = [dist.isend(buf, peer) if env.rank == 0 else dist.irecv(buf, peer) for _ in range(a.iters)]
        for r in reqs:
            r.wait()
        sync()
        dt = time.perf_counter() - t0
        rec = {"bytes": n, "half_rtt_us": lat * 1e6, "stream_GBps": n * a.iters / dt / 1e9}
        if a.transport == "ipc":
            # one-way stream of the same messages through the peer-copy transport (rank 0 -> rank 1)
            from llm_inference_in_distributed_edge_networks_amd.parallel.ipc import IpcP2P
            tr = IpcP2P(dev, capacity=max(n, 1 << 20))
            tr.setup(env.rank, 0 if env.rank == 1 else None, 1 if env.rank == 0 else None)
            sync()
            t0 = time.perf_counter()
            for _ in range(a.iters):   # the receiver consumes each message before posting the next receive
                h = tr.send(buf, 1) if env.rank == 0 else tr.recv(buf, 0)
                if env.rank == 1:
                    h.wait()
            tr.quiesce()
            sync()
            dist.barrier()
            rec["ipc_stream_GBps"] = n * a.iters / (time.perf_counter() - t0) / 1e9
            tr.close()
        if a.transport == "rccl":
            # one-way stream over the native channel of the edge (0, 1): per-op events, no host blocking
            from llm_inference_in_distributed_edge_networks_amd.parallel.rccl import RcclComm
            if not hasattr(main, "_rc"):
                main._rc = RcclComm(env.rank, env.world_size, dev.index or 0, peers=[peer])
            rc = main._rc
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            hs = [rc.send(buf, 1) if env.rank == 0 else rc.recv(buf, 0) for _ in range(a.iters)]
            for h in hs:
                h.wait()
            sync()
            rec["rccl_native_stream_GBps"] = n * a.iters / (time.perf_counter() - t0) / 1e9
        res.append(rec)
        if env.rank == 0:
            print(json.dumps(res[-1]), flush=True)
    if env.rank == 0 and a.json_out:
        with open(a.json_out, "w") as f:
            json.dump({"backend": env.backend, "results": res}, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
