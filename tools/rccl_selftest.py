"""Single-GPU self-test of the native RCCL transport (loopback send/recv + all-reduce)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd.parallel import rccl  # noqa: E402


def say(*a):
    print(*a, flush=True)


say("lib", rccl.COMM_LIB_PATH)
L = rccl.lib()
say("id bytes", L.edge_rccl_id_bytes())
uid = rccl.RcclComm.make_unique_id()
say("unique id ok", len(uid))
c = rccl.RcclComm(0, 1, torch.cuda.current_device(), uid)
say("init ok", c.h)
src = torch.randint(0, 255, (11_075_584,), dtype=torch.uint8, device="cuda")
dst = torch.zeros_like(src)
c.sendrecv(src, dst, 0).wait()
torch.cuda.synchronize()
say("loopback equal", torch.equal(src, dst))
t = torch.arange(10, dtype=torch.float64, device="cuda")
c.all_reduce_sum_f64(t)
torch.cuda.synchronize()
say("allreduce ok", t.tolist())
c.close()
say("RCCL_SELFTEST_OK")
