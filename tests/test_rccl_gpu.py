"""Native RCCL transport (csrc/comm/rccl_comm.cpp) on one GPU: self-loopback send/recv + all-reduce."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rccl_self_loopback_and_allreduce():
    from llm_inference_in_distributed_edge_networks_amd.parallel.rccl import RcclComm
    c = RcclComm(0, 1, torch.cuda.current_device())
    src = torch.randint(0, 255, (11_075_584,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros_like(src)
    c.sendrecv(src, dst, 0).wait()
    assert torch.equal(src, dst)
    t = torch.arange(10, dtype=torch.float64, device="cuda")
    c.all_reduce_sum_f64(t)
    assert torch.equal(t, torch.arange(10, dtype=torch.float64, device="cuda"))
    c.close()
