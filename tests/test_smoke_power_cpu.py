"""``__graft_entry__.smoke()``'s checks have power: the stage-by-stage oracle comparison (boundary hidden state,
decoded boundary tensor, final-norm input, NLL) passes for an unperturbed run and FAILS the fp32 tolerances under a
1e-3 relative perturbation of the boundary or of the final hidden state (run here CPU-vs-CPU; on the GPU box the
same checks compare cuda:0 with the CPU oracle)."""
import pytest
import torch

import __graft_entry__ as g


def test_unperturbed_passes():
    res = g.stage_oracle("cpu", torch.float32)
    assert g.smoke_failures(res, "fp32") == []
    assert res["message_bytes"] == res["message_bytes_codec"] > 0


@pytest.mark.parametrize("where", ["boundary", "final"])
def test_1e3_perturbation_fails(where):
    res = g.stage_oracle("cpu", torch.float32, perturb={where: 1e-3})
    bad = g.smoke_failures(res, "fp32")
    assert bad and any(b.startswith(where) for b in bad), (res, bad)
    assert res[where] == pytest.approx(1e-3, rel=1e-2)
