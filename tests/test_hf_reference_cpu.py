"""The same-node reference path (``eval.hf_reference``, recorded by ``bench.py``): HF transformers + eager running
the reference's per-window work.  CPU, tiny Qwen2 config."""
import torch

from llm_inference_in_distributed_edge_networks_amd.eval.hf_reference import ReferencePath, int4_global_lowest
from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2


def test_reference_path_runs_and_times_on_cpu():
    ref = ReferencePath(TINY_QWEN2, "cpu")
    r = ref.throughput(batch=2, windows=4, warmup=1, layer=1, ratio=0.5, max_length=64, stride=16)
    assert r["windows"] == 4 and r["window_tokens_per_s"] > 0
    assert abs(r["forward_tokens_per_s"] - 2 * r["window_tokens_per_s"]) < 1.0   # importance + one split forward


def test_reference_path_ratio_zero_is_the_unquantized_forward():
    """ratio 0 leaves the boundary untouched: the split forward's NLL equals HF's own full forward loss."""
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    ref = ReferencePath(TINY_QWEN2, "cpu")
    toks = synthetic_stream(4096, TINY_QWEN2.vocab_size, 0)
    wins = [w for w in sliding_windows(toks.shape[1], 64, 16) if w.length == 64][:3]
    b = next(batches(toks, wins, 3))
    nll0 = ref.run(b, layer=1, ratio=0.0)[0]
    nll1 = ref.run(b, layer=1, ratio=1.0)[0]
    ids = b.ids
    with torch.no_grad():
        logits = ref.split(input_ids=ids).logits[:, :-1]
    first = torch.tensor([w.first_scored for w in b.windows])
    tmask = torch.arange(64)[None] >= first[:, None] + 1
    tgt = torch.where(tmask[:, 1:], ids[:, 1:], torch.full_like(ids[:, 1:], -100))
    want = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), tgt.reshape(-1),
                                             ignore_index=-100, reduction="sum")
    assert torch.allclose(nll0, want, rtol=1e-5, atol=1e-4)
    assert not torch.allclose(nll1, want, rtol=1e-5, atol=1e-4)


def test_int4_global_lowest_quantizes_only_the_lowest_tokens():
    h = torch.randn(2, 8, 4)
    imp = torch.arange(16, dtype=torch.float32).view(2, 8)
    q = int4_global_lowest(h, imp, 0.5)
    assert torch.equal(q[:, 4:], h[:, 4:])
    sel = h[:, :4]
    mx = sel.abs().amax(dim=(1, 2), keepdim=True)
    assert torch.allclose(q[:, :4], torch.round(torch.clamp(sel / mx * 7, -8, 7)) / 7 * mx)
