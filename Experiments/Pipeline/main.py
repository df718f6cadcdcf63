"""N-stage split inference with quantized boundaries (BASELINE.json configs 1-5).

The reference simulates its two "edge devices" with an in-place fake quantization inside one
process (``Experiments/Qwen2-0.5B/qwen_layer_wise.py:54-70``).  This entry point runs the real
pipeline: layers are partitioned into ``num_stages`` stages (or at ``split_layers``), each stage
scores its boundary tokens (``methods``), encodes its output with ``codec`` into one byte message
and hands it to the next stage.

    python main.py --params configs/config1_pythia_split3_passthrough_cpu.json       # 1 process, CPU
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        main.py --params configs/config2_pythia_2stage_int8.json                      # 2 GPUs, RCCL
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        main.py --params configs/config5_qwen2_8stage_relevance.json                  # 8 GPUs

A world size that is a multiple of the stage count adds data-parallel pipeline replicas; a single
process runs every stage locally (same codec, same numerics).  Results: ``pipeline_results.json``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from llm_inference_in_distributed_edge_networks_amd.config import Params  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.experiments import pipeline_experiment  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel.dist import shutdown  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="params.json")
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-windows", type=int, default=None)
    ap.add_argument("--dataset", default=None)
    a = ap.parse_args()
    p = Params.load(a.params, device=a.device, max_windows=a.max_windows, dataset=a.dataset)
    p.experiment = "pipeline"
    pipeline_experiment(p, p.model or "qwen2-0.5b")
    shutdown()  # all ranks done: barrier + destroy the process group before interpreter exit
