import torch

from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM


def hf_qwen2(cfg, seed=0):
    from transformers import Qwen2Config, Qwen2ForCausalLM
    torch.manual_seed(seed)
    hc = Qwen2Config(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                     num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                     num_key_value_heads=cfg.num_kv_heads, max_position_embeddings=cfg.max_position,
                     rope_theta=cfg.rope_theta, tie_word_embeddings=cfg.tie_embeddings, rms_norm_eps=cfg.norm_eps,
                     attn_implementation="eager")
    m = Qwen2ForCausalLM(hc).eval()
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if k.endswith("bias"):
                v.normal_(0, 0.1)
            elif "norm" in k:
                v.normal_(1, 0.1)
    return m


def hf_neox(cfg, seed=0):
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM
    torch.manual_seed(seed)
    hc = GPTNeoXConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                       intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
                       num_attention_heads=cfg.num_heads, rotary_pct=cfg.rotary_dim / cfg.head_dim,
                       max_position_embeddings=cfg.max_position, layer_norm_eps=cfg.norm_eps,
                       attn_implementation="eager", hidden_act="gelu", tie_word_embeddings=False)
    m = GPTNeoXForCausalLM(hc).eval()
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if k.endswith("bias"):
                v.normal_(0, 0.1)
    return m


def ours_from_hf(cfg, hf):
    return DecoderLM.from_state_dict(cfg, hf.state_dict())
