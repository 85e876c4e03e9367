"""HF-layout checkpoint IO (safetensors) for the native fused-parameter models.

``save_pretrained`` writes config.json + generation_config.json + model.safetensors (sharded with
model.safetensors.index.json above ``max_shard_bytes``) using HF tensor names, so the output loads
with ``transformers.AutoModelForCausalLM.from_pretrained`` and vice versa — the ``{tag}_policy/``
artifact of the reference's save_checkpoint (reinforcement_learning_optimization_after_rag.py:365-370).
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, List, Tuple

import torch

from .config import ModelConfig, config_from_hf, config_to_hf

# (hf_name, native_param_name, row_start, row_count) ; row_count None = whole tensor
Mapping = List[Tuple[str, str, int, int]]


def decoder_mapping(cfg: ModelConfig) -> Mapping:
    m: Mapping = []
    Hq, Hkv, D, F = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, cfg.intermediate_size
    if cfg.arch == "opt":
        p = "model.decoder"
        m += [(f"{p}.embed_tokens.weight", "embed", 0, None), (f"{p}.embed_positions.weight", "pos_embed", 0, None),
              (f"{p}.final_layer_norm.weight", "norm_w", 0, None), (f"{p}.final_layer_norm.bias", "norm_b", 0, None)]
        for i in range(cfg.num_layers):
            L, n = f"{p}.layers.{i}", f"layers.{i}"
            m += [(f"{L}.self_attn_layer_norm.weight", f"{n}.ln1_w", 0, None),
                  (f"{L}.self_attn_layer_norm.bias", f"{n}.ln1_b", 0, None),
                  (f"{L}.final_layer_norm.weight", f"{n}.ln2_w", 0, None),
                  (f"{L}.final_layer_norm.bias", f"{n}.ln2_b", 0, None),
                  (f"{L}.self_attn.out_proj.weight", f"{n}.o_w", 0, None),
                  (f"{L}.self_attn.out_proj.bias", f"{n}.o_b", 0, None),
                  (f"{L}.fc1.weight", f"{n}.fc1_w", 0, None), (f"{L}.fc1.bias", f"{n}.fc1_b", 0, None),
                  (f"{L}.fc2.weight", f"{n}.fc2_w", 0, None), (f"{L}.fc2.bias", f"{n}.fc2_b", 0, None)]
            for proj, r0, rn in (("q_proj", 0, Hq * D), ("k_proj", Hq * D, Hkv * D), ("v_proj", (Hq + Hkv) * D, Hkv * D)):
                m += [(f"{L}.self_attn.{proj}.weight", f"{n}.qkv_w", r0, rn),
                      (f"{L}.self_attn.{proj}.bias", f"{n}.qkv_b", r0, rn)]
        return m
    m += [("model.embed_tokens.weight", "embed", 0, None), ("model.norm.weight", "norm_w", 0, None)]
    if not cfg.tie_embeddings:
        m.append(("lm_head.weight", "lm_head", 0, None))
    for i in range(cfg.num_layers):
        L, n = f"model.layers.{i}", f"layers.{i}"
        m += [(f"{L}.input_layernorm.weight", f"{n}.ln1_w", 0, None),
              (f"{L}.post_attention_layernorm.weight", f"{n}.ln2_w", 0, None),
              (f"{L}.self_attn.q_proj.weight", f"{n}.qkv_w", 0, Hq * D),
              (f"{L}.self_attn.k_proj.weight", f"{n}.qkv_w", Hq * D, Hkv * D),
              (f"{L}.self_attn.v_proj.weight", f"{n}.qkv_w", (Hq + Hkv) * D, Hkv * D),
              (f"{L}.self_attn.o_proj.weight", f"{n}.o_w", 0, None),
              (f"{L}.mlp.gate_proj.weight", f"{n}.gate_up_w", 0, F),
              (f"{L}.mlp.up_proj.weight", f"{n}.gate_up_w", F, F),
              (f"{L}.mlp.down_proj.weight", f"{n}.down_w", 0, None)]
    return m


def encoder_mapping(cfg: ModelConfig) -> Mapping:
    H = cfg.hidden_size
    m: Mapping = [("embeddings.word_embeddings.weight", "word_embed", 0, None),
                  ("embeddings.position_embeddings.weight", "pos_embed", 0, None),
                  ("embeddings.LayerNorm.weight", "emb_ln_w", 0, None),
                  ("embeddings.LayerNorm.bias", "emb_ln_b", 0, None)]
    if cfg.type_vocab_size:
        m.append(("embeddings.token_type_embeddings.weight", "type_embed", 0, None))
    if cfg.arch == "mpnet":
        m.append(("encoder.relative_attention_bias.weight", "rel_bias", 0, None))
    for i in range(cfg.num_layers):
        L, n = f"encoder.layer.{i}", f"layers.{i}"
        if cfg.arch == "bert":
            qkv = [(f"{L}.attention.self.query", 0), (f"{L}.attention.self.key", H), (f"{L}.attention.self.value", 2 * H)]
            o, ln1 = f"{L}.attention.output.dense", f"{L}.attention.output.LayerNorm"
        else:
            qkv = [(f"{L}.attention.attn.q", 0), (f"{L}.attention.attn.k", H), (f"{L}.attention.attn.v", 2 * H)]
            o, ln1 = f"{L}.attention.attn.o", f"{L}.attention.LayerNorm"
        for base, r0 in qkv:
            m += [(f"{base}.weight", f"{n}.qkv_w", r0, H), (f"{base}.bias", f"{n}.qkv_b", r0, H)]
        m += [(f"{o}.weight", f"{n}.o_w", 0, None), (f"{o}.bias", f"{n}.o_b", 0, None),
              (f"{ln1}.weight", f"{n}.ln1_w", 0, None), (f"{ln1}.bias", f"{n}.ln1_b", 0, None),
              (f"{L}.intermediate.dense.weight", f"{n}.fc1_w", 0, None),
              (f"{L}.intermediate.dense.bias", f"{n}.fc1_b", 0, None),
              (f"{L}.output.dense.weight", f"{n}.fc2_w", 0, None), (f"{L}.output.dense.bias", f"{n}.fc2_b", 0, None),
              (f"{L}.output.LayerNorm.weight", f"{n}.ln2_w", 0, None),
              (f"{L}.output.LayerNorm.bias", f"{n}.ln2_b", 0, None)]
    return m


def mapping_for(model) -> Mapping:
    return decoder_mapping(model.cfg) if model.cfg.is_decoder else encoder_mapping(model.cfg)


def to_hf_state_dict(model, dtype=None) -> Dict[str, torch.Tensor]:
    params = dict(model.named_parameters())
    out = {}
    for hf, nat, r0, rn in mapping_for(model):
        t = params[nat].detach()
        if rn is not None:
            t = t[r0:r0 + rn]
        t = t.to("cpu")
        out[hf] = (t.to(dtype) if dtype is not None else t).contiguous()
    return out


@torch.no_grad()
def load_hf_state_dict(model, sd: Dict[str, torch.Tensor], strict: bool = True, prefix_strip: str = ""):
    params = dict(model.named_parameters())
    missing = []
    for hf, nat, r0, rn in mapping_for(model):
        key = hf
        if key not in sd:
            alt = [k for k in sd if k.endswith(hf)]
            key = alt[0] if alt else None
        if key is None:
            missing.append(hf)
            continue
        src = sd[key]
        dst = params[nat]
        if rn is not None:
            dst = dst[r0:r0 + rn]
        dst.copy_(src.to(dst.device, dst.dtype).view_as(dst))
    if strict and missing:
        raise KeyError(f"missing tensors in checkpoint: {missing[:8]}{'...' if len(missing) > 8 else ''}")
    return missing


def save_pretrained(model, path: str, max_shard_bytes: int = 5 * 1024 ** 3, dtype=torch.bfloat16,
                    generation_config: dict = None, write_weights: bool = True):
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        d = config_to_hf(model.cfg)
        d["_ragtl_preset"] = model.cfg.name
        json.dump(d, f, indent=2)
    if model.cfg.is_decoder:
        gc = {"bos_token_id": model.cfg.bos_token_id, "eos_token_id": model.cfg.eos_token_id,
              "pad_token_id": model.cfg.pad_token_id, "do_sample": True, "temperature": 0.7, "max_length": 512}
        gc.update(generation_config or {})
        with open(os.path.join(path, "generation_config.json"), "w") as f:
            json.dump(gc, f, indent=2)
    if not write_weights:
        return
    sd = to_hf_state_dict(model, dtype)
    total = sum(t.numel() * t.element_size() for t in sd.values())
    if total <= max_shard_bytes:
        save_file(sd, os.path.join(path, "model.safetensors"), metadata={"format": "pt"})
        return
    shards, cur, cur_b = [], {}, 0
    for k, t in sd.items():
        b = t.numel() * t.element_size()
        if cur and cur_b + b > max_shard_bytes:
            shards.append(cur)
            cur, cur_b = {}, 0
        cur[k] = t
        cur_b += b
    if cur:
        shards.append(cur)
    wm = {}
    for i, sh in enumerate(shards):
        name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(path, name), metadata={"format": "pt"})
        for k in sh:
            wm[k] = name
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": wm}, f, indent=2)


def read_state_dict(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            wm = json.load(f)["weight_map"]
        sd = {}
        for name in sorted(set(wm.values())):
            sd.update(load_file(os.path.join(path, name)))
        return sd
    st = os.path.join(path, "model.safetensors")
    if os.path.exists(st):
        return load_file(st)
    pt = os.path.join(path, "pytorch_model.bin")
    if os.path.exists(pt):
        return torch.load(pt, map_location="cpu", weights_only=True)
    raise FileNotFoundError(f"no weights found in {path}")


def load_config(path: str) -> ModelConfig:
    with open(os.path.join(path, "config.json")) as f:
        return config_from_hf(json.load(f))


def from_pretrained(path: str, device="cpu", dtype=torch.bfloat16):
    from .decoder import CausalLM
    from .encoder import SentenceEncoder

    cfg = load_config(path)
    cls = CausalLM if cfg.is_decoder else SentenceEncoder
    model = cls(cfg, device=device, dtype=dtype, init=False)
    load_hf_state_dict(model, read_state_dict(path))
    return model
