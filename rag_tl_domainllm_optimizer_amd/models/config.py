"""Model configurations and named presets (shapes from SURVEY Appendix E).

The presets reproduce the architectures the reference names or implies — Llama-2-7B (its
``main()`` default, reinforcement_learning_optimization_after_rag.py:469), Mistral-7B / Llama-2-13B
(north-star configs), OPT-125m (CPU plumbing) and the all-MiniLM-L6-v2 / all-mpnet-base-v2
sentence encoders (reference default reward encoder, rl.py:22,54) — with random-init weights,
since no checkpoints can be downloaded. ``"<preset>:random"`` selects a preset by name.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class ModelConfig:
    arch: str = "llama"                 # llama | mistral | opt | bert | mpnet
    vocab_size: int = 32000
    hidden_size: int = 4096
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 32
    head_dim: int = 128
    intermediate_size: int = 11008
    max_position: int = 4096
    norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    sliding_window: int = 0             # 0 = full attention
    hidden_act: str = "silu"
    tie_embeddings: bool = False
    bias: bool = False                  # linear biases (OPT/BERT/MPNet)
    # token ids
    bos_token_id: int = 1
    eos_token_id: int = 2
    pad_token_id: int = 0
    # encoder specifics
    type_vocab_size: int = 0
    relative_buckets: int = 0
    relative_max_distance: int = 128
    position_offset: int = 0            # OPT learned positions start at index 2; MPNet at pad+1
    # misc
    name: str = "custom"
    initializer_range: float = 0.02

    @property
    def is_decoder(self) -> bool:
        return self.arch in ("llama", "mistral", "opt")

    @property
    def qkv_dim(self) -> int:
        return (self.num_heads + 2 * self.num_kv_heads) * self.head_dim

    def to_dict(self):
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d):
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    def num_params(self) -> int:
        H, F, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        attn = H * self.qkv_dim + self.num_heads * self.head_dim * H
        if self.arch in ("llama", "mistral"):
            mlp = 3 * H * F
            per = attn + mlp + 2 * H
            emb = V * H * (1 if self.tie_embeddings else 2)
            return L * per + emb + H
        mlp = 2 * H * F
        return L * (attn + mlp) + V * H


PRESETS = {
    "mistral-7b": ModelConfig(arch="mistral", vocab_size=32000, hidden_size=4096, num_layers=32, num_heads=32,
                              num_kv_heads=8, head_dim=128, intermediate_size=14336, max_position=32768,
                              norm_eps=1e-5, rope_theta=10000.0, sliding_window=4096, name="mistral-7b"),
    # OpenChat-3.5 (README.md:25 lists OpenChat): the Mistral-7B architecture with two added
    # chat tokens (vocab 32002), rope theta 1e4, 8k context
    "openchat-3.5": ModelConfig(arch="mistral", vocab_size=32002, hidden_size=4096, num_layers=32, num_heads=32,
                                num_kv_heads=8, head_dim=128, intermediate_size=14336, max_position=8192,
                                norm_eps=1e-5, rope_theta=10000.0, sliding_window=4096, name="openchat-3.5"),
    "llama2-7b": ModelConfig(arch="llama", vocab_size=32000, hidden_size=4096, num_layers=32, num_heads=32,
                             num_kv_heads=32, head_dim=128, intermediate_size=11008, max_position=4096,
                             norm_eps=1e-5, name="llama2-7b"),
    "llama2-13b": ModelConfig(arch="llama", vocab_size=32000, hidden_size=5120, num_layers=40, num_heads=40,
                              num_kv_heads=40, head_dim=128, intermediate_size=13824, max_position=4096,
                              norm_eps=1e-5, name="llama2-13b"),
    "opt-125m": ModelConfig(arch="opt", vocab_size=50272, hidden_size=768, num_layers=12, num_heads=12,
                            num_kv_heads=12, head_dim=64, intermediate_size=3072, max_position=2048,
                            norm_eps=1e-5, hidden_act="relu", tie_embeddings=True, bias=True, bos_token_id=2,
                            eos_token_id=2, pad_token_id=1, position_offset=2, name="opt-125m"),
    "minilm-l6": ModelConfig(arch="bert", vocab_size=30522, hidden_size=384, num_layers=6, num_heads=12,
                             num_kv_heads=12, head_dim=32, intermediate_size=1536, max_position=512,
                             norm_eps=1e-12, hidden_act="gelu", bias=True, type_vocab_size=2, pad_token_id=0,
                             bos_token_id=101, eos_token_id=102, name="all-MiniLM-L6-v2"),
    "mpnet-base": ModelConfig(arch="mpnet", vocab_size=30527, hidden_size=768, num_layers=12, num_heads=12,
                              num_kv_heads=12, head_dim=64, intermediate_size=3072, max_position=514,
                              norm_eps=1e-5, hidden_act="gelu", bias=True, relative_buckets=32,
                              pad_token_id=1, bos_token_id=0, eos_token_id=2, position_offset=2,
                              name="all-mpnet-base-v2"),
    # small shapes for tests and smoke runs (GPU-kernel compatible head dims)
    "tiny-llama": ModelConfig(arch="llama", vocab_size=512, hidden_size=256, num_layers=2, num_heads=4,
                              num_kv_heads=2, head_dim=64, intermediate_size=512, max_position=512,
                              norm_eps=1e-5, name="tiny-llama"),
    "tiny-mistral": ModelConfig(arch="mistral", vocab_size=512, hidden_size=256, num_layers=2, num_heads=4,
                                num_kv_heads=2, head_dim=64, intermediate_size=512, max_position=512,
                                norm_eps=1e-5, sliding_window=64, name="tiny-mistral"),
    "tiny-opt": ModelConfig(arch="opt", vocab_size=512, hidden_size=256, num_layers=2, num_heads=4,
                            num_kv_heads=4, head_dim=64, intermediate_size=512, max_position=512, norm_eps=1e-5,
                            hidden_act="relu", tie_embeddings=True, bias=True, bos_token_id=2, eos_token_id=2,
                            pad_token_id=1, position_offset=2, name="tiny-opt"),
    "tiny-bert": ModelConfig(arch="bert", vocab_size=512, hidden_size=128, num_layers=2, num_heads=4,
                             num_kv_heads=4, head_dim=32, intermediate_size=256, max_position=128, norm_eps=1e-12,
                             hidden_act="gelu", bias=True, type_vocab_size=2, name="tiny-bert"),
    "tiny-mpnet": ModelConfig(arch="mpnet", vocab_size=512, hidden_size=128, num_layers=2, num_heads=4,
                              num_kv_heads=4, head_dim=32, intermediate_size=256, max_position=130,
                              norm_eps=1e-5, hidden_act="gelu", bias=True, relative_buckets=32, pad_token_id=1,
                              bos_token_id=0, eos_token_id=2, position_offset=2, name="tiny-mpnet"),
}

ALIASES = {
    "mistralai/mistral-7b-v0.1": "mistral-7b",
    "mistral": "mistral-7b",
    "openchat/openchat_3.5": "openchat-3.5",
    "openchat": "openchat-3.5",
    "meta-llama/llama-2-7b-hf": "llama2-7b",
    "meta-llama/llama-2-13b-hf": "llama2-13b",
    "facebook/opt-125m": "opt-125m",
    "sentence-transformers/all-minilm-l6-v2": "minilm-l6",
    "all-minilm-l6-v2": "minilm-l6",
    "sentence-transformers/all-mpnet-base-v2": "mpnet-base",
    "all-mpnet-base-v2": "mpnet-base",
}


def resolve_preset(name: str) -> Optional[ModelConfig]:
    """Map ``"mistral-7b:random"``, an HF hub id, or a preset name to a config (or None)."""
    key = name.split(":")[0].strip().lower()
    key = ALIASES.get(key, key)
    cfg = PRESETS.get(key)
    return dataclasses.replace(cfg) if cfg is not None else None


def config_from_hf(d: dict) -> ModelConfig:
    """Build a ModelConfig from an HF config.json dict (llama / mistral / opt / bert / mpnet)."""
    mt = d.get("model_type", "llama")
    if mt in ("llama", "mistral"):
        H = d["hidden_size"]
        nh = d["num_attention_heads"]
        return ModelConfig(arch=mt, vocab_size=d["vocab_size"], hidden_size=H, num_layers=d["num_hidden_layers"],
                           num_heads=nh, num_kv_heads=d.get("num_key_value_heads", nh),
                           head_dim=d.get("head_dim") or H // nh, intermediate_size=d["intermediate_size"],
                           max_position=d.get("max_position_embeddings", 4096), norm_eps=d.get("rms_norm_eps", 1e-6),
                           rope_theta=d.get("rope_theta", 10000.0), sliding_window=d.get("sliding_window") or 0,
                           tie_embeddings=d.get("tie_word_embeddings", False), bos_token_id=d.get("bos_token_id", 1),
                           eos_token_id=d.get("eos_token_id", 2), pad_token_id=d.get("pad_token_id") or 0,
                           name=d.get("_name_or_path", mt))
    if mt == "opt":
        H = d["hidden_size"]
        nh = d["num_attention_heads"]
        return ModelConfig(arch="opt", vocab_size=d["vocab_size"], hidden_size=H, num_layers=d["num_hidden_layers"],
                           num_heads=nh, num_kv_heads=nh, head_dim=H // nh, intermediate_size=d["ffn_dim"],
                           max_position=d.get("max_position_embeddings", 2048), norm_eps=1e-5,
                           hidden_act=d.get("activation_function", "relu"), tie_embeddings=True, bias=True,
                           bos_token_id=d.get("bos_token_id", 2), eos_token_id=d.get("eos_token_id", 2),
                           pad_token_id=d.get("pad_token_id", 1), position_offset=2, name=d.get("_name_or_path", mt))
    if mt in ("bert", "mpnet"):
        H = d["hidden_size"]
        nh = d["num_attention_heads"]
        return ModelConfig(arch=mt, vocab_size=d["vocab_size"], hidden_size=H, num_layers=d["num_hidden_layers"],
                           num_heads=nh, num_kv_heads=nh, head_dim=H // nh, intermediate_size=d["intermediate_size"],
                           max_position=d.get("max_position_embeddings", 512),
                           norm_eps=d.get("layer_norm_eps", 1e-12), hidden_act=d.get("hidden_act", "gelu"),
                           bias=True, type_vocab_size=d.get("type_vocab_size", 0) if mt == "bert" else 0,
                           relative_buckets=d.get("relative_attention_num_buckets", 32) if mt == "mpnet" else 0,
                           pad_token_id=d.get("pad_token_id", 0), bos_token_id=d.get("bos_token_id", 0),
                           eos_token_id=d.get("eos_token_id", 2), position_offset=2 if mt == "mpnet" else 0,
                           name=d.get("_name_or_path", mt))
    raise ValueError(f"unsupported model_type {mt!r}")


def config_to_hf(cfg: ModelConfig) -> dict:
    """HF config.json dict for save_pretrained-compatible checkpoints."""
    if cfg.arch in ("llama", "mistral"):
        d = {
            "architectures": ["MistralForCausalLM" if cfg.arch == "mistral" else "LlamaForCausalLM"],
            "model_type": cfg.arch, "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden_size,
            "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
            "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
            "intermediate_size": cfg.intermediate_size, "max_position_embeddings": cfg.max_position,
            "rms_norm_eps": cfg.norm_eps, "rope_theta": cfg.rope_theta, "hidden_act": "silu",
            "tie_word_embeddings": cfg.tie_embeddings, "bos_token_id": cfg.bos_token_id,
            "eos_token_id": cfg.eos_token_id, "pad_token_id": cfg.pad_token_id, "torch_dtype": "bfloat16",
            "attention_bias": False, "initializer_range": cfg.initializer_range,
        }
        if cfg.arch == "mistral":
            d["sliding_window"] = cfg.sliding_window or None
        return d
    if cfg.arch == "opt":
        return {"architectures": ["OPTForCausalLM"], "model_type": "opt", "vocab_size": cfg.vocab_size,
                "hidden_size": cfg.hidden_size, "num_hidden_layers": cfg.num_layers,
                "num_attention_heads": cfg.num_heads, "ffn_dim": cfg.intermediate_size,
                "max_position_embeddings": cfg.max_position, "activation_function": cfg.hidden_act,
                "do_layer_norm_before": True, "word_embed_proj_dim": cfg.hidden_size,
                "bos_token_id": cfg.bos_token_id, "eos_token_id": cfg.eos_token_id, "pad_token_id": cfg.pad_token_id,
                "enable_bias": True, "layer_norm_elementwise_affine": True, "torch_dtype": "bfloat16",
                "tie_word_embeddings": True}
    if cfg.arch == "bert":
        return {"architectures": ["BertModel"], "model_type": "bert", "vocab_size": cfg.vocab_size,
                "hidden_size": cfg.hidden_size, "num_hidden_layers": cfg.num_layers,
                "num_attention_heads": cfg.num_heads, "intermediate_size": cfg.intermediate_size,
                "max_position_embeddings": cfg.max_position, "hidden_act": cfg.hidden_act,
                "layer_norm_eps": cfg.norm_eps, "type_vocab_size": cfg.type_vocab_size,
                "pad_token_id": cfg.pad_token_id}
    if cfg.arch == "mpnet":
        return {"architectures": ["MPNetModel"], "model_type": "mpnet", "vocab_size": cfg.vocab_size,
                "hidden_size": cfg.hidden_size, "num_hidden_layers": cfg.num_layers,
                "num_attention_heads": cfg.num_heads, "intermediate_size": cfg.intermediate_size,
                "max_position_embeddings": cfg.max_position, "hidden_act": cfg.hidden_act,
                "layer_norm_eps": cfg.norm_eps, "relative_attention_num_buckets": cfg.relative_buckets,
                "pad_token_id": cfg.pad_token_id, "bos_token_id": cfg.bos_token_id,
                "eos_token_id": cfg.eos_token_id}
    raise ValueError(cfg.arch)


def dump(cfg: ModelConfig) -> str:
    return json.dumps(cfg.to_dict(), indent=1)
