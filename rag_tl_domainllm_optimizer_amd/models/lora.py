"""LoRA adapters (PEFT-compatible) on the fused projections of the decoder.

Adapters are stored per HF target module (q_proj, k_proj, ..., down_proj) so PEFT checkpoints map
1:1; at run time the adapters of one fused projection form a :class:`ops.LoRAGroup` and are
executed inside the projection's MFMA GEMM. This is the "Transfer Learning (LoRA/PEFT)" stage the
reference README declares (README.md:15,29) but does not implement.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .. import ops

# projection name -> (fused group, row offset function)
_LLAMA_GROUPS = {
    "q_proj": "qkv", "k_proj": "qkv", "v_proj": "qkv", "o_proj": "o",
    "gate_proj": "gate_up", "up_proj": "gate_up", "down_proj": "down",
}
_OPT_GROUPS = {"q_proj": "qkv", "k_proj": "qkv", "v_proj": "qkv", "out_proj": "o", "fc1": "fc1", "fc2": "fc2"}


@dataclass
class LoraConfig:
    r: int = 16
    lora_alpha: float = 32.0
    lora_dropout: float = 0.0
    target_modules: List[str] = field(default_factory=lambda: ["q_proj", "v_proj"])
    bias: str = "none"
    task_type: str = "CAUSAL_LM"
    peft_type: str = "LORA"
    base_model_name_or_path: str = ""
    fan_in_fan_out: bool = False
    inference_mode: bool = False
    init_lora_weights: bool = True
    modules_to_save: Optional[List[str]] = None
    layers_to_transform: Optional[List[int]] = None
    use_rslora: bool = False

    @property
    def scaling(self) -> float:
        return self.lora_alpha / (math.sqrt(self.r) if self.use_rslora else self.r)

    def to_json(self) -> dict:
        d = asdict(self)
        d["target_modules"] = sorted(self.target_modules)
        return d


def _proj_rows(cfg, proj: str):
    """(row offset, rows) of an HF projection inside its fused weight."""
    Hq, Hkv, D, F, H = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, cfg.intermediate_size, cfg.hidden_size
    table = {
        "q_proj": (0, Hq * D), "k_proj": (Hq * D, Hkv * D), "v_proj": ((Hq + Hkv) * D, Hkv * D),
        "o_proj": (0, H), "out_proj": (0, H), "gate_proj": (0, F), "up_proj": (F, F), "down_proj": (0, H),
        "fc1": (0, F), "fc2": (0, H),
    }
    return table[proj]


def _proj_in(cfg, proj: str) -> int:
    if proj in ("o_proj", "out_proj"):
        return cfg.num_heads * cfg.head_dim
    if proj in ("down_proj", "fc2"):
        return cfg.intermediate_size
    return cfg.hidden_size


def group_map(cfg) -> Dict[str, str]:
    return _OPT_GROUPS if cfg.arch == "opt" else _LLAMA_GROUPS


def _group_out(cfg, group: str) -> int:
    return {"qkv": cfg.qkv_dim, "o": cfg.hidden_size, "gate_up": 2 * cfg.intermediate_size,
            "down": cfg.hidden_size, "fc1": cfg.intermediate_size, "fc2": cfg.hidden_size}[group]


def attach_lora(model, r=16, alpha=32.0, targets=None, dropout=0.0, seed=0):
    cfg = model.cfg
    gm = group_map(cfg)
    if targets is None or targets == "all":
        targets = list(gm.keys())
    targets = [t for t in targets if t in gm]
    if not 0.0 <= dropout < 1.0:
        raise ValueError(f"lora_dropout must be in [0, 1), got {dropout}")
    lcfg = LoraConfig(r=r, lora_alpha=alpha, lora_dropout=dropout, target_modules=list(targets),
                      base_model_name_or_path=cfg.name)
    g = torch.Generator(device="cpu").manual_seed(seed)
    dev = model.embed.device
    for layer in model.layers:
        layer.lora = {}
        layer.lora_params = nn.ParameterDict()
        groups: Dict[str, list] = {}
        for proj in targets:
            groups.setdefault(gm[proj], []).append(proj)
        for grp, projs in groups.items():
            a_list, b_list, c0s, scales = [], [], [], []
            for proj in projs:
                k_in = _proj_in(cfg, proj)
                row0, n = _proj_rows(cfg, proj)
                a = torch.empty(r, k_in)
                # PEFT init: A ~ kaiming_uniform(a=sqrt(5)), B = 0
                bound = 1.0 / math.sqrt(k_in)
                a.uniform_(-bound, bound, generator=g)
                pa = nn.Parameter(a.to(dev))
                pb = nn.Parameter(torch.zeros(n, r, device=dev))
                layer.lora_params[f"{proj}_A"] = pa
                layer.lora_params[f"{proj}_B"] = pb
                a_list.append(pa)
                b_list.append(pb)
                c0s.append(row0)
                scales.append(lcfg.scaling)
            layer.lora[grp] = ops.LoRAGroup(projs, a_list, b_list, c0s, scales, _group_out(cfg, grp),
                                            dropout=float(dropout))
    model.lora_config = lcfg
    model.refresh_lora()
    return lcfg


def _layer_prefix(cfg, i):
    return f"base_model.model.model.decoder.layers.{i}" if cfg.arch == "opt" else f"base_model.model.model.layers.{i}"


def _module_path(cfg, proj):
    if cfg.arch == "opt":
        return f"self_attn.{proj}" if proj in ("q_proj", "k_proj", "v_proj", "out_proj") else proj
    return f"self_attn.{proj}" if proj in ("q_proj", "k_proj", "v_proj", "o_proj") else f"mlp.{proj}"


def adapter_state_dict(model) -> Dict[str, torch.Tensor]:
    """PEFT key layout: base_model.model.model.layers.{i}.self_attn.q_proj.lora_A.weight [r, in]."""
    cfg = model.cfg
    out = {}
    for i, layer in enumerate(model.layers):
        for key, p in layer.lora_params.items():
            proj, ab = key.rsplit("_", 1)
            name = f"{_layer_prefix(cfg, i)}.{_module_path(cfg, proj)}.lora_{ab}.weight"
            out[name] = p.detach().float().cpu().contiguous()
    return out


def save_adapter(model, path: str):
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    save_file(adapter_state_dict(model), os.path.join(path, "adapter_model.safetensors"), metadata={"format": "pt"})
    with open(os.path.join(path, "adapter_config.json"), "w") as f:
        json.dump(model.lora_config.to_json(), f, indent=2)


def load_adapter(model, path: str):
    from safetensors.torch import load_file

    with open(os.path.join(path, "adapter_config.json")) as f:
        d = json.load(f)
    lc = LoraConfig(**{k: v for k, v in d.items() if k in LoraConfig.__dataclass_fields__})
    if not hasattr(model, "lora_config") or model.lora_config.r != lc.r or \
            sorted(model.lora_config.target_modules) != sorted(lc.target_modules):
        attach_lora(model, lc.r, lc.lora_alpha, lc.target_modules, lc.lora_dropout)
    sd = load_file(os.path.join(path, "adapter_model.safetensors"))
    cfg = model.cfg
    with torch.no_grad():
        for i, layer in enumerate(model.layers):
            for key, p in layer.lora_params.items():
                proj, ab = key.rsplit("_", 1)
                name = f"{_layer_prefix(cfg, i)}.{_module_path(cfg, proj)}.lora_{ab}.weight"
                p.copy_(sd[name].to(p.device, p.dtype))
    model.lora_config = lc
    model.refresh_lora()
    return lc


@torch.no_grad()
def merge_lora(model, sign: float = 1.0):
    """W += sign * s * B A for every adapter (sign=-1 unmerges). Used to export a merged HF model."""
    cfg = model.cfg
    for layer in model.layers:
        for grp_name, grp in layer.lora.items():
            w = _group_weight(layer, cfg, grp_name)
            for a, b, c0, s in zip(grp.a, grp.b, grp.col0, grp.scale):
                delta = (b.float() @ a.float()) * s * sign
                w[c0:c0 + b.shape[0]] += delta.to(w.dtype)


@torch.no_grad()
def merge_and_drop_lora(model):
    """Fold every adapter into its base weight (W += s B A) and remove the adapters, leaving a plain
    model (full fine-tuning after a LoRA stage, merged export)."""
    if getattr(model, "lora_config", None) is None:
        return
    merge_lora(model)
    for layer in model.layers:
        layer.lora = {}
        layer.lora_params = nn.ParameterDict()
    del model.lora_config


def _group_weight(layer, cfg, grp):
    return {"qkv": layer.qkv_w, "o": layer.o_w, "gate_up": getattr(layer, "gate_up_w", None),
            "down": getattr(layer, "down_w", None), "fc1": getattr(layer, "fc1_w", None),
            "fc2": getattr(layer, "fc2_w", None)}[grp]
