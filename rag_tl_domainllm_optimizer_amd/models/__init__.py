"""Model zoo: Llama-2 / Mistral / OPT decoders, BERT / MPNet sentence encoders, LoRA, value head."""
from __future__ import annotations

import os

import torch

from .config import PRESETS, ModelConfig, resolve_preset  # noqa: F401
from .decoder import CausalLM, fast_random_init_, pack_enabled, packed_index  # noqa: F401
from .encoder import SentenceEncoder  # noqa: F401
from .lora import LoraConfig, attach_lora, load_adapter, merge_lora, save_adapter  # noqa: F401
from .value_head import ValueHead  # noqa: F401
from . import io  # noqa: F401


def build_model(name_or_path: str, device="cpu", dtype=None, seed: int = 0, fast_init: bool = False):
    """Load a local HF-format directory, or build a random-init preset (``"mistral-7b:random"``)."""
    if dtype is None:
        dtype = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
    if os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "config.json")):
        return io.from_pretrained(name_or_path, device=device, dtype=dtype)
    cfg = resolve_preset(name_or_path)
    if cfg is None:
        raise ValueError(f"unknown model {name_or_path!r}: not a local HF dir and not a preset ({sorted(PRESETS)})")
    cls = CausalLM if cfg.is_decoder else SentenceEncoder
    if fast_init:
        m = cls(cfg, device=device, dtype=dtype, init=False)
        fast_random_init_(m, seed, cfg.initializer_range)
        return m
    return cls(cfg, device=device, dtype=dtype, init=True, seed=seed)
