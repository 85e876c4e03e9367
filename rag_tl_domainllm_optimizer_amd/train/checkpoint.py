"""Checkpoint / resume.

Writes the reference's three artifacts (reinforcement_learning_optimization_after_rag.py:365-370,
layout SURVEY App. D.3) plus what the reference lacks:

  {prefix}_policy/         HF save_pretrained layout (LoRA merged into the weights, so any HF
                           loader gets the fine-tuned policy)
  {prefix}_tokenizer/      tokenizer.json + tokenizer_config.json + special_tokens_map.json
  {prefix}_value_head.pt   {"weight": [1, H], "bias": [1]} (torch.nn.Linear(H, 1) state_dict)
  {prefix}_adapter/        PEFT adapter (adapter_config.json + adapter_model.safetensors)
  {prefix}_trainer_state/  optimizer moments, step/epoch/best metric, RNG states (resume)

Every directory is written to a temporary name and renamed into place (atomic on one filesystem);
only rank 0 writes.
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Optional

import torch

from ..models import io as mio
from ..models.lora import adapter_state_dict, load_adapter, save_adapter


def _atomic_dir(final: str):
    tmp = final + ".tmp"
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    os.makedirs(tmp)
    return tmp


def _commit(tmp: str, final: str):
    if os.path.exists(final):
        shutil.rmtree(final)
    os.replace(tmp, final)


def merged_hf_state_dict(model, dtype=torch.bfloat16):
    """HF state dict with every LoRA adapter folded in (W + s B A), computed in fp32 on the host."""
    sd = mio.to_hf_state_dict(model, dtype=torch.float32)
    if getattr(model, "lora_config", None) is not None:
        ad = adapter_state_dict(model)
        s = model.lora_config.scaling
        for k in list(ad):
            if ".lora_A.weight" not in k:
                continue
            base = k.replace("base_model.model.", "").replace(".lora_A.weight", ".weight")
            a = ad[k]
            b = ad[k.replace("lora_A", "lora_B")]
            sd[base] = sd[base] + s * (b @ a)
    return {k: v.to(dtype).contiguous() for k, v in sd.items()}


def save_policy(model, path: str, dtype=torch.bfloat16, max_shard_bytes: int = 5 * 1024 ** 3):
    from safetensors.torch import save_file

    tmp = _atomic_dir(path)
    sd = merged_hf_state_dict(model, dtype)
    # reuse save_pretrained's config/generation config writing, then overwrite weights with merged
    mio.save_pretrained(model, tmp, max_shard_bytes=max_shard_bytes, dtype=dtype)
    for f in os.listdir(tmp):
        if f.endswith(".safetensors") or f.endswith(".index.json"):
            os.remove(os.path.join(tmp, f))
    total = sum(t.numel() * t.element_size() for t in sd.values())
    if total <= max_shard_bytes:
        save_file(sd, os.path.join(tmp, "model.safetensors"), metadata={"format": "pt"})
    else:
        shards, cur, cur_b = [], {}, 0
        for k, t in sd.items():
            b = t.numel() * t.element_size()
            if cur and cur_b + b > max_shard_bytes:
                shards.append(cur)
                cur, cur_b = {}, 0
            cur[k] = t
            cur_b += b
        shards.append(cur)
        wm = {}
        for i, sh in enumerate(shards):
            name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
            save_file(sh, os.path.join(tmp, name), metadata={"format": "pt"})
            wm.update({k: name for k in sh})
        with open(os.path.join(tmp, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": total}, "weight_map": wm}, f, indent=2)
    _commit(tmp, path)


def save_checkpoint(prefix: str, model, tokenizer, value_head=None, optimizer=None, trainer_state: Optional[dict] = None,
                    save_full_policy: bool = True):
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    if save_full_policy:
        save_policy(model, f"{prefix}_policy")
    if tokenizer is not None:
        tmp = _atomic_dir(f"{prefix}_tokenizer")
        tokenizer.save_pretrained(tmp)
        _commit(tmp, f"{prefix}_tokenizer")
    if value_head is not None:
        tmpf = f"{prefix}_value_head.pt.tmp"
        torch.save(value_head.reference_state_dict(), tmpf)
        os.replace(tmpf, f"{prefix}_value_head.pt")
    if getattr(model, "lora_config", None) is not None:
        tmp = _atomic_dir(f"{prefix}_adapter")
        save_adapter(model, tmp)
        _commit(tmp, f"{prefix}_adapter")
    if optimizer is not None or trainer_state is not None:
        from safetensors.torch import save_file

        tmp = _atomic_dir(f"{prefix}_trainer_state")
        st = dict(trainer_state or {})
        if optimizer is not None:
            osd = optimizer.state_dict()
            save_file({"exp_avg": osd["exp_avg"].cpu().contiguous(), "exp_avg_sq": osd["exp_avg_sq"].cpu().contiguous(),
                       "params": optimizer.flat.data.cpu().contiguous()},
                      os.path.join(tmp, "optimizer.safetensors"))
            st["optimizer"] = {k: v for k, v in osd.items() if k not in ("exp_avg", "exp_avg_sq", "skipped")}
            st["optimizer"]["skipped"] = int(osd["skipped"])
        rng = st.pop("rng", None)
        if rng is not None:  # safetensors + JSON: nothing in a checkpoint needs unpickling
            from ..utils.seed import rng_state_pack

            rt, rm = rng_state_pack(rng)
            save_file(rt, os.path.join(tmp, "rng.safetensors"))
            with open(os.path.join(tmp, "rng.json"), "w") as f:
                json.dump(rm, f)
        with open(os.path.join(tmp, "state.json"), "w") as f:
            json.dump(st, f, indent=2, default=float)
        _commit(tmp, f"{prefix}_trainer_state")
    print(f"Checkpoint saved at {prefix}")


def load_checkpoint(prefix: str, model, value_head=None, optimizer=None, load_policy_weights: bool = False):
    """Restore adapter (or full policy), value head, optimizer moments and trainer state; returns
    the trainer-state dict (with "rng" when saved). The optimizer keeps pointing at the live
    parameters (they are views of its flat buffer), unlike the reference."""
    st = {}
    if os.path.isdir(f"{prefix}_adapter") and getattr(model, "lora_config", None) is not None:
        load_adapter(model, f"{prefix}_adapter")
    elif load_policy_weights and os.path.isdir(f"{prefix}_policy"):
        mio.load_hf_state_dict(model, mio.read_state_dict(f"{prefix}_policy"))
    if value_head is not None and os.path.exists(f"{prefix}_value_head.pt"):
        value_head.load_reference_state_dict(torch.load(f"{prefix}_value_head.pt", map_location="cpu",
                                                        weights_only=True))
    tsd = f"{prefix}_trainer_state"
    if os.path.isdir(tsd):
        with open(os.path.join(tsd, "state.json")) as f:
            st = json.load(f)
        if optimizer is not None and os.path.exists(os.path.join(tsd, "optimizer.safetensors")):
            from safetensors.torch import load_file

            t = load_file(os.path.join(tsd, "optimizer.safetensors"))
            osd = dict(st.get("optimizer", {}))
            osd.update({"exp_avg": t["exp_avg"], "exp_avg_sq": t["exp_avg_sq"],
                        "skipped": torch.tensor(osd.get("skipped", 0), dtype=torch.int32)})
            optimizer.load_state_dict(osd)
            with torch.no_grad():
                optimizer.flat.data.copy_(t["params"].to(optimizer.flat.data.device))
            if hasattr(optimizer.flat, "refresh_shadow"):  # full fine-tuning: bf16 copies <- master
                optimizer.flat.refresh_shadow()
        if os.path.exists(os.path.join(tsd, "rng.safetensors")):
            from safetensors.torch import load_file

            from ..utils.seed import rng_state_unpack

            with open(os.path.join(tsd, "rng.json")) as f:
                st["rng"] = rng_state_unpack(load_file(os.path.join(tsd, "rng.safetensors")), json.load(f))
    if hasattr(model, "refresh_lora"):
        model.refresh_lora()
    print(f"Checkpoint loaded from {prefix}")
    return st
