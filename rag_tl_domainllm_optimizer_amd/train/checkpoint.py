"""Checkpoint / resume.

Writes the reference's three artifacts (reinforcement_learning_optimization_after_rag.py:365-370,
layout SURVEY App. D.3) plus what the reference lacks:

  {prefix}_policy/         HF save_pretrained layout (LoRA merged into the weights, so any HF
                           loader gets the fine-tuned policy)
  {prefix}_tokenizer/      tokenizer.json + tokenizer_config.json + special_tokens_map.json
  {prefix}_value_head.pt   {"weight": [1, H], "bias": [1]} (torch.nn.Linear(H, 1) state_dict)
                           + the TRL AutoModelForCausalLMWithValueHead names (v_head.summary.*) in
                           {prefix}_value_head.safetensors and inside the policy's weight files
  {prefix}_adapter/        PEFT adapter (adapter_config.json + adapter_model.safetensors)
  {prefix}_trainer_state/  optimizer moments, step / epoch / position in the epoch, best metric,
                           RNG states of EVERY rank (rng_rank{r}.*), the sampler's device RNG counter

The merged policy is produced tensor by tensor: each LoRA-adapted projection is folded on the
device (W + s B A as one GEMM with W as the epilogue's residual input, bf16 out) and copied to the
host, which holds one safetensors shard at a time — never an fp32 copy of the model.
Every directory is written to a temporary name and renamed into place (atomic on one filesystem);
rank 0 writes the artifacts, every other rank only its RNG state.
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


def _lora_group_of(model, native_name: str):
    """LoRAGroup of a fused decoder projection parameter ("layers.{i}.qkv_w" -> layer i, "qkv")."""
    if getattr(model, "lora_config", None) is None or not native_name.startswith("layers."):
        return None
    _, i, pname = native_name.split(".", 2)
    grp = {"qkv_w": "qkv", "o_w": "o", "gate_up_w": "gate_up", "down_w": "down", "fc1_w": "fc1",
           "fc2_w": "fc2"}.get(pname)
    layer = model.layers[int(i)]
    return layer.lora.get(grp) if grp else None


@torch.no_grad()
def iter_merged_hf_tensors(model, dtype=torch.bfloat16):
    """Yield (hf_name, host tensor) in mapping order with every LoRA adapter folded in. A fused
    weight is merged once on its device and sliced into its HF tensors; only one merged projection
    lives at a time."""
    from .. import ops

    params = dict(model.named_parameters())
    cur_name, cur = None, None
    for hf, nat, r0, rn in mio.mapping_for(model):
        t = params[nat].detach()
        grp = _lora_group_of(model, nat)
        if grp is not None:
            if cur_name != nat:
                if grp.a_pad is None or grp.a_pad.device != t.device:
                    grp.refresh(dtype=t.dtype)
                if ops.on_gpu(t) and t.dtype == torch.bfloat16:
                    cur = torch.empty_like(t)
                    ops.native().gemm_big(grp.ub, grp.a_pad, ops.ROW, ops.KMAJ, None, None, None, 0, 0, 1, cur, None, t)
                else:
                    cur = t.float() + grp.ub.float() @ grp.a_pad.float()
                cur_name = nat
            t = cur
        if rn is not None:
            t = t[r0:r0 + rn]
        yield hf, t.to("cpu").to(dtype).contiguous()


def merged_hf_state_dict(model, dtype=torch.bfloat16):
    """HF state dict with every LoRA adapter folded in (W + s B A) — tests / small models; large
    policies stream through ``save_policy``."""
    return dict(iter_merged_hf_tensors(model, dtype))


def save_policy(model, path: str, dtype=torch.bfloat16, max_shard_bytes: int = 5 * 1024 ** 3, extra=None):
    """HF layout (config + generation config + safetensors shards + index). ``extra`` tensors
    (e.g. the TRL value head) are stored with the last shard."""
    from safetensors.torch import save_file

    tmp = _atomic_dir(path)
    mio.save_pretrained(model, tmp, max_shard_bytes=max_shard_bytes, dtype=dtype, write_weights=False)
    shards, cur, cur_b, total = [], {}, 0, 0

    def flush():
        nonlocal cur, cur_b
        name = f"shard-{len(shards):05d}.safetensors"
        save_file(cur, os.path.join(tmp, name), metadata={"format": "pt"})
        shards.append((name, list(cur)))
        cur, cur_b = {}, 0

    for k, t in iter_merged_hf_tensors(model, dtype):
        b = t.numel() * t.element_size()
        if cur and cur_b + b > max_shard_bytes:
            flush()
        cur[k] = t
        cur_b += b
        total += b
    for k, t in (extra or {}).items():
        cur[k] = t.detach().to("cpu").contiguous()
        total += t.numel() * t.element_size()
    flush()
    if len(shards) == 1:
        os.replace(os.path.join(tmp, shards[0][0]), os.path.join(tmp, "model.safetensors"))
    else:
        wm = {}
        for i, (name, keys) in enumerate(shards):
            final = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
            os.replace(os.path.join(tmp, name), os.path.join(tmp, final))
            wm.update({k: final for k in keys})
        with open(os.path.join(tmp, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": total}, "weight_map": wm}, f, indent=2)
    _commit(tmp, path)


def save_rank_rng(prefix: str, rank: int, rng: dict, d: Optional[str] = None):
    """RNG state of one data-parallel rank into {prefix}_trainer_state/rng_rank{rank}.* (or into
    ``d``, the not-yet-committed trainer-state directory of :func:`save_checkpoint_dp`)."""
    from safetensors.torch import save_file

    from ..utils.seed import rng_state_pack

    d = d or f"{prefix}_trainer_state"
    os.makedirs(d, exist_ok=True)
    rt, rm = rng_state_pack(rng)
    save_file(rt, os.path.join(d, f"rng_rank{rank}.safetensors.tmp"))
    os.replace(os.path.join(d, f"rng_rank{rank}.safetensors.tmp"), os.path.join(d, f"rng_rank{rank}.safetensors"))
    with open(os.path.join(d, f"rng_rank{rank}.json"), "w") as f:
        json.dump(rm, f)


def load_rank_rng(prefix: str, rank: int):
    """This rank's saved RNG state. Never another rank's: copying rank 0's streams onto rank r
    would make dropout masks and sampling draws identical across ranks. When rank r's file is
    missing (world-size change, crash between the save barriers) the caller gets None plus a
    warning and keeps its own freshly seeded streams. Rank 0 also reads the single-file layout of
    older checkpoints (``rng.safetensors`` / ``rng.json``)."""
    import warnings

    from safetensors.torch import load_file

    from ..utils.seed import rng_state_unpack

    d = f"{prefix}_trainer_state"
    names = [f"rng_rank{rank}"] + (["rng"] if rank == 0 else [])
    for n in names:
        f = os.path.join(d, f"{n}.safetensors")
        if os.path.exists(f):
            with open(os.path.join(d, f"{n}.json")) as fh:
                return rng_state_unpack(load_file(f), json.load(fh))
    if os.path.isdir(d):
        warnings.warn(f"{d}: no RNG state saved for rank {rank}; this rank keeps its own seeded RNG streams",
                      RuntimeWarning)
    return None


def save_checkpoint_dp(prefix: str, model, tokenizer, value_head=None, optimizer=None,
                       trainer_state: Optional[dict] = None, save_full_policy: bool = True):
    """Data-parallel save (every rank calls it): rank 0 writes the artifacts and the trainer state
    into ``{prefix}_trainer_state.tmp``; after a barrier every other rank adds its RNG state and,
    under ZeRO-1, every rank its optimizer shard to that same directory; rank 0 renames it into
    place only after a second barrier behind all of those writes. A crash anywhere before the
    rename leaves the previous checkpoint of this prefix intact (never a state.json without its
    shards or RNG files)."""
    from ..parallel import barrier
    from ..parallel import info as dist_info
    from ..utils import rng_state

    di = dist_info()
    tmp = f"{prefix}_trainer_state.tmp"
    if di.is_main:
        save_checkpoint(prefix, model, tokenizer, value_head, optimizer, trainer_state, save_full_policy,
                        defer_commit=True)
    barrier()
    if not di.is_main:
        save_rank_rng(prefix, di.rank, rng_state(), d=tmp)
    if optimizer is not None and getattr(optimizer, "sharded", False):
        optimizer.save_shard(tmp)
    barrier()
    if di.is_main:
        _commit(tmp, f"{prefix}_trainer_state")
    barrier()


def save_checkpoint(prefix: str, model, tokenizer, value_head=None, optimizer=None, trainer_state: Optional[dict] = None,
                    save_full_policy: bool = True, defer_commit: bool = False):
    """Rank-local save of every artifact. ``defer_commit``: leave the trainer state in
    ``{prefix}_trainer_state.tmp`` for :func:`save_checkpoint_dp` to complete and rename."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    if save_full_policy:
        save_policy(model, f"{prefix}_policy", extra=value_head.trl_state_dict() if value_head is not None else None)
    if tokenizer is not None:
        tmp = _atomic_dir(f"{prefix}_tokenizer")
        tokenizer.save_pretrained(tmp)
        _commit(tmp, f"{prefix}_tokenizer")
    if value_head is not None:
        tmpf = f"{prefix}_value_head.pt.tmp"
        torch.save(value_head.reference_state_dict(), tmpf)
        os.replace(tmpf, f"{prefix}_value_head.pt")
        from safetensors.torch import save_file

        save_file(value_head.trl_state_dict(), f"{prefix}_value_head.safetensors.tmp", metadata={"format": "pt"})
        os.replace(f"{prefix}_value_head.safetensors.tmp", f"{prefix}_value_head.safetensors")
    if getattr(model, "lora_config", None) is not None:
        tmp = _atomic_dir(f"{prefix}_adapter")
        save_adapter(model, tmp)
        _commit(tmp, f"{prefix}_adapter")
    if optimizer is not None or trainer_state is not None:
        from safetensors.torch import save_file

        tmp = _atomic_dir(f"{prefix}_trainer_state")
        st = dict(trainer_state or {})
        if optimizer is not None:
            # how the optimizer state is laid out: 0 = one optimizer.safetensors, N = ZeRO-1 shards
            # of a world of N (load_checkpoint refuses a mismatching optimizer)
            st["zero_world"] = int(optimizer.world) if getattr(optimizer, "sharded", False) else 0
        if optimizer is not None and getattr(optimizer, "sharded", False):
            # ZeRO-1: metadata here, tensors per rank (ZeroAdamW.save_shard, called on every rank)
            osd = optimizer.state_dict()
            st["optimizer"] = {k: v for k, v in osd.items() if k != "skipped"}
            st["optimizer"]["skipped"] = int(osd["skipped"])
        elif optimizer is not None:
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
            save_file(rt, os.path.join(tmp, "rng_rank0.safetensors"))
            with open(os.path.join(tmp, "rng_rank0.json"), "w") as f:
                json.dump(rm, f)
        with open(os.path.join(tmp, "state.json"), "w") as f:
            json.dump(st, f, indent=2, default=float)
        if not defer_commit:
            _commit(tmp, f"{prefix}_trainer_state")
    print(f"Checkpoint saved at {prefix}")


def _check_optimizer_layout(tsd: str, st: dict, optimizer):
    """Refuse to resume an optimizer from a checkpoint whose optimizer state has another layout:
    ZeRO-1 shards of a different world size, shards into an unsharded optimizer or the reverse —
    silently skipping the moments (and, under full fine-tuning, the fp32 masters that carry the
    weights) would resume from the initial weights with a restored step counter."""
    import glob

    sharded = bool(getattr(optimizer, "sharded", False))
    world = int(getattr(optimizer, "world", 1)) if sharded else 0
    if "zero_world" in st:
        zw = int(st["zero_world"])
    elif glob.glob(os.path.join(tsd, "optimizer_zero*_rank*.safetensors")):  # written before "zero_world"
        zw = -1
    else:
        zw = 0 if os.path.exists(os.path.join(tsd, "optimizer.safetensors")) or "optimizer" not in st else -2
    if zw == -2:
        raise RuntimeError(f"{tsd}: state.json records optimizer state but optimizer.safetensors is missing")
    if zw == 0 and sharded:
        raise RuntimeError(f"{tsd}: unsharded optimizer checkpoint, but the optimizer is ZeRO-1 sharded over "
                           f"{world} ranks; resume with zero=False (or world 1)")
    if zw != 0 and not sharded:
        raise RuntimeError(f"{tsd}: ZeRO-1 sharded optimizer checkpoint (world {zw if zw > 0 else '?'}), but the "
                           f"optimizer is unsharded; resume with zero=True at the saving world size")
    if zw > 0 and zw != world:
        raise RuntimeError(f"{tsd}: ZeRO-1 shards of world {zw}, resuming at world {world}")


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
        if optimizer is not None:
            _check_optimizer_layout(tsd, st, optimizer)
        if optimizer is not None and getattr(optimizer, "sharded", False):
            osd = dict(st.get("optimizer", {}))
            optimizer.load_state_dict(osd)
            optimizer.load_shard(tsd)  # collective: every rank loads its shard, bf16 copy all-gathered
        elif optimizer is not None and os.path.exists(os.path.join(tsd, "optimizer.safetensors")):
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
        from ..parallel import info as dist_info

        rng = load_rank_rng(prefix, dist_info().rank)
        if rng is not None:
            st["rng"] = rng
    if hasattr(model, "refresh_lora"):
        model.refresh_lora()
    print(f"Checkpoint loaded from {prefix}")
    return st
